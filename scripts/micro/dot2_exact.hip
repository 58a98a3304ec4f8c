// v_dot2c_f32_f16 semantics on gfx950 (the refine screen's bound assumes them): for random half pairs, including
// subnormal and tiny operands, the dot2 result a0*b0 + a1*b1 + acc is compared with the exact fp64 value. Prints the
// largest error in units of 2^-24 * (|a0 b0| + |a1 b1| + |acc|) (<= 2 if at most two fp32 roundings) and the count
// of results that differ from exact by more than that, which a flushed subnormal would produce.
// build: hipcc --offload-arch=gfx950 -O3 -o dot2_exact dot2_exact.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

typedef _Float16 h2 __attribute__((ext_vector_type(2)));

__global__ void k(const h2* a, const h2* b, const float* acc, float* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = __builtin_amdgcn_fdot2(a[i], b[i], acc[i], false);
}

int main() {
  const int n = 1 << 22;
  std::mt19937 g(7);
  std::vector<h2> a(n), b(n);
  std::vector<float> acc(n), out(n);
  std::uniform_real_distribution<float> U(-1.f, 1.f);
  std::uniform_int_distribution<int> E(-30, 2);
  for (int i = 0; i < n; i++) {
    auto r = [&]() { return (_Float16)(U(g) * std::ldexp(1.0f, E(g))); };
    a[i] = h2{r(), r()};
    b[i] = h2{r(), r()};
    acc[i] = (i % 4 == 0) ? 0.f : U(g) * std::ldexp(1.0f, E(g) - 4);
  }
  h2 *da, *db;
  float *dc, *dout;
  (void)hipMalloc(&da, n * 4);
  (void)hipMalloc(&db, n * 4);
  (void)hipMalloc(&dc, n * 4);
  (void)hipMalloc(&dout, n * 4);
  (void)hipMemcpy(da, a.data(), n * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(db, b.data(), n * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(dc, acc.data(), n * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3((n + 255) / 256), dim3(256), 0, 0, da, db, dc, dout, n);
  (void)hipMemcpy(out.data(), dout, n * 4, hipMemcpyDeviceToHost);
  double worst = 0, worst_n = 0, max_excess = 0;
  long bad = 0, sub = 0, bad_n = 0, shown = 0;
  for (int i = 0; i < n; i++) {
    const double p0 = (double)a[i].x * (double)b[i].x, p1 = (double)a[i].y * (double)b[i].y;
    const double ex = p0 + p1 + (double)acc[i];
    const double mag = std::fabs(p0) + std::fabs(p1) + std::fabs((double)acc[i]);
    const double err = std::fabs((double)out[i] - ex);
    const double u = mag > 0 ? err / (mag * std::ldexp(1.0, -24)) : (err > 0 ? 1e30 : 0);
    if (std::fabs((double)a[i].x) < 6.1e-5 || std::fabs((double)b[i].x) < 6.1e-5) sub++;
    const bool anysub = std::fabs((double)a[i].x) < 6.1035e-5 || std::fabs((double)b[i].x) < 6.1035e-5 ||
                        std::fabs((double)a[i].y) < 6.1035e-5 || std::fabs((double)b[i].y) < 6.1035e-5;
    const double excess = err - 3.0 * std::ldexp(1.0, -24) * mag;
    if (excess > max_excess) max_excess = excess;
    if (u > worst && mag > 1e-37) worst = u;
    if (!anysub && u > worst_n && mag > 1e-37) worst_n = u;
    if (u > 2.0 && err > 1e-37) {
      bad++;
      if (!anysub) bad_n++;
      if (shown < 12 && (!anysub || shown < 4)) {
        shown++;
        printf("  a=(%g,%g) b=(%g,%g) acc=%g exact=%.9g got=%.9g sub=%d\n", (double)a[i].x, (double)a[i].y,
               (double)b[i].x, (double)b[i].y, (double)acc[i], ex, (double)out[i], (int)anysub);
      }
    }
  }
  printf("dot2c: n=%d (subnormal-operand cases %ld), worst error %.3f x 2^-24 * magnitude, %ld beyond 2 roundings;"
         " all operands normal: worst %.3f, %ld beyond\n", n, sub, worst, bad, worst_n, bad_n);
  printf("largest absolute error beyond 3 x 2^-24 * magnitude: %.3e (2^%.1f)\n", max_excess,
         max_excess > 0 ? std::log2(max_excess) : -999.0);
  return 0;
}
