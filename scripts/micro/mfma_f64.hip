// Micro-benchmark: v_mfma_f64_16x16x4f64 issue/latency and v_fma_f64 rate on one wave (gfx950).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4v __attribute__((ext_vector_type(4)));
template <int CH>
__global__ void k_mfma(double* out, unsigned long long* t, int iters) {
  d4v acc[CH];
  for (int c = 0; c < CH; c++) acc[c] = d4v{0, 0, 0, 0};
  double a = threadIdx.x * 1e-3, b = 1.0 - a;
  unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; i++)
#pragma unroll
    for (int c = 0; c < CH; c++) acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[c], 0, 0, 0);
  unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  double s = 0;
  for (int c = 0; c < CH; c++) s += acc[c][0] + acc[c][3];
  out[blockIdx.x * 64 + threadIdx.x] = s;
  if (threadIdx.x == 0) t[blockIdx.x] = t1 - t0;
}
template <int CH>
__global__ void k_fma(double* out, unsigned long long* t, int iters) {
  double acc[CH];
  for (int c = 0; c < CH; c++) acc[c] = c;
  double a = threadIdx.x * 1e-3, b = 1.0 - a;
  unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; i++)
#pragma unroll
    for (int c = 0; c < CH; c++) acc[c] = fma(acc[c], a, b);
  unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  double s = 0;
  for (int c = 0; c < CH; c++) s += acc[c];
  out[blockIdx.x * 64 + threadIdx.x] = s;
  if (threadIdx.x == 0) t[blockIdx.x] = t1 - t0;
}
template <typename K>
void run(const char* name, K kern, int per_iter, double* o, unsigned long long* t, int iters) {
  hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, o, t, iters);
  hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, o, t, iters);
  unsigned long long h;
  hipMemcpy(&h, t, 8, hipMemcpyDeviceToHost);
  const double ns = h * 10.0;  // 100 MHz
  printf("%-28s %8.2f ns per instruction (one wave)\n", name, ns / (double)(iters * per_iter));
}
int main() {
  double* o;
  unsigned long long* t;
  hipMalloc(&o, 64 * 8 * 8);
  hipMalloc(&t, 64);
  const int it = 20000;
  run("mfma_f64 dependent chain", k_mfma<1>, 1, o, t, it);
  run("mfma_f64 2 chains", k_mfma<2>, 2, o, t, it);
  run("mfma_f64 4 chains", k_mfma<4>, 4, o, t, it);
  run("mfma_f64 8 chains", k_mfma<8>, 8, o, t, it);
  run("v_fma_f64 dependent", k_fma<1>, 1, o, t, it);
  run("v_fma_f64 8 chains", k_fma<8>, 8, o, t, it);
  return 0;
}
