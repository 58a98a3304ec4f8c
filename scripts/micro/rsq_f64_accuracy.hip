// Accuracy of the gfx950 v_rsq_f64 / v_rcp_f64 estimates (and after one Newton step) vs correctly rounded
// 1/sqrt(d), 1/d, over d in [1e-6, 1e6] (log-uniform).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
__global__ void k(const double* d, double* o, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double x = d[i];
  const double y = __builtin_amdgcn_rsq(x);
  const double y1 = fma(y, fma(-0.5 * x * y, y, 0.5), y);
  const double r = __builtin_amdgcn_rcp(x);
  const double r1 = fma(r, fma(-x, r, 1.0), r);
  o[4 * i] = y; o[4 * i + 1] = y1; o[4 * i + 2] = r; o[4 * i + 3] = r1;
}
int main() {
  const int n = 1 << 20;
  double *hd = new double[n], *ho = new double[4 * n], *dd, *dout;
  unsigned long long s = 12345;
  for (int i = 0; i < n; i++) {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    const double u = (double)(s >> 11) / 9007199254740992.0;
    hd[i] = pow(10.0, -6.0 + 12.0 * u);
  }
  (void)hipMalloc(&dd, n * 8); (void)hipMalloc(&dout, 4 * n * 8);
  (void)hipMemcpy(dd, hd, n * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, dd, dout, n);
  (void)hipMemcpy(ho, dout, 4 * n * 8, hipMemcpyDeviceToHost);
  double e[4] = {0, 0, 0, 0};
  for (int i = 0; i < n; i++) {
    const double rs = 1.0 / sqrt(hd[i]), rc = 1.0 / hd[i];
    e[0] = fmax(e[0], fabs(ho[4 * i] / rs - 1)); e[1] = fmax(e[1], fabs(ho[4 * i + 1] / rs - 1));
    e[2] = fmax(e[2], fabs(ho[4 * i + 2] / rc - 1)); e[3] = fmax(e[3], fabs(ho[4 * i + 3] / rc - 1));
  }
  printf("max rel err: rsq %.3g  rsq+1NR %.3g  rcp %.3g  rcp+1NR %.3g\n", e[0], e[1], e[2], e[3]);
  return 0;
}
