// Semantics check of the DPP / permlane primitives used by the BA pivot chain (gfx950):
// replicate row 0 (lanes 0..15) of a double across the 4 rows with v_permlane32_swap + v_permlane16_swap,
// then v_fmac_f64_dpp row_newbcast:c.
#include <hip/hip_runtime.h>
#include <cstdio>
__device__ __forceinline__ double rep_row0(double v) {
  int2 a = *reinterpret_cast<int2*>(&v), b = a;
  asm volatile("s_nop 1\n v_permlane32_swap_b32 %0, %1\n s_nop 1" : "+v"(a.x), "+v"(b.x));
  asm volatile("s_nop 1\n v_permlane32_swap_b32 %0, %1\n s_nop 1" : "+v"(a.y), "+v"(b.y));
  int2 c = a;
  asm volatile("s_nop 1\n v_permlane16_swap_b32 %0, %1\n s_nop 1" : "+v"(a.x), "+v"(c.x));
  asm volatile("s_nop 1\n v_permlane16_swap_b32 %0, %1\n s_nop 1" : "+v"(a.y), "+v"(c.y));
  return *reinterpret_cast<double*>(&a);
}
__global__ void k(double* o) {
  const int l = threadIdx.x;
  const double x = 100.0 + l;
  const double rep = rep_row0(x);
  double acc = 0.5;
  const double y = 2.0;
  asm volatile("s_nop 2\n v_fmac_f64_dpp %0, %1, %2 row_newbcast:5 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(rep), "v"(y));
  o[l] = rep;
  o[64 + l] = acc;
}
int main() {
  double* d;
  (void)hipMalloc(&d, 128 * 8);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  double h[128];
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  int bad = 0;
  for (int l = 0; l < 64; l++) {
    if (h[l] != 100.0 + (l % 16)) bad++;
    if (h[64 + l] != 0.5 + 2.0 * 105.0) bad++;
  }
  printf("rep lanes: %g %g %g %g | fmac_dpp lanes: %g %g %g %g | bad=%d\n", h[0], h[17], h[35], h[63], h[64], h[80],
         h[100], h[127], bad);
  return bad != 0;
}
