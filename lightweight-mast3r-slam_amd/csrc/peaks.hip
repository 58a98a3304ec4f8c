// Measured-peak probe for the bench's roofline lines ("re-measure with a STREAM-like copy
// and an FMA loop on the box"). Not on the tracking / BA path.
#include <hip/hip_runtime.h>

namespace m3s {

// 8 independent v_fma_f32 chains per lane, `iters` rounds; 4 waves per SIMD at the launch below.
__global__ void __launch_bounds__(256) peak_fma_f32_kernel(float* __restrict__ out, int iters) {
  float acc[8];
#pragma unroll
  for (int c = 0; c < 8; c++) acc[c] = (float)(threadIdx.x + c);
  const float a = 1.0000001f, b = 1e-7f;
  for (int i = 0; i < iters; i++)
#pragma unroll
    for (int c = 0; c < 8; c++) acc[c] = fmaf(acc[c], a, b);
  float s = 0.0f;
#pragma unroll
  for (int c = 0; c < 8; c++) s += acc[c];
  if (s == 1234.5f) out[threadIdx.x] = s;  // keeps the loop alive; never true for these inputs
}

}  // namespace m3s

// flops = blocks * 256 * iters * 8 * 2
extern "C" hipError_t m3s_launch_peak_fma_f32(float* out, int blocks, int iters, hipStream_t s) {
  hipLaunchKernelGGL(m3s::peak_fma_f32_kernel, dim3(blocks), dim3(256), 0, s, out, iters);
  return hipGetLastError();
}
