// VALU issue rates on gfx950 with several waves per SIMD: v_fma_f64 vs v_fma_f32 vs v_pk_fma_f32,
// one block of T threads on one CU (T/256 waves per SIMD), 8 independent chains per lane.
#include <hip/hip_runtime.h>
#include <cstdio>
template <typename T>
__global__ void k(T* out, unsigned long long* t, int iters) {
  T acc[8];
  for (int c = 0; c < 8; c++) acc[c] = (T)(c + threadIdx.x);
  const T a = (T)1.0000001, b = (T)1e-7;
  __syncthreads();
  unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; i++)
#pragma unroll
    for (int c = 0; c < 8; c++) acc[c] = acc[c] * a + b;
  __syncthreads();
  unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  T s = 0;
  for (int c = 0; c < 8; c++) s += acc[c];
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) *t = t1 - t0;
}
typedef float f2 __attribute__((ext_vector_type(2)));
__global__ void kp(float* out, unsigned long long* t, int iters) {
  f2 acc[8];
  for (int c = 0; c < 8; c++) acc[c] = f2{(float)c, (float)threadIdx.x};
  const f2 a = {1.0000001f, 1.0000001f}, b = {1e-7f, 1e-7f};
  __syncthreads();
  unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; i++)
#pragma unroll
    for (int c = 0; c < 8; c++) acc[c] = __builtin_elementwise_fma(acc[c], a, b);
  __syncthreads();
  unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  float s = 0;
  for (int c = 0; c < 8; c++) s += acc[c].x + acc[c].y;
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) *t = t1 - t0;
}
int main() {
  void* o;
  unsigned long long* t;
  (void)hipMalloc(&o, 1024 * 8);
  (void)hipMalloc(&t, 8);
  const int it = 20000;
  for (int T : {256, 512, 1024}) {
    unsigned long long h;
    hipLaunchKernelGGL(k<double>, dim3(1), dim3(T), 0, 0, (double*)o, t, it);
    hipLaunchKernelGGL(k<double>, dim3(1), dim3(T), 0, 0, (double*)o, t, it);
    (void)hipMemcpy(&h, t, 8, hipMemcpyDeviceToHost);
    const double w = T / 256.0;  // waves per SIMD
    printf("T=%4d (%.0f waves/SIMD) v_fma_f64: %.2f ns per wave-instr per SIMD", T, w, h * 10.0 / (it * 8.0 * w));
    hipLaunchKernelGGL(k<float>, dim3(1), dim3(T), 0, 0, (float*)o, t, it);
    hipLaunchKernelGGL(k<float>, dim3(1), dim3(T), 0, 0, (float*)o, t, it);
    (void)hipMemcpy(&h, t, 8, hipMemcpyDeviceToHost);
    printf(" | v_fma_f32: %.2f", h * 10.0 / (it * 8.0 * w));
    hipLaunchKernelGGL(kp, dim3(1), dim3(T), 0, 0, (float*)o, t, it);
    hipLaunchKernelGGL(kp, dim3(1), dim3(T), 0, 0, (float*)o, t, it);
    (void)hipMemcpy(&h, t, 8, hipMemcpyDeviceToHost);
    printf(" | v_pk_fma_f32: %.2f\n", h * 10.0 / (it * 8.0 * w));
  }
  return 0;
}
