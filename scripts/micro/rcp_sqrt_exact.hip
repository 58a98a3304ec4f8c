// Exhaustive checks on gfx950 for the short reciprocal and square root proj_occlusion's LM step uses inside a
// guarded range (csrc/matching.hip rcp_rn / sqrt_rn):
//   rcp1(x) = fma(fma(-x, y, 1), y, y), y = v_rcp_f32(x)          vs IEEE 1.0f / x     for every |x| in [2^-125, 2^126)
//   sqrt_c(s) = v_sqrt_f32 + the +-1 ulp residual correction     vs IEEE sqrtf(s)     for every s in [2^-95, 2^128)
//   rcp1(sqrt_c(s))                                              vs 1.0f / sqrtf(s)   on the same s
// Every bit pattern of the range, both signs for the reciprocal; bitwise equality.
// build: hipcc --offload-arch=gfx950 -O3 -o bin/rcp_sqrt_exact rcp_sqrt_exact.hip
#include <hip/hip_runtime.h>

#include <cstdio>

__device__ __forceinline__ float rcp1(float x) {
  const float y = __builtin_amdgcn_rcpf(x);
  const float e = __builtin_fmaf(-x, y, 1.0f);
  return __builtin_fmaf(e, y, y);
}

__device__ __forceinline__ float sqrt_c(float s) {
  const float r = __builtin_amdgcn_sqrtf(s);
  const float rm = __uint_as_float(__float_as_uint(r) - 1u), rp = __uint_as_float(__float_as_uint(r) + 1u);
  const float em = __builtin_fmaf(-rm, r, s), ep = __builtin_fmaf(-rp, r, s);
  float o = em <= 0.0f ? rm : r;
  o = ep > 0.0f ? rp : o;
  return o;
}

__global__ void check(unsigned hi, unsigned long long* bad, unsigned* first) {
  // blockIdx.x * 256 + threadIdx.x: the low 24 bits of a pattern; hi: the top 8 bits
  const unsigned bits = (hi << 24) | (blockIdx.x * 256u + threadIdx.x);
  const unsigned ex = (bits >> 23) & 0xff;
  const float x = __uint_as_float(bits);
  if (ex >= 2 && ex <= 252) {
    if (__float_as_uint(rcp1(x)) != __float_as_uint(1.0f / x)) {
      atomicAdd(&bad[0], 1ull);
      atomicCAS(&first[0], 0xffffffffu, bits);
    }
  }
  if ((bits >> 31) == 0 && ex >= 32 && ex <= 254) {
    const float a = sqrtf(x);
    const float b = sqrt_c(x);
    if (__float_as_uint(a) != __float_as_uint(b)) {
      atomicAdd(&bad[1], 1ull);
      atomicCAS(&first[1], 0xffffffffu, bits);
    }
    if (__float_as_uint(1.0f / a) != __float_as_uint(rcp1(b))) {
      atomicAdd(&bad[2], 1ull);
      atomicCAS(&first[2], 0xffffffffu, bits);
    }
  }
}

int main() {
  unsigned long long* bad;
  unsigned* first;
  (void)hipMalloc(&bad, 3 * 8);
  (void)hipMalloc(&first, 3 * 4);
  (void)hipMemset(bad, 0, 3 * 8);
  (void)hipMemset(first, 0xff, 3 * 4);
  for (unsigned hi = 0; hi < 256; hi++) hipLaunchKernelGGL(check, dim3(65536), dim3(256), 0, 0, hi, bad, first);
  unsigned long long hb[3] = {0, 0, 0};
  unsigned hf[3] = {0, 0, 0};
  (void)hipMemcpy(hb, bad, sizeof(hb), hipMemcpyDeviceToHost);
  (void)hipMemcpy(hf, first, sizeof(hf), hipMemcpyDeviceToHost);
  const char* name[3] = {"rcp1 vs 1.0f/x, |x| in [2^-125, 2^126)", "sqrt_c vs sqrtf, s in [2^-95, 2^128)",
                         "rcp1(sqrt_c) vs 1.0f/sqrtf, same s"};
  for (int k = 0; k < 3; k++) {
    printf("%s: %llu mismatches", name[k], hb[k]);
    if (hb[k]) printf(" (first 0x%08x)", hf[k]);
    printf("\n");
  }
  return (hb[0] || hb[1] || hb[2]) ? 1 : 0;
}
