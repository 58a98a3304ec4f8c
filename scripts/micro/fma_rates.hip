// VALU issue rates on gfx950 (MI355X) per instruction, at 1, 2 and 4 waves per SIMD: the measured constants
// behind the issue floors in DESIGN.md §4 (refine: v_pk_mul_f16 / v_add_f16 / v_cvt_f16_f32 / v_pk_add_f16;
// BA linearisation: v_pk_fma_f32 / v_fma_f32; the factorisation: v_fma_f64).
//
// One kernel per instruction: every lane runs `iters` x 8 independent instances (8 accumulators, inline asm so
// the compiler can neither fold nor reorder them), timed by s_memtime (shader clock) between two barriers.
// Grid: one block of T threads per CU on every CU (256 blocks), T = 256 / 512 / 1024 = 1 / 2 / 4 waves per SIMD.
// cycles per wave-instruction per SIMD = dcycles / (waves_per_SIMD x iters x 8); the median block is printed.
// build: hipcc --offload-arch=gfx950 -O3 -o fma_rates fma_rates.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define BODY8(ASM)                          \
  asm volatile(ASM : "+v"(r0) : "v"(k)); \
  asm volatile(ASM : "+v"(r1) : "v"(k)); \
  asm volatile(ASM : "+v"(r2) : "v"(k)); \
  asm volatile(ASM : "+v"(r3) : "v"(k)); \
  asm volatile(ASM : "+v"(r4) : "v"(k)); \
  asm volatile(ASM : "+v"(r5) : "v"(k)); \
  asm volatile(ASM : "+v"(r6) : "v"(k)); \
  asm volatile(ASM : "+v"(r7) : "v"(k));

#define KERNEL(NAME, T, ASM)                                                                          \
  __global__ void NAME(T* out, unsigned long long* cyc, int iters) {                                  \
    T r0 = (T)threadIdx.x, r1 = r0 + (T)1, r2 = r0 + (T)2, r3 = r0 + (T)3, r4 = r0 + (T)4, r5 = r0 + (T)5, \
      r6 = r0 + (T)6, r7 = r0 + (T)7;                                                                 \
    const T k = (T)1;                                                                                 \
    __syncthreads();                                                                                  \
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();                                       \
    const unsigned long long r0t = __builtin_amdgcn_s_memrealtime();                                  \
    for (int i = 0; i < iters; i++) {                                                                 \
      BODY8(ASM)                                                                                      \
    }                                                                                                 \
    __syncthreads();                                                                                  \
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();                                       \
    const unsigned long long r1t = __builtin_amdgcn_s_memrealtime();                                  \
    out[blockIdx.x * blockDim.x + threadIdx.x] = r0 + r1 + r2 + r3 + r4 + r5 + r6 + r7;               \
    if (threadIdx.x == 0) {                                                                           \
      cyc[blockIdx.x] = t1 - t0;                                                                      \
      cyc[gridDim.x + blockIdx.x] = r1t - r0t;                                                        \
    }                                                                                                 \
  }

// 32-bit operand instructions (f16 / packed f16 / packed-f32 halves live in 32-bit VGPRs)
KERNEL(k_fma_f32, float, "v_fma_f32 %0, %0, %1, %1")
KERNEL(k_add_f32, float, "v_add_f32 %0, %0, %1")
KERNEL(k_pk_mul_f16, unsigned, "v_pk_mul_f16 %0, %0, %1")
KERNEL(k_pk_add_f16, unsigned, "v_pk_add_f16 %0, %0, %1")
KERNEL(k_pk_fma_f16, unsigned, "v_pk_fma_f16 %0, %0, %1, %1")
KERNEL(k_add_f16, unsigned, "v_add_f16 %0, %0, %1")
KERNEL(k_mul_f16, unsigned, "v_mul_f16 %0, %0, %1")
KERNEL(k_cvt_f16_f32, unsigned, "v_cvt_f16_f32 %0, %1")
KERNEL(k_cvt_f32_f16, unsigned, "v_cvt_f32_f16 %0, %1")
KERNEL(k_perm_b32, unsigned, "v_perm_b32 %0, %0, %1, %1")
// encodings of the same f16 add: VOP3 (e64) and SDWA (high-half source, high-half destination with the low half kept)
KERNEL(k_add_f16_e64, unsigned, "v_add_f16_e64 %0, %0, %1")
KERNEL(k_add_f16_sdwa_s1, unsigned, "v_add_f16_sdwa %0, %0, %1 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_1")
KERNEL(k_add_f16_sdwa_d1, unsigned, "v_add_f16_sdwa %0, %0, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1")
KERNEL(k_pack_b32_f16, unsigned, "v_pack_b32_f16 %0, %0, %1")
KERNEL(k_add_f32_e64, float, "v_add_f32_e64 %0, %0, %1")
// the odd-channel add of a half-sum chain as a 3-operand f16 op reading the high half (VOP3 op_sel), the
// multiplier an inline 1.0: s = fma(p.hi, 1.0, s) (v_add_f16_e64 takes no op_sel on gfx950)
KERNEL(k_fma_f16_hi1, unsigned, "v_fma_f16 %0, %1, 1.0, %0 op_sel:[1,0,0,0]")
KERNEL(k_mad_f16_hi1, unsigned, "v_mad_f16 %0, %1, 1.0, %0 op_sel:[1,0,0,0]")
KERNEL(k_fma_f16_v3, unsigned, "v_fma_f16 %0, %1, %1, %0")
KERNEL(k_pk_add_f16_sel, unsigned, "v_pk_add_f16 %0, %0, %1 op_sel:[0,1] op_sel_hi:[1,1]")
// 64-bit operands
KERNEL(k_pk_fma_f32, double, "v_pk_fma_f32 %0, %0, %1, %1")
KERNEL(k_pk_mul_f32, double, "v_pk_mul_f32 %0, %0, %1")
KERNEL(k_fma_f64, double, "v_fma_f64 %0, %0, %1, %1")
KERNEL(k_add_f64, double, "v_add_f64 %0, %0, %1")
// refine screening (bit-exact screened refine): fp32 dot of two half pairs, VOP2 accumulate and VOP3P forms
KERNEL(k_dot2c_f32_f16, float, "v_dot2c_f32_f16 %0, %1, %1")
KERNEL(k_dot2_f32_f16, float, "v_dot2_f32_f16 %0, %1, %1, %0")
KERNEL(k_max3_f32, float, "v_max3_f32 %0, %0, %1, %1")

typedef void (*kfn)(void*, unsigned long long*, int);

int main() {
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int blocks = cus;
  void* out;
  unsigned long long* cyc;
  (void)hipMalloc(&out, (size_t)blocks * 1024 * 8);
  (void)hipMalloc(&cyc, (size_t)blocks * 16);
  struct K {
    const char* name;
    const void* fn;
    int size;
  };
  const K ks[] = {
      {"v_fma_f32", (const void*)k_fma_f32, 4},       {"v_add_f32", (const void*)k_add_f32, 4},
      {"v_pk_fma_f32", (const void*)k_pk_fma_f32, 8}, {"v_pk_mul_f32", (const void*)k_pk_mul_f32, 8},
      {"v_pk_mul_f16", (const void*)k_pk_mul_f16, 4}, {"v_pk_add_f16", (const void*)k_pk_add_f16, 4},
      {"v_pk_fma_f16", (const void*)k_pk_fma_f16, 4}, {"v_add_f16", (const void*)k_add_f16, 4},
      {"v_mul_f16", (const void*)k_mul_f16, 4},       {"v_cvt_f16_f32", (const void*)k_cvt_f16_f32, 4},
      {"v_cvt_f32_f16", (const void*)k_cvt_f32_f16, 4}, {"v_perm_b32", (const void*)k_perm_b32, 4},
      {"v_add_f16_e64", (const void*)k_add_f16_e64, 4}, {"v_add_f16_sdwa_s1", (const void*)k_add_f16_sdwa_s1, 4},
      {"v_add_f16_sdwa_d1", (const void*)k_add_f16_sdwa_d1, 4}, {"v_pack_b32_f16", (const void*)k_pack_b32_f16, 4},
      {"v_add_f32_e64", (const void*)k_add_f32_e64, 4},
      {"v_fma_f16_hi1", (const void*)k_fma_f16_hi1, 4}, {"v_mad_f16_hi1", (const void*)k_mad_f16_hi1, 4},
      {"v_fma_f16_v3", (const void*)k_fma_f16_v3, 4}, {"v_pk_add_f16_sel", (const void*)k_pk_add_f16_sel, 4},
      {"v_fma_f64", (const void*)k_fma_f64, 8},       {"v_add_f64", (const void*)k_add_f64, 8},
      {"v_dot2c_f32_f16", (const void*)k_dot2c_f32_f16, 4}, {"v_dot2_f32_f16", (const void*)k_dot2_f32_f16, 4},
      {"v_max3_f32", (const void*)k_max3_f32, 4},
  };
  const int iters = 4000;
  printf("gfx950 VALU issue cost per wave64 instruction per SIMD (median over %d CUs, one block per CU):\n"
         "s_memtime cycles | ns (s_memrealtime, 100 MHz) | cycles at 2.4 GHz from the ns\n", blocks);
  printf("%-18s %26s %26s %26s\n", "instruction", "1 w/SIMD", "2 w/SIMD", "4 w/SIMD");
  std::vector<unsigned long long> h(2 * blocks), hc(blocks), hr(blocks);
  for (const K& k : ks) {
    printf("%-18s", k.name);
    for (int T : {256, 512, 1024}) {
      void* args[] = {&out, &cyc, (void*)&iters};
      (void)args;
      for (int rep = 0; rep < 2; rep++) {
        void* a[] = {&out, &cyc, const_cast<int*>(&iters)};
        (void)hipLaunchKernel(k.fn, dim3(blocks), dim3(T), a, 0, 0);
      }
      (void)hipDeviceSynchronize();
      (void)hipMemcpy(h.data(), cyc, (size_t)blocks * 16, hipMemcpyDeviceToHost);
      for (int b = 0; b < blocks; b++) {
        hc[b] = h[b];
        hr[b] = h[blocks + b];
      }
      std::sort(hc.begin(), hc.end());
      std::sort(hr.begin(), hr.end());
      const double w = T / 256.0, n = w * iters * 8.0;
      const double ns = (double)hr[blocks / 2] * 10.0 / n;
      printf("   %7.2f | %6.3f | %6.2f", (double)hc[blocks / 2] / n, ns, ns * 2.4);
    }
    printf("\n");
  }
  return 0;
}
