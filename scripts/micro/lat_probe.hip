// Latency probe for the BA factor kernel design (one workgroup of 16 waves on one CU):
// dependent global load (L2-warm), store + vmcnt(0), workgroup barrier, LDS round trip, dependent
// fp64 FMA, v_rsq_f64. Times from s_memrealtime (100 MHz) and s_memtime (shader clock).
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void __launch_bounds__(1024) probe(double* buf, int* idx, unsigned long long* out, int iters) {
  __shared__ double lds[1024];
  __shared__ int ldsi[64];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  // warm: chain of indices in buf region
  if (t < 64) ldsi[t] = t;
  __syncthreads();
  unsigned long long r0, r1, c0, c1;
  // 1. dependent global loads (pointer chase over idx), wave 0 lane 0
  if (t == 0) {
    int p = 0;
    for (int i = 0; i < 64; i++) p = idx[p];  // warm
    r0 = __builtin_amdgcn_s_memrealtime();
    c0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; i++) p = __hip_atomic_load(idx + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    c1 = __builtin_amdgcn_s_memtime();
    r1 = __builtin_amdgcn_s_memrealtime();
    out[0] = r1 - r0; out[1] = c1 - c0; out[15] = p;
    // 2. store + wait
    r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; i++) {
      buf[i & 255] = (double)i;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    r1 = __builtin_amdgcn_s_memrealtime();
    out[2] = r1 - r0;
    // 4. dependent fp64 fma
    double x = buf[1], y = buf[2];
    r0 = __builtin_amdgcn_s_memrealtime();
    c0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; i++) {
#pragma unroll
      for (int u = 0; u < 16; u++) x = fma(x, y, 0.5);
      asm volatile("" : "+v"(x));
    }
    c1 = __builtin_amdgcn_s_memtime();
    r1 = __builtin_amdgcn_s_memrealtime();
    out[4] = r1 - r0; out[5] = c1 - c0; buf[300] = x;
    // 5. dependent rsq f64
    x = buf[3] + 2.0;
    r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; i++) {
#pragma unroll
      for (int u = 0; u < 16; u++) x = __builtin_amdgcn_rsq(x) + 1.5;
      asm volatile("" : "+v"(x));
    }
    r1 = __builtin_amdgcn_s_memrealtime();
    out[6] = r1 - r0; buf[301] = x;
    // 6. dependent fp32 fma
    float xf = buf[4], yf = buf[5];
    r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; i++) {
#pragma unroll
      for (int u = 0; u < 16; u++) xf = fmaf(xf, yf, 0.5f);
      asm volatile("" : "+v"(xf));
    }
    r1 = __builtin_amdgcn_s_memrealtime();
    out[7] = r1 - r0; buf[302] = xf;
    // 7. LDS dependent chain
    int q = 0;
    r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; i++) q = ldsi[(q + 1) & 63];
    r1 = __builtin_amdgcn_s_memrealtime();
    out[8] = r1 - r0; out[14] = q;
    // 8. global load after own store (L2 round trip incl. the write)
    r0 = __builtin_amdgcn_s_memrealtime();
    double acc = 0;
    for (int i = 0; i < iters; i++) {
      buf[512 + (i & 63)] = acc + i;
      acc += __hip_atomic_load(buf + 512 + (i & 63), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    r1 = __builtin_amdgcn_s_memrealtime();
    out[9] = r1 - r0; buf[303] = acc;
  }
  __syncthreads();
  // 3. barrier cost, all 16 waves
  r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; i++) __syncthreads();
  r1 = __builtin_amdgcn_s_memrealtime();
  if (t == 0) out[3] = r1 - r0;
  // 3b. barrier with global stores outstanding from every wave
  r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; i++) {
    buf[1024 + t] = (double)i;
    __syncthreads();
  }
  r1 = __builtin_amdgcn_s_memrealtime();
  if (t == 0) out[10] = r1 - r0;
  // 3c. LDS-only barrier: lds store + s_barrier without waiting for global stores
  r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; i++) {
    buf[1024 + t] = (double)i;
    lds[t] = i;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
  }
  r1 = __builtin_amdgcn_s_memrealtime();
  if (t == 0) out[11] = r1 - r0;
  (void)w; (void)lane;
}

int main() {
  double* buf; int* idx; unsigned long long* out;
  hipMalloc(&buf, 1 << 20); hipMalloc(&idx, 4096 * 4); hipMalloc(&out, 16 * 8);
  int h[4096];
  for (int i = 0; i < 4096; i++) h[i] = (i * 97 + 31) % 1024;  // chase within 4 KB (L1/L2)
  hipMemcpy(idx, h, sizeof(h), hipMemcpyHostToDevice);
  hipMemset(buf, 0, 1 << 20);
  const int it = 2000;
  for (int rep = 0; rep < 3; rep++) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(1024), 0, 0, buf, idx, out, it);
    hipDeviceSynchronize();
  }
  unsigned long long o[16];
  hipMemcpy(o, out, sizeof(o), hipMemcpyDeviceToHost);
  const double ns = 10.0 / it;  // 100 MHz ticks -> ns per iteration
  printf("clock %.2f GHz (memtime/realtime over the load chase)\n", (double)o[1] / (o[0] * 10.0));
  printf("dependent global load (sc0 relaxed, L1/L2 warm): %.1f ns\n", o[0] * ns);
  printf("store + vmcnt(0): %.1f ns\n", o[2] * ns);
  printf("__syncthreads (16 waves): %.1f ns\n", o[3] * ns);
  printf("__syncthreads with a global store per thread: %.1f ns\n", o[10] * ns);
  printf("LDS-only barrier with a global store per thread: %.1f ns\n", o[11] * ns);
  printf("dependent v_fma_f64: %.2f ns\n", o[4] * ns / 16);
  printf("dependent v_rsq_f64 + v_add_f64: %.2f ns\n", o[6] * ns / 16);
  printf("dependent v_fma_f32: %.2f ns\n", o[7] * ns / 16);
  printf("dependent ds_read_b32: %.2f ns\n", o[8] * ns);
  printf("store then load same address: %.1f ns\n", o[9] * ns);
  return 0;
}
