// Retrieval codebook quantization for MI355X (gfx950): the distance GEMM + top-k of
// RetrievalDatabase.quantize_custom (/root/reference/mast3r_slam/retrieval_database.py:96-105):
//
//   l2[m, c] = (|q_m|^2 + |c_c|^2) - 2 q_m . c_c        (fp32, torch broadcasting order)
//   topk(l2, k, dim=1, largest=False).indices           (ascending distance, int64)
//
// At the reference's shapes (asmk codebook 64k x 1024, 300 local features per keyframe, k = 5 for a
// query, 1 for a database add: mast3r/retrieval/processor.py:91-97, model.py:108-109) this is a
// 300 x 65536 x 1024 GEMM whose 256 MB codebook is streamed once per call. The reference runs it as a
// TF32 GEMM (main.py:168 enables TF32 matmuls) followed by torch.topk.
//
// MI355X design:
//   * Matrix cores in bf16 with a hi/lo split: x = hi + lo (both bf16, |lo| <= 2^-9 |x|) and
//     q.c ~= qh.ch + qh.cl + ql.ch, fp32 accumulation (v_mfma_f32_16x16x32_bf16). Per-product error
//     ~2^-16 relative: ~100x tighter than the reference's own TF32 product (10-bit mantissas), at
//     3 MFMA per product = 3 x 2.5 PF/s dense bf16 instead of the 157 TF/s fp32 MFMA rate.
//   * Both operands are pre-arranged in MFMA fragment order (one 16-B unit per lane per 16x32
//     tile): the codebook once (m3s_codebook_prepare), the queries per call. A k-step's operands are
//     then contiguous, staged by lane-linear global_load_lds copies, and read back conflict-free.
//   * One 512-thread block per 256 codebook rows (256 blocks = one per CU at 64k rows), two waves
//     per SIMD: wave w owns 32 rows (two 16-row tiles) against all 19 query tiles of the group, i.e.
//     38 16x16 fp32 accumulator tiles = 152 registers per lane (no spills at 256 per wave).
//     Query k-step images (38 KB) are double-buffered in LDS (global_load_lds one step ahead); each wave's
//     codebook fragments (4 KB per step) stream global -> VGPR two steps ahead through a 3-slot register ring.
//     Each query fragment pair read feeds 6 MFMAs, each codebook fragment pair 57.
//   * Epilogue (exact block top-k per query, keys = order-preserving fp32 bits << 32 | row): a
//     query's 256 block distances sit in 32 lanes, 8 each. tau = the k-th smallest of the 32 lane
//     minima bounds the k-th best, so only distances <= tau (typically ~6 per query and block) are
//     appended to LDS lists and sorted. rq_merge_kernel reduces the blocks' keys (one wave per
//     query) and writes the indices. Ties break to the lower codebook row (torch.topk leaves them
//     unspecified).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace m3s {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f4v __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const void* rq_gptr;
typedef __attribute__((address_space(3))) void* rq_lptr;

#define RQ_NQT 19                 // query column tiles (16 queries) per group
#define RQ_QG (RQ_NQT * 16)       // 304 queries per group
#define RQ_NR 2                   // codebook row tiles (16 rows) per wave
#define RQ_ROWS 256               // codebook rows per block: 8 waves x 32
#define RQ_THREADS 512            // 8 waves
#define RQ_NL 32                  // lane slots per query in a block: 8 waves x 4 lane groups
#define RQ_BT (RQ_ROWS / 16)      // codebook row tiles per block
#define RQ_QU (RQ_NQT * 2 * 64)   // 16-B query units per (group, k-step): 19 tiles x {hi, lo} x 64 lanes
#define RQ_AU (RQ_BT * 2 * 64)    // 16-B codebook units per (block, k-step): 16 tiles x {hi, lo} x 64 lanes
#define RQ_CAP 24                 // epilogue candidate list length per query

__device__ __forceinline__ unsigned bf16_rne_bits(float x) {
  unsigned u = __float_as_uint(x);
  u += 0x7fffu + ((u >> 16) & 1u);
  return u >> 16;
}

// Split 8 consecutive fp32 values into bf16 hi / lo fragments (8 x bf16 each, packed in a uint4).
__device__ __forceinline__ void split8(const float (&v)[8], uint4& hi, uint4& lo) {
  unsigned h[8], l[8];
#pragma unroll
  for (int j = 0; j < 8; j++) {
    h[j] = bf16_rne_bits(v[j]);
    l[j] = bf16_rne_bits(v[j] - __uint_as_float(h[j] << 16));
  }
  hi = make_uint4(h[0] | (h[1] << 16), h[2] | (h[3] << 16), h[4] | (h[5] << 16), h[6] | (h[7] << 16));
  lo = make_uint4(l[0] | (l[1] << 16), l[2] | (l[3] << 16), l[4] | (l[5] << 16), l[6] | (l[7] << 16));
}

// Fragment layout: tile T (16 rows) of k-step s, part p (hi/lo), lane l holds rows 16T + (l & 15),
// columns 32s + 8(l >> 4) .. +7. Unit index (((T / inner_n) * S + s) * inner_n + T % inner_n) * 2 + p)
// * 64 + l: inner_n = RQ_BT for the codebook (a block's k-step contiguous, 32 KB), RQ_NQT for the
// queries (a group's k-step contiguous, 38 KB). Rows >= R and columns >= D are zero.
__global__ void __launch_bounds__(256) rq_prep_kernel(const float* __restrict__ X, int R, int D, int S, int ntiles,
                                                      int inner_n, uint4* __restrict__ frag, int nfrag, int Rp,
                                                      float pad_value, float* __restrict__ nrm) {
  // blocks [nfrag, ..): the squared row norms |x_r|^2 in fp32, one wave per row; rows in [R, Rp) get pad_value
  // (+inf for the codebook, so padded rows never rank; 0 for padded queries, whose results are not written)
  if ((int)blockIdx.x >= nfrag) {
    const int row = (blockIdx.x - nfrag) * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (row >= Rp) return;
    float s0 = 0.0f, s1 = 0.0f, s2 = 0.0f, s3 = 0.0f;
    if (row < R) {
      const float* x = X + (size_t)row * D;
      int k = lane;
      for (; k + 192 < D; k += 256) {
        const float a = x[k], b = x[k + 64], c = x[k + 128], d = x[k + 192];
        s0 += a * a;
        s1 += b * b;
        s2 += c * c;
        s3 += d * d;
      }
      for (; k < D; k += 64) s0 += x[k] * x[k];
    }
    float s = (s0 + s1) + (s2 + s3);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    if (lane == 0) nrm[row] = row < R ? s : pad_value;
    return;
  }
  const size_t gid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t total = (size_t)ntiles * S * 64;
  if (gid >= total) return;
  const int lane = (int)(gid & 63);
  const size_t ts = gid >> 6;
  const int s = (int)(ts % S);
  const int T = (int)(ts / S);
  const int row = 16 * T + (lane & 15), k0 = 32 * s + 8 * (lane >> 4);
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; j++) v[j] = (row < R && k0 + j < D) ? X[(size_t)row * D + k0 + j] : 0.0f;
  uint4 hi, lo;
  split8(v, hi, lo);
  const size_t u = ((((size_t)(T / inner_n) * S + s) * inner_n + T % inner_n) * 2) * 64 + lane;
  frag[u] = hi;
  frag[u + 64] = lo;
}

__device__ __forceinline__ unsigned long long dist_key(float d, unsigned row) {
  unsigned u = __float_as_uint(d);
  u ^= (u & 0x80000000u) ? 0xffffffffu : 0x80000000u;  // order-preserving fp32 -> u32
  return ((unsigned long long)u << 32) | row;
}

// insert key into the ascending list L (keeps the K smallest)
template <int K>
__device__ __forceinline__ void kins(unsigned long long (&L)[K], unsigned long long key) {
#pragma unroll
  for (int j = 0; j < K; j++) {
    const unsigned long long o = L[j];
    const bool lt = key < o;
    L[j] = lt ? key : o;
    key = lt ? o : key;
  }
}

template <int K>
__device__ __forceinline__ void kmerge_xor(unsigned long long (&L)[K], int off) {
  unsigned long long P[K];
#pragma unroll
  for (int j = 0; j < K; j++) P[j] = __shfl_xor(L[j], off, 64);
#pragma unroll
  for (int j = 0; j < K; j++) kins<K>(L, P[j]);
}

// grid (Cp / 256, groups); block 512. cand[((g * nblk + b) * RQ_QG + q) * K + j]: the block's K best keys.
template <int K>
__global__ void __launch_bounds__(RQ_THREADS) __attribute__((amdgpu_waves_per_eu(2, 2)))
rq_gemm_topk_kernel(const uint4* __restrict__ cfrag, const float* __restrict__ cn, const uint4* __restrict__ qfrag,
                    const float* __restrict__ qn, int S, unsigned long long* __restrict__ cand) {
  // query k-step images: two separate arrays (not one indexed by parity) so the compiler can prove that a
  // step's ds_reads never alias the global_load_lds writing the other image; with one array it waits
  // vmcnt(0) before every read and the staging no longer overlaps the MFMAs
  __shared__ uint4 sb0_[RQ_QU];
  __shared__ uint4 sb1_[RQ_QU];
  __shared__ uint4 sa_[2][RQ_AU];  // epilogue scratch (candidate lists)
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  const int g = blockIdx.y;
  // this wave's codebook units of a k-step: tiles 2w, 2w+1 x {hi, lo} = 4 x 1 KB, contiguous
  const uint4* ca = cfrag + (size_t)blockIdx.x * S * RQ_AU + (size_t)(w * RQ_NR * 2) * 64 + lane;
  const uint4* qa = qfrag + (size_t)g * S * RQ_QU + lane;
  f4v acc[RQ_NR][RQ_NQT];
#pragma unroll
  for (int r = 0; r < RQ_NR; r++)
#pragma unroll
    for (int q = 0; q < RQ_NQT; q++) acc[r][q] = f4v{0.0f, 0.0f, 0.0f, 0.0f};
  // queries: lane-linear 1-KB global_load_lds copies into the idle LDS image, one k-step ahead
  // (issued by inline asm: the compiler's own wait insertion would otherwise drain every outstanding load with
  // vmcnt(0) before any read of either image, serialising the staging; the explicit waits below order them)
  auto stage_b = [&](int s, uint4* dst) {
    for (int i = w; i < RQ_QU / 64; i += RQ_THREADS / 64) {
      const unsigned m0 = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(rq_lptr)&dst[i * 64]);
      // one wait state between the M0 write and the LDS DMA that reads it (CDNA3/4 manually inserted wait states;
      // the compiler's own global_load_lds sequences keep one instruction there)
      asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(qa + (size_t)s * RQ_QU + i * 64), "{m0}"(m0)
                   : "memory");  // M0 an operand: the compiler writes it before the asm and knows its value
    }
  };
  // codebook: global -> VGPR two k-steps ahead (a 3-slot register ring), by inline-asm loads the compiler does
  // not wait for: every step ends with s_waitcnt vmcnt(4), which leaves exactly the 4 loads of step s+2 in
  // flight and retires everything older (the query copies of step s+1 and the codebook of step s+1).
  auto aload = [&](u32x4 (&A)[4], int s) {
    const uint4* src = ca + (size_t)s * RQ_AU;
#pragma unroll
    for (int j = 0; j < 4; j++) asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(A[j]) : "v"(src + j * 64) : "memory");
  };
  auto step = [&](auto parity, int s, const u32x4 (&Ac)[4], u32x4 (&An)[4]) {
    constexpr int buf = decltype(parity)::value;  // == s & 1
    if (s + 1 < S) stage_b(s + 1, buf ? sb0_ : sb1_);
    aload(An, min(s + 2, S - 1));  // past the end: a harmless re-load keeps the vmcnt arithmetic fixed
    const bf16x8 ah[RQ_NR] = {__builtin_bit_cast(bf16x8, Ac[0]), __builtin_bit_cast(bf16x8, Ac[2])};
    const bf16x8 al[RQ_NR] = {__builtin_bit_cast(bf16x8, Ac[1]), __builtin_bit_cast(bf16x8, Ac[3])};
    const uint4* sb = (buf ? sb1_ : sb0_) + lane;
    uint4 bh = sb[0], bl = sb[64];
#pragma unroll
    for (int q = 0; q < RQ_NQT; q++) {
      uint4 nh = bh, nl = bl;
      if (q + 1 < RQ_NQT) {  // next tile's fragments in flight behind this tile's 6 MFMAs
        nh = sb[(2 * q + 2) * 64];
        nl = sb[(2 * q + 3) * 64];
      }
      const bf16x8 vh = __builtin_bit_cast(bf16x8, bh), vl = __builtin_bit_cast(bf16x8, bl);
#pragma unroll
      for (int r = 0; r < RQ_NR; r++) acc[r][q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[r], vh, acc[r][q], 0, 0, 0);
#pragma unroll
      for (int r = 0; r < RQ_NR; r++) acc[r][q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[r], vl, acc[r][q], 0, 0, 0);
#pragma unroll
      for (int r = 0; r < RQ_NR; r++) acc[r][q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[r], vh, acc[r][q], 0, 0, 0);
      bh = nh;
      bl = nl;
    }
    asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)" ::: "memory");  // this wave's k-step s+1 query copies landed ...
    __builtin_amdgcn_s_barrier();                      // ... and every wave's; image `buf` no longer read
    // the ring registers are defined by the asm loads, so the compiler sees no dependence on the wait above:
    // a scheduling fence keeps the next step's MFMAs (pure register ops) from being hoisted across it
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
  };
  const std::integral_constant<int, 0> I0;
  const std::integral_constant<int, 1> I1;
  u32x4 A0[4], A1[4], A2[4];
  aload(A0, 0);
  aload(A1, min(1, S - 1));
  stage_b(0, sb0_);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  __syncthreads();
  for (int s = 0; s < S; s += 6) {  // 6 = lcm(3 register slots, 2 LDS images): every selection compile-time
    step(I0, s, A0, A2);
    if (s + 1 < S) step(I1, s + 1, A1, A0);
    if (s + 2 < S) step(I0, s + 2, A2, A1);
    if (s + 3 < S) step(I1, s + 3, A0, A2);
    if (s + 4 < S) step(I0, s + 4, A1, A0);
    if (s + 5 < S) step(I1, s + 5, A2, A1);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing re-loads
  __builtin_amdgcn_sched_barrier(0);
  __syncthreads();

  // ---- epilogue: exact block top-K per query by a threshold filter ----
#ifdef RQ_EXP_NOEPI  // (experiment builds only) skip the top-k: one checksum store per lane
  {
    float sum = 0.0f;
#pragma unroll
    for (int r = 0; r < RQ_NR; r++)
#pragma unroll
      for (int q = 0; q < RQ_NQT; q++) sum += acc[r][q][0] + acc[r][q][1] + acc[r][q][2] + acc[r][q][3];
    if (sum == 12345.0f) cand[t] = 0;
    return;
  }
#endif
  //   1. every lane takes the minimum of its 8 distances of a query; tau[q] = the K-th smallest of the
  //      query's 32 lane minima, so at least K distances are <= tau[q] and the K best all are;
  //   2. every lane appends its distances <= tau[q] to the query's LDS list (one LDS atomic per lane and
  //      query tile reserves the slots);
  //   3. one thread per query keeps the K best of the list (the (distance, row) order of a full sort).
  // A list longer than RQ_CAP (many equal distances, or tau = +inf when fewer than K lanes hold codebook
  // rows) is redone for its query tile by exhaustive per-lane insertion + merges.
  const unsigned row0 = blockIdx.x * RQ_ROWS + w * (16 * RQ_NR) + (lane >> 4) * 4;
  float cv[RQ_NR][4];
#pragma unroll
  for (int r = 0; r < RQ_NR; r++)
#pragma unroll
    for (int i = 0; i < 4; i++) cv[r][i] = cn[row0 + 16 * r + i];
  float* smin = reinterpret_cast<float*>(&sb0_[0]);  // [RQ_QG][RQ_NL] lane minima
  float* tau = reinterpret_cast<float*>(&sb1_[0]);   // [RQ_QG]
  int* cnt = reinterpret_cast<int*>(tau + RQ_QG);    // [RQ_QG] list lengths
  int* ovf = cnt + RQ_QG;                            // [32] query-tile overflow flags
  unsigned long long* lst = reinterpret_cast<unsigned long long*>(&sa_[0][0]);  // [RQ_QG][RQ_CAP]
  static_assert(4 * RQ_QG * RQ_NL <= (int)sizeof(sb0_), "lane minima fit a query image");
  static_assert(4 * (2 * RQ_QG + 32) <= (int)sizeof(sb1_), "epilogue scalars fit a query image");
  static_assert(8 * RQ_QG * RQ_CAP <= (int)sizeof(sa_), "candidate lists fit the codebook images");
  static_assert(8 * 16 * K <= RQ_QG * RQ_CAP, "fallback lists fit the candidate lists");
  const int col = lane & 15, lg = w * 4 + (lane >> 4);  // query column in the tile; lane slot of the query
#pragma unroll 19  // explicit count: a plain full-unroll request is declined for large K (acc -> scratch)
  for (int q = 0; q < RQ_NQT; q++) {
    const int ql = 16 * q + col;
    const float qv = qn[g * RQ_QG + ql];
    float m = __builtin_inff();
#pragma unroll
    for (int r = 0; r < RQ_NR; r++)
#pragma unroll
      for (int i = 0; i < 4; i++) m = fminf(m, (qv + cv[r][i]) - 2.0f * acc[r][q][i]);
    smin[ql * RQ_NL + lg] = m;
  }
  __syncthreads();
  for (int ql = t; ql < RQ_QG; ql += RQ_THREADS) {
    float L[K];
#pragma unroll
    for (int j = 0; j < K; j++) L[j] = __builtin_inff();
#pragma unroll
    for (int u = 0; u < RQ_NL; u++) {
      float v = smin[ql * RQ_NL + u];
#pragma unroll
      for (int j = 0; j < K; j++) {  // sorted insertion (values only)
        const float o = L[j];
        L[j] = fminf(o, v);
        v = fmaxf(o, v);
      }
    }
    tau[ql] = L[K - 1];
    cnt[ql] = 0;
  }
  if (t < 32) ovf[t] = 0;
  __syncthreads();
#pragma unroll 19  // explicit count: a plain full-unroll request is declined for large K (acc -> scratch)
  for (int q = 0; q < RQ_NQT; q++) {
    const int ql = 16 * q + col;
    const float qv = qn[g * RQ_QG + ql];
    const float tq = tau[ql];
    unsigned mask = 0;
#pragma unroll
    for (int r = 0; r < RQ_NR; r++)
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const float d = (qv + cv[r][i]) - 2.0f * acc[r][q][i];
        mask |= (d <= tq && d < __builtin_inff()) ? 1u << (4 * r + i) : 0u;
      }
    if (mask) {
      int slot = atomicAdd(&cnt[ql], __popc(mask));
#pragma unroll
      for (int r = 0; r < RQ_NR; r++)
#pragma unroll
        for (int i = 0; i < 4; i++)
          if (mask & (1u << (4 * r + i))) {
            if (slot < RQ_CAP)
              lst[ql * RQ_CAP + slot] = dist_key((qv + cv[r][i]) - 2.0f * acc[r][q][i], row0 + 16 * r + i);
            slot++;
          }
    }
  }
  __syncthreads();
  for (int ql = t; ql < RQ_QG; ql += RQ_THREADS) {
    const int n = cnt[ql];
    if (n > RQ_CAP) {
      ovf[ql >> 4] = 1;
      continue;
    }
    unsigned long long L[K];
#pragma unroll
    for (int j = 0; j < K; j++) L[j] = ~0ull;
    for (int u = 0; u < n; u++) kins<K>(L, lst[ql * RQ_CAP + u]);
    unsigned long long* o = cand + ((size_t)(g * gridDim.x + blockIdx.x) * RQ_QG + ql) * K;
#pragma unroll
    for (int j = 0; j < K; j++) o[j] = L[j];
  }
  __syncthreads();
  unsigned long long* sk = lst;  // fallback merge lists [8 waves][16][K]
#pragma unroll 19  // explicit count: a plain full-unroll request is declined for large K (acc -> scratch)
  for (int q = 0; q < RQ_NQT; q++) {
    if (ovf[q]) {  // block-uniform
      const float qv = qn[g * RQ_QG + 16 * q + col];
      unsigned long long L[K];
#pragma unroll
      for (int j = 0; j < K; j++) L[j] = ~0ull;
#pragma unroll
      for (int r = 0; r < RQ_NR; r++)
#pragma unroll
        for (int i = 0; i < 4; i++) kins<K>(L, dist_key((qv + cv[r][i]) - 2.0f * acc[r][q][i], row0 + 16 * r + i));
      kmerge_xor<K>(L, 16);
      kmerge_xor<K>(L, 32);
      if (lane < 16) {
#pragma unroll
        for (int j = 0; j < K; j++) sk[(w * 16 + lane) * K + j] = L[j];
      }
      __syncthreads();
      if (t < 16 && cnt[16 * q + t] > RQ_CAP) {
        unsigned long long M[K];
#pragma unroll
        for (int j = 0; j < K; j++) M[j] = sk[t * K + j];
#pragma unroll
        for (int ww = 1; ww < RQ_THREADS / 64; ww++)
#pragma unroll
          for (int j = 0; j < K; j++) kins<K>(M, sk[(ww * 16 + t) * K + j]);
        unsigned long long* o = cand + ((size_t)(g * gridDim.x + blockIdx.x) * RQ_QG + 16 * q + t) * K;
#pragma unroll
        for (int j = 0; j < K; j++) o[j] = M[j];
      }
      __syncthreads();
    }
  }
}

// one wave per query: the K best of the nblk blocks' K keys (each block list sorted ascending), written as int64
// row indices. Lane l holds the lists of blocks l + 64 m; K rounds of: wave minimum of the lanes' head keys
// (keys are unique: they carry the row), the owning lane pops its head.
#define RQ_ML 4  // block lists per lane (nblk <= 64 * RQ_ML per pass; more blocks are folded in first)
template <int K>
__global__ void __launch_bounds__(256) rq_merge_kernel(const unsigned long long* __restrict__ cand, int nblk, int M,
                                                       int64_t* __restrict__ out) {
  const int q = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (q >= M) return;
  const int g = q / RQ_QG, ql = q % RQ_QG;
  unsigned long long L[RQ_ML][K];
#pragma unroll
  for (int m = 0; m < RQ_ML; m++) {
    const int b = lane + 64 * m;
    const unsigned long long* c = cand + ((size_t)(g * nblk + min(b, nblk - 1)) * RQ_QG + ql) * K;
#pragma unroll
    for (int j = 0; j < K; j++) L[m][j] = b < nblk ? c[j] : ~0ull;
  }
  for (int b = lane + 64 * RQ_ML; b < nblk; b += 64) {  // codebooks beyond 64k rows: fold into list 0
    const unsigned long long* c = cand + ((size_t)(g * nblk + b) * RQ_QG + ql) * K;
#pragma unroll
    for (int j = 0; j < K; j++) {
      const unsigned long long key = c[j];
      if (key < L[0][K - 1]) kins<K>(L[0], key);
    }
  }
  unsigned long long res = ~0ull;
#pragma unroll
  for (int r = 0; r < K; r++) {
    unsigned long long h = L[0][0];
    int hm = 0;
#pragma unroll
    for (int m = 1; m < RQ_ML; m++)
      if (L[m][0] < h) {
        h = L[m][0];
        hm = m;
      }
    unsigned long long wmin = h;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const unsigned long long o = __shfl_xor(wmin, off, 64);
      wmin = o < wmin ? o : wmin;
    }
    if (lane == r) res = wmin;
    if (h == wmin) {  // this lane owns the minimum: pop that list's head
#pragma unroll
      for (int m = 0; m < RQ_ML; m++)
        if (m == hm) {
#pragma unroll
          for (int j = 0; j + 1 < K; j++) L[m][j] = L[m][j + 1];
          L[m][K - 1] = ~0ull;
        }
    }
  }
  if (lane < K) out[(size_t)q * K + lane] = (int64_t)(res & 0xffffffffull);
}

}  // namespace m3s

// ------------------------------------------------------------------------------------------
extern "C" hipError_t m3s_launch_rq_prep(const float* X, int R, int D, int S, int ntiles, int inner_n, uint4* frag,
                                         int Rp, float pad_value, float* nrm, hipStream_t s) {
  const size_t total = (size_t)ntiles * S * 64;
  const int nfrag = (int)((total + 255) / 256);
  hipLaunchKernelGGL(m3s::rq_prep_kernel, dim3(nfrag + (Rp + 3) / 4), dim3(256), 0, s, X, R, D, S, ntiles, inner_n,
                     frag, nfrag, Rp, pad_value, nrm);
  return hipGetLastError();
}

template <int K>
static hipError_t rq_launch_k(const uint4* cfrag, const float* cn, const uint4* qfrag, const float* qn, int S,
                              int nblk, int groups, int M, unsigned long long* cand, int64_t* out, hipStream_t s) {
  hipLaunchKernelGGL(m3s::rq_gemm_topk_kernel<K>, dim3(nblk, groups), dim3(RQ_THREADS), 0, s, cfrag, cn, qfrag, qn, S,
                     cand);
  hipLaunchKernelGGL(m3s::rq_merge_kernel<K>, dim3((M + 3) / 4), dim3(256), 0, s, cand, nblk, M, out);
  return hipGetLastError();
}

extern "C" hipError_t m3s_launch_rq_topk(const uint4* cfrag, const float* cn, const uint4* qfrag, const float* qn,
                                         int S, int nblk, int groups, int M, int k, unsigned long long* cand,
                                         int64_t* out, hipStream_t s) {
  switch (k) {
    case 1: return rq_launch_k<1>(cfrag, cn, qfrag, qn, S, nblk, groups, M, cand, out, s);
    case 2: return rq_launch_k<2>(cfrag, cn, qfrag, qn, S, nblk, groups, M, cand, out, s);
    case 3: return rq_launch_k<3>(cfrag, cn, qfrag, qn, S, nblk, groups, M, cand, out, s);
    case 4: return rq_launch_k<4>(cfrag, cn, qfrag, qn, S, nblk, groups, M, cand, out, s);
    case 5: return rq_launch_k<5>(cfrag, cn, qfrag, qn, S, nblk, groups, M, cand, out, s);
    case 6: return rq_launch_k<6>(cfrag, cn, qfrag, qn, S, nblk, groups, M, cand, out, s);
    case 7: return rq_launch_k<7>(cfrag, cn, qfrag, qn, S, nblk, groups, M, cand, out, s);
    case 8: return rq_launch_k<8>(cfrag, cn, qfrag, qn, S, nblk, groups, M, cand, out, s);
    default: return hipErrorInvalidValue;
  }
}
