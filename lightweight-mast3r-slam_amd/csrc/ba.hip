// Global bundle adjustment (keyframe Sim(3) poses, pointmap edges) for MI355X (gfx950).
//
// Reference semantics:
//   point_align_kernel / ray_align_kernel / calib_proj_kernel
//                     /root/reference/mast3r_slam/backend/src/gn_kernels.cu:455-723, 813-1138, 1231-1543
//   SparseBlock update_lhs/rhs + SimplicialLLT solve   gn_kernels.cu:57-159
//   pose_retr_kernel  gn_kernels.cu:415-453
//   host GN loop      gn_kernels.cu:725-811, 1140-1228, 1546-1637
//
// MI355X design (not a translation):
//   * ba_lin: (edge, point-chunk) blocks. Because Ji = -Jj and Jj = A_i J_local with a per-edge
//     7x7 adjoint map A_i (gn_kernels.cu:277-297 is linear in the row), each lane accumulates only
//     the 28-entry local normal matrix L = sum w J J^T and the 7-entry v = sum w e J in registers
//     (instead of 105 + 14 transformed entries, products/sums in fp64, structural zeros skipped)
//     and the per-edge transform is applied once.
//   * ba_edge: per-edge fp64 reduction of the chunk partials and M = A L A^T, g = A v.
//     The (E,36) edge-sum rows are the only data a multi-GPU run all-reduces.
//   * ba_assemble: deterministic block-sparse assembly (host-built CSR of contributions per 7x7
//     factor block, fixed order) of the pose system; every rank therefore solves an identical system
//     and keeps identical poses.
//   * ba_sparse_factor: the block-sparse fp64 Cholesky of that system in the plan's minimum-degree
//     order, level by level of the elimination tree inside ONE workgroup (right-looking updates, the
//     forward substitution carried as the rhs block row), the back substitution, then the Sim(3)
//     retraction + |dx| early-exit flag on device: no host synchronisation inside the GN loop.
#include "m3s_common.hpp"
#include "m3s_ba.h"
#include "ba_pattern.h"  // BA_BS_* flags of the dataflow back-substitution lists
#include <cstring>

namespace m3s {

#define BA_NSUM 36

// ------------------------------------------------------------------------------------------
// linearisation
// ------------------------------------------------------------------------------------------
typedef float f2 __attribute__((ext_vector_type(2)));

// MASK: the row's structurally nonzero Jacobian entries (bit c). Products with a structural zero are skipped:
// for finite weights they add an exact +-0 to the sum, so the result is unchanged (the reference computes
// them; ~45% of the FMAs in rays mode). Products and sums in fp32 (packed: two points per instruction) over
// runs of BA_RUN_LEN rounds per slot, each run then added to the fp64 accumulators (the kernel is VALU-issue
// bound; fp64 products put no measurable accuracy gain against the fp64 truth once runs are short).
#ifndef BA_RUN_LEN  // rounds per fp32 run (points per slot): 8 -> 16 took C5 2.25 -> 2.19 ms, C4 1.91 -> 1.83 ms.
// Round 5: 64 (a chunk is <= 48 rounds, so one fp32 run per slot and chunk, flushed once): with the fp64 retraction and
// relative pose (m3s_common.hpp) the fp32 runs no longer carry the error budget: every BA fixture <= 3.5e-6 from the
// fp64 truth (16: <= 7.2e-6; scripts/ba_acc.py), linearisation -2 % (C5 2.28 -> 2.22 ms, C4 1.86 -> 1.82 ms in
// scripts/ba_exp.py spans; profiles/r05_ba_runlen.txt)
#define BA_RUN_LEN 64
#endif
template <unsigned MASK>
__device__ __forceinline__ void acc_local_f2(f2* L, f2* v, const f2 J[7], f2 w, f2 e) {
  int l = 0;
#pragma unroll
  for (int c = 0; c < 7; c++) {
    const f2 wj = w * J[c];
#pragma unroll
    for (int d = c; d < 7; d++) {
      if ((MASK >> c) & (MASK >> d) & 1u) L[l] = __builtin_elementwise_fma(wj, J[d], L[l]);
      l++;
    }
    if ((MASK >> c) & 1u) v[c] = __builtin_elementwise_fma(wj, e, v[c]);
  }
}

// huber weight (gn_kernels.cu:172-175, k = 1.345 as a double) of two residuals. The reference's quotient is
// the double division k / |r| rounded to float; here the float quotient of the two-float k = KH + KL by |r|,
// refined by one FMA residual step (equal to the double route but for a rounding tie within ~2^-48), so no
// fp64 division sequence runs for every row (the select evaluated it unconditionally).
__device__ __forceinline__ f2 huber_ba2(f2 r) {
  constexpr float KH = 1.345f;
  constexpr float KL = (float)(1.345 - (double)1.345f);
  const f2 ra = {fabsf(r.x), fabsf(r.y)};
  const f2 y = {__builtin_amdgcn_rcpf(ra.x), __builtin_amdgcn_rcpf(ra.y)};
  const f2 q0 = KH * y;
  const f2 e = __builtin_elementwise_fma(-q0, ra, f2{KH, KH}) + KL;
  const f2 q = __builtin_elementwise_fma(e, y, q0);
  // |r| < k -> 1, else k/|r| (<= 1): min(1, q), with |r| = 0 (q NaN from rcp(0) * 0) -> 1 by min's NaN rule
  return f2{fminf(1.0f, q.x), fminf(1.0f, q.y)};
}

// 1/sqrt(x) and 1/x of two values: the hardware estimates (~1 ulp) refined by one Newton step each (packed), which
// takes out the estimates' bias against the reference's IEEE sqrtf and divisions: without it the K = 256 EuRoC rays
// graph sat 1.14e-5 from the fp64 truth (6.8e-6 with it, for +2 % linearisation time; scripts/ba_acc.py)
#ifndef BA_RAYS_NEWTON
#define BA_RAYS_NEWTON 1
#endif
__device__ __forceinline__ f2 rsq2(f2 x) {
  f2 y = {__builtin_amdgcn_rsqf(x.x), __builtin_amdgcn_rsqf(x.y)};
#if BA_RAYS_NEWTON
  y = y * __builtin_elementwise_fma(-0.5f * x * y, y, f2{1.5f, 1.5f});
#endif
  return y;
}
__device__ __forceinline__ f2 rcp2(f2 x) {
  f2 y = {__builtin_amdgcn_rcpf(x.x), __builtin_amdgcn_rcpf(x.y)};
#if BA_RAYS_NEWTON
  y = y * __builtin_elementwise_fma(-x, y, f2{2.0f, 2.0f});
#endif
  return y;
}

// BA_LIN_MATRIX: the per-point Sim(3) action as X + (D X + t) with the per-edge D = s R - I (3 packed FMAs + an add
// per component instead of the quaternion expression's 12 ops under -ffp-contract=off). BA_LIN_FMA: explicit FMAs in
// the calib rows' product-sums (pixel projection, the (1 + x^2) Jacobian terms). Measured on MI355X (scripts/
// gpu_r03s2_i.sh, scripts/ba_acc.py): lin C5 2.20 -> 1.94 ms, C4 1.88 -> 1.80 ms; every BA fixture <= 8e-6 from the
// fp64 truth (max: K=256 EuRoC rays 8.0e-6). FMAs in the rays rows gained 1.4 % and cost accuracy (EuRoC 8.6e-6):
// not used.
#ifndef BA_LIN_MATRIX
#define BA_LIN_MATRIX 1
#endif
#ifndef BA_LIN_FMA
#define BA_LIN_FMA 1
#endif
__device__ __forceinline__ f2 BA_FMA2(f2 a, f2 b, f2 c) {
#if BA_LIN_FMA
  return __builtin_elementwise_fma(a, b, c);
#else
  return a * b + c;
#endif
}

// actSO3 of two points (component arrays), same expression as actSO3
__device__ __forceinline__ void actSO3_v(const float* q, const f2* X, f2* Y) {
  const f2 uv0 = 2.0f * (q[1] * X[2] - q[2] * X[1]);
  const f2 uv1 = 2.0f * (q[2] * X[0] - q[0] * X[2]);
  const f2 uv2 = 2.0f * (q[0] * X[1] - q[1] * X[0]);
  Y[0] = X[0] + q[3] * uv0 + (q[1] * uv2 - q[2] * uv1);
  Y[1] = X[1] + q[3] * uv1 + (q[2] * uv0 - q[0] * uv2);
  Y[2] = X[2] + q[3] * uv2 + (q[0] * uv1 - q[1] * uv0);
}

// The fp64 accumulation is split between the two lanes of a lane pair (even lane: sums 0..17, odd lane: 18..34). At
// a flush a lane hands the partner the run sums the partner owns (DPP swaps) and adds its own and the partner's fp32
// run sums of both points in fp64: the same BA_RUN_LEN-point fp32 runs as with per-lane accumulators (folding a
// lane's two points in fp32 first took the 6-KF rays fixture to 1.6e-5 from the fp64 truth, over the 1e-5 contract),
// half the fp64 values to move through LDS.
#ifndef BA_LIN_WAVES  // waves per SIMD the linearisation is compiled for (VGPR budget 512 / waves)
#define BA_LIN_WAVES 3
#endif
#define BA_PAIR_HALF 18  // sums owned per lane of a pair (35 = 18 + 17)

__device__ __forceinline__ float dpp_swap1(float x) {  // quad_perm [1,0,3,2]: the value of lane ^ 1
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), 0xB1, 0xF, 0xF, false));
}

// each lane of the pair (lane ^ 1) adds the fp32 run sums (28 L + 7 v, both points) of the sums it owns, its
// own and the partner's, into its fp64 accumulators
__device__ __forceinline__ void pair_flush(double* acc, const f2* fL, const f2* fv, bool odd) {
  const f2 z2 = {0.0f, 0.0f};
#pragma unroll
  for (int m = 0; m < BA_PAIR_HALF; m++) {
    const f2 lo = m < 28 ? fL[m] : fv[m - 28];
    const int c = BA_PAIR_HALF + m;
    const f2 hi = c < 28 ? fL[c] : (c < 35 ? fv[c - 28] : z2);
    const f2 own = odd ? hi : lo;
    const f2 give = odd ? lo : hi;  // the partner owns the other half
    const f2 got = {dpp_swap1(give.x), dpp_swap1(give.y)};
    acc[m] += (double)own.x;
    acc[m] += (double)own.y;
    acc[m] += (double)got.x;
    acc[m] += (double)got.y;
  }
}

// Per-call point records (once per gauss_newton call; the GN iterations only move the poses):
//   rec[e][k] = {Xi (points / rays) ; sw} (16 B) or, calib, {u_t | v_t << 16, log z_i | NaN if z_i <= z_eps, sw}
//   (12 B: the lin kernel streams E x N records every iteration, so a quarter less HBM traffic) with
//   Xi = Xs[i][valid ? idx : 0]
//   (gn_kernels.cu reads index 0 for an invalid match) and sw = sqrt(q) when the match is valid and
//   q > Q_thresh, c_i > C_thresh, c_j > C_thresh, else 0 (gn_kernels.cu:880-906) — the per-iteration
//   gathers, int64 index loads and threshold tests leave the linearisation loop.
// Only the edges of a.pack_list when the plan reuses records (m3s_ba_make_plan_reuse: the rest kept theirs), each
// into its record slot.
// the record of point k of shard edge e (ix, jx: its pose ranks); rays: *n = |Xi| (the record holds Xi / |Xi|,
// computed with the linearisation's own instruction sequence, so the rows are bit-identical to normalising there)
#ifndef BA_PACK_NT
#define BA_PACK_NT 1
#endif
#if BA_PACK_NT
#define BA_NT_LOAD(ptr) __builtin_nontemporal_load(ptr)
#else
#define BA_NT_LOAD(ptr) (*(ptr))
#endif
// the record of a matched point from its gathered X_i (ind: its pixel in keyframe i) and its folded validity
template <int MODE>
__device__ __forceinline__ float4 pack_finish(const BaParams& p, const float* Xi, int64_t ind, float q, bool valid,
                                              float* n) {
  // hardware sqrt (<= 1 ulp): parity is checked against the fp64 truth (1e-5)
  const float sw = valid ? __builtin_amdgcn_sqrtf(q) : 0.0f;
  if constexpr (MODE == BA_MODE_CALIB) {
    const int ind32 = (int)ind;  // < H*W < 2^31: 32-bit division
    const unsigned v_t = (unsigned)(ind32 / p.W), u_t = (unsigned)ind32 - v_t * (unsigned)p.W;  // W, H < 2^16 (plan)
    // log z_i once per call (the same __logf the linearisation applied every iteration), NaN marks z_i <= z_eps
    const float zi = Xi[2];
    return make_float4(__builtin_bit_cast(float, u_t | (v_t << 16)), zi > p.z_eps ? __logf(zi) : __builtin_nanf(""),
                       sw, 0.0f);
  } else if constexpr (MODE == BA_MODE_RAYS) {
    const f2 X[3] = {f2{Xi[0], Xi[0]}, f2{Xi[1], Xi[1]}, f2{Xi[2], Xi[2]}};
    const f2 n2 = X[0] * X[0] + X[1] * X[1] + X[2] * X[2];
    const f2 inv = rsq2(n2);
    *n = (n2 * inv).x;
    return make_float4((inv * X[0]).x, (inv * X[1]).x, (inv * X[2]).x, sw);
  } else {
    return make_float4(Xi[0], Xi[1], Xi[2], sw);
  }
}

// the record of point k of shard edge e (ix, jx: its pose ranks), every load in order (the fused pack of the first
// linearisation, ba_lin_kernel<PACK>); the per-edge streams are non-temporal
template <int MODE>
__device__ __forceinline__ float4 pack_record(const BaArgs& a, const BaParams& p, int e, int ix, int jx, int k,
                                              float* n) {
  const size_t g = (size_t)(e + p.edge_offset) * p.N + k;
  const bool vm = BA_NT_LOAD(&a.valid[g]) != 0;
  const int64_t ind = vm ? BA_NT_LOAD(&a.idx[g]) : 0;
  const float* Xi = a.Xkf[ix] + (size_t)ind * 3;
  const float q = BA_NT_LOAD(&a.Q[g]);
  const bool valid = vm && (q > p.Q_thresh) && (a.Ckf[ix][ind] * a.Cscale[ix] > p.C_thresh) &&
                     (BA_NT_LOAD(&a.Ckf[jx][k]) * a.Cscale[jx] > p.C_thresh);
  return pack_finish<MODE>(p, Xi, ind, q, valid, n);
}

// a record as stored (pack_record) -> as computed on: calib {u_t, v_t, log z_i, sw} (exact: integers < 2^16)
template <int MODE>
__device__ __forceinline__ float4 rec_expand(float4 r) {
  if constexpr (MODE == BA_MODE_CALIB) {
    const unsigned uv = __builtin_bit_cast(unsigned, r.x);
    return make_float4((float)(uv & 0xffffu), (float)(uv >> 16), r.y, r.z);
  } else {
    return r;
  }
}
template <int MODE>
__device__ __forceinline__ void rec_store(float4* slot, int k, float4 r) {
  // records: streamed out once per call (non-temporal under BA_PACK_NT, like the pack's input streams)
#if BA_PACK_NT
  if constexpr (MODE == BA_MODE_CALIB) {
    // three 4-B stores, 12 B by construction: a vec3 store may legally be widened to 16 B, which would overwrite the
    // next record's first word (the backend merges these into one dwordx3)
    float* d = reinterpret_cast<float*>(slot) + 3 * (size_t)k;
    __builtin_nontemporal_store(r.x, d);
    __builtin_nontemporal_store(r.y, d + 1);
    __builtin_nontemporal_store(r.z, d + 2);
  } else {
    typedef float f4v __attribute__((ext_vector_type(4)));
    __builtin_nontemporal_store(f4v{r.x, r.y, r.z, r.w}, reinterpret_cast<f4v*>(slot + k));
  }
#else
  if constexpr (MODE == BA_MODE_CALIB) reinterpret_cast<float3*>(slot)[k] = make_float3(r.x, r.y, r.z);
  else slot[k] = r;
#endif
}
template <int MODE>
__device__ __forceinline__ float4 rec_load(const float4* slot, int k) {
  if constexpr (MODE == BA_MODE_CALIB) {
    const float3 c = reinterpret_cast<const float3*>(slot)[k];
    return make_float4(c.x, c.y, c.z, 0.0f);
  } else {
    return slot[k];
  }
}

// record slot s (m3s_ba.h ba_rec_slot_bytes): N records, then the rays' |Xi| at rec + N
__device__ __forceinline__ float4* rec_of_slot(const BaArgs& a, int s, int N) {
  return reinterpret_cast<float4*>(reinterpret_cast<char*>(a.rec) + (size_t)s * ba_rec_slot_bytes(N));
}

// One block per tile of BA_PACK_TILE points of one edge: the edge's slot, ranks, keyframe pointers and confidence
// scales are block-uniform (scalar loads, once per block, not per point). A lane takes BA_PACK_UNROLL points per trip
// (256 apart): every per-point stream load (valid, idx, Q, C_j; non-temporal, unconditional at a clamped index) is
// issued first, then the X_i / C_i gathers, then the stores, so a point's chain is two loads deep and the trip's
// points overlap. Tiles in XCD-contiguous order: the blocks of XCD x (blockIdx % 8 == x) take the x-th eighth of
// the tile list, whose edges the plan orders by source keyframe, so an XCD gathers its own source keyframes' X_i / C_i.
#ifndef BA_PACK_TILE
#define BA_PACK_TILE 4096
#endif
#ifndef BA_PACK_UNROLL
#define BA_PACK_UNROLL 4
#endif
template <int MODE>
__global__ void __launch_bounds__(256) ba_pack_kernel(BaArgs a, BaParams p, int n_pack, int tiles_per_edge) {
  constexpr int U = BA_PACK_UNROLL;
  const int N = p.N;
  const int n_tiles = n_pack * tiles_per_edge;
  const int tile = (blockIdx.x % 8) * (gridDim.x / 8) + blockIdx.x / 8;  // gridDim.x: a multiple of 8
  if (tile >= n_tiles) return;
  const int t = tile / tiles_per_edge, c = tile - t * tiles_per_edge;
  const int e = a.pack_list ? a.pack_list[t] : t;
  const int ix = a.ii_rank[e], jx = a.jj_rank[e];
  const float* __restrict__ Xi = a.Xkf[ix];
  const float* __restrict__ Ci = a.Ckf[ix];
  const float* __restrict__ Cj = a.Ckf[jx];
  const float si = a.Cscale[ix], sj = a.Cscale[jx];
  float4* rec = rec_of_slot(a, a.rec_slot ? a.rec_slot[e] : e, N);
  const size_t g0 = (size_t)(e + p.edge_offset) * N;
  const int k_begin = c * BA_PACK_TILE, k_end = min(N, k_begin + BA_PACK_TILE);
  for (int k0 = k_begin + (int)threadIdx.x; k0 < k_end; k0 += 256 * U) {
    unsigned char vm[U];
    int64_t id[U];
    float q[U], cj[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int k = min(k0 + 256 * u, k_end - 1);
      vm[u] = BA_NT_LOAD(&a.valid[g0 + k]);
      id[u] = BA_NT_LOAD(&a.idx[g0 + k]);
      q[u] = BA_NT_LOAD(&a.Q[g0 + k]);
      cj[u] = BA_NT_LOAD(&Cj[k]);
    }
    float X[U][3], ci[U];
    int64_t ind[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      ind[u] = vm[u] ? id[u] : 0;  // gn_kernels.cu reads index 0 for an invalid match
      X[u][0] = Xi[(size_t)ind[u] * 3];
      X[u][1] = Xi[(size_t)ind[u] * 3 + 1];
      X[u][2] = Xi[(size_t)ind[u] * 3 + 2];
      ci[u] = Ci[ind[u]];
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int k = k0 + 256 * u;
      if (k >= k_end) continue;
      const bool valid = vm[u] && (q[u] > p.Q_thresh) && (ci[u] * si > p.C_thresh) && (cj[u] * sj > p.C_thresh);
      float n = 0.0f;
      rec_store<MODE>(rec, k, pack_finish<MODE>(p, X[u], ind[u], q[u], valid, &n));
      if constexpr (MODE == BA_MODE_RAYS) __builtin_nontemporal_store(n, reinterpret_cast<float*>(rec + N) + k);
    }
  }
}

// Record reuse: keyframe k's points and confidences against the library's copy from the previous plan (exact bit
// compare, 3N + N words), dirty[k] = 1 on any difference and the copy refreshed. One block row per keyframe; a
// null entry (a keyframe no edge of this shard touches) is skipped. 16-B accesses where the buffers allow.
__device__ __forceinline__ bool cmp_refresh(const unsigned* __restrict__ src, unsigned* __restrict__ dst, size_t n) {
  bool diff = false;
  const size_t t0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x, st = (size_t)gridDim.x * blockDim.x;
  if (n % 4 == 0 && ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15) == 0) {
    const uint4* s4 = reinterpret_cast<const uint4*>(src);
    uint4* d4 = reinterpret_cast<uint4*>(dst);
    for (size_t i = t0; i < n / 4; i += st) {
      const uint4 v = s4[i], d = d4[i];
      if (v.x != d.x || v.y != d.y || v.z != d.z || v.w != d.w) {
        d4[i] = v;
        diff = true;
      }
    }
  } else {
    for (size_t i = t0; i < n; i += st)
      if (dst[i] != src[i]) {
        dst[i] = src[i];
        diff = true;
      }
  }
  return diff;
}

__global__ void __launch_bounds__(256) ba_kf_compare_kernel(const BaKfCopy* __restrict__ kf, int N, uint8_t* dirty) {
  const int k = blockIdx.y;
  const BaKfCopy c = kf[k];
  if (c.copy == nullptr) return;
  unsigned* sx = reinterpret_cast<unsigned*>(c.copy);
  bool diff = cmp_refresh(reinterpret_cast<const unsigned*>(c.X), sx, (size_t)3 * N);
  diff |= cmp_refresh(reinterpret_cast<const unsigned*>(c.C), sx + (size_t)3 * N, (size_t)N);
  if (__any(diff) && (threadIdx.x & 63) == 0) dirty[k] = 1;
}

// PACK: the first GN iteration of a call that packs every edge builds each point's record itself (pack_record, the
// same values) and stores it for the later iterations: the pack's gathers (HBM-bound) run under this kernel's
// VALU-bound rows instead of as a separate launch before it.
template <int MODE, bool PACK>  // specialised per residual type: one mode's registers, not the union of three
__global__ void __launch_bounds__(256, BA_LIN_WAVES) ba_lin_kernel(BaArgs a, BaParams p) {
  if (*a.done) return;
  // the plan's block table: edges grouped by target keyframe, consecutive blocks on one XCD (xcd_remap)
  const int code = a.lin_tab[xcd_remap(blockIdx.x, gridDim.x)];
  const int e = code / p.chunks;
  const int chunk = code - e * p.chunks;
  const int N = p.N;
  const int ix = a.ii_rank[e], jx = a.jj_rank[e];
  float Ti[8], Tj[8], Tij[8];
#pragma unroll
  for (int c = 0; c < 8; c++) {
    Ti[c] = a.Twc[ix * 8 + c];
    Tj[c] = a.Twc[jx * 8 + c];
  }
#if BA_LIN_MATRIX
  // T_ij in double (relSim3_d): in fp32 its translation t_j - t_i rounds at |t_i| (metres), an error coherent over
  // every point of the edge (C4 EuRoC graph: 2.6e-6 -> 5e-7 from the fp64 truth, scripts/ba_prec_exp.py)
  double Td[8];
  relSim3_d(Ti, Tj, Td);
#pragma unroll
  for (int c = 0; c < 8; c++) Tij[c] = (float)Td[c];
#else
  relSim3(Ti, Tj, Tij);
#endif
#if BA_LIN_MATRIX
  // the linear map of actSO3 (Y = X + 2w q x X + 2 q x (q x X), any |q|) times s, formed in fp64 once per block:
  // s (I + 2w[q]x + 2([q][q]^T - |q|^2 I)), kept as its difference from the identity, D = s R - I (Y = X + (D X + t)):
  // D is small for the near-identity relative poses of co-visible keyframes, so rounding it to fp32 costs far less
  // than rounding s R itself (which put the ill-conditioned 6-KF fixtures at 1.6-1.8e-5 from the fp64 truth)
  float M[9];
  {
    const double x = Td[3], y = Td[4], z = Td[5], w = Td[6], sc = Td[7];
    const double R[9] = {1.0 - 2.0 * (y * y + z * z), 2.0 * (x * y - z * w),       2.0 * (x * z + y * w),
                         2.0 * (x * y + z * w),       1.0 - 2.0 * (x * x + z * z), 2.0 * (y * z - x * w),
                         2.0 * (x * z - y * w),       2.0 * (y * z + x * w),       1.0 - 2.0 * (x * x + y * y)};
#pragma unroll
    for (int c = 0; c < 9; c++) {  // block-uniform: kept in SGPRs (the packed FMAs read them as scalar operands)
      const double d = sc * R[c] - ((c % 4 == 0) ? 1.0 : 0.0);
      M[c] = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, (float)d)));
    }
#pragma unroll
    for (int c = 0; c < 3; c++)
      Tij[c] = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, Tij[c])));
  }
#endif
  // the block's fp64 sums: a flush transposes the lanes' fp64 pair sums through LDS (s_fl: conflict-free, one
  // column per thread) and 7 threads per sum add its 128 lanes, then the 7 partials in order: ~40 instructions per
  // thread instead of a 6-level fp64 shuffle butterfly per sum (~110 VALU per sum and wave, ~15 % of the kernel)
  __shared__ double s_fl[BA_PAIR_HALF][256];
  __shared__ double s_red[35][7];
  __shared__ double s_tot[BA_NSUM];
  if (threadIdx.x < BA_NSUM) s_tot[threadIdx.x] = 0.0;
  float4* rec = rec_of_slot(a, a.rec_slot ? a.rec_slot[e] : e, N);
  float* rec_n = reinterpret_cast<float*>(rec + N);  // rays: |Xi|
  const float* Xj_base = a.Xkf[jx];
  const int per = (N + p.chunks - 1) / p.chunks;
  const int k_begin = chunk * per;
  const int k_end = min(N, k_begin + per);
  f2 fL[28], fv[7];  // fp32 run sums, one slot per point of the pair
#pragma unroll
  for (int c = 0; c < 28; c++) fL[c] = f2{0.0f, 0.0f};
#pragma unroll
  for (int c = 0; c < 7; c++) fv[c] = f2{0.0f, 0.0f};
  // a run's fp32 sums into the block's fp64 sums: the lanes of a pair trade the halves they own (pair_flush: fp64
  // adds from 0 in the order a per-lane accumulator would make them), then the LDS transpose above. A chunk is at
  // most BA_RUN_LEN rounds (ba_chunks), so this runs once per block and no fp64 accumulator is live across the point
  // loop: its VGPRs carry the next round's prefetched records instead. Block-uniform (barriers): every thread of
  // the block reaches every flush (the trip count is the block's).
  auto flush = [&]() {
    const int t = threadIdx.x;
    const bool odd = t & 1;
    double acc[BA_PAIR_HALF];
#pragma unroll
    for (int m = 0; m < BA_PAIR_HALF; m++) acc[m] = 0.0;
    pair_flush(acc, fL, fv, odd);
#pragma unroll
    for (int m = 0; m < BA_PAIR_HALF; m++) s_fl[m][t] = acc[m];
    __syncthreads();
    if (t < 35 * 7) {  // sum c: even lanes own 0..17, odd lanes 18..34
      const int c = t / 7, part = t - 7 * c;
      const int par = c >= BA_PAIR_HALF ? 1 : 0, m = c - BA_PAIR_HALF * par;
      double r = 0.0;
      for (int i = part; i < 128; i += 7) r += s_fl[m][2 * i + par];
      s_red[c][part] = r;
    }
    __syncthreads();
    if (t < 35) {
      double r = s_tot[t];
#pragma unroll
      for (int q = 0; q < 7; q++) r += s_red[t][q];
      s_tot[t] = r;
    }
#pragma unroll
    for (int c = 0; c < 28; c++) fL[c] = f2{0.0f, 0.0f};
#pragma unroll
    for (int c = 0; c < 7; c++) fv[c] = f2{0.0f, 0.0f};
  };
  // the rows of one round: two points per lane, (k0, k0 + blockDim): every per-point float operation runs on both at
  // once as one packed fp32 instruction (v_pk_fma/mul/add_f32; float2 lanes), the transcendentals per component.
  // R0, R1: the records as computed on (rec_expand); a missing second point (has1 false) repeats the first with
  // weight 0: it adds exact zeros unless the first point's own row is non-finite, which poisons the sums anyway
  // (another point as filler changed the rays sums)
  auto rows = [&](const float4& R0, const float4& R1, f2 nI, const f2* Xj, bool has1) {
    const f2 Rx = {R0.x, R1.x}, Ry = {R0.y, R1.y}, Rz = {R0.z, R1.z};
    // sqrt(q), 0 for an invalid match (ba_pack) and for the missing second point of a ragged tail
    const f2 sqq = {R0.w, has1 ? R1.w : 0.0f};
    f2 Y[3];
#if BA_LIN_MATRIX
    // actSim3 (gn_kernels.cu:207-219) as the edge's map X + (D X + t): three packed FMAs and an add per component
#pragma unroll
    for (int c = 0; c < 3; c++)
      Y[c] = Xj[c] + __builtin_elementwise_fma(
                         f2{M[3 * c], M[3 * c]}, Xj[0],
                         __builtin_elementwise_fma(f2{M[3 * c + 1], M[3 * c + 1]}, Xj[1],
                                                   __builtin_elementwise_fma(f2{M[3 * c + 2], M[3 * c + 2]}, Xj[2],
                                                                             f2{Tij[c], Tij[c]})));
#else
    actSO3_v(&Tij[3], Xj, Y);  // actSim3 (gn_kernels.cu:207-219): rotate, scale, translate
#pragma unroll
    for (int c = 0; c < 3; c++) Y[c] = Y[c] * Tij[7] + Tij[c];
#endif
    if constexpr (MODE == BA_MODE_POINTS) {
      const f2 err[3] = {Y[0] - Rx, Y[1] - Ry, Y[2] - Rz};
      const f2 sw = p.inv_a * sqq;
      const f2 wc = sw * sw;
      const f2 z2 = {0.0f, 0.0f}, o2 = {1.0f, 1.0f};
      const f2 J0[7] = {o2, z2, z2, z2, Y[2], -Y[1], Y[0]};
      const f2 J1[7] = {z2, o2, z2, -Y[2], z2, Y[0], Y[1]};
      const f2 J2[7] = {z2, z2, o2, Y[1], -Y[0], z2, Y[2]};
      acc_local_f2<0b1110001>(fL, fv, J0, huber_ba2(sw * err[0]) * wc, err[0]);  // {0,4,5,6}
      acc_local_f2<0b1101010>(fL, fv, J1, huber_ba2(sw * err[1]) * wc, err[1]);  // {1,3,5,6}
      acc_local_f2<0b1011100>(fL, fv, J2, huber_ba2(sw * err[2]) * wc, err[2]);  // {2,3,4,6}
    } else if constexpr (MODE == BA_MODE_RAYS) {
      // the record holds ri = Xi / |Xi| and rec_n |Xi| (pack_record: the same operations, once per call)
      const f2 n1i = nI;
      const f2 n2j = Y[0] * Y[0] + Y[1] * Y[1] + Y[2] * Y[2];
      const f2 n1j_inv = rsq2(n2j);
      const f2 n1j = n2j * n1j_inv;
      const f2 rj[3] = {n1j_inv * Y[0], n1j_inv * Y[1], n1j_inv * Y[2]};
      const f2 err[4] = {rj[0] - Rx, rj[1] - Ry, rj[2] - Rz, n1j - n1i};
      const f2 swr = p.inv_a * sqq;
      const f2 swd = p.inv_b * sqq;
      const f2 wr = swr * swr, wd = swd * swd;
      const f2 n3 = n1j_inv * rcp2(n2j);
      const f2 dxx = n1j_inv - Y[0] * Y[0] * n3;
      const f2 dyy = n1j_inv - Y[1] * Y[1] * n3;
      const f2 dzz = n1j_inv - Y[2] * Y[2] * n3;
      const f2 dxy = -Y[0] * Y[1] * n3;
      const f2 dxz = -Y[0] * Y[2] * n3;
      const f2 dyz = -Y[1] * Y[2] * n3;
      const f2 z2 = {0.0f, 0.0f};
      const f2 J0[7] = {dxx, dxy, dxz, z2, rj[2], -rj[1], z2};
      const f2 J1[7] = {dxy, dyy, dyz, -rj[2], z2, rj[0], z2};
      const f2 J2[7] = {dxz, dyz, dzz, rj[1], -rj[0], z2, z2};
      const f2 J3[7] = {rj[0], rj[1], rj[2], z2, z2, z2, n1j};
      acc_local_f2<0b0110111>(fL, fv, J0, huber_ba2(swr * err[0]) * wr, err[0]);  // {0,1,2,4,5}
      acc_local_f2<0b0101111>(fL, fv, J1, huber_ba2(swr * err[1]) * wr, err[1]);  // {0,1,2,3,5}
      acc_local_f2<0b0011111>(fL, fv, J2, huber_ba2(swr * err[2]) * wr, err[2]);  // {0,1,2,3,4}
      acc_local_f2<0b1000111>(fL, fv, J3, huber_ba2(swd * err[3]) * wd, err[3]);  // {0,1,2,6}
    } else {  // calib
      const f2 u_t = Rx, v_t = Ry, lzi = Rz;  // lzi: log z_i, NaN where z_i <= z_eps (pack_record)
      const auto valid_z = (Y[2] > p.z_eps) & (lzi == lzi);
      const f2 z2 = {0.0f, 0.0f};
      const f2 zj_inv = valid_z ? f2{__builtin_amdgcn_rcpf(Y[2].x), __builtin_amdgcn_rcpf(Y[2].y)} : z2;
      const f2 zj_log = valid_z ? f2{__logf(Y[2].x), __logf(Y[2].y)} : z2;
      const f2 zi_log = valid_z ? lzi : z2;
      const f2 xz = Y[0] * zj_inv, yz = Y[1] * zj_inv;
      const f2 u = BA_FMA2(f2{p.fx, p.fx}, xz, f2{p.cx, p.cx}), vv = BA_FMA2(f2{p.fy, p.fy}, yz, f2{p.cy, p.cy});
      const float ub = (float)p.pixel_border, uh = (float)(p.W - 1 - p.pixel_border),
                  vh = (float)(p.H - 1 - p.pixel_border);
      const auto valid = (u > ub) & (u < uh) & (vv > ub) & (vv < vh) & valid_z;
      const f2 err[3] = {u - u_t, vv - v_t, zj_log - zi_log};
      const f2 swp = valid ? p.inv_a * sqq : z2;
      const f2 swd = valid ? p.inv_b * sqq : z2;
      const f2 wp = swp * swp, wd = swd * swd;
      const float fx = p.fx, fy = p.fy;
      const f2 o2 = {1.0f, 1.0f};
      const f2 J0[7] = {fx * zj_inv, z2, -fx * xz * zj_inv, -fx * xz * yz, fx * BA_FMA2(xz, xz, o2), -fx * yz, z2};
      const f2 J1[7] = {z2, fy * zj_inv, -fy * yz * zj_inv, -fy * BA_FMA2(yz, yz, o2), fy * xz * yz, fy * xz, z2};
      const f2 J2[7] = {z2, z2, zj_inv, yz, -xz, z2, o2};
      acc_local_f2<0b0111101>(fL, fv, J0, huber_ba2(swp * err[0]) * wp, err[0]);  // {0,2,3,4,5}
      acc_local_f2<0b0111110>(fL, fv, J1, huber_ba2(swp * err[1]) * wp, err[1]);  // {1,2,3,4,5}
      acc_local_f2<0b1011100>(fL, fv, J2, huber_ba2(swd * err[2]) * wd, err[2]);  // {2,3,4,6}
    }
  };
  int run = 0;
  // a block-uniform trip count: every lane reaches each run flush together (the pair flush swaps run sums between
  // the lanes of a pair); a lane past the chunk's end skips the point work
  if constexpr (PACK) {
    for (int k00 = k_begin; k00 < k_end; k00 += 2 * blockDim.x) {
      const int k0 = k00 + (int)threadIdx.x;
      if (k0 < k_end) {
        const int k1 = k0 + (int)blockDim.x;
        const bool has1 = k1 < k_end;
        const int k1c = has1 ? k1 : k0;
        float n0 = 0.0f, n1 = 0.0f;
        float4 R0 = pack_record<MODE>(a, p, e, ix, jx, k0, &n0), R1;
        n1 = n0;
        if (has1) R1 = pack_record<MODE>(a, p, e, ix, jx, k1, &n1);
        else R1 = R0;
        rec_store<MODE>(rec, k0, R0);
        if (has1) rec_store<MODE>(rec, k1, R1);
        if constexpr (MODE == BA_MODE_RAYS) {
          rec_n[k0] = n0;
          if (has1) rec_n[k1] = n1;
        }
        f2 Xj[3];
#pragma unroll
        for (int c = 0; c < 3; c++) Xj[c] = f2{Xj_base[(size_t)k0 * 3 + c], Xj_base[(size_t)k1c * 3 + c]};
        rows(rec_expand<MODE>(R0), rec_expand<MODE>(R1), f2{n0, n1}, Xj, has1);
      }
      if (++run == BA_RUN_LEN) {
        run = 0;
        flush();
      }
    }
  } else {
    // software-pipelined: a lane loads the next round's records and X_j before it computes this round's rows, so
    // the loads' HBM latency runs under the VALU work (the kernel holds 3 waves per SIMD, too few to hide it alone).
    // Every load is unconditional (a lane past the chunk's end loads point k_begin and skips the rows): the hand-over
    // nxt -> cur at the end of a round is then the only use of a load in flight, after the round's rows.
    struct Round {
      float4 R0, R1;  // as stored (rec_load)
      f2 nI;          // rays: |Xi| of both points
      f2 Xj[3];
    };
    auto fetch = [&](int k00, Round& r) {
      const int k0 = k00 + (int)threadIdx.x < k_end ? k00 + (int)threadIdx.x : k_begin;
      const int k1 = k0 + (int)blockDim.x < k_end ? k0 + (int)blockDim.x : k0;
      r.R0 = rec_load<MODE>(rec, k0);
      r.R1 = rec_load<MODE>(rec, k1);
      if constexpr (MODE == BA_MODE_RAYS) r.nI = f2{rec_n[k0], rec_n[k1]};
#pragma unroll
      for (int c = 0; c < 3; c++) r.Xj[c] = f2{Xj_base[(size_t)k0 * 3 + c], Xj_base[(size_t)k1 * 3 + c]};
    };
    Round cur;
    fetch(k_begin, cur);
    for (int k00 = k_begin; k00 < k_end; k00 += 2 * blockDim.x) {
      const int k0 = k00 + (int)threadIdx.x;
      Round nxt;
      fetch(k00 + 2 * blockDim.x, nxt);
      if (k0 < k_end) {
        f2 nI = {0.0f, 0.0f};
        if constexpr (MODE == BA_MODE_RAYS) nI = cur.nI;
        rows(rec_expand<MODE>(cur.R0), rec_expand<MODE>(cur.R1), nI, cur.Xj, k0 + (int)blockDim.x < k_end);
      }
      if (++run == BA_RUN_LEN) {
        run = 0;
        flush();
      }
      cur = nxt;
    }
  }
  flush();
  if (threadIdx.x < 35) a.partials[(size_t)code * BA_NSUM + threadIdx.x] = s_tot[threadIdx.x];  // its own entry
}

// per-edge: sum chunk partials, M = A L A^T, g = A v with A the adjoint-inverse map of T_i.
// Writes edge_sums[(e + edge_offset) * 36 + {0..27: M upper, 28..34: g}].
__global__ void __launch_bounds__(64) ba_edge_kernel(BaArgs a, BaParams p, int E_local) {
  if (*a.done) return;
  const int e = blockIdx.x;
  if (e >= E_local) return;
  __shared__ double s_L[7][7], s_v[7], s_A[7][7], s_AL[7][7];
  const int t = threadIdx.x;
  if (t < 35) {
    // the chunk partials in chunk order, eight loads in flight at a time (one at a time they were a chain of
    // dependent round trips per edge); clamped loads past the last chunk are not added
    double s = 0.0;
    const double* pe = a.partials + (size_t)e * p.chunks * BA_NSUM + t;
    for (int c0 = 0; c0 < p.chunks; c0 += 8) {
      double v[8];
#pragma unroll
      for (int k = 0; k < 8; k++) v[k] = pe[(size_t)min(c0 + k, p.chunks - 1) * BA_NSUM];
#pragma unroll
      for (int k = 0; k < 8; k++)
        if (c0 + k < p.chunks) s += v[k];
    }
    if (t < 28) {
      int r = 0, l = t;
      while (l >= 7 - r) {
        l -= 7 - r;
        r++;
      }
      const int c = r + l;
      s_L[r][c] = s;
      s_L[c][r] = s;
    } else {
      s_v[t - 28] = s;
    }
  }
  if (t < 7) {  // column t of A: adj_inv_row(e_t) (linear map, gn_kernels.cu:277-297), in float as the reference
    const int ix = a.ii_rank[e];
    float Ti[8];
    for (int c = 0; c < 8; c++) Ti[c] = a.Twc[ix * 8 + c];
    float X[7] = {0, 0, 0, 0, 0, 0, 0}, Y[7];
    X[t] = 1.0f;
    adj_inv_row(Ti, X, Y);
    for (int r = 0; r < 7; r++) s_A[r][t] = (double)Y[r];
  }
  __syncthreads();
  if (t < 49) {
    const int r = t / 7, c = t % 7;
    double s = 0.0;
    for (int k = 0; k < 7; k++) s += s_A[r][k] * s_L[k][c];
    s_AL[r][c] = s;
  }
  __syncthreads();
  double* out = a.edge_sums + (size_t)(e + p.edge_offset) * BA_NSUM;
  if (t < 28) {
    int r = 0, l = t;
    while (l >= 7 - r) {
      l -= 7 - r;
      r++;
    }
    const int c = r + l;
    double s = 0.0;
    for (int k = 0; k < 7; k++) s += s_AL[r][k] * s_A[c][k];
    out[t] = s;
  } else if (t < 35) {
    const int r = t - 28;
    double s = 0.0;
    for (int k = 0; k < 7; k++) s += s_A[r][k] * s_v[k];
    out[t] = s;
  }
}

// ------------------------------------------------------------------------------------------
// Block-sparse pose system (SparseBlock + SimplicialLLT, gn_kernels.cu:57-159), pattern analysed once
// per plan on the host (ba_pattern.cpp: minimum-degree order, 7x7-block factor pattern, elimination-tree
// levels, per-level update lists).
//
// ba_assemble_kernel: one 64-lane block per factor block (fill blocks are written as zeros, so the
// factor storage needs no clearing) and one per rhs block row; contributions summed in the plan's
// fixed edge order (deterministic: identical on every rank).
//
// ba_sparse_factor_kernel: ONE workgroup of 16 waves factors, solves and retracts. The work is a few
// MFLOP, so what bounds it is the dependency chain through the elimination tree, not throughput; in one
// workgroup every hand-off is a __syncthreads (tens of ns) instead of a cross-CU flag (1-3 us each,
// MI355X_MICROARCH.md "handoff-flag"), and the factor (<= 1 MB at K = 256) stays in this CU's L1/L2.
// Level by level of the elimination tree:
//   A. every column of the level (one wave each): 7x7 Cholesky of the diagonal block (lane-redundant,
//      in registers), then one lane per row of its off-diagonal blocks and of its rhs block solves
//      x L_jj^T = a  -> L_ij, and the forward substitution y_j = L_jj^-1 b_j;
//   B. every column j that the level's columns update (one wave each, sources in ascending order):
//      L(i,j) -= L_ik L_jk^T for the rows i >= j of column k, and b_j -= L_jk y_k (right-looking, so
//      the update work of a level runs in parallel instead of on the chain of the column it feeds).
// Then the back substitution x_j = L_jj^-T (y_j - sum_i L_ij^T x_i), levels from the root down; then
// dx = -x in pose order (0 on a failed pivot: the reference's silent zero step), the Sim(3) retraction
// and the |dx| early exit.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void ba_assemble_one(const BaArgs& a, int nL, int b, int t);

// xcd_stride 8: only the blocks dispatched to XCD 0 work, each on items b / 8, b / 8 + nwork, ... (the factor steps and
// the one-workgroup kernel then read the assembled blocks from that XCD's L2)
__global__ void __launch_bounds__(64) ba_assemble_kernel(BaArgs a, int nL, int xcd_stride) {
  if (*a.done) return;
  if (xcd_stride > 1 && blockIdx.x % xcd_stride != 0) return;
  const int nwork = gridDim.x / xcd_stride;
  for (int b = blockIdx.x / xcd_stride; b < nL + a.nb; b += nwork) ba_assemble_one(a, nL, b, threadIdx.x);
}

__device__ __forceinline__ void ba_assemble_one(const BaArgs& a, int nL, int b, int t) {
  if (b == 0 && t == 0) *a.bad = 0;  // the multi-workgroup factor steps of this solve start clean
  const int* ptr = b < nL ? a.asm_ptr + b : a.rhs_ptr + (b - nL);
  const int* ent = b < nL ? a.asm_ent : a.rhs_ent;
  int li;
  double* out;
  if (b < nL) {
    if (t >= 49) return;
    const int rr = t / 7, cc = t - 7 * (t / 7);
    // M stored upper: index of (min,max)
    const int lo = min(rr, cc), hi = max(rr, cc);
    li = lo * 7 - lo * (lo - 1) / 2 + (hi - lo);
    out = a.L + (size_t)b * 64 + rr * 8 + cc;
  } else {
    if (t >= 7) return;
    li = 28 + t;
    out = a.y + (size_t)(b - nL) * 8 + t;
  }
  // contributions summed in CSR order (deterministic); indices and values of 4 at a time in flight
  double s = 0.0;
  const int kb = ptr[0], ke = ptr[1];
  int k = kb;
  for (; k + 4 <= ke; k += 4) {
    int e[4];
    double v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) e[u] = ent[k + u];
#pragma unroll
    for (int u = 0; u < 4; u++) v[u] = a.edge_sums[(size_t)(e[u] >> 1) * BA_NSUM + li];
#pragma unroll
    for (int u = 0; u < 4; u++) s += ((e[u] & 1) ? -1.0 : 1.0) * v[u];
  }
  for (; k < ke; k++) {
    const int e = ent[k];
    s += ((e & 1) ? -1.0 : 1.0) * a.edge_sums[(size_t)(e >> 1) * BA_NSUM + li];
  }
  *out = s;
}

constexpr int SP_WAVES = 16;                 // waves of the factor workgroup
static_assert(SP_WAVES == M3S_BA_SP_WAVES, "the host's schedules assume the kernel's wave count");
constexpr int SP_PLAN_BYTES = 144 * 1024;   // LDS for the plan's loop tables and the solution x

// 1/sqrt(d) for d > 0: the v_rsq_f64 estimate (~2^-22 relative) refined by ONE Newton step (~2^-44)
__device__ __forceinline__ double rsqrt_nr(double d) {
  const double y = __builtin_amdgcn_rsq(d);
  return fma(y, fma(-0.5 * d * y, y, 0.5), y);
}

// lanes of one wave exchanging data through LDS: a compiler memory barrier (the hardware returns a
// wave's LDS accesses in order)
__device__ __forceinline__ void wave_sync() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ double bcast_lane(double v, int src) {
  int2 x = *reinterpret_cast<int2*>(&v);
  x.x = __builtin_amdgcn_readlane(x.x, src);
  x.y = __builtin_amdgcn_readlane(x.y, src);
  return *reinterpret_cast<double*>(&x);
}

// one 8-double row of a factor block (64-B aligned) as four 16-B accesses
__device__ __forceinline__ void ld_row(double (&v)[8], const double* p) {
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const double2 t = reinterpret_cast<const double2*>(p)[q];
    v[2 * q] = t.x;
    v[2 * q + 1] = t.y;
  }
}
__device__ __forceinline__ void st_row(double* p, const double (&v)[8]) {
#pragma unroll
  for (int q = 0; q < 4; q++) reinterpret_cast<double2*>(p)[q] = make_double2(v[2 * q], v[2 * q + 1]);
}

#ifdef M3S_SP_STAMPS  // (experiment builds only) s_memrealtime after every barrier of the factor kernel
__device__ unsigned long long g_sp_stamps[4096];
#define SPST(k)                                                                               \
  do {                                                                                        \
    if (threadIdx.x == 0 && (k) < 3000) g_sp_stamps[k] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#define FST(k)                                                                              \
  do {                                                                                      \
    if (lane == 0) g_sp_stamps[3000 + (k)] = __builtin_amdgcn_s_memrealtime();            \
  } while (0)
#define TST(k)                                                                                   \
  do {                                                                                           \
    if (lane == 0 && (k) < 2000) g_sp_stamps[1000 + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define TST(k) \
  do {         \
  } while (0)
#define SPST(k) \
  do {          \
  } while (0)
#define FST(k) \
  do {         \
  } while (0)
#endif

// the plan's loop tables (LDS when they fit)
struct SpTables {
  const int* col_ptr;
  const int* rowL;
  const int* lev_ptr;
  const int* lev_col;
  const int* grp_ptr;
  const int4* grp;
  const int* pull_grp;
  const int4* src;
  const int* sidx;
  const int* sched;
};

// the loop tables at `base`: the plan's table region [plan_lo, plan_lo + plan_bytes) staged to `base` (LDS), or
// base = plan_lo itself (global)
__device__ __forceinline__ SpTables sp_tables(const BaArgs& a, const int* base) {
  const int* g = reinterpret_cast<const int*>(a.plan_lo);
  SpTables T;
  T.col_ptr = base + (a.col_ptr - g);
  T.rowL = base + (a.rowL - g);
  T.lev_ptr = base + (a.lev_ptr - g);
  T.lev_col = base + (a.lev_col - g);
  T.grp_ptr = base + (a.grp_ptr - g);
  T.grp = reinterpret_cast<const int4*>(base + (reinterpret_cast<const int*>(a.grp) - g));
  T.pull_grp = base + (a.pull_grp - g);
  T.src = reinterpret_cast<const int4*>(base + (reinterpret_cast<const int*>(a.src) - g));
  T.sidx = base + (a.sidx - g);
  T.sched = base + (a.sched - g);
  return T;
}

// the rows of a column: row p < 7 (noff + 1) is row p % 7 of the column's block p / 7 (block 0 = the
// diagonal block), row 7 (noff + 1) is the rhs block y_j
__device__ __forceinline__ double* sp_row_addr(const BaArgs& a, int b0, int noff, int j, int p) {
  return p < 7 * (noff + 1) ? a.L + (size_t)(b0 + p / 7) * 64 + (p - 7 * (p / 7)) * 8 : a.y + (size_t)j * 8;
}

// the source row of row p of column j for one group source (pl: block of L_jk, k, sidx offset): row p % 7
// of the block of column k at the same block row, y_k for the rhs row, nullptr where struct(k) misses it
__device__ __forceinline__ const double* sp_src_addr(const BaArgs& a, const SpTables& T, const int4& pl, int noff,
                                                     int p) {
  if (p == 7 * (noff + 1)) return a.y + (size_t)pl.y * 8;
  const int sb = T.sidx[pl.z + p / 7];
  return sb >= 0 ? a.L + (size_t)sb * 64 + (p - 7 * (p / 7)) * 8 : nullptr;
}

// v[0..6] -= x L_jk^T with L_jk (49 doubles, row-major 7x7) in LDS: a short dependency tree per output
__device__ __forceinline__ void sp_apply(double (&v)[8], const double (&x)[8], const double* bjk) {
#pragma unroll
  for (int c = 0; c < 7; c++) {
    const double* bc = bjk + c * 7;
    const double p0 = fma(x[0], bc[0], x[1] * bc[1]);
    const double p1 = fma(x[2], bc[2], x[3] * bc[3]);
    const double p2 = fma(x[4], bc[4], x[5] * bc[5]);
    v[c] -= (p0 + p1) + fma(x[6], bc[6], p2);
  }
}

__device__ __forceinline__ double sp_ljk(const BaArgs& a, int blk, int lane) {
  return lane < 49 ? a.L[(size_t)blk * 64 + (lane / 7) * 8 + lane - 7 * (lane / 7)] : 0.0;
}

// apply the sources of group g to the rows p1 = lane and p2 = lane + 64 of column j held in v1 / v2
// (rows beyond nrow are idle). Columns of at most 64 rows (the common case) issue the next source's
// loads before the current one is applied.
__device__ __forceinline__ void sp_group_regs(const BaArgs& a, const SpTables& T, int2 gr, int noff, int nrow,
                                              double (&v1)[8], double (&v2)[8], int lane, double* bjk) {
  if (gr.x >= gr.y) return;
  const int p1 = lane, p2 = lane + 64;
  if (nrow <= 64) {
    int4 pl = T.src[gr.x];
    const double* s1 = p1 < nrow ? sp_src_addr(a, T, pl, noff, p1) : nullptr;
    double bv = sp_ljk(a, pl.x, lane);
    double x1[8];
    if (s1) ld_row(x1, s1);
    for (int e = gr.x; e < gr.y; e++) {
      const bool more = e + 1 < gr.y;
      const double* n1 = nullptr;
      double nbv = 0.0, y1[8];
      if (more) {
        const int4 nl = T.src[e + 1];
        n1 = p1 < nrow ? sp_src_addr(a, T, nl, noff, p1) : nullptr;
        nbv = sp_ljk(a, nl.x, lane);
        if (n1) ld_row(y1, n1);
      }
      wave_sync();  // the previous source's reads of bjk are done
      if (lane < 49) bjk[lane] = bv;
      wave_sync();
      if (s1) sp_apply(v1, x1, bjk);
      s1 = n1;
      bv = nbv;
#pragma unroll
      for (int c = 0; c < 8; c++) x1[c] = y1[c];
    }
  } else {
    for (int e = gr.x; e < gr.y; e++) {
      const int4 pl = T.src[e];
      const double* s1 = sp_src_addr(a, T, pl, noff, p1);
      const double* s2 = p2 < nrow ? sp_src_addr(a, T, pl, noff, p2) : nullptr;
      const double bv = sp_ljk(a, pl.x, lane);
      double x1[8], x2[8];
      if (s1) ld_row(x1, s1);
      if (s2) ld_row(x2, s2);
      wave_sync();
      if (lane < 49) bjk[lane] = bv;
      wave_sync();
      if (s1) sp_apply(v1, x1, bjk);
      if (s2) sp_apply(v2, x2, bjk);
    }
  }
  wave_sync();
}

// rows p >= 128 of column j (columns with more than 17 off-diagonal blocks), one pass of 64 rows at a
// time: group g's sources applied, then (when inv != nullptr) the triangular solve with L_jj
__device__ __forceinline__ void sp_rows_extra(const BaArgs& a, const SpTables& T, int j, int b0, int noff, int nrow,
                                              bool has_g, int2 gr, const double* lo, const double* inv, int lane,
                                              double* bjk) {
  for (int base = 128; base < nrow; base += 64) {
    const int p = base + lane;
    const bool act = p < nrow;
    double v[8];
    double* tp = act ? sp_row_addr(a, b0, noff, j, p) : nullptr;
    if (act) ld_row(v, tp);
    if (has_g) {
      for (int e = gr.x; e < gr.y; e++) {
        const int4 pl = T.src[e];
        const double bv = sp_ljk(a, pl.x, lane);
        const double* sp = act ? sp_src_addr(a, T, pl, noff, p) : nullptr;
        double x[8];
        if (sp) ld_row(x, sp);
        wave_sync();
        if (lane < 49) bjk[lane] = bv;
        wave_sync();
        if (sp) sp_apply(v, x, bjk);
      }
      wave_sync();
    }
    if (inv) {  // x L_jj^T = a, right-looking
#pragma unroll
      for (int m = 0; m < 7; m++) {
        v[m] *= inv[m];
#pragma unroll
        for (int c = m + 1; c < 7; c++) v[c] = fma(-v[m], lo[c * (c - 1) / 2 + m], v[c]);
      }
    }
    if (act) st_row(tp, v);
  }
}

// A. column j (one wave): its children's-level update group, then the register-row factorisation (lane
// p holds row p of the column; the diagonal rows' right-looking Cholesky steps are, for the rows below
// them, the triangular solve L_ij = A_ij L_jj^-T, and for the rhs row the forward substitution
// y_j = L_jj^-1 b_j), then the stores. Diagonal block afterwards: lower = L_jj, column 7 = 1/L_mm.
// j's blocks [b0, b1), its pull group's source range gr (has_g) come from the caller: the plan tables (factor
// kernel) or one task record (wide steps)
__device__ __forceinline__ void sp_factor_column_at(const BaArgs& a, const SpTables& T, int j, int b0, int b1,
                                                    bool has_g, int2 gr, int lane, double* bjk, int* bad) {
  const int noff = b1 - b0 - 1, nrow = 7 * (noff + 1) + 1;
  const bool has1 = lane < nrow, has2 = lane + 64 < nrow;
  double v1[8], v2[8];
  double* p1 = has1 ? sp_row_addr(a, b0, noff, j, lane) : nullptr;
  double* p2 = has2 ? sp_row_addr(a, b0, noff, j, lane + 64) : nullptr;
  if (has1) ld_row(v1, p1);
  if (has2) ld_row(v2, p2);
  if (has_g) sp_group_regs(a, T, gr, noff, nrow, v1, v2, lane, bjk);
  bool fail = false;
  double inv[7], lo[21];
#pragma unroll
  for (int m = 0; m < 7; m++) {
    double d = bcast_lane(v1[m], m);
    if (!(d > 0.0)) {  // not positive definite: the step is discarded (dx = 0), as SimplicialLLT's info
      fail = true;
      d = 1.0;
    }
    inv[m] = rsqrt_nr(d);
    const double l1 = v1[m] * inv[m], l2 = v2[m] * inv[m];
    v1[m] = lane == m ? d * inv[m] : l1;
    v2[m] = l2;
#pragma unroll
    for (int c = m + 1; c < 7; c++) {
      const double lc = bcast_lane(l1, c);
      lo[c * (c - 1) / 2 + m] = lc;
      v1[c] = fma(-l1, lc, v1[c]);
      v2[c] = fma(-l2, lc, v2[c]);
    }
  }
  if (fail && lane == 0) atomicOr(bad, BA_BAD_LLT);
  if (lane < 7) {  // 1/L_mm in column 7 of the diagonal block (used by the back substitution)
    double iv = inv[0];
#pragma unroll
    for (int m = 1; m < 7; m++) iv = lane == m ? inv[m] : iv;
    v1[7] = iv;
  }
  if (has1) st_row(p1, v1);
  if (has2) st_row(p2, v2);
  if (nrow > 128) sp_rows_extra(a, T, j, b0, noff, nrow, has_g, gr, lo, inv, lane, bjk);
}

__device__ __forceinline__ void sp_factor_column(const BaArgs& a, const SpTables& T, int j, int lane, double* bjk,
                                                 int* bad) {
  const int g = T.pull_grp[j];
  const int4 gq = g >= 0 ? T.grp[g] : make_int4(0, 0, 0, 0);
  sp_factor_column_at(a, T, j, T.col_ptr[j], T.col_ptr[j + 1], g >= 0, make_int2(gq.y, gq.z), lane, bjk, bad);
}

// B. update group g (one wave): the rows of its target column take the group's sources, loaded and
// stored once per group
__device__ __forceinline__ void sp_update_group_at(const BaArgs& a, const SpTables& T, int j, int b0, int b1, int2 gr,
                                                   int lane, double* bjk) {
  const int noff = b1 - b0 - 1, nrow = 7 * (noff + 1) + 1;
  const bool has1 = lane < nrow, has2 = lane + 64 < nrow;
  double v1[8], v2[8];
  double* p1 = has1 ? sp_row_addr(a, b0, noff, j, lane) : nullptr;
  double* p2 = has2 ? sp_row_addr(a, b0, noff, j, lane + 64) : nullptr;
  if (has1) ld_row(v1, p1);
  if (has2) ld_row(v2, p2);
  sp_group_regs(a, T, gr, noff, nrow, v1, v2, lane, bjk);
  if (has1) st_row(p1, v1);
  if (has2) st_row(p2, v2);
  if (nrow > 128) sp_rows_extra(a, T, j, b0, noff, nrow, true, gr, nullptr, nullptr, lane, bjk);
}

__device__ __forceinline__ void sp_update_group(const BaArgs& a, const SpTables& T, int g, int lane, double* bjk) {
  const int4 gq = T.grp[g];
  sp_update_group_at(a, T, gq.x, T.col_ptr[gq.x], T.col_ptr[gq.x + 1], make_int2(gq.y, gq.z), lane, bjk);
}

// back substitution of column j: x_j = L_jj^-T (y_j - sum_{i in struct(j)} L_ij^T x_i); X = the solution
// (LDS when it fits), 8 doubles per column
__device__ __forceinline__ void sp_back_column(const BaArgs& a, const SpTables& T, double* X, int j, int lane,
                                               double* red) {
  const int b0 = T.col_ptr[j], b1 = T.col_ptr[j + 1];
  const int q = lane / 7, m = lane - 7 * (lane / 7);
  const double* D = a.L + (size_t)b0 * 64;
  double dl[8][8];  // L_jj (lower) and 1/L_mm (column 7), issued before the sums
#pragma unroll
  for (int r = 0; r < 7; r++) {
    double row[8];
    ld_row(row, D + r * 8);
#pragma unroll
    for (int c = 0; c < 8; c++) dl[r][c] = row[c];
  }
  const double yv = lane < 7 ? a.y[(size_t)j * 8 + lane] : 0.0;
  double acc = 0.0;
  if (lane < 63)
    for (int b = b0 + 1 + q; b < b1; b += 9) {
      const double* Lb = a.L + (size_t)b * 64 + m;
      const double* xi = X + (size_t)T.rowL[b] * 8;
#pragma unroll
      for (int r = 0; r < 7; r++) acc = fma(Lb[r * 8], xi[r], acc);
    }
  red[lane] = acc;
  wave_sync();
  if (lane < 7) {
    double sacc = yv;
#pragma unroll
    for (int qq = 0; qq < 9; qq++) sacc -= red[qq * 7 + lane];  // fixed order: deterministic
    red[lane] = sacc;
  }
  wave_sync();
  double z[7];
#pragma unroll
  for (int mm = 0; mm < 7; mm++) z[mm] = red[mm];
  double x[7];
#pragma unroll
  for (int mm = 6; mm >= 0; mm--) {
    double vv = z[mm];
#pragma unroll
    for (int p = mm + 1; p < 7; p++) vv = fma(-dl[p][mm], x[p], vv);
    x[mm] = vv * dl[mm][7];
  }
  if (lane == 0) {
#pragma unroll
    for (int mm = 0; mm < 7; mm++) X[(size_t)j * 8 + mm] = x[mm];
  }
  wave_sync();
}

// ---- dataflow schedule (ba_pattern.h ba_flow_schedule): flags in LDS instead of a barrier per level ----
// Producers publish with a workgroup-scope release (their global stores of factor blocks, or LDS writes of x,
// complete first); consumers spin on an acquire load. All waves of the workgroup share one CU and its L1.
__device__ __forceinline__ int flow_ld(const int* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void flow_st(int* p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// wait until every source column of group range gr is factored and `cnt` (when non-null) reads q; wave-uniform
// Spins are bounded (~2^20 polls, tens of ms): a schedule that could not complete sets the STALL bit of `bad`
// (BA_BAD_STALL: dx = 0, the GN loop ends, and the host returns M3S_ESTALL) instead of hanging the workgroup. A
// wait abandoned because another wave already failed (a non-positive pivot, BA_BAD_LLT) is not a stall.
// force_stall (M3S_BA_FORCE_STALL, tests only): the wait is never satisfied.
constexpr int FLOW_MAX_SPINS = 1 << 20;
__device__ __forceinline__ void flow_wait_task(const SpTables& T, int2 gr, const int* fac, const int* cnt, int q,
                                               int lane, int* bad, bool force_stall) {
  const int ns = gr.y - gr.x;
  for (int base = 0; base == 0 || base < ns; base += 63) {
    const bool cs = lane < 63 && base + lane < ns;
    const int k = cs ? T.src[gr.x + base + lane].y : 0;
    const bool cc = lane == 63 && base == 0 && cnt != nullptr;
    int spins = 0;
    while (__ballot((cs && flow_ld(&fac[k]) == 0) || (cc && flow_ld(cnt) != q) || force_stall) != 0) {
      __builtin_amdgcn_s_sleep(1);
      if (*(volatile int*)bad) return;  // already failed (or stalled) elsewhere: stop waiting
      if (++spins > FLOW_MAX_SPINS) {
        if (lane == 0) atomicOr(bad, BA_BAD_STALL);
        return;
      }
    }
  }
}

// sp_back_column with its factor-block loads issued before the wait for x of struct(j) (flags xd); same
// arithmetic in the same order (bit-identical x)
__device__ __forceinline__ void sp_back_column_flow(const BaArgs& a, const SpTables& T, double* X, int* xd, int j,
                                                    bool wait, int lane, double* red, int* bad) {
  const int b0 = T.col_ptr[j], b1 = T.col_ptr[j + 1];
  const int q = lane / 7, m = lane - 7 * (lane / 7);
  const double* D = a.L + (size_t)b0 * 64;
  double dl[8][8];
#pragma unroll
  for (int r = 0; r < 7; r++) {
    double row[8];
    ld_row(row, D + r * 8);
#pragma unroll
    for (int c = 0; c < 8; c++) dl[r][c] = row[c];
  }
  const double yv = lane < 7 ? a.y[(size_t)j * 8 + lane] : 0.0;
  // this lane's first two blocks (b0 + 1 + q, + 9), loaded ahead of the wait
  const int bA = b0 + 1 + q, bB = bA + 9;
  const bool hA = lane < 63 && bA < b1, hB = lane < 63 && bB < b1;
  double LA[7], LB[7];
#pragma unroll
  for (int r = 0; r < 7; r++) {
    LA[r] = hA ? a.L[(size_t)bA * 64 + m + r * 8] : 0.0;
    LB[r] = hB ? a.L[(size_t)bB * 64 + m + r * 8] : 0.0;
  }
  const int iA = hA ? T.rowL[bA] : 0, iB = hB ? T.rowL[bB] : 0;
  for (int base = b0 + 1; wait && (base == b0 + 1 || base < b1); base += 64) {
    const bool c = base + lane < b1;
    const int i = c ? T.rowL[base + lane] : 0;
    int spins = 0;
    while (__ballot(c && flow_ld(&xd[i]) == 0) != 0) {
      __builtin_amdgcn_s_sleep(1);
      if (*(volatile int*)bad) break;
      if (++spins > FLOW_MAX_SPINS) {
        if (lane == 0) atomicOr(bad, BA_BAD_STALL);
        break;
      }
    }
  }
  double acc = 0.0;
  if (hA) {
    const double* xi = X + (size_t)iA * 8;
#pragma unroll
    for (int r = 0; r < 7; r++) acc = fma(LA[r], xi[r], acc);
  }
  if (hB) {
    const double* xi = X + (size_t)iB * 8;
#pragma unroll
    for (int r = 0; r < 7; r++) acc = fma(LB[r], xi[r], acc);
  }
  if (lane < 63)
    for (int b = bB + 9; b < b1; b += 9) {
      const double* Lb = a.L + (size_t)b * 64 + m;
      const double* xi = X + (size_t)T.rowL[b] * 8;
#pragma unroll
      for (int r = 0; r < 7; r++) acc = fma(Lb[r * 8], xi[r], acc);
    }
  red[lane] = acc;
  wave_sync();
  if (lane < 7) {
    double sacc = yv;
#pragma unroll
    for (int qq = 0; qq < 9; qq++) sacc -= red[qq * 7 + lane];  // fixed order: deterministic
    red[lane] = sacc;
  }
  wave_sync();
  double z[7];
#pragma unroll
  for (int mm = 0; mm < 7; mm++) z[mm] = red[mm];
  double x[7];
#pragma unroll
  for (int mm = 6; mm >= 0; mm--) {
    double vv = z[mm];
#pragma unroll
    for (int p = mm + 1; p < 7; p++) vv = fma(-dl[p][mm], x[p], vv);
    x[mm] = vv * dl[mm][7];
  }
  if (lane == 0) {
#pragma unroll
    for (int mm = 0; mm < 7; mm++) X[(size_t)j * 8 + mm] = x[mm];
    flow_st(&xd[j], 1);
  }
  wave_sync();
}

// One wide factor step l of the elimination tree (its level's factor tasks + the update groups whose sources
// sit one level below) as a multi-workgroup launch: one wave per task, the same per-task code and therefore
// the same arithmetic as inside ba_sparse_factor_kernel (bit-identical factor). The launch boundary orders
// the steps. The leaf end of a minimum-degree tree is wide (one workgroup's 16 waves took ~12 rounds per
// step there), the root end a chain of single columns, which stays inside the one-workgroup kernel.
// Each task reads one 32-B record built with the plan ({j, b0, b1, pull group} and the group's source range), in
// the same round trip as the early-exit flag: the level / column / group table lookups that used to precede the
// column's own loads (four dependent global round trips) are gone.
__global__ void __launch_bounds__(64) ba_sparse_step_kernel(BaArgs a, int rec_base, int na, int xcd_stride) {
  __shared__ double s_red[64];
  const int lane = threadIdx.x;
  // xcd_stride 8 (M3S_BA_XCD0, default): only the blocks dispatched to XCD 0 (blockIdx % 8 == 0) work, so every
  // step and the one-workgroup kernel share one XCD's L2
  if (xcd_stride > 1 && blockIdx.x % xcd_stride != 0) return;
  const int task = blockIdx.x / xcd_stride;
  const int4 r0 = a.step_rec[2 * (rec_base + task)], r1 = a.step_rec[2 * (rec_base + task) + 1];
  if (*a.done) return;
  const SpTables T = sp_tables(a, reinterpret_cast<const int*>(a.plan_lo));
  if (task < na) sp_factor_column_at(a, T, r0.x, r0.y, r0.z, r0.w >= 0, make_int2(r1.x, r1.y), lane, s_red, a.bad);
  else sp_update_group_at(a, T, r0.x, r0.y, r0.z, make_int2(r1.x, r1.y), lane, s_red);
}

template <bool LT>  // LT: the loop tables and x fit in LDS (index lookups are ds_reads), else global
__global__ void __launch_bounds__(1024) ba_sparse_factor_kernel(BaArgs a, int K, int nL, float delta_thresh) {
  if (*a.done) return;
  __shared__ __attribute__((aligned(16))) int s_plan[LT ? SP_PLAN_BYTES / 4 : 4];
  __shared__ double s_red[SP_WAVES][64];  // per-wave staging: L_jk and the back-substitution sums
  __shared__ float s_n2[SP_WAVES];
  __shared__ int s_bad;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  SPST(0);
  const int* g = reinterpret_cast<const int*>(a.plan_lo);
  const int xoff = ((a.plan_bytes + 15) & ~15) / 4;  // ints
  if constexpr (LT) {  // the loop tables into LDS: every thread's loads in flight at once
    const int4* src = reinterpret_cast<const int4*>(a.plan_lo);
    int4* dst = reinterpret_cast<int4*>(s_plan);
    const int n16 = (a.plan_bytes + 15) / 16;
    int4 tmp[8];
    for (int i0 = 0; i0 < n16; i0 += 8 * 1024) {
#pragma unroll
      for (int u = 0; u < 8; u++) tmp[u] = src[min(i0 + u * 1024 + (int)threadIdx.x, n16 - 1)];
#pragma unroll
      for (int u = 0; u < 8; u++) {
        const int i = i0 + u * 1024 + (int)threadIdx.x;
        if (i < n16) dst[i] = tmp[u];
      }
    }
  }
  const int* base = LT ? static_cast<const int*>(s_plan) : g;
  double* X = LT ? reinterpret_cast<double*>(s_plan + xoff) : a.xs;
  const SpTables T = sp_tables(a, base);
  const int nb = a.nb;
  // dataflow flags after x: update groups landed per column, factored per column, x done per column
  int* f_app = s_plan + xoff + 16 * nb;
  int* f_fac = f_app + nb;
  int* f_xd = f_fac + nb;
  const bool flow = LT && a.flow;
  if (flow) {
    const int* fac_init = a.sched + 2 * (SP_WAVES + 1);
    for (int i = threadIdx.x; i < nb; i += 1024) {
      f_app[i] = 0;
      f_fac[i] = fac_init[i];
      f_xd[i] = 0;
    }
  }
  if (threadIdx.x == 0) s_bad = 0;
  __syncthreads();
  SPST(1);
  const int nlev = a.nlev;
  if (flow) {
    // every wave walks its own task list (step order); a task waits only for its inputs
    const int* S = T.sched;
    const int2* wl = reinterpret_cast<const int2*>(S + 2 * (SP_WAVES + 1) + nb);
    for (int t = S[w]; t < S[w + 1]; t++) {
      const int2 tk = wl[t];
      if (tk.x >= 0) {
        const int j = tk.x, gp = T.pull_grp[j];
        const int4 gq = gp >= 0 ? T.grp[gp] : make_int4(0, 0, 0, 0);
        const int2 gr = make_int2(gq.y, gq.z);
        flow_wait_task(T, gr, f_fac, &f_app[j], tk.y, lane, &s_bad, a.force_stall);
        TST(2 * t);
        sp_factor_column_at(a, T, j, T.col_ptr[j], T.col_ptr[j + 1], gp >= 0, gr, lane, s_red[w], &s_bad);
        if (lane == 0) flow_st(&f_fac[j], 1);
      } else {
        const int4 gq = T.grp[-1 - tk.x];
        const int2 gr = make_int2(gq.y, gq.z);
        flow_wait_task(T, gr, f_fac, &f_app[gq.x], tk.y, lane, &s_bad, a.force_stall);
        TST(2 * t);
        sp_update_group_at(a, T, gq.x, T.col_ptr[gq.x], T.col_ptr[gq.x + 1], gr, lane, s_red[w]);
        if (lane == 0) flow_st(&f_app[gq.x], tk.y + 1);
      }
      TST(2 * t + 1);
      wave_sync();
    }
    __syncthreads();
    SPST(2 + nlev);
    const int* bs_ptr = S + SP_WAVES + 1;
    const int* bs_col = S + 2 * (SP_WAVES + 1) + nb + 2 * S[SP_WAVES];
    for (int t = bs_ptr[w]; t < bs_ptr[w + 1]; t++) {
      const int code = bs_col[t];
      sp_back_column_flow(a, T, X, f_xd, code & BA_BS_COL, (code & BA_BS_NOWAIT) == 0, lane, s_red[w], &s_bad);
      FST(t);
    }
  }
  // step l: factor the columns of level l (each pulls its children's-level updates first) beside the
  // push updates of level l-1 into the columns above level l
  for (int l = flow ? nlev + 1 : a.wide_steps; l <= nlev; l++) {
    const int c0 = l < nlev ? T.lev_ptr[l] : 0, na = l < nlev ? T.lev_ptr[l + 1] - c0 : 0;
    const int t0 = T.grp_ptr[l], nt = T.grp_ptr[l + 1] - t0;
    for (int task = w; task < na + nt; task += SP_WAVES) {
      if (task < na) sp_factor_column(a, T, T.lev_col[c0 + task], lane, s_red[w], &s_bad);
      else sp_update_group(a, T, t0 + task - na, lane, s_red[w]);
    }
    __syncthreads();
    SPST(2 + l);
  }
  // back substitution, levels from the root down; runs of single-column levels stay on wave 0 with no
  // barrier between them (X in LDS: a wave's LDS accesses are ordered)
  for (int l = flow ? -1 : nlev - 1; l >= 0; l--) {
    const int c0 = T.lev_ptr[l], c1 = T.lev_ptr[l + 1];
    for (int c = c0 + w; c < c1; c += SP_WAVES) sp_back_column(a, T, X, T.lev_col[c], lane, s_red[w]);
    const bool chain = LT && c1 - c0 == 1 && l > 0 && T.lev_ptr[l] - T.lev_ptr[l - 1] == 1;
    if (!chain) {
      __syncthreads();
      SPST(3 + nlev + (nlev - 1 - l));
    }
  }
  __syncthreads();
  SPST(3 + 2 * nlev);
  // the multi-workgroup factor launches (the wide steps) report through *a.bad
  const int ext_bad = a.wide_steps > 0 ? *(volatile int*)a.bad : 0;
  const bool failed = s_bad != 0 || ext_bad != 0;
  const bool stalled = ((s_bad | ext_bad) & BA_BAD_STALL) != 0;
  const int n = a.nb * 7;
  float n2 = 0.0f;
  for (int i = threadIdx.x; i < n; i += 1024) {
    const int j = i / 7, m = i - 7 * (i / 7);
    const float d = failed ? 0.0f : (float)(-X[(size_t)j * 8 + m]);
    a.dx[a.perm[j] * 7 + m] = d;
    n2 += d * d;
  }
  __syncthreads();
  for (int k = 1 + threadIdx.x; k < K; k += 1024) {
    float Tw[8], xi[7];
    for (int c = 0; c < 8; c++) Tw[c] = a.Twc[k * 8 + c];
    for (int c = 0; c < 7; c++) xi[c] = a.dx[(k - 1) * 7 + c];
    retrSim3_d(xi, Tw);  // fp64 retraction (m3s_common.hpp: fp32 expSim3 cancels for small steps)
    for (int c = 0; c < 8; c++) a.Twc[k * 8 + c] = Tw[c];
  }
  n2 = wave_sum(n2);
  if (lane == 0) s_n2[w] = n2;
  __syncthreads();
  if (threadIdx.x == 0) {
    float sum = 0.0f;
    for (int q = 0; q < SP_WAVES; q++) sum += s_n2[q];
    *a.iters += 1;
    if (sqrtf(sum) < delta_thresh) *a.done = 1;
    *a.info = failed ? 1 : 0;
    if (stalled) {  // sticky until the next plan; the loop ends (the host reports M3S_ESTALL)
      *a.stalled = 1;
      *a.done = 1;
    }
  }
  SPST(4 + 2 * nlev);
}

}  // namespace m3s

#ifdef M3S_SP_STAMPS
extern "C" int m3s_debug_sp_stamps(unsigned long long* out) {
  (void)hipDeviceSynchronize();
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(m3s::g_sp_stamps), sizeof(unsigned long long) * 4096) == hipSuccess ? 0 : -1;
}
#endif

// ------------------------------------------------------------------------------------------
extern "C" hipError_t m3s_launch_ba_kf_compare(const BaKfCopy* kf, int Kp, int N, uint8_t* dirty, hipStream_t s) {
  if (Kp <= 0) return hipSuccess;
  const unsigned bx = (unsigned)std::min<size_t>(((size_t)4 * N + 255) / 256, 64);
  hipLaunchKernelGGL(m3s::ba_kf_compare_kernel, dim3(bx, Kp), dim3(256), 0, s, kf, N, dirty);
  return hipGetLastError();
}

extern "C" hipError_t m3s_launch_ba_pack(const BaArgs* a, const BaParams* p, int n_pack, hipStream_t s) {
  if (n_pack <= 0) return hipSuccess;
  const int tiles = (p->N + BA_PACK_TILE - 1) / BA_PACK_TILE;
  const size_t blocks = ((size_t)n_pack * tiles + 7) & ~(size_t)7;  // a multiple of 8: the XCD-contiguous tile order
  if (blocks > 0x7fffffff) return hipErrorInvalidValue;
  const dim3 g((unsigned)blocks);
  if (p->mode == BA_MODE_CALIB)
    hipLaunchKernelGGL(m3s::ba_pack_kernel<BA_MODE_CALIB>, g, dim3(256), 0, s, *a, *p, n_pack, tiles);
  else if (p->mode == BA_MODE_RAYS)
    hipLaunchKernelGGL(m3s::ba_pack_kernel<BA_MODE_RAYS>, g, dim3(256), 0, s, *a, *p, n_pack, tiles);
  else
    hipLaunchKernelGGL(m3s::ba_pack_kernel<BA_MODE_POINTS>, g, dim3(256), 0, s, *a, *p, n_pack, tiles);
  return hipGetLastError();
}

// pack (first iteration of a call whose pack was deferred): the linearisation also builds and stores the records
extern "C" hipError_t m3s_launch_ba_lin(const BaArgs* a, const BaParams* p, int E_local, int pack, hipStream_t s) {
  if (E_local <= 0) return hipSuccess;
  const dim3 g(E_local * p->chunks);
#define BA_LIN_LAUNCH(M)                                                                        \
  do {                                                                                          \
    if (pack)                                                                                   \
      hipLaunchKernelGGL((m3s::ba_lin_kernel<M, true>), g, dim3(256), 0, s, *a, *p);              \
    else                                                                                        \
      hipLaunchKernelGGL((m3s::ba_lin_kernel<M, false>), g, dim3(256), 0, s, *a, *p);             \
  } while (0)
  if (p->mode == BA_MODE_POINTS)
    BA_LIN_LAUNCH(BA_MODE_POINTS);
  else if (p->mode == BA_MODE_RAYS)
    BA_LIN_LAUNCH(BA_MODE_RAYS);
  else
    BA_LIN_LAUNCH(BA_MODE_CALIB);
#undef BA_LIN_LAUNCH
  hipLaunchKernelGGL(m3s::ba_edge_kernel, dim3(E_local), dim3(64), 0, s, *a, *p, E_local);
  return hipGetLastError();
}

// assembly (nL factor blocks + nb rhs rows), then the one-workgroup factor / solve / retraction
// step_tasks / step_base / step_na: per wide step its tasks, its first task record, its factor tasks (the rest are
// update groups)

// XCD affinity of the solve (M3S_BA_XCD0, default on): every multi-workgroup factor step and the one-workgroup kernel
// (block 0) run on XCD 0, so each step reads the previous one's blocks from that XCD's L2 instead of across the
// fabric. Measured (scripts/gpu_r05_xcd.sh, same box, two pairs): solve C5 0.393 -> 0.375 ms, C4 0.424 -> 0.409 ms.
// The stride assumes the round-robin workgroup dispatch over 8 XCDs of an MI3xx part in SPX mode (one device = the
// whole package): it is used only when the device is a gfx94x / gfx950 that reports at least 8 x 32 CUs. A partition
// (CPX: one XCD per device, 32 CUs) or any other part gets stride 1, where the 7 of 8 idle blocks would be wasted
// dispatches and the L2 locality would not exist.
static int ba_xcd_stride() {
  static const int xs = [] {
    const char* e = getenv("M3S_BA_XCD0");
    if (e && atoi(e) == 0) return 1;
    int dev = 0, cus = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess) return 1;
    cus = prop.multiProcessorCount;
    const bool mi3xx = strncmp(prop.gcnArchName, "gfx94", 5) == 0 || strncmp(prop.gcnArchName, "gfx950", 6) == 0;
    return (mi3xx && cus >= 8 * 32 && cus % 8 == 0) ? 8 : 1;
  }();
  return xs;
}

extern "C" hipError_t m3s_launch_ba_solve(const BaArgs* a, int K, int nL, float delta_thresh, const int* step_tasks,
                                          const int* step_base, const int* step_na, hipStream_t s) {
  const int xs = ba_xcd_stride();
  // the assembly stays spread over every XCD: pinned to XCD 0 (32 CUs, item-strided) it took longer than the L2 reads
  // it saved the first step (solve C5 0.381 vs 0.375 ms)
  if (a->nb > 0) hipLaunchKernelGGL(m3s::ba_assemble_kernel, dim3(nL + a->nb), dim3(64), 0, s, *a, nL, 1);
  // LDS: the plan tables, x (8 doubles per column) and, for the dataflow schedule, 3 flags per column
  const size_t lds = ((a->plan_bytes + 15) & ~15) + (size_t)a->nb * 64;
  const bool flow_fits = a->flow && lds + (size_t)a->nb * 12 <= (size_t)m3s::SP_PLAN_BYTES;
  for (int l = 0; l < a->wide_steps; l++)
    if (step_tasks[l] > 0)
      hipLaunchKernelGGL(m3s::ba_sparse_step_kernel, dim3(step_tasks[l] * xs), dim3(64), 0, s, *a, step_base[l],
                         step_na[l], xs);
  if (flow_fits)
    hipLaunchKernelGGL(m3s::ba_sparse_factor_kernel<true>, dim3(1), dim3(1024), 0, s, *a, K, nL, delta_thresh);
  else if (lds <= (size_t)m3s::SP_PLAN_BYTES) {
    BaArgs b = *a;
    b.flow = 0;
    hipLaunchKernelGGL(m3s::ba_sparse_factor_kernel<true>, dim3(1), dim3(1024), 0, s, b, K, nL, delta_thresh);
  }
  else
    hipLaunchKernelGGL(m3s::ba_sparse_factor_kernel<false>, dim3(1), dim3(1024), 0, s, *a, K, nL, delta_thresh);
  return hipGetLastError();
}
