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
//   * ba_assemble: deterministic block-sparse scatter (host-built CSR of contributions per 7x7
//     block, fixed order) into a dense fp64 [H; g^T] system; every rank therefore solves an
//     identical system and keeps identical poses.
//   * dense right-looking blocked fp64 Cholesky (64-wide panels) with the rhs carried as an extra
//     row (forward substitution for free), blocked back substitution, and the Sim(3) retraction +
//     |dx| early-exit flag on device: no host synchronisation inside the GN loop.
#include "m3s_common.hpp"
#include "m3s_ba.h"

namespace m3s {

#define BA_NSUM 36

// ------------------------------------------------------------------------------------------
// linearisation
// ------------------------------------------------------------------------------------------
// MASK: the row's structurally nonzero Jacobian entries (bit c). Products with a structural zero
// are skipped: for finite weights they add an exact +-0 to the sum, so the result is unchanged
// (the reference computes them; ~45% of the FMAs in rays mode).
// Products and sums in fp64 from the fp32 rows: fp64 FMA issues at the fp32 (unpacked) rate on
// CDNA, and it keeps the whole BA within 1e-5 of the fp64 truth (fp32 products put the
// ill-conditioned 6-KF golden at ~1.2e-5).
template <unsigned MASK>
__device__ __forceinline__ void acc_local(double* L, double* v, const float J[7], float w, float e) {
  double Jd[7];
#pragma unroll
  for (int c = 0; c < 7; c++) Jd[c] = (double)J[c];
  const double wd = (double)w, ed = (double)e;
  int l = 0;
#pragma unroll
  for (int c = 0; c < 7; c++) {
    const double wj = wd * Jd[c];
#pragma unroll
    for (int d = c; d < 7; d++) {
      if ((MASK >> c) & (MASK >> d) & 1u) L[l] += wj * Jd[d];
      l++;
    }
    if ((MASK >> c) & 1u) v[c] += wj * ed;
  }
}

template <int MODE>  // specialised per residual type: one mode's registers, not the union of three
__global__ void __launch_bounds__(256, 4) ba_lin_kernel(BaArgs a, BaParams p) {
  if (*a.done) return;
  const int e = blockIdx.x / p.chunks;
  const int chunk = blockIdx.x % p.chunks;
  const int N = p.N;
  const int ix = a.ii_rank[e], jx = a.jj_rank[e];
  float Ti[8], Tj[8], Tij[8];
#pragma unroll
  for (int c = 0; c < 8; c++) {
    Ti[c] = a.Twc[ix * 8 + c];
    Tj[c] = a.Twc[jx * 8 + c];
  }
  relSim3(Ti, Tj, Tij);
  double L[28], v[7];
#pragma unroll
  for (int c = 0; c < 28; c++) L[c] = 0.0;
#pragma unroll
  for (int c = 0; c < 7; c++) v[c] = 0.0;
  const size_t eoff = (size_t)(e + p.edge_offset) * N;
  const float* Xi_base = a.Xs + (size_t)ix * N * 3;
  const float* Xj_base = a.Xs + (size_t)jx * N * 3;
  const float* Ci_base = a.Cs + (size_t)ix * N;
  const float* Cj_base = a.Cs + (size_t)jx * N;
  const int per = (N + p.chunks - 1) / p.chunks;
  const int k_begin = chunk * per;
  const int k_end = min(N, k_begin + per);
  for (int k = k_begin + threadIdx.x; k < k_end; k += blockDim.x) {
    const bool vm = a.valid[eoff + k] != 0;
    const int64_t ind = vm ? a.idx[eoff + k] : 0;
    const float Xi[3] = {Xi_base[ind * 3], Xi_base[ind * 3 + 1], Xi_base[ind * 3 + 2]};
    const float Xj[3] = {Xj_base[(size_t)k * 3], Xj_base[(size_t)k * 3 + 1], Xj_base[(size_t)k * 3 + 2]};
    float Y[3];
    actSO3(&Tij[3], Xj, Y);  // actSim3 (gn_kernels.cu:207-219): rotate, scale, translate
    Y[0] = Y[0] * Tij[7];
    Y[1] = Y[1] * Tij[7];
    Y[2] = Y[2] * Tij[7];
    Y[0] += Tij[0];
    Y[1] += Tij[1];
    Y[2] += Tij[2];
    const float q = a.Q[eoff + k];
    const float ci = Ci_base[ind];
    const float cj = Cj_base[k];
    bool valid = vm && (q > p.Q_thresh) && (ci > p.C_thresh) && (cj > p.C_thresh);
    // hardware sqrt/rsq/rcp (<= 1 ulp) instead of the correctly rounded sequences: the rows are
    // VALU-bound here and the products are formed in fp64 afterwards; parity is checked against
    // the fp64 truth (1e-5)
    const float sqq = __builtin_amdgcn_sqrtf(q);
    if constexpr (MODE == BA_MODE_POINTS) {
      const float err[3] = {Y[0] - Xi[0], Y[1] - Xi[1], Y[2] - Xi[2]};
      const float sw = valid ? p.inv_a * sqq : 0.0f;
      const float wc = sw * sw;
      const float J0[7] = {1.0f, 0.0f, 0.0f, 0.0f, Y[2], -Y[1], Y[0]};
      const float J1[7] = {0.0f, 1.0f, 0.0f, -Y[2], 0.0f, Y[0], Y[1]};
      const float J2[7] = {0.0f, 0.0f, 1.0f, Y[1], -Y[0], 0.0f, Y[2]};
      acc_local<0b1110001>(L, v, J0, huber_ba(sw * err[0]) * wc, err[0]);  // {0,4,5,6}
      acc_local<0b1101010>(L, v, J1, huber_ba(sw * err[1]) * wc, err[1]);  // {1,3,5,6}
      acc_local<0b1011100>(L, v, J2, huber_ba(sw * err[2]) * wc, err[2]);  // {2,3,4,6}
    } else if constexpr (MODE == BA_MODE_RAYS) {
      const float n2i = Xi[0] * Xi[0] + Xi[1] * Xi[1] + Xi[2] * Xi[2];
      const float n1i_inv = __builtin_amdgcn_rsqf(n2i);
      const float n1i = n2i * n1i_inv;
      const float n2j = Y[0] * Y[0] + Y[1] * Y[1] + Y[2] * Y[2];
      const float n1j_inv = __builtin_amdgcn_rsqf(n2j);
      const float n1j = n2j * n1j_inv;
      const float rj[3] = {n1j_inv * Y[0], n1j_inv * Y[1], n1j_inv * Y[2]};
      const float err[4] = {rj[0] - n1i_inv * Xi[0], rj[1] - n1i_inv * Xi[1], rj[2] - n1i_inv * Xi[2], n1j - n1i};
      const float swr = valid ? p.inv_a * sqq : 0.0f;
      const float swd = valid ? p.inv_b * sqq : 0.0f;
      const float wr = swr * swr, wd = swd * swd;
      const float n3 = n1j_inv * __builtin_amdgcn_rcpf(n2j);
      const float dxx = n1j_inv - Y[0] * Y[0] * n3;
      const float dyy = n1j_inv - Y[1] * Y[1] * n3;
      const float dzz = n1j_inv - Y[2] * Y[2] * n3;
      const float dxy = -Y[0] * Y[1] * n3;
      const float dxz = -Y[0] * Y[2] * n3;
      const float dyz = -Y[1] * Y[2] * n3;
      const float J0[7] = {dxx, dxy, dxz, 0.0f, rj[2], -rj[1], 0.0f};
      const float J1[7] = {dxy, dyy, dyz, -rj[2], 0.0f, rj[0], 0.0f};
      const float J2[7] = {dxz, dyz, dzz, rj[1], -rj[0], 0.0f, 0.0f};
      const float J3[7] = {rj[0], rj[1], rj[2], 0.0f, 0.0f, 0.0f, n1j};
      acc_local<0b0110111>(L, v, J0, huber_ba(swr * err[0]) * wr, err[0]);  // {0,1,2,4,5}
      acc_local<0b0101111>(L, v, J1, huber_ba(swr * err[1]) * wr, err[1]);  // {0,1,2,3,5}
      acc_local<0b0011111>(L, v, J2, huber_ba(swr * err[2]) * wr, err[2]);  // {0,1,2,3,4}
      acc_local<0b1000111>(L, v, J3, huber_ba(swd * err[3]) * wd, err[3]);  // {0,1,2,6}
    } else {  // calib
      const int ind32 = (int)ind;  // < H*W < 2^31: 32-bit division instead of 64-bit
      const int v_t = ind32 / p.W, u_t = ind32 - v_t * p.W;
      const bool valid_z = (Y[2] > p.z_eps) && (Xi[2] > p.z_eps);
      const float zj_inv = valid_z ? __builtin_amdgcn_rcpf(Y[2]) : 0.0f;
      const float zj_log = valid_z ? __logf(Y[2]) : 0.0f;
      const float zi_log = valid_z ? __logf(Xi[2]) : 0.0f;
      const float xz = Y[0] * zj_inv, yz = Y[1] * zj_inv;
      const float u = p.fx * xz + p.cx, vv = p.fy * yz + p.cy;
      const bool valid_u = (u > (float)p.pixel_border) && (u < (float)(p.W - 1 - p.pixel_border));
      const bool valid_v = (vv > (float)p.pixel_border) && (vv < (float)(p.H - 1 - p.pixel_border));
      valid = valid && valid_u && valid_v && valid_z;
      const float err[3] = {u - (float)u_t, vv - (float)v_t, zj_log - zi_log};
      const float swp = valid ? p.inv_a * sqq : 0.0f;
      const float swd = valid ? p.inv_b * sqq : 0.0f;
      const float wp = swp * swp, wd = swd * swd;
      const float fx = p.fx, fy = p.fy;
      const float J0[7] = {fx * zj_inv, 0.0f, -fx * xz * zj_inv, -fx * xz * yz, fx * (1 + xz * xz), -fx * yz, 0.0f};
      const float J1[7] = {0.0f, fy * zj_inv, -fy * yz * zj_inv, -fy * (1 + yz * yz), fy * xz * yz, fy * xz, 0.0f};
      const float J2[7] = {0.0f, 0.0f, zj_inv, yz, -xz, 0.0f, 1.0f};
      acc_local<0b0111101>(L, v, J0, huber_ba(swp * err[0]) * wp, err[0]);  // {0,2,3,4,5}
      acc_local<0b0111110>(L, v, J1, huber_ba(swp * err[1]) * wp, err[1]);  // {1,2,3,4,5}
      acc_local<0b1011100>(L, v, J2, huber_ba(swd * err[2]) * wd, err[2]);  // {2,3,4,6}
    }
  }
  // wave64 butterfly in fp64, then 4 waves through LDS
  __shared__ double s_part[4][BA_NSUM];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int c = 0; c < 28; c++) {
    const double t = wave_sum(L[c]);
    if (lane == 0) s_part[wid][c] = t;
  }
#pragma unroll
  for (int c = 0; c < 7; c++) {
    const double t = wave_sum(v[c]);
    if (lane == 0) s_part[wid][28 + c] = t;
  }
  __syncthreads();
  if (threadIdx.x < 35) {
    const int c = threadIdx.x;
    a.partials[(size_t)blockIdx.x * BA_NSUM + c] = s_part[0][c] + s_part[1][c] + s_part[2][c] + s_part[3][c];
  }
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
    double s = 0.0;
    for (int c = 0; c < p.chunks; c++) s += a.partials[((size_t)e * p.chunks + c) * BA_NSUM + t];
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
// deterministic assembly: one 64-lane block per nonzero lower 7x7 block (CSR of contributions),
// rhs rows from the same CSR (sign -1 for the i side, +1 for the j side).
// Dense system Hs (n+1, n) row-major, row n = g^T (carried through the factorisation).
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(64) ba_assemble_kernel(BaArgs a, int n, int nblocks) {
  if (*a.done) return;
  const int b = blockIdx.x;
  const int t = threadIdx.x;
  if (b < nblocks) {
    const int r = a.blk_row[b], c = a.blk_col[b];
    if (t < 49) {
      const int rr = t / 7, cc = t % 7;
      // M stored upper: index of (min,max)
      const int lo = min(rr, cc), hi = max(rr, cc);
      const int li = lo * 7 - lo * (lo - 1) / 2 + (hi - lo);
      double s = 0.0;
      for (int k = a.blk_ptr[b]; k < a.blk_ptr[b + 1]; k++) {
        const int ent = a.blk_ent[k];
        const int e = ent >> 1;
        const double sign = (ent & 1) ? -1.0 : 1.0;
        s += sign * a.edge_sums[(size_t)e * BA_NSUM + li];
      }
      a.H[(size_t)(r * 7 + rr) * n + c * 7 + cc] = s;
    }
  } else {
    const int row = b - nblocks;  // rhs block row
    if (t < 7) {
      double s = 0.0;
      for (int k = a.rhs_ptr[row]; k < a.rhs_ptr[row + 1]; k++) {
        const int ent = a.rhs_ent[k];
        const int e = ent >> 1;
        const double sign = (ent & 1) ? -1.0 : 1.0;
        s += sign * a.edge_sums[(size_t)e * BA_NSUM + 28 + t];
      }
      a.H[(size_t)n * n + row * 7 + t] = s;
    }
  }
}

// ------------------------------------------------------------------------------------------
// dense blocked Cholesky, lower, rows 0..n (row n = rhs), columns 0..n-1.
// Panels of PNB = 32 columns: the serial work per panel (diagonal factorisation, one wave) grows
// with PNB^2 per lane, so a narrow panel keeps the critical path short; the trailing update runs
// on 64x64 tiles of depth PNB.
// ------------------------------------------------------------------------------------------
#define PNB 32
#define UT 64

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

// Right-looking column step J of the register-row diagonal factorisation: pivot and column
// multipliers broadcast with readlane, rank-1 update of the lane's own row. Rows/columns >= kb are
// padded with the identity, so every step is valid and the padding stays inert.
template <int J>
__device__ __forceinline__ void diag_step(double (&r)[PNB], int lane, bool& bad) {
  if constexpr (J < PNB) {
    double d = bcast_lane(r[J], J);
    if (!(d > 0.0)) {
      bad = true;
      d = 1.0;
    }
    const double sj = sqrt(d);
    const double inv = 1.0 / sj;
    // unconditional multiplier (a lane-dependent select here makes the allocator spill r[]); lanes
    // <= J only disturb their own strictly-upper entries, which are never read
    const double l = r[J] * inv;
    r[J] = lane == J ? sj : (lane > J ? l : r[J]);
#pragma unroll
    for (int c = J + 1; c < PNB; c++) r[c] -= l * bcast_lane(l, c);
    diag_step<J + 1>(r, lane, bad);
  }
}

// Right-looking step J of the register-row forward substitution: x_J *= 1/L_JJ, then fold x_J into
// the later columns with column J of L11 (= row J of Ls = L11^T in LDS: broadcast reads; no compiler
// barrier here — a memory clobber inside the unrolled steps makes the allocator spill x[]).
template <int J>
__device__ __forceinline__ void trsm_step(double (&x)[PNB], const double (*Ls)[PNB + 2]) {
  if constexpr (J < PNB) {
    x[J] *= Ls[J][PNB];  // reciprocal of the pivot, stored after the row
#pragma unroll
    for (int k0 = J + 1; k0 < PNB; k0 += 8) {
#pragma unroll
      for (int k = k0; k < (k0 + 8 < PNB ? k0 + 8 : PNB); k++) x[k] -= x[J] * Ls[J][k];
    }
    trsm_step<J + 1>(x, Ls);
  }
}

// One panel: every block (one wave, 64 rows) factors the PNBxPNB diagonal block itself (lanes
// 0..31 = rows in registers, readlane broadcasts) — redundant across blocks but it removes a launch
// and a dependency from the critical path — then solves its rows r in [k0+kb, n] (row n = rhs):
// L21 = A21 L11^-T. L11 goes to Ldiag[panel] (block 0), never back into H: other blocks may still
// be reading A11 from H.
__global__ void __launch_bounds__(64) chol_panel_kernel(double* __restrict__ H, double* __restrict__ Ldiag, int n,
                                                        int k0, int* __restrict__ info, const int* __restrict__ done) {
  if (*done) return;
  const int kb = min(PNB, n - k0);
  __shared__ double S[PNB][PNB + 1];
  __shared__ double Ls[PNB][PNB + 2];
  const int lane = threadIdx.x;
  const int li = min(lane, PNB - 1);
  {
    double v[PNB];
#pragma unroll
    for (int t = 0; t < PNB; t++) v[t] = H[(size_t)(k0 + min(t, kb - 1)) * n + k0 + min(li, kb - 1)];
    if (lane < PNB)
#pragma unroll
      for (int t = 0; t < PNB; t++) S[t][lane] = (t < kb && lane < kb && lane <= t) ? v[t] : 0.0;
  }
  wave_sync();
  {
    double r[PNB];
#pragma unroll
    for (int c = 0; c < PNB; c++) r[c] = (li < kb && c < kb) ? S[li][c] : (c == li ? 1.0 : 0.0);
    bool bad = false;
    diag_step<0>(r, lane, bad);
    if (bad && lane == 0 && blockIdx.x == 0) *info = 1;
    wave_sync();
    if (lane < PNB)
#pragma unroll
      for (int c = 0; c < PNB; c++) S[lane][c] = c <= lane ? r[c] : 0.0;
  }
  wave_sync();
  if (lane < PNB) {
    for (int t = 0; t < PNB; t++) Ls[t][lane] = S[lane][t];  // Ls = L11^T (padded)
    Ls[lane][PNB] = 1.0 / S[lane][lane];
    if (blockIdx.x == 0) {
      double* Ld = Ldiag + (size_t)(k0 / PNB) * PNB * PNB;
      for (int t = 0; t < PNB; t++) Ld[t * PNB + lane] = S[t][lane];  // row-major L11 (padded)
    }
  }
  wave_sync();
  const int r = k0 + kb + blockIdx.x * 64 + lane;
  const int rr = min(r, n);
  double* row = H + (size_t)rr * n + k0;
  double x[PNB];
#pragma unroll
  for (int c = 0; c < PNB; c++) x[c] = c < kb ? row[min(c, kb - 1)] : 0.0;
  trsm_step<0>(x, Ls);
  if (r <= n) {
    // branch-free stores (a per-column `if (c < kb)` makes the allocator spill x[]): columns past
    // kb rewrite column kb-1 with its own value
    double keep = x[0];  // x[kb - 1], selected without dynamic indexing
#pragma unroll
    for (int c = 1; c < PNB; c++) keep = (c == kb - 1) ? x[c] : keep;
#pragma unroll
    for (int c = 0; c < PNB; c++) row[min(c, kb - 1)] = c < kb ? x[c] : keep;
  }
}

// trailing update A22 -= L21 L21^T over UTxUT lower tiles, depth kb <= PNB; rows [s, n], cols [s, n-1]
__global__ void __launch_bounds__(256) chol_update_kernel(double* __restrict__ H, int n, int k0,
                                                          const int* __restrict__ done) {
  if (*done) return;
  const int kb = min(PNB, n - k0);
  const int s = k0 + kb;
  const int ti = blockIdx.x, tj = blockIdx.y;
  if (tj > ti) return;
  const int r0 = s + ti * UT, c0 = s + tj * UT;
  if (c0 >= n) return;
  const int nr = min(UT, n + 1 - r0), nc = min(UT, n - c0);
  __shared__ double A[UT][PNB + 1];
  __shared__ double B[UT][PNB + 1];
  {  // 8 + 8 per lane, branch-free, all loads issued before the LDS stores
    double av[8], bv[8];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int t = threadIdx.x + 256 * u, i = t / PNB, k = t % PNB;
      const int kc = min(k, kb - 1);
      av[u] = H[(size_t)(r0 + min(i, nr - 1)) * n + k0 + kc];
      bv[u] = H[(size_t)(c0 + min(i, nc - 1)) * n + k0 + kc];
    }
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int t = threadIdx.x + 256 * u, i = t / PNB, k = t % PNB;
      A[i][k] = (i < nr && k < kb) ? av[u] : 0.0;
      B[i][k] = (i < nc && k < kb) ? bv[u] : 0.0;
    }
  }
  __syncthreads();
  const int ty = threadIdx.x / 16, tx = threadIdx.x % 16;  // 4x4 outputs per lane
  double acc[4][4];
#pragma unroll
  for (int x = 0; x < 4; x++)
#pragma unroll
    for (int y = 0; y < 4; y++) acc[x][y] = 0.0;
#pragma unroll 8
  for (int k = 0; k < PNB; k++) {
    double av[4], bv[4];
#pragma unroll
    for (int x = 0; x < 4; x++) av[x] = A[ty + 16 * x][k];
#pragma unroll
    for (int y = 0; y < 4; y++) bv[y] = B[tx + 16 * y][k];
#pragma unroll
    for (int x = 0; x < 4; x++)
#pragma unroll
      for (int y = 0; y < 4; y++) acc[x][y] += av[x] * bv[y];
  }
#pragma unroll
  for (int x = 0; x < 4; x++) {
    const int i = ty + 16 * x;
    if (i >= nr) continue;
#pragma unroll
    for (int y = 0; y < 4; y++) {
      const int j = tx + 16 * y;
      if (j >= nc) continue;
      if (r0 + i < n && c0 + j > r0 + i) continue;  // strictly-upper part unused
      H[(size_t)(r0 + i) * n + c0 + j] -= acc[x][y];
    }
  }
}

// Whole back substitution L^T x = y (y = row n after the factorisation) in ONE block: 64-column
// panels from the end; per panel the solved tail is folded in by a 16-group x 64-column GEMV, then
// wave 0 back-solves the 64x64 diagonal block with lane shuffles. x stays in LDS (n <= 8192).
#define BK_NB 64
__global__ void __launch_bounds__(1024) chol_back_all_kernel(const double* __restrict__ H,
                                                             const double* __restrict__ Ldiag, double* __restrict__ xg,
                                                             int n, const int* __restrict__ done) {
  if (*done) return;
  __shared__ double xs[8192];
  __shared__ double part[16][BK_NB];
  __shared__ double Ld[BK_NB][BK_NB + 1];
  const int c = threadIdx.x % BK_NB, g = threadIdx.x / BK_NB;
  for (int k0 = ((n - 1) / BK_NB) * BK_NB; k0 >= 0; k0 -= BK_NB) {
    const int kb = min(BK_NB, n - k0);
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    if (c < kb) {
      int r = k0 + kb + g;
      for (; r + 48 < n; r += 64) {
#pragma unroll
        for (int u = 0; u < 4; u++) acc[u] += H[(size_t)(r + 16 * u) * n + k0 + c] * xs[r + 16 * u];
      }
      for (; r < n; r += 16) acc[0] += H[(size_t)r * n + k0 + c] * xs[r];
    }
    part[g][c] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
    for (int t = threadIdx.x; t < BK_NB * BK_NB; t += 1024) {
      const int i = t / BK_NB, j = t % BK_NB;
      double v = 0.0;
      if (i < kb && j <= i) {
        if (i / PNB == j / PNB)  // inside a PNB diagonal block: kept in Ldiag by the panel kernel
          v = Ldiag[(size_t)((k0 + i) / PNB) * PNB * PNB + (i % PNB) * PNB + (j % PNB)];
        else
          v = H[(size_t)(k0 + i) * n + k0 + j];
      }
      Ld[i][j] = v;
    }
    __syncthreads();
    if (threadIdx.x < 64) {
      const int lane = threadIdx.x;
      double y = 0.0;
      if (lane < kb) {
        double sp = 0.0;
#pragma unroll
        for (int q = 0; q < 16; q++) sp += part[q][lane];
        y = H[(size_t)n * n + k0 + lane] - sp;
      }
      for (int cc = kb - 1; cc >= 0; cc--) {
        const double xc = __shfl(y, cc, 64) / Ld[cc][cc];
        if (lane == cc) y = xc;
        if (lane < cc) y -= Ld[cc][lane] * xc;
      }
      if (lane < kb) xs[k0 + lane] = y;
    }
    __syncthreads();
  }
  for (int i = threadIdx.x; i < n; i += 1024) xg[i] = xs[i];
}

// dx = -x (or 0 when the factorisation failed), poses k >= 1 retracted, |dx| early exit.
__global__ void __launch_bounds__(256) ba_retr_kernel(BaArgs a, int K, int n, float delta_thresh) {
  if (*a.done) return;
  const bool failed = *a.info != 0;
  __shared__ float s_n2[4];
  float n2 = 0.0f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const float d = failed ? 0.0f : (float)(-a.x[i]);
    a.dx[i] = d;
    n2 += d * d;
  }
  __syncthreads();
  for (int k = 1 + threadIdx.x; k < K; k += blockDim.x) {
    float T[8], xi[7];
    for (int c = 0; c < 8; c++) T[c] = a.Twc[k * 8 + c];
    for (int c = 0; c < 7; c++) xi[c] = a.dx[(k - 1) * 7 + c];
    retrSim3(xi, T);
    for (int c = 0; c < 8; c++) a.Twc[k * 8 + c] = T[c];
  }
  n2 = wave_sum(n2);
  if ((threadIdx.x & 63) == 0) s_n2[threadIdx.x >> 6] = n2;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float nrm = sqrtf(s_n2[0] + s_n2[1] + s_n2[2] + s_n2[3]);
    *a.iters += 1;
    if (nrm < delta_thresh) *a.done = 1;
    *a.info = 0;
  }
}

}  // namespace m3s

// ------------------------------------------------------------------------------------------
extern "C" hipError_t m3s_launch_ba_lin(const BaArgs* a, const BaParams* p, int E_local, hipStream_t s) {
  if (E_local <= 0) return hipSuccess;
  const dim3 g(E_local * p->chunks);
  if (p->mode == BA_MODE_POINTS)
    hipLaunchKernelGGL(m3s::ba_lin_kernel<BA_MODE_POINTS>, g, dim3(256), 0, s, *a, *p);
  else if (p->mode == BA_MODE_RAYS)
    hipLaunchKernelGGL(m3s::ba_lin_kernel<BA_MODE_RAYS>, g, dim3(256), 0, s, *a, *p);
  else
    hipLaunchKernelGGL(m3s::ba_lin_kernel<BA_MODE_CALIB>, g, dim3(256), 0, s, *a, *p);
  hipLaunchKernelGGL(m3s::ba_edge_kernel, dim3(E_local), dim3(64), 0, s, *a, *p, E_local);
  return hipGetLastError();
}

extern "C" hipError_t m3s_launch_ba_solve(const BaArgs* a, int K, int nblocks, int nrhs_rows, float delta_thresh,
                                          hipStream_t s) {
  const int n = (K - 1) * 7;
  if (n > 0) {
    if (hipMemsetAsync(a->H, 0, sizeof(double) * (size_t)(n + 1) * n, s) != hipSuccess) return hipGetLastError();
    hipLaunchKernelGGL(m3s::ba_assemble_kernel, dim3(nblocks + nrhs_rows), dim3(64), 0, s, *a, n, nblocks);
    for (int k0 = 0; k0 < n; k0 += PNB) {
      const int kb = n - k0 < PNB ? n - k0 : PNB;
      const int rows = n + 1 - (k0 + kb);  // >= 1: the rhs row
      hipLaunchKernelGGL(m3s::chol_panel_kernel, dim3((rows + 63) / 64), dim3(64), 0, s, a->H, a->Lt, n, k0, a->info,
                         a->done);
      const int tr = (rows + UT - 1) / UT;
      const int tc = (n - (k0 + kb) + UT - 1) / UT;
      if (tc > 0) hipLaunchKernelGGL(m3s::chol_update_kernel, dim3(tr, tc), dim3(256), 0, s, a->H, n, k0, a->done);
    }
    hipLaunchKernelGGL(m3s::chol_back_all_kernel, dim3(1), dim3(1024), 0, s, a->H, a->Lt, a->x, n, a->done);
  }
  hipLaunchKernelGGL(m3s::ba_retr_kernel, dim3(1), dim3(256), 0, s, *a, K, n, delta_thresh);
  return hipGetLastError();
}
