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
//   * dense right-looking blocked fp64 Cholesky (64-wide panels, 16-wide register-row sub-steps
//     between matrix-core updates) with the rhs and the identity carried as extra rows: the forward
//     substitution comes for free and the carried identity becomes L^-T, so the back substitution is
//     one parallel mat-vec; the Sim(3) retraction + |dx| early-exit flag on device: no host
//     synchronisation inside the GN loop.
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

// Per-call point records (once per gauss_newton call; the GN iterations only move the poses):
//   rec[e][k] = {Xi (points / rays) or (u_t, v_t, z_i) (calib) ; sw} with Xi = Xs[i][valid ? idx : 0]
//   (gn_kernels.cu reads index 0 for an invalid match) and sw = sqrt(q) when the match is valid and
//   q > Q_thresh, c_i > C_thresh, c_j > C_thresh, else 0 (gn_kernels.cu:880-906) — the per-iteration
//   gathers, int64 index loads and threshold tests leave the linearisation loop.
template <int MODE>
__global__ void __launch_bounds__(256) ba_pack_kernel(BaArgs a, BaParams p, int E_local) {
  const int N = p.N;
  const size_t total = (size_t)E_local * N;
  for (size_t o = (size_t)blockIdx.x * blockDim.x + threadIdx.x; o < total; o += (size_t)gridDim.x * blockDim.x) {
    const int e = (int)(o / N), k = (int)(o - (size_t)e * N);
    const size_t g = (size_t)(e + p.edge_offset) * N + k;
    const int ix = a.ii_rank[e], jx = a.jj_rank[e];
    const bool vm = a.valid[g] != 0;
    const int64_t ind = vm ? a.idx[g] : 0;
    const float* Xi = a.Xkf[ix] + (size_t)ind * 3;
    const float q = a.Q[g];
    const bool valid = vm && (q > p.Q_thresh) && (a.Ckf[ix][ind] * a.Cscale[ix] > p.C_thresh) &&
                       (a.Ckf[jx][k] * a.Cscale[jx] > p.C_thresh);
    // hardware sqrt (<= 1 ulp): parity is checked against the fp64 truth (1e-5)
    const float sw = valid ? __builtin_amdgcn_sqrtf(q) : 0.0f;
    float4 r;
    if constexpr (MODE == BA_MODE_CALIB) {
      const int ind32 = (int)ind;  // < H*W < 2^31: 32-bit division
      const int v_t = ind32 / p.W, u_t = ind32 - v_t * p.W;
      r = make_float4((float)u_t, (float)v_t, Xi[2], sw);
    } else {
      r = make_float4(Xi[0], Xi[1], Xi[2], sw);
    }
    a.rec[o] = r;
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
  const float4* rec = a.rec + (size_t)e * N;
  const float* Xj_base = a.Xkf[jx];
  const int per = (N + p.chunks - 1) / p.chunks;
  const int k_begin = chunk * per;
  const int k_end = min(N, k_begin + per);
  for (int k = k_begin + threadIdx.x; k < k_end; k += blockDim.x) {
    const float4 R = rec[k];
    const float Xj[3] = {Xj_base[(size_t)k * 3], Xj_base[(size_t)k * 3 + 1], Xj_base[(size_t)k * 3 + 2]};
    float Y[3];
    actSO3(&Tij[3], Xj, Y);  // actSim3 (gn_kernels.cu:207-219): rotate, scale, translate
    Y[0] = Y[0] * Tij[7];
    Y[1] = Y[1] * Tij[7];
    Y[2] = Y[2] * Tij[7];
    Y[0] += Tij[0];
    Y[1] += Tij[1];
    Y[2] += Tij[2];
    const float sqq = R.w;  // sqrt(q), 0 for an invalid match (ba_pack)
    if constexpr (MODE == BA_MODE_POINTS) {
      const float Xi[3] = {R.x, R.y, R.z};
      const float err[3] = {Y[0] - Xi[0], Y[1] - Xi[1], Y[2] - Xi[2]};
      const float sw = p.inv_a * sqq;
      const float wc = sw * sw;
      const float J0[7] = {1.0f, 0.0f, 0.0f, 0.0f, Y[2], -Y[1], Y[0]};
      const float J1[7] = {0.0f, 1.0f, 0.0f, -Y[2], 0.0f, Y[0], Y[1]};
      const float J2[7] = {0.0f, 0.0f, 1.0f, Y[1], -Y[0], 0.0f, Y[2]};
      acc_local<0b1110001>(L, v, J0, huber_ba(sw * err[0]) * wc, err[0]);  // {0,4,5,6}
      acc_local<0b1101010>(L, v, J1, huber_ba(sw * err[1]) * wc, err[1]);  // {1,3,5,6}
      acc_local<0b1011100>(L, v, J2, huber_ba(sw * err[2]) * wc, err[2]);  // {2,3,4,6}
    } else if constexpr (MODE == BA_MODE_RAYS) {
      const float Xi[3] = {R.x, R.y, R.z};
      const float n2i = Xi[0] * Xi[0] + Xi[1] * Xi[1] + Xi[2] * Xi[2];
      const float n1i_inv = __builtin_amdgcn_rsqf(n2i);
      const float n1i = n2i * n1i_inv;
      const float n2j = Y[0] * Y[0] + Y[1] * Y[1] + Y[2] * Y[2];
      const float n1j_inv = __builtin_amdgcn_rsqf(n2j);
      const float n1j = n2j * n1j_inv;
      const float rj[3] = {n1j_inv * Y[0], n1j_inv * Y[1], n1j_inv * Y[2]};
      const float err[4] = {rj[0] - n1i_inv * Xi[0], rj[1] - n1i_inv * Xi[1], rj[2] - n1i_inv * Xi[2], n1j - n1i};
      const float swr = p.inv_a * sqq;
      const float swd = p.inv_b * sqq;
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
      const float u_t = R.x, v_t = R.y, zi = R.z;
      const bool valid_z = (Y[2] > p.z_eps) && (zi > p.z_eps);
      const float zj_inv = valid_z ? __builtin_amdgcn_rcpf(Y[2]) : 0.0f;
      const float zj_log = valid_z ? __logf(Y[2]) : 0.0f;
      const float zi_log = valid_z ? __logf(zi) : 0.0f;
      const float xz = Y[0] * zj_inv, yz = Y[1] * zj_inv;
      const float u = p.fx * xz + p.cx, vv = p.fy * yz + p.cy;
      const bool valid_u = (u > (float)p.pixel_border) && (u < (float)(p.W - 1 - p.pixel_border));
      const bool valid_v = (vv > (float)p.pixel_border) && (vv < (float)(p.H - 1 - p.pixel_border));
      const bool valid = valid_u && valid_v && valid_z;
      const float err[3] = {u - u_t, vv - v_t, zj_log - zi_log};
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
// Dense system H (2n+1, n) row-major, row n = g^T, rows n+1.. = identity (carried through the factorisation).
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(64) ba_assemble_kernel(BaArgs a, int n, int nblocks, int nrhs) {
  if (*a.done) return;
  const int b = blockIdx.x;
  const int t = threadIdx.x;
  if (b >= nblocks + nrhs) {  // carried identity rows (H row n+1+i = e_i^T)
    const int i = (b - nblocks - nrhs) * 64 + t;
    if (i < n) a.H[(size_t)(n + 1 + i) * n + i] = 1.0;
    return;
  }
  if (b < nblocks) {
    const int r = a.blk_row[b], c = a.blk_col[b];
    if (t < 49) {
      const int rr = t / 7, cc = t % 7;
      // M stored upper: index of (min,max)
      const int lo = min(rr, cc), hi = max(rr, cc);
      const int li = lo * 7 - lo * (lo - 1) / 2 + (hi - lo);
      // contributions summed in CSR order (deterministic); indices and values of 4 at a time in flight
      double s = 0.0;
      const int kb = a.blk_ptr[b], ke = a.blk_ptr[b + 1];
      int k = kb;
      for (; k + 4 <= ke; k += 4) {
        int ent[4];
        double v[4];
#pragma unroll
        for (int u = 0; u < 4; u++) ent[u] = a.blk_ent[k + u];
#pragma unroll
        for (int u = 0; u < 4; u++) v[u] = a.edge_sums[(size_t)(ent[u] >> 1) * BA_NSUM + li];
#pragma unroll
        for (int u = 0; u < 4; u++) s += ((ent[u] & 1) ? -1.0 : 1.0) * v[u];
      }
      for (; k < ke; k++) {
        const int ent = a.blk_ent[k];
        s += ((ent & 1) ? -1.0 : 1.0) * a.edge_sums[(size_t)(ent >> 1) * BA_NSUM + li];
      }
      a.H[(size_t)(r * 7 + rr) * n + c * 7 + cc] = s;
    }
  } else {
    const int row = b - nblocks;  // rhs block row
    if (t < 7) {
      double s = 0.0;
      const int kb = a.rhs_ptr[row], ke = a.rhs_ptr[row + 1];
      int k = kb;
      for (; k + 4 <= ke; k += 4) {
        int ent[4];
        double v[4];
#pragma unroll
        for (int u = 0; u < 4; u++) ent[u] = a.rhs_ent[k + u];
#pragma unroll
        for (int u = 0; u < 4; u++) v[u] = a.edge_sums[(size_t)(ent[u] >> 1) * BA_NSUM + 28 + t];
#pragma unroll
        for (int u = 0; u < 4; u++) s += ((ent[u] & 1) ? -1.0 : 1.0) * v[u];
      }
      for (; k < ke; k++) {
        const int ent = a.rhs_ent[k];
        s += ((ent & 1) ? -1.0 : 1.0) * a.edge_sums[(size_t)(ent >> 1) * BA_NSUM + 28 + t];
      }
      a.H[(size_t)n * n + row * 7 + t] = s;
    }
  }
}

// ------------------------------------------------------------------------------------------
// dense blocked Cholesky with carried inverse rows.
// H is ((2n+1) x n) row-major: rows 0..n-1 the system (lower triangle used), row n = g^T, row n+1+i =
// e_i^T. The right-looking factorisation applies its forward elimination to every row below the
// diagonal, so row n ends as y^T = (L^-1 g)^T and row n+1+i as (L^-1 e_i)^T: the carried block is L^-T
// and x = L^-T y is one parallel mat-vec (chol_apply_kernel) instead of a serial back substitution.
// Carried row i stays zero in the columns before i, so it joins the elimination at the panel that
// holds column i (the "active" carried rows of panel s are i < end of panel s).
// One launch per PNB-column (64) panel with a one-panel look-ahead: launch s factors panel s while panel
// s-1's trailing update of the columns beyond panel s runs beside it in the same grid. The panel blocks
// apply panel s-1's update to their own column block first, so the update of the rest of the matrix
// is off the critical path.
// ------------------------------------------------------------------------------------------
#ifndef PNB
#define PNB 64  // panel width (columns factorised per launch)
#endif
#ifndef SB
#define SB 16  // sub-panel width
#endif  // of the in-block factorisation (register-row steps between MFMA updates)
#define UT 64

typedef double d4v __attribute__((ext_vector_type(4)));

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

// 1/sqrt(d) and 1/d for d > 0: the v_rsq_f64 / v_rcp_f64 estimates (~2^-22 relative) refined by ONE
// Newton step (~2^-44): the pivot chain is latency-bound (a dependent v_fma_f64 costs ~13 ns on gfx950,
// measured by scripts/micro/mfma_f64.hip), and 1e-13 relative pivots are far inside the 1e-5 pose
// contract (the LAPACK parity test bounds the solve at 2e-6 of the step).
__device__ __forceinline__ double rsqrt_nr(double d) {
  const double y = __builtin_amdgcn_rsq(d);
  return fma(y, fma(-0.5 * d * y, y, 0.5), y);
}

__device__ __forceinline__ double rcp_nr(double d) {
  const double y = __builtin_amdgcn_rcp(d);
  return fma(y, fma(-d, y, 1.0), y);
}

// Right-looking column step J of the register-row factorisation of a W-column sub-panel: lane l holds
// row l (of the sub-panel's rows) in r[0..W); pivot and column multipliers broadcast with readlane,
// rank-1 update of the lane's own row. Lanes >= W are the rows below the sub-block: the same steps
// are their triangular solve. Lanes < J only disturb their own strictly-upper entries (never read).
template <int J, int W>
__device__ __forceinline__ void diag_step(double (&r)[W], int lane, bool& bad) {
  if constexpr (J < W) {
    double d = bcast_lane(r[J], J);
    if (!(d > 0.0)) {
      bad = true;
      d = 1.0;
    }
    const double inv = rsqrt_nr(d);  // serial chain: hardware estimate + two Newton steps
    const double sj = d * inv;
    // unconditional multiplier (a lane-dependent select here makes the allocator spill r[])
    const double l = r[J] * inv;
    r[J] = lane == J ? sj : (lane > J ? l : r[J]);
#pragma unroll
    for (int c = J + 1; c < W; c++) r[c] -= l * bcast_lane(l, c);
    diag_step<J + 1, W>(r, lane, bad);
  }
}

// Right-looking step J of the register-row forward substitution x <- x L^-T over a W-column
// sub-block: x_J *= 1/L_JJ, then fold x_J into the later columns with column J of L (row J of
// Ls = L^T, reciprocal pivot stored after the row). Row J+1 is read from LDS before step J's FMAs.
template <int J, int W>
__device__ __forceinline__ void trsm_pipe(double (&x)[W], const double (*Ls)[W + 2], const double (&cur)[W + 2]) {
  if constexpr (J < W) {
    double nxt[W + 2];
    if constexpr (J + 1 < W) {
#pragma unroll
      for (int c = (J + 2) & ~1; c < W + 2; c += 2) {
        const double2 v = *reinterpret_cast<const double2*>(&Ls[J + 1][c]);
        nxt[c] = v.x;
        nxt[c + 1] = v.y;
      }
    }
    x[J] *= cur[W];
#pragma unroll
    for (int k = J + 1; k < W; k++) x[k] -= x[J] * cur[k];
    trsm_pipe<J + 1, W>(x, Ls, nxt);
  }
}

constexpr int LP = PNB + 2;   // LDS row pitch (doubles) of the panel arrays

// Factorisation results are stored write-through (agent-scope sc1 stores): the next launch reads them
// on other XCDs anyway, and a launch that left ~28 MB of dirty trailing-matrix lines in L2 paid their
// write-back at its end (the kernel boundary), on the critical path.
__device__ __forceinline__ void st_wt(double* p, double v) {
#ifdef M3S_CHOL_PLAIN_STORES
  *p = v;
#else
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
}
constexpr int PR = 64;        // rows per panel block
constexpr int RS = 256 / PNB;  // rows covered by one pass of the block's 256 loading lanes

constexpr int NSUB = PNB / SB;  // sub-panels per panel

#ifdef M3S_CHOL_STAMPS  // (experiment builds only) s_memrealtime stamps of panel block 0, per launch
__device__ unsigned long long g_chol_stamps[64 * 16];
__shared__ unsigned long long s_stamp[16];
#define CST(k)                                                                              \
  do {                                                                                       \
    if (blockIdx.x == 0 && (threadIdx.x & 63) == 0) s_stamp[k] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define CST(k) \
  do {         \
  } while (0)
#endif

// In-block hand-offs between the waves of one panel block go through LDS words (all waves of a block
// are resident together). Spins are bounded: a logic error would surface as info = 2 (dx = 0), never
// as a hung GPU.
__device__ __forceinline__ void lds_wait_ge(int* f, int v, int* info) {
  int spins = 0;
  while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < v) {
    __builtin_amdgcn_s_sleep(1);
    if (++spins > (1 << 22)) {
      *info = 2;
      break;
    }
  }
}

__device__ __forceinline__ void lds_signal(int* f, int lane) {
  if (lane == 0) __hip_atomic_fetch_add(f, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Look-ahead tile (ti, tj) of the diagonal block: S[16ti.., 16tj..] -= P1 P1^T (K = PNB), operand reads
// issued before the MFMA chain, two interleaved accumulators.
__device__ __forceinline__ void la_tile(double (*S)[LP], const double (*P1)[LP], int ti, int tj, int lr, int lk) {
  double fa[PNB / 4], fb[PNB / 4];
#pragma unroll
  for (int q = 0; q < PNB; q += 4) {
    fa[q / 4] = P1[16 * ti + lr][q + lk];
    fb[q / 4] = P1[16 * tj + lr][q + lk];
  }
  d4v c2[2] = {{0.0, 0.0, 0.0, 0.0}, {0.0, 0.0, 0.0, 0.0}};
#pragma unroll
  for (int q = 0; q < PNB / 4; q++) c2[q & 1] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[q], fb[q], c2[q & 1], 0, 0, 0);
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const int si = 16 * ti + lk + 4 * r, sj = 16 * tj + lr;
    if (sj <= si) S[si][sj] -= c2[0][r] + c2[1][r];
  }
}

// Wave 0, sub-panel C0: factor rows C0..PNB-1 of the diagonal block on columns C0..C0+SB in registers
// (the rows below the SB x SB sub-block get their triangular solve from the same steps), write them back
// to S, publish L_qq^T + reciprocal pivots in Lq; then S[C0+SB.., C0+SB..] -= L21 L21^T (matrix cores).
template <int C0>
__device__ __forceinline__ void diag_chain(double (*S)[LP], double (*Lq)[SB][SB + 2], int* flags, int lane, int* info) {
  if constexpr (C0 < PNB) {
    constexpr int q = C0 / SB, REST = PNB - C0 - SB;
    const int row = C0 + lane;
    double r[SB];
#pragma unroll
    for (int c = 0; c < SB; c++) r[c] = row < PNB ? S[row][C0 + c] : 0.0;
    bool bad = false;
    diag_step<0, SB>(r, lane, bad);
    if (bad && lane == 0 && blockIdx.x == 0) *info = 1;
    if (row < PNB) {
#pragma unroll
      for (int c = 0; c < SB; c++) S[row][C0 + c] = (lane < SB && c > lane) ? 0.0 : r[c];
    }
    if (lane < SB) {
#pragma unroll
      for (int J = 0; J < SB; J++) Lq[q][J][lane] = J <= lane ? r[J] : 0.0;  // Lq[q][J][c] = L[C0+c][C0+J]
      Lq[q][lane][SB] = rcp_nr(r[lane]);
      Lq[q][lane][SB + 1] = 0.0;
    }
    lds_signal(&flags[q], lane);  // L_qq and L21 (S columns C0..C0+SB) published
    CST(3 + q);
    if constexpr (REST > 0) {
      // near update: only the next sub-panel's column block (its factorisation waits on it); the far
      // tiles are updated by waves 1/2 (far_update), which also touch column block q+2 -> wait for
      // sub-panel q-1's far tiles first
      if constexpr (q > 0) lds_wait_ge(&flags[4 * NSUB + q - 1], 2, info);
      else lds_wait_ge(&flags[5 * NSUB], 3, info);  // the look-ahead of the later column blocks is in
      const int lr = lane & 15, lk = lane >> 4;
      double bf[SB / 4];
#pragma unroll
      for (int k = 0; k < SB; k += 4) bf[k / 4] = S[C0 + SB + lr][C0 + k + lk];
#pragma unroll
      for (int ti = 0; ti < REST / 16; ti++) {
        d4v acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int k = 0; k < SB; k += 4)
          acc = __builtin_amdgcn_mfma_f64_16x16x4f64(S[C0 + SB + 16 * ti + lr][C0 + k + lk], bf[k / 4], acc, 0, 0, 0);
#pragma unroll
        for (int r4 = 0; r4 < 4; r4++) {
          const int i = 16 * ti + lk + 4 * r4;
          if (lr <= i) S[C0 + SB + i][C0 + SB + lr] -= acc[r4];
        }
      }
    }
    diag_chain<C0 + SB>(S, Lq, flags, lane, info);
  }
}

// Waves 1/2, sub-panel C0: the far tiles of S[C0+SB.., C0+SB..] -= L21 L21^T (column blocks q+2..),
// dealt alternately to the two waves; flags[4 NSUB + q] counts the two waves.
template <int C0>
__device__ __forceinline__ void far_update(double (*S)[LP], int* flags, int w, int lane, int* info) {
  constexpr int q = C0 / SB, RT = (PNB - C0 - SB) / 16;
  const int lr = lane & 15, lk = lane >> 4;
  int u = 0;
#pragma unroll
  for (int ti = 1; ti < RT; ti++)
#pragma unroll
    for (int tj = 1; tj <= ti; tj++, u++) {
      if ((u & 1) != w - 1) continue;
      d4v acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int k = 0; k < SB; k += 4)
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(S[C0 + SB + 16 * ti + lr][C0 + k + lk],
                                                   S[C0 + SB + 16 * tj + lr][C0 + k + lk], acc, 0, 0, 0);
#pragma unroll
      for (int r4 = 0; r4 < 4; r4++) {
        const int i = 16 * ti + lk + 4 * r4, j = 16 * tj + lr;
        if (j <= i) S[C0 + SB + i][C0 + SB + j] -= acc[r4];
      }
    }
  lds_signal(&flags[4 * NSUB + q], lane);
}

// Row side (waves 1..3) of the panel block. Row tiles (16 rows of X) are owned by one wave each
// (wave 1: tiles 0 and 2, wave 2: tiles 1 and 3; wave 3 only solves), so every element's update order
// is fixed (deterministic). Per column block j, R[j] = flags[2 NSUB + j] counts the finished contributions:
// the look-ahead of panel s-1 (la_rows<j>) and the X-updates of sub-panels p < j, one signal per wave
// each; wave 3 solves X[:, block q] <- X L_qq^-T (lane = row) once L_qq is published (flags[q]) and
// R[q] = 3 (q + 1), then signals flags[NSUB + q]. Each wave then looks ahead on block q+1 and applies
// sub-panel q's update to its row tiles: block q+1 first (the next solve waits on it), then the rest.
// flags: [q] L_qq published (wave 0); [NSUB + q] block q solved (wave 3); [2 NSUB + j] R[j];
// [4 NSUB + q] far S-update q (waves 2/3); [5 NSUB] the diagonal block's later look-ahead tiles.
__device__ __forceinline__ bool owns_tile(int w, int rt) { return w <= 2 && (rt & 1) == w - 1; }

template <int J>
__device__ __forceinline__ void la_rows(double (*X)[LP], const double (*LR)[LP], const double (*P1)[LP], int* flags, int w,
                                        int lane, bool upd) {
  const int lr = lane & 15, lk = lane >> 4;
  if (upd) {  // X[own rows][block J] -= L_{R,s-1} L_{s,s-1}[block J]^T
#pragma unroll
    for (int rt = 0; rt < PR / 16; rt++) {
      if (!owns_tile(w, rt)) continue;
      d4v c2[2] = {{0.0, 0.0, 0.0, 0.0}, {0.0, 0.0, 0.0, 0.0}};
#pragma unroll
      for (int q = 0; q < PNB; q += 4)
        c2[(q >> 2) & 1] = __builtin_amdgcn_mfma_f64_16x16x4f64(LR[16 * rt + lr][q + lk], P1[16 * J + lr][q + lk],
                                                                c2[(q >> 2) & 1], 0, 0, 0);
#pragma unroll
      for (int r = 0; r < 4; r++) X[16 * rt + lk + 4 * r][16 * J + lr] -= c2[0][r] + c2[1][r];
    }
  }
  lds_signal(&flags[2 * NSUB + J], lane);
}

// X[own rows][block J] -= X[own rows][block q] L[block J rows][block q]^T, then R[J] += 1
template <int C0, int J>
__device__ __forceinline__ void x_update(double (*S)[LP], double (*X)[LP], int* flags, int w, int lane) {
  const int lr = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int rt = 0; rt < PR / 16; rt++) {
    if (!owns_tile(w, rt)) continue;
    d4v acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int k = 0; k < SB; k += 4)
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(X[16 * rt + lr][C0 + k + lk], S[16 * J + lr][C0 + k + lk], acc, 0, 0, 0);
#pragma unroll
    for (int r4 = 0; r4 < 4; r4++) X[16 * rt + lk + 4 * r4][16 * J + lr] -= acc[r4];
  }
  lds_signal(&flags[2 * NSUB + J], lane);
}

template <int C0, int J>
__device__ __forceinline__ void x_update_far(double (*S)[LP], double (*X)[LP], int* flags, int w, int lane) {
  if constexpr (J < NSUB) {
    x_update<C0, J>(S, X, flags, w, lane);
    x_update_far<C0, J + 1>(S, X, flags, w, lane);
  }
}

template <int C0>
__device__ __forceinline__ void row_chain(double (*S)[LP], double (*X)[LP], const double (*LR)[LP], const double (*P1)[LP],
                                          double (*Lq)[SB][SB + 2], int* flags, int w, int lane, bool upd, int* info) {
  static_assert(SB == 16 && PR == 64, "row tiles are 16 x 16 column blocks");
  if constexpr (C0 < PNB) {
    constexpr int q = C0 / SB;
    if (w == 3) {
      lds_wait_ge(&flags[q], 1, info);
      lds_wait_ge(&flags[2 * NSUB + q], 3 * (q + 1), info);
      double x[SB], row0[SB + 2];
#pragma unroll
      for (int c = 0; c < SB; c++) x[c] = X[lane][C0 + c];
#pragma unroll
      for (int c = 0; c < SB + 2; c += 2) {
        const double2 v = *reinterpret_cast<const double2*>(&Lq[q][0][c]);
        row0[c] = v.x;
        row0[c + 1] = v.y;
      }
      trsm_pipe<0, SB>(x, Lq[q], row0);
#pragma unroll
      for (int c = 0; c < SB; c++) X[lane][C0 + c] = x[c];
      lds_signal(&flags[NSUB + q], lane);
      CST(9 + q);
    } else if constexpr (PNB - C0 - SB > 16) {
      if (w <= 2) {  // far S tiles of sub-panel q (column blocks q+2..) while wave 3 solves
        lds_wait_ge(&flags[q], 1, info);
        if constexpr (q == 0) lds_wait_ge(&flags[5 * NSUB], 3, info);
        far_update<C0>(S, flags, w, lane, info);
      }
    }
    if constexpr (q + 1 < NSUB) {
      la_rows<q + 1>(X, LR, P1, flags, w, lane, upd);
      lds_wait_ge(&flags[NSUB + q], 1, info);
      x_update<C0, q + 1>(S, X, flags, w, lane);      // the next solve waits on this block
      x_update_far<C0, q + 2>(S, X, flags, w, lane);  // later blocks
    }
    row_chain<C0 + SB>(S, X, LR, P1, Lq, flags, w, lane, upd, info);
  }
}

// Launch s of the factorisation (k0 = s*PNB, kb = panel width, st = k0 + kb).
// Blocks [0, P1): PR rows each of rows st..n (system rows below the diagonal block + the rhs row);
// blocks [P1, P): PR rows each of the active carried rows n+1+i, i < st. Each panel block:
//   1. coalesced loads of A11 (diagonal block), its rows A21 and, for s > 0, the matching rows of
//      panel s-1 (L_{s,s-1} and L_{R,s-1}), all in flight at once;
//   2. s > 0: A11 -= L_{s,s-1} L_{s,s-1}^T, A21 -= L_{R,s-1} L_{s,s-1}^T (the look-ahead update, MFMA);
//   3. factors A11 redundantly (no extra launch on the critical path) in SB-column sub-steps and solves
//      its rows L21 = A21 L11^-T along (panel_substep), stores L21 coalesced.
// Blocks [P, P+U): panel s-1's update A22 -= L21 L21^T over the UTxUT tiles of the columns beyond panel
// s: lower-triangle tiles of the system rows (+ the rhs row), then full tiles of the carried rows
// active at panel s-1 (i < k0).
__global__ void __launch_bounds__(256) chol_step_kernel(double* __restrict__ H, int n, int k0, int P1, int P,
                                                        int* __restrict__ info, const int* __restrict__ done) {
  if (threadIdx.x < 64) CST(0);
  if (*done) return;
  static_assert(UT == 64 && PR == 64 && PNB % 16 == 0 && 256 % PNB == 0, "tiling");
  __shared__ double smem[2 * PNB * LP + 2 * PR * LP + NSUB * SB * (SB + 2) + 3 * NSUB + 1];  // >= 2 * UT * LP (update tiles)
  const int kb = min(PNB, n - k0);
  const int st = k0 + kb;
  const int t = threadIdx.x;
  if ((int)blockIdx.x >= P) {
    // ---- trailing update of panel s-1 (columns PNB wide at kp) beyond panel s ----
    const int kp = k0 - PNB;
    const int T = (n - st + UT - 1) / UT;  // column tiles
    const int R = (n + 1 - st + UT - 1) / UT;
    const int tri = T * (T + 1) / 2, xr = R > T ? T : 0;
    const int u = blockIdx.x - P;
    int r0, c0, nr;
    if (u < tri) {
      int ti = (int)((sqrtf(8.0f * (float)u + 1.0f) - 1.0f) * 0.5f);
      while (ti * (ti + 1) / 2 > u) ti--;
      while ((ti + 1) * (ti + 2) / 2 <= u) ti++;
      const int tj = u - ti * (ti + 1) / 2;
      r0 = st + ti * UT;
      c0 = st + tj * UT;
      nr = min(UT, n + 1 - r0);
    } else if (u < tri + xr) {  // the extra tile row holding only the rhs row (n - st a multiple of UT)
      r0 = st + T * UT;
      c0 = st + (u - tri) * UT;
      nr = min(UT, n + 1 - r0);
    } else {  // carried rows active at panel s-1 (i < k0), every column tile
      const int v = u - tri - xr;
      r0 = n + 1 + (v / T) * UT;
      c0 = st + (v % T) * UT;
      nr = min(UT, n + 1 + k0 - r0);
    }
    const int nc = min(UT, n - c0);
    double(*A)[LP] = reinterpret_cast<double(*)[LP]>(smem);
    double(*B)[LP] = reinterpret_cast<double(*)[LP]>(smem + UT * LP);
    // matrix cores (v_mfma_f64_16x16x4): wave w owns the 32x32 quadrant (w/2, w%2) = 2x2 MFMA tiles
    const int w = t >> 6, lr = t & 15, lk = (t >> 4) & 3, wy = w >> 1, wx = w & 1;
    constexpr int NQ = UT * PNB / 256;
    {  // the panel loads and the 16 output-tile loads per lane, all issued before any use
      double av[NQ], bv[NQ];
#pragma unroll
      for (int q = 0; q < NQ; q++) {
        const int e = t + 256 * q, i = e / PNB, k = e % PNB;
        av[q] = H[(size_t)(r0 + min(i, nr - 1)) * n + kp + k];
        bv[q] = H[(size_t)(c0 + min(i, nc - 1)) * n + kp + k];
      }
#pragma unroll
      for (int q = 0; q < NQ; q++) {
        const int e = t + 256 * q, i = e / PNB, k = e % PNB;
        A[i][k] = i < nr ? av[q] : 0.0;
        B[i][k] = i < nc ? bv[q] : 0.0;
      }
    }
    double cold[2][2][4];
#pragma unroll
    for (int x = 0; x < 2; x++)
#pragma unroll
      for (int y = 0; y < 2; y++)
#pragma unroll
        for (int r = 0; r < 4; r++)
          cold[x][y][r] = H[(size_t)(r0 + min(32 * wy + 16 * x + lk + 4 * r, nr - 1)) * n + c0 +
                            min(32 * wx + 16 * y + lr, nc - 1)];
    __syncthreads();
    d4v acc[2][2];
#pragma unroll
    for (int x = 0; x < 2; x++)
#pragma unroll
      for (int y = 0; y < 2; y++) acc[x][y] = d4v{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int q = 0; q < PNB; q += 4) {
      double fa[2], fb[2];
#pragma unroll
      for (int x = 0; x < 2; x++) fa[x] = A[32 * wy + 16 * x + lr][q + lk];
#pragma unroll
      for (int y = 0; y < 2; y++) fb[y] = B[32 * wx + 16 * y + lr][q + lk];
#pragma unroll
      for (int x = 0; x < 2; x++)
#pragma unroll
        for (int y = 0; y < 2; y++) acc[x][y] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[x], fb[y], acc[x][y], 0, 0, 0);
    }
#pragma unroll
    for (int x = 0; x < 2; x++)
#pragma unroll
      for (int y = 0; y < 2; y++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
          const int i = 32 * wy + 16 * x + lk + 4 * r, j = 32 * wx + 16 * y + lr;
          if (i < nr && j < nc && !(r0 + i < n && c0 + j > r0 + i))  // strictly-upper part unused
            st_wt(&H[(size_t)(r0 + i) * n + c0 + j], cold[x][y][r] - acc[x][y][r]);
        }
    return;
  }
  // ---- panel s ----
  double(*S)[LP] = reinterpret_cast<double(*)[LP]>(smem);                  // A11 -> L11
  double(*P1s)[LP] = reinterpret_cast<double(*)[LP]>(smem + PNB * LP);     // L_{s,s-1}
  double(*X)[LP] = reinterpret_cast<double(*)[LP]>(smem + 2 * PNB * LP);   // A21 -> L21 (PR rows)
  double(*LR)[LP] = reinterpret_cast<double(*)[LP]>(smem + (2 * PNB + PR) * LP);  // L_{R,s-1}
  double(*Lq)[SB][SB + 2] = reinterpret_cast<double(*)[SB][SB + 2]>(smem + 2 * (PNB + PR) * LP);
  int* flags = reinterpret_cast<int*>(smem + 2 * (PNB + PR) * LP + NSUB * SB * (SB + 2));  // 5 NSUB + 1 words
  if (t < 5 * NSUB + 1) flags[t] = 0;
  const bool upd = k0 > 0;
  const int kp = k0 - PNB;
  const bool carried = (int)blockIdx.x >= P1;
  const int rbase = carried ? n + 1 + ((int)blockIdx.x - P1) * PR : st + (int)blockIdx.x * PR;
  const int rlim = carried ? n + st : n;  // last row of this block's range (inclusive)
  const int col = t % PNB, rs = t / PNB;  // loads: column col of rows rs + RS q
  {
    constexpr int QS = PNB / RS, QX = PR / RS;
    const int cc = min(col, kb - 1);
    double sv[QS], pv[QS], xv[QX], lv[QX];
#pragma unroll
    for (int q = 0; q < QS; q++) {
      const int rr = k0 + min(rs + RS * q, kb - 1);
      sv[q] = H[(size_t)rr * n + k0 + cc];
      if (upd) pv[q] = H[(size_t)rr * n + kp + col];
    }
#pragma unroll
    for (int q = 0; q < QX; q++) {
      const int rr = min(rbase + rs + RS * q, rlim);
      xv[q] = H[(size_t)rr * n + k0 + cc];
      if (upd) lv[q] = H[(size_t)rr * n + kp + col];
    }
#pragma unroll
    for (int q = 0; q < QS; q++) {
      const int i = rs + RS * q;
      // rows / columns past kb padded with the identity: the padding stays inert through every step
      S[i][col] = (i < kb && col < kb) ? (col <= i ? sv[q] : 0.0) : (i == col ? 1.0 : 0.0);
      P1s[i][col] = (upd && i < kb) ? pv[q] : 0.0;
    }
#pragma unroll
    for (int q = 0; q < QX; q++) {
      const int i = rs + RS * q;
      X[i][col] = col < kb ? xv[q] : 0.0;
      LR[i][col] = upd ? lv[q] : 0.0;
    }
  }
  __syncthreads();
  if (t < 64) CST(1);
  const int w = t >> 6, lane = t & 63, lr = t & 15, lk = (t >> 4) & 3;
  if (upd) {  // look-ahead update of the diagonal block's first column block by panel s-1:
    // A11[:, 0:16] -= L_{s,s-1} L_{s,s-1}[0:16]^T, tile (w, 0) per wave (the rest: la_far_tiles, off the chain)
    la_tile(S, P1s, w, 0, lr, lk);
  }
  __syncthreads();  // first column block of the diagonal block complete, flags zeroed
  if (w == 0) {
    CST(2);
    diag_chain<0>(S, Lq, flags, lane, info);  // the serial chain runs ahead on its own wave
    CST(7);
  } else {
    if (upd) {  // the diagonal block's other look-ahead tiles (ti, tj), 1 <= tj <= ti: two per wave
      constexpr int CT = PNB / 16;
      int u = 0;
#pragma unroll
      for (int ti = 1; ti < CT; ti++)
#pragma unroll
        for (int tj = 1; tj <= ti; tj++, u++)
          if (u % 3 == w - 1) la_tile(S, P1s, ti, tj, lr, lk);
    }
    lds_signal(&flags[5 * NSUB], lane);
    la_rows<0>(X, LR, P1s, flags, w, lane, upd);
    if (w == 1) CST(8);
    row_chain<0>(S, X, LR, P1s, Lq, flags, w, lane, upd, info);
  }
  __syncthreads();
  if (w == 0) CST(13);
  {
    constexpr int QX = PR / RS;
#pragma unroll
    for (int q = 0; q < QX; q++) {
      const int i = rs + RS * q, rw = rbase + i;
      if (rw <= rlim && col < kb) st_wt(&H[(size_t)rw * n + k0 + col], X[i][col]);
    }
  }
#ifdef M3S_CHOL_STAMPS
  if (blockIdx.x == 0 && t == 0 && k0 / PNB < 64) {
    s_stamp[14] = __builtin_amdgcn_s_memrealtime();
    for (int k = 0; k < 16; k++) g_chol_stamps[(k0 / PNB) * 16 + k] = s_stamp[k];
  }
#endif
}

// x = L^-T y: row i of the carried block (H row n+1+i, zero before column i) dotted with y (row n),
// one wave per row, fixed summation order (deterministic across ranks).
__global__ void __launch_bounds__(256) chol_apply_kernel(const double* __restrict__ H, double* __restrict__ x, int n,
                                                         const int* __restrict__ done) {
  if (*done) return;
  const int i = (int)((blockIdx.x * 256u + threadIdx.x) >> 6), lane = threadIdx.x & 63;
  if (i >= n) return;
  const double* c = H + (size_t)(n + 1 + i) * n;
  const double* y = H + (size_t)n * n;
  double s0 = 0.0, s1 = 0.0;  // two interleaved partial sums, four row loads per lane in flight
  int j = (i & ~63) + lane;
  for (; j + 192 < n; j += 256) {
    const double c0 = c[j], c1 = c[j + 64], c2 = c[j + 128], c3 = c[j + 192];
    const double y0 = y[j], y1 = y[j + 64], y2 = y[j + 128], y3 = y[j + 192];
    s0 += (j >= i ? c0 * y0 : 0.0) + (j + 128 >= i ? c2 * y2 : 0.0);
    s1 += (j + 64 >= i ? c1 * y1 : 0.0) + (j + 192 >= i ? c3 * y3 : 0.0);
  }
  for (; j < n; j += 64) s0 += j >= i ? c[j] * y[j] : 0.0;
  double s = s0 + s1;
  s = wave_sum(s);
  if (lane == 0) x[i] = s;
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

#ifdef M3S_CHOL_STAMPS
extern "C" int m3s_debug_chol_stamps(unsigned long long* out) {
  (void)hipDeviceSynchronize();
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(m3s::g_chol_stamps), sizeof(unsigned long long) * 1024) == hipSuccess ? 0 : -1;
}
#endif


// ------------------------------------------------------------------------------------------
extern "C" hipError_t m3s_launch_ba_pack(const BaArgs* a, const BaParams* p, int E_local, hipStream_t s) {
  if (E_local <= 0) return hipSuccess;
  const size_t total = (size_t)E_local * p->N;
  const dim3 g((unsigned)std::min<size_t>((total + 255) / 256, 8192));
  if (p->mode == BA_MODE_CALIB)
    hipLaunchKernelGGL(m3s::ba_pack_kernel<BA_MODE_CALIB>, g, dim3(256), 0, s, *a, *p, E_local);
  else if (p->mode == BA_MODE_RAYS)
    hipLaunchKernelGGL(m3s::ba_pack_kernel<BA_MODE_RAYS>, g, dim3(256), 0, s, *a, *p, E_local);
  else
    hipLaunchKernelGGL(m3s::ba_pack_kernel<BA_MODE_POINTS>, g, dim3(256), 0, s, *a, *p, E_local);
  return hipGetLastError();
}

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
    // system + rhs + carried identity rows (the identity itself is written by the assembly launch)
    if (hipMemsetAsync(a->H, 0, sizeof(double) * (size_t)(2 * n + 1) * n, s) != hipSuccess) return hipGetLastError();
    hipLaunchKernelGGL(m3s::ba_assemble_kernel, dim3(nblocks + nrhs_rows + (n + 63) / 64), dim3(64), 0, s, *a, n,
                       nblocks, nrhs_rows);
    for (int k0 = 0; k0 < n; k0 += PNB) {
      const int kb = n - k0 < PNB ? n - k0 : PNB;
      const int st = k0 + kb;
      const int P1 = (n + 1 - st + m3s::PR - 1) / m3s::PR;  // >= 1: the rhs row
      const int P2 = (st + m3s::PR - 1) / m3s::PR;          // carried rows i < st
      int U = 0;
      if (k0 > 0 && st < n) {
        const int T = (n - st + UT - 1) / UT, R = (n + 1 - st + UT - 1) / UT, Rc = (k0 + UT - 1) / UT;
        U = T * (T + 1) / 2 + (R > T ? T : 0) + Rc * T;
      }
      hipLaunchKernelGGL(m3s::chol_step_kernel, dim3(P1 + P2 + U), dim3(256), 0, s, a->H, n, k0, P1, P1 + P2, a->info,
                         a->done);
    }
    hipLaunchKernelGGL(m3s::chol_apply_kernel, dim3((n + 3) / 4), dim3(256), 0, s, a->H, a->x, n, a->done);
  }
  hipLaunchKernelGGL(m3s::ba_retr_kernel, dim3(1), dim3(256), 0, s, *a, K, n, delta_thresh);
  return hipGetLastError();
}
