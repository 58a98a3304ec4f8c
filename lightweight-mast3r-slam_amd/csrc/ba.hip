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
// dense blocked Cholesky, lower, rows 0..n (row n = rhs), columns 0..n-1, right-looking with a
// one-panel look-ahead: launch s factors panel s (PNB = 32 columns) while panel s-1's trailing
// update of the columns beyond panel s runs beside it in the same grid. The panel blocks apply
// panel s-1's update to their own column block first, so the update of the rest of the matrix is
// off the critical path (one launch per panel instead of a panel launch + an update launch).
// ------------------------------------------------------------------------------------------
#define PNB 32
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

// 1/sqrt(d) for d > 0 to ~1 ulp: v_rsq_f64 estimate refined by two Newton steps — a fraction of the
// latency of the correctly rounded sqrt + divide sequences on the pivot chain.
__device__ __forceinline__ double rsqrt_nr(double d) {
  double y = __builtin_amdgcn_rsq(d);
  const double h = 0.5 * d;
#pragma unroll
  for (int it = 0; it < 2; it++) y = fma(y, fma(-h * y, y, 0.5), y);
  return y;
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
    const double inv = rsqrt_nr(d);  // 1/sqrt(d): hardware estimate + two Newton steps (serial chain)
    const double sj = d * inv;
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
// the later columns with column J of L11 (row J of Ls = L11^T in LDS). Row J+1 is read from LDS
// before step J's FMAs (software pipelining: the broadcast reads' latency hides behind them).
template <int J>
__device__ __forceinline__ void trsm_pipe(double (&x)[PNB], const double (*Ls)[PNB + 2], const double (&cur)[PNB + 2]) {
  if constexpr (J < PNB) {
    double nxt[PNB + 2];
    if constexpr (J + 1 < PNB) {
#pragma unroll
      for (int c = (J + 2) & ~1; c < PNB + 2; c += 2) {
        const double2 v = *reinterpret_cast<const double2*>(&Ls[J + 1][c]);
        nxt[c] = v.x;
        nxt[c + 1] = v.y;
      }
    }
    x[J] *= cur[PNB];  // reciprocal of the pivot, stored after the row
#pragma unroll
    for (int k = J + 1; k < PNB; k++) x[k] -= x[J] * cur[k];
    trsm_pipe<J + 1>(x, Ls, nxt);
  }
}

// Launch s of the factorisation (k0 = s*PNB, kb = panel width). Blocks [0, P): 64 rows each of
// panel s below its diagonal block (row n = rhs included):
//   1. coalesced loads of A11 (diagonal block), the block's rows A21 and, for s > 0, the matching
//      rows of panel s-1 (L_{s,s-1} and L_{R,s-1});
//   2. s > 0: A11 -= L_{s,s-1} L_{s,s-1}^T, A21 -= L_{R,s-1} L_{s,s-1}^T (the look-ahead update);
//   3. wave 0 factors A11 (every block redundantly: no extra launch or dependency on the critical
//      path; lanes = rows in registers, readlane broadcasts), block 0 keeps L11 in Ldiag;
//   4. wave 0 solves L21 = A21 L11^-T (lane = row) and the block stores it coalesced.
// Blocks [P, P+U): panel s-1's update A22 -= L21 L21^T over the UTxUT lower tiles of the columns
// beyond panel s (rows and columns from k0+kb; the lower-triangle tiles enumerated, none idle).
// L11 never goes back into H; later launches read the diagonal blocks from Ldiag.
__global__ void __launch_bounds__(256) chol_step_kernel(double* __restrict__ H, double* __restrict__ Ldiag, int n,
                                                        int k0, int P, int* __restrict__ info,
                                                        const int* __restrict__ done) {
  if (*done) return;
  constexpr int LD = PNB + 1;
  __shared__ double smem[2 * 32 * LD + 2 * 64 * LD + 32 * (PNB + 2)];  // >= 2 * 64 * (PNB + 2) (update)
  const int kb = min(PNB, n - k0);
  const int t = threadIdx.x;
  if ((int)blockIdx.x >= P) {
    // ---- trailing update of panel s-1 (columns PNB wide at kp) beyond panel s ----
    const int kp = k0 - PNB, st = k0 + kb;
    const int T = (n - st + UT - 1) / UT;  // column tiles
    const int tri = T * (T + 1) / 2;
    const int u = blockIdx.x - P;
    int ti, tj;
    if (u < tri) {
      ti = (int)((sqrtf(8.0f * (float)u + 1.0f) - 1.0f) * 0.5f);
      while (ti * (ti + 1) / 2 > u) ti--;
      while ((ti + 1) * (ti + 2) / 2 <= u) ti++;
      tj = u - ti * (ti + 1) / 2;
    } else {  // the extra tile row holding only the rhs row (when n - st is a multiple of UT)
      ti = T;
      tj = u - tri;
    }
    const int r0 = st + ti * UT, c0 = st + tj * UT;
    const int nr = min(UT, n + 1 - r0), nc = min(UT, n - c0);
    constexpr int LU = PNB + 2;  // row pitch: the MFMA fragment reads below are conflict-free
    double(*A)[LU] = reinterpret_cast<double(*)[LU]>(smem);
    double(*B)[LU] = reinterpret_cast<double(*)[LU]>(smem + 64 * LU);
    // matrix cores (v_mfma_f64_16x16x4): wave w owns the 32x32 quadrant (w/2, w%2) = 2x2 MFMA tiles
    const int w = t >> 6, lr = t & 15, lk = (t >> 4) & 3, wy = w >> 1, wx = w & 1;
    {  // 8 + 8 panel loads and the 16 output-tile loads per lane, all issued before any use
      double av[8], bv[8];
#pragma unroll
      for (int q = 0; q < 8; q++) {
        const int e = t + 256 * q, i = e / PNB, k = e % PNB;
        av[q] = H[(size_t)(r0 + min(i, nr - 1)) * n + kp + k];
        bv[q] = H[(size_t)(c0 + min(i, nc - 1)) * n + kp + k];
      }
#pragma unroll
      for (int q = 0; q < 8; q++) {
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
            H[(size_t)(r0 + i) * n + c0 + j] = cold[x][y][r] - acc[x][y][r];
        }
    return;
  }
  // ---- panel s ----
  double(*S)[LD] = reinterpret_cast<double(*)[LD]>(smem);             // A11 -> L11
  double(*P1)[LD] = reinterpret_cast<double(*)[LD]>(smem + 32 * LD);  // L_{s,s-1}
  double(*X)[LD] = reinterpret_cast<double(*)[LD]>(smem + 64 * LD);   // A21 -> L21 (64 rows)
  double(*LR)[LD] = reinterpret_cast<double(*)[LD]>(smem + 128 * LD); // L_{R,s-1}
  double(*Ls)[PNB + 2] = reinterpret_cast<double(*)[PNB + 2]>(smem + 192 * LD);
  const bool upd = k0 > 0;
  const int kp = k0 - PNB;
  const int rbase = k0 + kb + blockIdx.x * 64;
  const int col = t & 31, rs = t >> 5;  // loads: column col of rows rs + 8q
  {
    const int cc = min(col, kb - 1);
    double sv[4], pv[4], xv[8], lv[8];
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int rr = k0 + min(rs + 8 * q, kb - 1);
      sv[q] = H[(size_t)rr * n + k0 + cc];
      if (upd) pv[q] = H[(size_t)rr * n + kp + col];
    }
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const int rr = min(rbase + rs + 8 * q, n);
      xv[q] = H[(size_t)rr * n + k0 + cc];
      if (upd) lv[q] = H[(size_t)rr * n + kp + col];
    }
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int i = rs + 8 * q;
      S[i][col] = (i < kb && col < kb && col <= i) ? sv[q] : 0.0;
      P1[i][col] = (upd && i < kb) ? pv[q] : 0.0;
    }
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const int i = rs + 8 * q;
      X[i][col] = col < kb ? xv[q] : 0.0;
      LR[i][col] = upd ? lv[q] : 0.0;
    }
  }
  __syncthreads();
#ifdef CHOL_NOUPD
  if (false) {
#else
  if (upd) {  // look-ahead update of this column block by panel s-1
#endif
    // on the matrix cores (v_mfma_f64_16x16x4): wave w takes rows 16w..16w+15 of A21 (both 16-column
    // halves) and the 16x16 tile (w/2, w%2) of A11. Operand maps: A[l&15][k=l>>4], B[k=l>>4][l&15];
    // result row (l>>4)+4r, column l&15. Rows of P1 past kb are zero, so the padding stays zero.
    const int w = t >> 6, lr = t & 15, lk = (t >> 4) & 3;
    const int ti = w >> 1, tj = w & 1;
    d4v c0 = {0.0, 0.0, 0.0, 0.0}, c1 = c0, cs = c0;
#pragma unroll
    for (int q = 0; q < PNB; q += 4) {
      const double av = LR[16 * w + lr][q + lk];
      c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(av, P1[lr][q + lk], c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(av, P1[16 + lr][q + lk], c1, 0, 0, 0);
      cs = __builtin_amdgcn_mfma_f64_16x16x4f64(P1[16 * ti + lr][q + lk], P1[16 * tj + lr][q + lk], cs, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int i = 16 * w + lk + 4 * r;
      X[i][lr] -= c0[r];
      X[i][16 + lr] -= c1[r];
      const int si = 16 * ti + lk + 4 * r, sj = 16 * tj + lr;
      if (sj <= si) S[si][sj] -= cs[r];
    }
    __syncthreads();
  }
  if (t < 64) {
    const int lane = t, li = min(lane, PNB - 1);
    {
      double r[PNB];
#pragma unroll
      for (int c = 0; c < PNB; c++) r[c] = (li < kb && c < kb) ? S[li][c] : (c == li ? 1.0 : 0.0);
      bool bad = false;
#ifndef CHOL_NODIAG
      diag_step<0>(r, lane, bad);
#endif
      if (bad && lane == 0 && blockIdx.x == 0) *info = 1;
      wave_sync();
      if (lane < PNB)
#pragma unroll
        for (int c = 0; c < PNB; c++) S[lane][c] = c <= lane ? r[c] : 0.0;
    }
    wave_sync();
    if (lane < PNB) {
      for (int q = 0; q < PNB; q++) Ls[q][lane] = S[lane][q];  // Ls = L11^T (padded)
      const double dj = S[lane][lane];
      double y = __builtin_amdgcn_rcp(dj);  // 1/L_jj: estimate + two Newton steps
      y = fma(y, fma(-dj, y, 1.0), y);
      y = fma(y, fma(-dj, y, 1.0), y);
      Ls[lane][PNB] = y;
      Ls[lane][PNB + 1] = 0.0;
      if (blockIdx.x == 0) {
        double* Ld = Ldiag + (size_t)(k0 / PNB) * PNB * PNB;
        for (int q = 0; q < PNB; q++) Ld[q * PNB + lane] = S[q][lane];  // row-major L11 (padded)
      }
    }
    wave_sync();
    double x[PNB], row0[PNB + 2];
#pragma unroll
    for (int c = 0; c < PNB; c++) x[c] = X[lane][c];
#pragma unroll
    for (int c = 0; c < PNB + 2; c += 2) {
      const double2 v = *reinterpret_cast<const double2*>(&Ls[0][c]);
      row0[c] = v.x;
      row0[c + 1] = v.y;
    }
#ifndef CHOL_NOTRSM
    trsm_pipe<0>(x, Ls, row0);
#endif
#pragma unroll
    for (int c = 0; c < PNB; c++) X[lane][c] = x[c];
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 8; q++) {
    const int i = rs + 8 * q, rw = rbase + i;
    if (rw <= n && col < kb) H[(size_t)rw * n + k0 + col] = X[i][col];
  }
}

// Back substitution L^T x = y (y = row n after the factorisation), one launch per BS_NB-column
// panel from the end (right-looking):
//   A (every block, redundantly): load the panel's diagonal block of L into LDS (its PNB-diagonal
//     blocks from Ldiag) and back-solve it with one wave (lanes hold two unknowns each; x_c broadcast
//     by readlane, the next row of L prefetched from LDS);
//   B (block b, columns [b*BS_NB, (b+1)*BS_NB) below k0): y_j -= sum_r L[k0+r][j] x_r, read row-wise
//     (coalesced) by two half-blocks, written back into row n for the next launch.
// Replaces a single-block solve that streamed all of L through one CU.
#define BS_NB 128
__global__ void __launch_bounds__(1024) chol_back_step_kernel(double* __restrict__ H, const double* __restrict__ Ldiag,
                                                              double* __restrict__ xg, int n, int k0,
                                                              const int* __restrict__ done) {
  if (*done) return;
  const int kb = min(BS_NB, n - k0);
  __shared__ double Ld[BS_NB][BS_NB + 1];
  __shared__ double rd[BS_NB];
  __shared__ double xs[BS_NB];
  __shared__ double part[8][BS_NB];
  const int t = threadIdx.x;
  const double* yrow = H + (size_t)n * n;
  // every global load of the launch is issued up front: the diagonal block (16 per thread) and the
  // panel rows phase B multiplies (16 per thread; they do not depend on x)
  double v[16], pb[16];
#pragma unroll
  for (int u = 0; u < 16; u++) {
    const int e = u * 1024 + t, i = e / BS_NB, j = e % BS_NB;
    const int ic = min(i, kb - 1), jc = min(j, ic);
    v[u] = (ic / PNB == jc / PNB) ? Ldiag[(size_t)((k0 + ic) / PNB) * PNB * PNB + (ic % PNB) * PNB + (jc % PNB)]
                                  : H[(size_t)(k0 + ic) * n + k0 + jc];
  }
  const int jl = t & (BS_NB - 1), rg = t >> 7;  // phase B: column jl, rows rg + 8u
  const int j = blockIdx.x * BS_NB + jl;
  if (k0 > 0) {
    const int jc = min(j, k0 - 1);
#pragma unroll
    for (int u = 0; u < 16; u++) pb[u] = H[(size_t)(k0 + min(rg + 8 * u, kb - 1)) * n + jc];
  }
#pragma unroll
  for (int u = 0; u < 16; u++) {  // rows/columns past kb padded with the identity
    const int e = u * 1024 + t, i = e / BS_NB, jj = e % BS_NB;
    Ld[i][jj] = (i < kb && jj <= i) ? v[u] : (i == jj ? 1.0 : 0.0);
  }
  __syncthreads();
  if (t < BS_NB) {
    const double d = Ld[t][t];
    double y = __builtin_amdgcn_rcp(d);  // 1/L_cc: estimate + two Newton steps
    y = fma(y, fma(-d, y, 1.0), y);
    rd[t] = fma(y, fma(-d, y, 1.0), y);
  }
  __syncthreads();
  if (t < 64) {  // one wave, two unknowns per lane, fully unrolled over the padded 128 columns
    double y0 = t < kb ? yrow[k0 + t] : 0.0, y1 = t + 64 < kb ? yrow[k0 + t + 64] : 0.0;
    // L[c][k] = 0 for k > c; k == c only disturbs the finished unknown c
#pragma unroll 8
    for (int c = BS_NB - 1; c >= 64; c--) {
      const double xc = bcast_lane(y1, c - 64) * rd[c];
      y0 -= Ld[c][t] * xc;
      y1 -= Ld[c][t + 64] * xc;
      if (t == 0) xs[c] = xc;
    }
#pragma unroll 8
    for (int c = 63; c >= 0; c--) {
      const double xc = bcast_lane(y0, c) * rd[c];
      y0 -= Ld[c][t] * xc;
      if (t == 0) xs[c] = xc;
    }
  }
  __syncthreads();
  if (blockIdx.x == 0 && t < kb) xg[k0 + t] = xs[t];
  if (k0 > 0) {
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int u = 0; u < 16; u++) acc[u & 3] += pb[u] * xs[rg + 8 * u];  // xs = 0 past kb
    part[rg][jl] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
    __syncthreads();
    if (t < BS_NB && j < k0) {
      double sum = 0.0;
#pragma unroll
      for (int g = 0; g < 8; g++) sum += part[g][t];
      H[(size_t)n * n + j] -= sum;
    }
  }
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
      const int st = k0 + kb;
      const int P = (n + 1 - st + 63) / 64;  // >= 1: the rhs row
      int U = 0;
      if (k0 > 0 && st < n) {
        const int T = (n - st + UT - 1) / UT, R = (n + 1 - st + UT - 1) / UT;
        U = T * (T + 1) / 2 + (R > T ? T : 0);
      }
      hipLaunchKernelGGL(m3s::chol_step_kernel, dim3(P + U), dim3(256), 0, s, a->H, a->Lt, n, k0, P, a->info,
                         a->done);
    }
    for (int k0 = ((n - 1) / BS_NB) * BS_NB; k0 >= 0; k0 -= BS_NB)
      hipLaunchKernelGGL(m3s::chol_back_step_kernel, dim3(k0 > 0 ? (k0 + BS_NB - 1) / BS_NB : 1), dim3(1024), 0, s,
                         a->H, a->Lt, a->x, n, k0, a->done);
  }
  hipLaunchKernelGGL(m3s::ba_retr_kernel, dim3(1), dim3(256), 0, s, *a, K, n, delta_thresh);
  return hipGetLastError();
}
