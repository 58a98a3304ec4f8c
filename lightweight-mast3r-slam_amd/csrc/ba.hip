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
//     (instead of 105 + 14 transformed entries) and the per-edge transform is applied once.
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
#define CH_NB 64

// ------------------------------------------------------------------------------------------
// linearisation
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void acc_local(float* L, float* v, const float J[7], float w, float e) {
  int l = 0;
#pragma unroll
  for (int c = 0; c < 7; c++) {
    const float wj = w * J[c];
#pragma unroll
    for (int d = c; d < 7; d++) L[l++] += wj * J[d];
    v[c] += wj * e;
  }
}

__global__ void __launch_bounds__(256) ba_lin_kernel(BaArgs a, BaParams p) {
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
  float L[28], v[7];
#pragma unroll
  for (int c = 0; c < 28; c++) L[c] = 0.0f;
#pragma unroll
  for (int c = 0; c < 7; c++) v[c] = 0.0f;
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
    const float sqq = sqrtf(q);
    if (p.mode == BA_MODE_POINTS) {
      const float err[3] = {Y[0] - Xi[0], Y[1] - Xi[1], Y[2] - Xi[2]};
      const float sw = valid ? p.inv_a * sqq : 0.0f;
      const float wc = sw * sw;
      const float J0[7] = {1.0f, 0.0f, 0.0f, 0.0f, Y[2], -Y[1], Y[0]};
      const float J1[7] = {0.0f, 1.0f, 0.0f, -Y[2], 0.0f, Y[0], Y[1]};
      const float J2[7] = {0.0f, 0.0f, 1.0f, Y[1], -Y[0], 0.0f, Y[2]};
      acc_local(L, v, J0, huber_ba(sw * err[0]) * wc, err[0]);
      acc_local(L, v, J1, huber_ba(sw * err[1]) * wc, err[1]);
      acc_local(L, v, J2, huber_ba(sw * err[2]) * wc, err[2]);
    } else if (p.mode == BA_MODE_RAYS) {
      const float n1i = sqrtf(Xi[0] * Xi[0] + Xi[1] * Xi[1] + Xi[2] * Xi[2]);
      const float n1i_inv = 1.0f / n1i;
      const float n2j = Y[0] * Y[0] + Y[1] * Y[1] + Y[2] * Y[2];
      const float n1j = sqrtf(n2j);
      const float n1j_inv = 1.0f / n1j;
      const float rj[3] = {n1j_inv * Y[0], n1j_inv * Y[1], n1j_inv * Y[2]};
      const float err[4] = {rj[0] - n1i_inv * Xi[0], rj[1] - n1i_inv * Xi[1], rj[2] - n1i_inv * Xi[2], n1j - n1i};
      const float swr = valid ? p.inv_a * sqq : 0.0f;
      const float swd = valid ? p.inv_b * sqq : 0.0f;
      const float wr = swr * swr, wd = swd * swd;
      const float n3 = n1j_inv / n2j;
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
      acc_local(L, v, J0, huber_ba(swr * err[0]) * wr, err[0]);
      acc_local(L, v, J1, huber_ba(swr * err[1]) * wr, err[1]);
      acc_local(L, v, J2, huber_ba(swr * err[2]) * wr, err[2]);
      acc_local(L, v, J3, huber_ba(swd * err[3]) * wd, err[3]);
    } else {  // calib
      const int u_t = (int)(ind % p.W), v_t = (int)(ind / p.W);
      const bool valid_z = (Y[2] > p.z_eps) && (Xi[2] > p.z_eps);
      const float zj_inv = valid_z ? 1.0f / Y[2] : 0.0f;
      const float zj_log = valid_z ? logf(Y[2]) : 0.0f;
      const float zi_log = valid_z ? logf(Xi[2]) : 0.0f;
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
      acc_local(L, v, J0, huber_ba(swp * err[0]) * wp, err[0]);
      acc_local(L, v, J1, huber_ba(swp * err[1]) * wp, err[1]);
      acc_local(L, v, J2, huber_ba(swd * err[2]) * wd, err[2]);
    }
  }
  // wave64 butterfly in fp64, then 4 waves through LDS
  __shared__ double s_part[4][BA_NSUM];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int c = 0; c < 28; c++) {
    const double t = wave_sum((double)L[c]);
    if (lane == 0) s_part[wid][c] = t;
  }
#pragma unroll
  for (int c = 0; c < 7; c++) {
    const double t = wave_sum((double)v[c]);
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
// dense blocked Cholesky, lower, rows 0..n (row n = rhs), columns 0..n-1
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) chol_diag_kernel(double* __restrict__ H, int n, int k0, int* __restrict__ info,
                                                        const int* __restrict__ done) {
  if (*done) return;
  const int kb = min(CH_NB, n - k0);
  __shared__ double T[CH_NB][CH_NB + 1];
  for (int t = threadIdx.x; t < kb * kb; t += blockDim.x) {
    const int i = t / kb, j = t % kb;
    T[i][j] = (j <= i) ? H[(size_t)(k0 + i) * n + k0 + j] : 0.0;
  }
  __syncthreads();
  for (int j = 0; j < kb; j++) {
    if (threadIdx.x == 0) {
      double d = T[j][j];
      if (!(d > 0.0)) {
        *info = 1;
        d = 1.0;
      }
      T[j][j] = sqrt(d);
    }
    __syncthreads();
    const double djj = T[j][j];
    for (int i = j + 1 + threadIdx.x; i < kb; i += blockDim.x) T[i][j] /= djj;
    __syncthreads();
    const int m = kb - j - 1;  // trailing (m x m) lower update
    for (int t = threadIdx.x; t < m * m; t += blockDim.x) {
      const int i = j + 1 + t / m, c = j + 1 + t % m;
      if (c <= i) T[i][c] -= T[i][j] * T[c][j];
    }
    __syncthreads();
  }
  for (int t = threadIdx.x; t < kb * kb; t += blockDim.x) {
    const int i = t / kb, j = t % kb;
    if (j <= i) H[(size_t)(k0 + i) * n + k0 + j] = T[i][j];
  }
}

// rows r in [k0+kb, n] (row n = rhs): L21 = A21 L11^-T, 64 rows per block, right-looking over
// the panel's columns so all 256 lanes work between the 2*kb barriers
__global__ void __launch_bounds__(256) chol_trsm_kernel(double* __restrict__ H, int n, int k0,
                                                        const int* __restrict__ done) {
  if (*done) return;
  const int kb = min(CH_NB, n - k0);
  __shared__ double Ls[CH_NB][CH_NB + 1];
  __shared__ double X[CH_NB][CH_NB + 1];
  for (int t = threadIdx.x; t < kb * kb; t += blockDim.x) {
    const int i = t / kb, j = t % kb;
    Ls[i][j] = (j <= i) ? H[(size_t)(k0 + i) * n + k0 + j] : 0.0;
  }
  const int r0 = k0 + kb + blockIdx.x * CH_NB;
  const int nr = min(CH_NB, n + 1 - r0);
  for (int t = threadIdx.x; t < nr * kb; t += blockDim.x) {
    const int i = t / kb, j = t % kb;
    X[i][j] = H[(size_t)(r0 + i) * n + k0 + j];
  }
  __syncthreads();
  for (int j = 0; j < kb; j++) {
    if (threadIdx.x < nr) X[threadIdx.x][j] /= Ls[j][j];
    __syncthreads();
    const int m = kb - j - 1;
    for (int t = threadIdx.x; t < nr * m; t += blockDim.x) {
      const int i = t / m, c = j + 1 + t % m;
      X[i][c] -= X[i][j] * Ls[c][j];
    }
    __syncthreads();
  }
  for (int t = threadIdx.x; t < nr * kb; t += blockDim.x) {
    const int ii = t / kb, j = t % kb;
    H[(size_t)(r0 + ii) * n + k0 + j] = X[ii][j];
  }
}

// trailing update A22 -= L21 L21^T over 64x64 lower tiles; rows [s, n], cols [s, n-1], s = k0+kb
__global__ void __launch_bounds__(256) chol_update_kernel(double* __restrict__ H, int n, int k0,
                                                          const int* __restrict__ done) {
  if (*done) return;
  const int kb = min(CH_NB, n - k0);
  const int s = k0 + kb;
  const int ti = blockIdx.x, tj = blockIdx.y;
  if (tj > ti) return;
  const int r0 = s + ti * CH_NB, c0 = s + tj * CH_NB;
  if (c0 >= n) return;
  const int nr = min(CH_NB, n + 1 - r0), nc = min(CH_NB, n - c0);
  __shared__ double A[CH_NB][CH_NB + 1];
  __shared__ double B[CH_NB][CH_NB + 1];
  for (int t = threadIdx.x; t < CH_NB * kb; t += blockDim.x) {
    const int i = t / kb, k = t % kb;
    A[i][k] = i < nr ? H[(size_t)(r0 + i) * n + k0 + k] : 0.0;
    B[i][k] = i < nc ? H[(size_t)(c0 + i) * n + k0 + k] : 0.0;
  }
  __syncthreads();
  const int ty = threadIdx.x / 16, tx = threadIdx.x % 16;  // 4x4 outputs per lane
  double acc[4][4];
#pragma unroll
  for (int x = 0; x < 4; x++)
#pragma unroll
    for (int y = 0; y < 4; y++) acc[x][y] = 0.0;
  for (int k = 0; k < kb; k++) {
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

// backward substitution L^T x = y for the panel at k0 (called for panels in reverse order):
// the already-solved tail is folded in by a 4x64-lane column GEMV, then wave 0 back-solves the
// 64x64 diagonal block with x broadcast by lane shuffles.
__global__ void __launch_bounds__(256) chol_back_kernel(const double* __restrict__ H, double* __restrict__ x, int n,
                                                        int k0, const int* __restrict__ done) {
  if (*done) return;
  const int kb = min(CH_NB, n - k0);
  __shared__ double part[4][CH_NB];
  __shared__ double Ld[CH_NB][CH_NB + 1];
  const int c = threadIdx.x % CH_NB, g = threadIdx.x / CH_NB;
  double s = 0.0;
  if (c < kb)
    for (int r = k0 + kb + g; r < n; r += 4) s += H[(size_t)r * n + k0 + c] * x[r];
  part[g][c] = s;
  for (int t = threadIdx.x; t < kb * kb; t += blockDim.x) {
    const int i = t / kb, j = t % kb;
    Ld[i][j] = (j <= i) ? H[(size_t)(k0 + i) * n + k0 + j] : 0.0;
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    double y = 0.0;
    if (lane < kb) y = H[(size_t)n * n + k0 + lane] - (part[0][lane] + part[1][lane] + part[2][lane] + part[3][lane]);
    for (int cc = kb - 1; cc >= 0; cc--) {
      const double xc = __shfl(y, cc, 64) / Ld[cc][cc];
      if (lane == cc) y = xc;
      if (lane < cc) y -= Ld[cc][lane] * xc;
    }
    if (lane < kb) x[k0 + lane] = y;
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
  hipLaunchKernelGGL(m3s::ba_lin_kernel, dim3(E_local * p->chunks), dim3(256), 0, s, *a, *p);
  hipLaunchKernelGGL(m3s::ba_edge_kernel, dim3(E_local), dim3(64), 0, s, *a, *p, E_local);
  return hipGetLastError();
}

extern "C" hipError_t m3s_launch_ba_solve(const BaArgs* a, int K, int nblocks, int nrhs_rows, float delta_thresh,
                                          hipStream_t s) {
  const int n = (K - 1) * 7;
  if (n > 0) {
    if (hipMemsetAsync(a->H, 0, sizeof(double) * (size_t)(n + 1) * n, s) != hipSuccess) return hipGetLastError();
    hipLaunchKernelGGL(m3s::ba_assemble_kernel, dim3(nblocks + nrhs_rows), dim3(64), 0, s, *a, n, nblocks);
    for (int k0 = 0; k0 < n; k0 += CH_NB) {
      const int kb = n - k0 < CH_NB ? n - k0 : CH_NB;
      hipLaunchKernelGGL(m3s::chol_diag_kernel, dim3(1), dim3(256), 0, s, a->H, n, k0, a->info, a->done);
      const int rows = n + 1 - (k0 + kb);
      if (rows > 0) {
        const int tr = (rows + CH_NB - 1) / CH_NB;
        hipLaunchKernelGGL(m3s::chol_trsm_kernel, dim3(tr), dim3(256), 0, s, a->H, n, k0, a->done);
        const int tc = (n - (k0 + kb) + CH_NB - 1) / CH_NB;
        if (tc > 0) hipLaunchKernelGGL(m3s::chol_update_kernel, dim3(tr, tc), dim3(256), 0, s, a->H, n, k0, a->done);
      }
    }
    for (int k0 = ((n - 1) / CH_NB) * CH_NB; k0 >= 0; k0 -= CH_NB)
      hipLaunchKernelGGL(m3s::chol_back_kernel, dim3(1), dim3(256), 0, s, a->H, a->x, n, k0, a->done);
  }
  hipLaunchKernelGGL(m3s::ba_retr_kernel, dim3(1), dim3(256), 0, s, *a, K, n, delta_thresh);
  return hipGetLastError();
}
