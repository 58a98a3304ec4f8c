// Dense fp64 Cholesky of the BA pose system (fallback for fill-heavy graphs).
//
// The block-sparse factorisation (ba.hip, ba_sparse_factor_kernel) runs down the elimination tree inside
// one workgroup; on graphs whose fill makes the factor nearly dense (e.g. loop closures to random earlier
// keyframes) its level count and update volume approach the dense case, and this multi-CU dense
// factorisation is faster. The plan picks one of the two from the symbolic factorisation (abi.cpp).
// Same system, same order (the plan's minimum-degree permutation), fp64, deterministic (every element
// has one owner and a fixed summation order), so ranks stay bit-identical either way.
//
// Layout: H is ((2n+1) x n) row-major, n = 7 (K-1): rows 0..n-1 the system (lower triangle used), row n
// the rhs g^T, rows n+1.. an identity carried through the factorisation (-> L^-T, so the back
// substitution is one parallel mat-vec).
#include "m3s_common.hpp"
#include "m3s_ba.h"

namespace m3s_dense {
using m3s::wave_sum;

#define BA_NSUM 36

// assembly of the dense system from the plan's per-factor-block contribution CSR (blocks of the
// permuted system; block (rowL[b], column j) -> H rows 7 rowL[b].., columns 7 j..), rhs rows and the
// carried identity
__global__ void __launch_bounds__(64) dense_assemble_kernel(BaArgs a, int n, int nL) {
  if (*a.done) return;
  const int b = blockIdx.x;
  const int t = threadIdx.x;
  if (b >= nL + a.nb) {  // carried identity rows (H row n+1+i = e_i^T)
    const int i = (b - nL - a.nb) * 64 + t;
    if (i < n) a.H[(size_t)(n + 1 + i) * n + i] = 1.0;
    return;
  }
  const int* ptr = b < nL ? a.asm_ptr + b : a.rhs_ptr + (b - nL);
  const int* ent = b < nL ? a.asm_ent : a.rhs_ent;
  int li;
  double* out;
  if (b < nL) {
    if (t >= 49) return;
    const int rr = t / 7, cc = t - 7 * (t / 7);
    const int lo = min(rr, cc), hi = max(rr, cc);
    li = lo * 7 - lo * (lo - 1) / 2 + (hi - lo);
    const int r = a.rowL[b];
    int j = 0;  // the column of block b: col_ptr[j] <= b < col_ptr[j+1]
    int lo_j = 0, hi_j = a.nb;
    while (hi_j - lo_j > 1) {
      const int mid = (lo_j + hi_j) >> 1;
      if (a.col_ptr[mid] <= b) lo_j = mid;
      else hi_j = mid;
    }
    j = lo_j;
    out = a.H + (size_t)(r * 7 + rr) * n + j * 7 + cc;
  } else {
    if (t >= 7) return;
    li = 28 + t;
    out = a.H + (size_t)n * n + (b - nL) * 7 + t;
  }
  double s = 0.0;
  const int kb = ptr[0], ke = ptr[1];
  for (int k = kb; k < ke; k++) {
    const int e = ent[k];
    s += ((e & 1) ? -1.0 : 1.0) * a.edge_sums[(size_t)(e >> 1) * BA_NSUM + li];
  }
  *out = s;
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

#define CST(k) \
  do {         \
  } while (0)

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

// dx = -x in pose order (0 when the factorisation failed), poses k >= 1 retracted, |dx| early exit
__global__ void __launch_bounds__(256) dense_finish_kernel(BaArgs a, int K, int n, float delta_thresh) {
  if (*a.done) return;
  const bool failed = *a.info != 0;
  __shared__ float s_n2[4];
  float n2 = 0.0f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int j = i / 7, m = i - 7 * (i / 7);
    const float d = failed ? 0.0f : (float)(-a.xs[i]);
    a.dx[a.perm[j] * 7 + m] = d;
    n2 += d * d;
  }
  __syncthreads();
  for (int k = 1 + threadIdx.x; k < K; k += blockDim.x) {
    float T[8], xi[7];
    for (int c = 0; c < 8; c++) T[c] = a.Twc[k * 8 + c];
    for (int c = 0; c < 7; c++) xi[c] = a.dx[(k - 1) * 7 + c];
    m3s::retrSim3_d(xi, T);  // fp64 retraction (m3s_common.hpp)
    for (int c = 0; c < 8; c++) a.Twc[k * 8 + c] = T[c];
  }
  n2 = wave_sum(n2);
  if ((threadIdx.x & 63) == 0) s_n2[threadIdx.x >> 6] = n2;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float nrm = sqrtf(s_n2[0] + s_n2[1] + s_n2[2] + s_n2[3]);
    *a.iters += 1;
    if (nrm < delta_thresh) *a.done = 1;
    if (*a.info == 2) {  // an LDS hand-off stalled (lds_wait_ge): sticky, the loop ends, the host reports M3S_ESTALL
      *a.stalled = 1;
      *a.done = 1;
    }
    *a.info = 0;
  }
}

}  // namespace m3s_dense

extern "C" hipError_t m3s_launch_ba_solve_dense(const BaArgs* a, int K, int nL, float delta_thresh, hipStream_t s) {
  const int n = a->nb * 7;
  if (n > 0) {
    // system + rhs + carried identity rows (the identity itself is written by the assembly launch)
    if (hipMemsetAsync(a->H, 0, sizeof(double) * (size_t)(2 * n + 1) * n, s) != hipSuccess) return hipGetLastError();
    hipLaunchKernelGGL(m3s_dense::dense_assemble_kernel, dim3(nL + a->nb + (n + 63) / 64), dim3(64), 0, s, *a, n, nL);
    for (int k0 = 0; k0 < n; k0 += PNB) {
      const int kb = n - k0 < PNB ? n - k0 : PNB;
      const int st = k0 + kb;
      const int P1 = (n + 1 - st + m3s_dense::PR - 1) / m3s_dense::PR;  // >= 1: the rhs row
      const int P2 = (st + m3s_dense::PR - 1) / m3s_dense::PR;          // carried rows i < st
      int U = 0;
      if (k0 > 0 && st < n) {
        const int T = (n - st + UT - 1) / UT, R = (n + 1 - st + UT - 1) / UT, Rc = (k0 + UT - 1) / UT;
        U = T * (T + 1) / 2 + (R > T ? T : 0) + Rc * T;
      }
      hipLaunchKernelGGL(m3s_dense::chol_step_kernel, dim3(P1 + P2 + U), dim3(256), 0, s, a->H, n, k0, P1, P1 + P2,
                         a->info, a->done);
    }
    hipLaunchKernelGGL(m3s_dense::chol_apply_kernel, dim3((n + 3) / 4), dim3(256), 0, s, a->H, a->xs, n, a->done);
  }
  hipLaunchKernelGGL(m3s_dense::dense_finish_kernel, dim3(1), dim3(256), 0, s, *a, K, n, delta_thresh);
  return hipGetLastError();
}
