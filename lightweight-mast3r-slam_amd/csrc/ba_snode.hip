// Supernodal Cholesky of the global-BA pose system (SparseBlock + SimplicialLLT, gn_kernels.cu:57-159) for MI355X.
//
// The plan (ba_snode.cpp, ba_pattern.h ba_snode_plan) groups chains of elimination-tree columns into supernodes. A
// supernode is factored by one GROUP of SN_GW = 4 waves (one per SIMD) as a dense panel in registers: group lane p
// (0..255) owns panel row p = 7 * (block row) + (row in the 7x7 block); the rhs is the last panel row (7R), so the
// forward substitution y = L^-1 b is the panel's augmented row. Per supernode:
//   1. wait until its child supernodes are done (LDS flags: every wave of the producing group adds 1 after its stores);
//   2. load A: the assembled factor blocks of its rows (zeros where the structure has none), the rhs rows;
//   3. pull (left-looking): for every descendant column k meeting its columns, ascending k, each lane's row of L(:, k)
//      (or y_k) times the 7x7 blocks L(c_t, k)^T of the hit columns: 49 FMAs per (k, t), fp64;
//   4. factor the panel column by column t: the 7x7 diagonal block (its rows are lanes 7t..7t+6 of the group's first
//      wave) is shared through LDS and factored redundantly in every lane; each row below takes the triangular solve
//      with it; rows of the later diagonal blocks share their new entries through LDS and every row below takes the
//      rank-7 update. Two group barriers per column (an LDS counter of the group's 4 waves);
//   5. store the factor rows into their blocks (diagonal blocks keep 1/L_mm in column 7, as the back substitution of
//      ba_sparse_factor_kernel expects) and y.
// The ONE multi-workgroup launch runs the supernodes below the plan's cut (whole subtrees per workgroup, nothing
// shared between workgroups); one workgroup runs the rest. Every order is fixed by the plan (pulls ascending, the
// panel arithmetic lane-local): deterministic, identical on every rank. A non-positive pivot sets BA_BAD_LLT (the
// reference's silent zero step), a timed-out wait BA_BAD_STALL, in *a.bad (read by the back-substitution launch).
#include "m3s_common.hpp"
#include "m3s_ba.h"

namespace m3s {

constexpr int SN_GW = 4;          // waves per group
constexpr int SN_MAXN = 4096;     // supernodes (<= poses)
constexpr int SN_SPINS = 1 << 20;  // bounded waits (a stall is an error, never a hang)

__device__ __forceinline__ int sn_ld(const int* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void sn_add(int* p, int v) {
  __hip_atomic_fetch_add(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// barrier of one group's 4 waves: a monotonic LDS counter (the workgroup barrier would hold every group)
__device__ __forceinline__ bool sn_gbar(int* ctr, int& phase, int lane, int* bad) {
  phase += SN_GW;
  if (lane == 0) sn_add(ctr, 1);
  int spins = 0;
  while (sn_ld(ctr) < phase) {
    if (++spins > SN_SPINS) {
      if (lane == 0) atomicOr(bad, BA_BAD_STALL);
      return false;
    }
  }
  return true;
}

__device__ __forceinline__ double sn_rsqrt(double d) {  // v_rsq_f64 + one Newton step (as rsqrt_nr in ba.hip)
  const double y = __builtin_amdgcn_rsq(d);
  return fma(y, fma(-0.5 * d * y, y, 0.5), y);
}

__device__ __forceinline__ void ld7(double (&v)[7], const double* p) {
  if (p) {
    const double2 a = reinterpret_cast<const double2*>(p)[0], b = reinterpret_cast<const double2*>(p)[1],
                  c = reinterpret_cast<const double2*>(p)[2];
    v[0] = a.x; v[1] = a.y; v[2] = b.x; v[3] = b.y; v[4] = c.x; v[5] = c.y; v[6] = p[6];
  } else {
#pragma unroll
    for (int c = 0; c < 7; c++) v[c] = 0.0;
  }
}

template <int SMAX>
__device__ bool sn_supernode(const BaArgs& a, const int* T, int S, int p, int lane, bool first_wave, const int* done,
                             int* bar, int& phase, double* sD, double* sE, int* bad) {
  const int* rec = T + T[2] + 8 * S;
  const int s = rec[0], R = rec[1];
  const int* rows = T + rec[2];
  const int* blk = T + rec[3];
  // 1. the child supernodes
  for (int c0 = rec[6]; c0 < rec[7]; c0 += 64) {
    const int ci = c0 + lane < rec[7] ? T[c0 + lane] : -1;
    int spins = 0;
    while (__ballot(ci >= 0 && sn_ld(&done[ci]) < SN_GW) != 0) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > SN_SPINS) {
        if (lane == 0) atomicOr(bad, BA_BAD_STALL);
        return false;
      }
    }
  }
  const int nrow = 7 * R + 1;
  const bool act = p < nrow, rhs = p == 7 * R;
  const int ib = p / 7, m = p - 7 * (p / 7);
  // 2. A
  double v[SMAX][7];
#pragma unroll
  for (int t = 0; t < SMAX; t++) {
    const double* src = nullptr;
    if (t < s && act) {
      if (rhs) {
        src = a.y + (size_t)rows[t] * 8;
      } else if (ib >= t) {
        const int b = blk[t * R + ib];
        if (b >= 0) src = a.L + (size_t)b * 64 + m * 8;
      }
    }
    ld7(v[t], src);
  }
  // 3. pulls
  const int* pl = T + T[3];
  for (int q = rec[4]; q < rec[5]; q++) {
    const int k = pl[2 * q];
    const int* map = T + pl[2 * q + 1];
    const double* src = nullptr;
    if (act) {
      if (rhs) {
        src = a.y + (size_t)k * 8;
      } else {
        const int b = map[ib];
        if (b >= 0) src = a.L + (size_t)b * 64 + m * 8;
      }
    }
    if (__ballot(src != nullptr) == 0) continue;  // none of this wave's rows lies in struct(k)
    double x[7];
    ld7(x, src);
#pragma unroll
    for (int t = 0; t < SMAX; t++) {
      if (t >= s) break;
      const int bt = map[t];
      if (bt < 0) continue;
      const double* B = a.L + (size_t)bt * 64;
#pragma unroll
      for (int c = 0; c < 7; c++) {
        double acc = x[0] * B[c * 8];
#pragma unroll
        for (int mm = 1; mm < 7; mm++) acc = fma(x[mm], B[c * 8 + mm], acc);
        v[t][c] -= acc;
      }
    }
  }
  // 4. the panel, column by column
  double myinv = 0.0;
  bool fail = false;
#pragma unroll
  for (int t = 0; t < SMAX; t++) {
    if (t >= s) break;
    // the diagonal block's rows (lanes 7t..7t+6 of the first wave) into LDS
    if (act && !rhs && ib == t) {
#pragma unroll
      for (int c = 0; c < 7; c++) sD[m * 8 + c] = v[t][c];
    }
    if (!sn_gbar(bar, phase, lane, bad)) return false;
    // lane-redundant 7x7 Cholesky (right-looking; the same operations as ba.hip's register-row factor)
    double D[7][7], inv[7];
#pragma unroll
    for (int i = 0; i < 7; i++)
#pragma unroll
      for (int c = 0; c <= i; c++) D[i][c] = sD[i * 8 + c];
#pragma unroll
    for (int c = 0; c < 7; c++) {
      double d = D[c][c];
      if (!(d > 0.0)) {  // not positive definite: the step is discarded (dx = 0), as SimplicialLLT's info
        fail = true;
        d = 1.0;
      }
      inv[c] = sn_rsqrt(d);
#pragma unroll
      for (int i = c + 1; i < 7; i++) D[i][c] *= inv[c];
#pragma unroll
      for (int i = c + 1; i < 7; i++)
#pragma unroll
        for (int jj = c + 1; jj <= i; jj++) D[i][jj] = fma(-D[i][c], D[jj][c], D[i][jj]);
    }
    // rows of block t and below (and the rhs): the row-wise right-looking solve with L_tt; a diagonal row m ends as
    // row m of L_tt (its entries past m are zeroed)
    if (act && (rhs || ib >= t)) {
#pragma unroll
      for (int c = 0; c < 7; c++) {
        v[t][c] *= inv[c];
#pragma unroll
        for (int c2 = c + 1; c2 < 7; c2++) v[t][c2] = fma(-v[t][c], D[c2][c], v[t][c2]);
      }
      if (!rhs && ib == t) {
#pragma unroll
        for (int c = 0; c < 7; c++) {
          if (c > m) v[t][c] = 0.0;
          if (c == m) myinv = inv[c];
        }
      }
    }
    // the later diagonal blocks' rows share their column-t entries (L(c_t2, c_t)) through LDS
    if (act && !rhs && ib > t && ib < s) {
#pragma unroll
      for (int c = 0; c < 7; c++) sE[(ib * 8 + m) * 8 + c] = v[t][c];
    }
    if (!sn_gbar(bar, phase, lane, bad)) return false;
#pragma unroll
    for (int t2 = t + 1; t2 < SMAX; t2++) {
      if (t2 >= s) break;
      if (act && (rhs || ib >= t2)) {
#pragma unroll
        for (int c = 0; c < 7; c++) {
          const double* e = sE + (t2 * 8 + c) * 8;
          double acc = v[t][0] * e[0];
#pragma unroll
          for (int mm = 1; mm < 7; mm++) acc = fma(v[t][mm], e[mm], acc);
          v[t2][c] -= acc;
        }
      }
    }
  }
  if (fail && p == 0) atomicOr(bad, BA_BAD_LLT);
  (void)first_wave;
  // 5. stores
  if (act) {
#pragma unroll
    for (int t = 0; t < SMAX; t++) {
      if (t >= s) break;
      double* dst = nullptr;
      if (rhs) {
        dst = a.y + (size_t)rows[t] * 8;
      } else if (ib >= t) {
        const int b = blk[t * R + ib];
        if (b >= 0) dst = a.L + (size_t)b * 64 + m * 8;
      }
      if (dst) {
        reinterpret_cast<double2*>(dst)[0] = make_double2(v[t][0], v[t][1]);
        reinterpret_cast<double2*>(dst)[1] = make_double2(v[t][2], v[t][3]);
        reinterpret_cast<double2*>(dst)[2] = make_double2(v[t][4], v[t][5]);
        reinterpret_cast<double2*>(dst)[3] = make_double2(v[t][6], (!rhs && ib == t) ? myinv : 0.0);
      }
    }
  }
  return true;
}

// one workgroup = NG groups of 4 waves; workgroup wg_base + blockIdx.x walks its lists of the plan
template <int NG, int SMAX>
__global__ void __launch_bounds__(NG * SN_GW * 64) ba_snode_kernel(BaArgs a, int wg_base) {
  if (*a.done) return;
  __shared__ int s_done[SN_MAXN];
  __shared__ int s_bar[NG];
  __shared__ int s_bad;
  __shared__ __attribute__((aligned(16))) double s_D[NG][64];
  __shared__ __attribute__((aligned(16))) double s_E[NG][SMAX * 64];
  constexpr int NT = NG * SN_GW * 64;
  const int* T = a.sn_tab;
  const int nsn = T[0];
  const int wg = wg_base + blockIdx.x;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int g = w / SN_GW, gl = (w % SN_GW) * 64 + lane;
  const int* lp = T + T[4] + wg * (NG + 1);
  for (int i = threadIdx.x; i < nsn; i += NT) s_done[i] = SN_GW;  // other workgroups' supernodes: done before
  if (threadIdx.x < NG) s_bar[threadIdx.x] = 0;
  if (threadIdx.x == 0) s_bad = 0;
  __syncthreads();
  for (int i = lp[0] + (int)threadIdx.x; i < lp[NG]; i += NT) s_done[T[i]] = 0;
  __syncthreads();
  int phase = 0;
  for (int it = lp[g]; it < lp[g + 1]; it++) {
    const int S = T[it];
    const bool ok = sn_supernode<SMAX>(a, T, S, gl, lane, (w % SN_GW) == 0, s_done, &s_bar[g], phase, s_D[g], s_E[g],
                                       &s_bad);
    if (lane == 0) sn_add(&s_done[S], 1);  // release: this wave's stores first
    if (!ok) break;
  }
  __syncthreads();
  if (threadIdx.x == 0 && s_bad) atomicOr(a.bad, s_bad);
}

}  // namespace m3s

// the supernodal factorisation: the multi-workgroup launch of the subtrees below the cut (nwg workgroups), then the
// one-workgroup launch of the rest; the back substitution and retraction follow (ba_sparse_factor_kernel, no factor
// tasks in its schedule)
extern "C" hipError_t m3s_launch_ba_snode(const BaArgs* a, int nwg, hipStream_t s) {
  if (nwg > 0)
    hipLaunchKernelGGL((m3s::ba_snode_kernel<M3S_BA_SN_GROUPS, M3S_BA_SN_SMAX>), dim3(nwg),
                       dim3(M3S_BA_SN_GROUPS * m3s::SN_GW * 64), 0, s, *a, 0);
  hipLaunchKernelGGL((m3s::ba_snode_kernel<M3S_BA_SN_GROUPS, M3S_BA_SN_SMAX>), dim3(1),
                     dim3(M3S_BA_SN_GROUPS * m3s::SN_GW * 64), 0, s, *a, nwg);
  return hipGetLastError();
}
