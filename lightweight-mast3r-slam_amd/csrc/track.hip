// Per-frame tracking Gauss-Newton (Sim(3), pointmap residuals) for MI355X (gfx950).
//
// Reference semantics:
//   FrameTracker.track pre-GN setup    /root/reference/mast3r_slam/tracker.py:35-70, 129-154
//   FrameTracker.solve                 tracker.py:156-171 (+ nonlinear_optimizer.huber :28-33)
//   opt_pose_ray_dist_sim3             tracker.py:173-214 (geometry.act_Sim3 :45-52, point_to_ray_dist :17-34)
//   opt_pose_calib_sim3                tracker.py:216-266 (geometry.project_calib :63-104,
//                                      constrain_points_to_ray / backproject :37-42, 107-115)
//   check_convergence                  nonlinear_optimizer.py:5-25
//   keyframe fusion + selection stats  tracker.py:95-114, frame.py:41-77 (weighted_pointmap)
//
// Device pipeline per frame, no host synchronisation inside:
//   track_init   : zero the state and the unique(idx[valid]) byte map, T_CkCf = T_WCk^-1 T_WCf
//   track_setup  : gather Xf[idx], Qk = sqrt(Qff[idx] Qkf), validity masks, a 32-byte per-point GN
//                  record, counts (valid_opt, valid_kf) and the byte map
//   gn_loop      : ONE persistent launch runs every GN iteration: per iteration every block
//                  accumulates the 28 (H upper) + 7 (g) + 1 (cost) sums in fp64, publishes them
//                  write-through (sc1) and takes an arrival ticket; the last-arriving block reduces all
//                  partials, solves the 7x7 system, retracts T <- Exp(tau) T, applies the convergence
//                  test, broadcasts the new T (GnBcast) and, once done, writes T_WCf = T_WCk T_CkCf
//                  (also to the caller's T_out); the other blocks poll the broadcast and go on.
//   fuse         : keyframe X <- (C X + C' T_CkCf Xkf) / (C + C'), C += C'
#include "m3s_common.hpp"
#include "m3s_track.h"

namespace m3s {

#define GN_NSUM 36
#define GN_PSTRIDE 40
#define GN_SLOTS 64  // partial-sum slots of the persistent GN launch: one per iteration

// lietorch group product with the product quaternion re-normalised (RxSO3 ctor), float.
__device__ __forceinline__ void sim3_mul_norm(const float* A, const float* B, float* C) {
  float q[4];
  quat_comp(&A[3], &B[3], q);
  const float ni = __builtin_amdgcn_rsqf(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  float t[3];
  actSO3(&A[3], &B[0], t);
  C[0] = A[0] + A[7] * t[0];
  C[1] = A[1] + A[7] * t[1];
  C[2] = A[2] + A[7] * t[2];
  C[3] = q[0] * ni;
  C[4] = q[1] * ni;
  C[5] = q[2] * ni;
  C[6] = q[3] * ni;
  C[7] = A[7] * B[7];
}

__device__ __forceinline__ void sim3_inv(const float* A, float* C) {
  const float qi[4] = {-A[3], -A[4], -A[5], A[6]};
  const float si = 1.0f / A[7];
  float t[3];
  actSO3(qi, &A[0], t);
  C[0] = -si * t[0];
  C[1] = -si * t[1];
  C[2] = -si * t[2];
  C[3] = qi[0];
  C[4] = qi[1];
  C[5] = qi[2];
  C[6] = qi[3];
  C[7] = si;
}

// the grid zeroes the unique-idx byte map, the setup counters and the GN tickets / broadcast record (the state
// itself is initialised by track_setup's first thread: nothing reads it before the GN launch)
__global__ void __launch_bounds__(256) track_init_kernel(uint4* flags, int n16, unsigned long long* cnt, unsigned* tick) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n16) flags[i] = make_uint4(0u, 0u, 0u, 0u);
  if (i < M3S_TRACK_SHARDS * 16) cnt[i] = 0ull;
  for (int j = i; j < M3S_TRACK_TICK_WORDS; j += gridDim.x * blockDim.x) tick[j] = 0u;  // tickets + granules
}

// state <- {0, T = T_WCk^-1 * T_WCf (tracker.py:180/225), T_WCk, old_cost = inf}
__device__ void track_state_init(TrackState* st, const float* T_WCf, const float* T_WCk) {
  *st = TrackState{};
  float Ti[8], Tf[8], Tk[8];
  for (int c = 0; c < 8; c++) {
    Tf[c] = T_WCf[c];
    Tk[c] = T_WCk[c];
    st->T_WCk[c] = Tk[c];
  }
  sim3_inv(Tk, Ti);
  sim3_mul_norm(Ti, Tf, st->T);
  st->old_cost = __builtin_inf();
}

// ------------------------------------------------------------------------------------------
// the 32-byte GN record of point n < N (r0, r1), its validity for the solve (v_opt) and for the keyframe stats
// (v_kf), and the unique-match byte map entry
__device__ __forceinline__ void setup_point(const TrackArgs& a, const TrackParams& p, int n, float4& r0, float4& r1,
                                            int& v_opt, int& v_kf) {
  if (p.direct) {  // opt_pose_* surface: Qff = Qk, valid_match = valid, Xf pre-gathered
    const float qk = a.Qff[n];
    const bool valid_opt = a.valid_match[n] != 0;
    v_opt = valid_opt;
    v_kf = valid_opt;
    const float sq = valid_opt ? sqrtf(qk) : 0.0f;
    const float* Xf = a.Xf + (size_t)n * 3;
    if (p.mode == 0) {
      const float* Xk = a.Xk + (size_t)n * 3;
      const float d = sqrtf(Xk[0] * Xk[0] + Xk[1] * Xk[1] + Xk[2] * Xk[2]);
      const float di = 1.0f / d;
      r0 = make_float4(Xf[0], Xf[1], Xf[2], di * Xk[0]);
      r1 = make_float4(di * Xk[1], di * Xk[2], d, sq);
    } else {
      const float* m = a.meas_k + (size_t)n * 3;
      r0 = make_float4(Xf[0], Xf[1], Xf[2], m[0]);
      r1 = make_float4(m[1], m[2], a.valid_meas[n] ? 1.0f : 0.0f, sq);
    }
  } else {
    const int64_t i = a.idx[n];
    const float qk = sqrtf(a.Qff[i] * a.Qkf[n]);
    const float cf = a.Cf[i] / p.Nf;  // frame.get_average_conf(): C / N
    const float ck = a.Ck[n] / p.Nk;
    const bool vm = a.valid_match[n] != 0;
    const bool valid_opt = vm && (cf > p.C_conf) && (ck > p.C_conf) && (qk > p.Q_conf);
    v_opt = valid_opt;
    v_kf = vm && (qk > p.Q_conf);
    if (vm) a.flags[i] = 1;  // benign same-value races; popcounted by the fuse launch
    const float sq = valid_opt ? sqrtf(qk) : 0.0f;
    const float* Xf = a.Xf + i * 3;
    const float* Xk = a.Xk + (size_t)n * 3;
    if (p.mode == 0) {  // rays: [Xf[idx], rd_k = (Xk/|Xk|, |Xk|), sqrtQ*valid]
      const float d = sqrtf(Xk[0] * Xk[0] + Xk[1] * Xk[1] + Xk[2] * Xk[2]);
      const float di = 1.0f / d;
      r0 = make_float4(Xf[0], Xf[1], Xf[2], di * Xk[0]);
      r1 = make_float4(di * Xk[1], di * Xk[2], d, sq);
    } else {  // calib: constrain_points_to_ray at pixel idx, meas_k = [u_n, v_n, log z_k]
      const int i32 = (int)i, vi = i32 / p.W;  // 32-bit: i < H*W
      const float uf = (float)(i32 - vi * p.W), vf = (float)vi;
      const float zf = Xf[2];
      const float xc = zf * ((uf - p.cx) / p.fx);
      const float yc = zf * ((vf - p.cy) / p.fy);
      const float zk = Xk[2];
      const bool vmeas = zk > p.depth_eps;
      const int vnn = n / p.W;
      const float un = (float)(n - vnn * p.W), vn = (float)vnn;
      r0 = make_float4(xc, yc, zf, vmeas ? un : 0.0f);
      r1 = make_float4(vmeas ? vn : 0.0f, vmeas ? logf(zk) : 0.0f, vmeas ? 1.0f : 0.0f, sq);
    }
  }
}

// setup_point (non-direct path) for K points of one thread at once, for the folded GN prologue: every point's own
// loads first (idx, Qkf, Ck, the match flag, Xk), then every gather at idx (Qff, Cf, Xf), then the math, then the
// byte-map stores, with no branch between the points: one point after another, each point's two dependent round
// trips and the branches around them stacked up in front of the first iteration. A point at n >= N computes point
// N - 1 again and counts, stores and marks nothing (its records are zero, as before). Same formulas as setup_point,
// so the records and counts are the same bit for bit.
template <int K>
__device__ __forceinline__ void setup_points(const TrackArgs& a, const TrackParams& p, const int (&nn)[K],
                                             float4 (&r0)[K], float4 (&r1)[K], int& v_opt, int& v_kf) {
  int n[K];
  bool act[K];
  int64_t i[K];
  float qkf[K], ck[K], xk[K][3];
  bool vm[K];
#pragma unroll
  for (int u = 0; u < K; u++) {
    act[u] = nn[u] < p.N;
    n[u] = act[u] ? nn[u] : p.N - 1;
    i[u] = a.idx[n[u]];
    qkf[u] = a.Qkf[n[u]];
    ck[u] = a.Ck[n[u]];
    vm[u] = a.valid_match[n[u]] != 0;
#pragma unroll
    for (int c = 0; c < 3; c++) xk[u][c] = a.Xk[(size_t)n[u] * 3 + c];
  }
  float qff[K], cf[K], xf[K][3];
#pragma unroll
  for (int u = 0; u < K; u++) {
    qff[u] = a.Qff[i[u]];
    cf[u] = a.Cf[i[u]];
#pragma unroll
    for (int c = 0; c < 3; c++) xf[u][c] = a.Xf[i[u] * 3 + c];
  }
#pragma unroll
  for (int u = 0; u < K; u++) {
    const float qk = sqrtf(qff[u] * qkf[u]);
    const float cfa = cf[u] / p.Nf;  // frame.get_average_conf(): C / N
    const float cka = ck[u] / p.Nk;
    const bool valid_opt = vm[u] && (cfa > p.C_conf) && (cka > p.C_conf) && (qk > p.Q_conf);
    v_opt += (act[u] && valid_opt) ? 1 : 0;
    v_kf += (act[u] && vm[u] && (qk > p.Q_conf)) ? 1 : 0;
    const float sq = valid_opt ? sqrtf(qk) : 0.0f;
    float4 q0, q1;
    if (p.mode == 0) {  // rays: [Xf[idx], rd_k = (Xk/|Xk|, |Xk|), sqrtQ*valid]
      const float d = sqrtf(xk[u][0] * xk[u][0] + xk[u][1] * xk[u][1] + xk[u][2] * xk[u][2]);
      const float di = 1.0f / d;
      q0 = make_float4(xf[u][0], xf[u][1], xf[u][2], di * xk[u][0]);
      q1 = make_float4(di * xk[u][1], di * xk[u][2], d, sq);
    } else {  // calib: constrain_points_to_ray at pixel idx, meas_k = [u_n, v_n, log z_k]
      const int i32 = (int)i[u], vi = i32 / p.W;  // 32-bit: i < H*W
      const float uf = (float)(i32 - vi * p.W), vf = (float)vi;
      const float zf = xf[u][2];
      const float xc = zf * ((uf - p.cx) / p.fx);
      const float yc = zf * ((vf - p.cy) / p.fy);
      const float zk = xk[u][2];
      const bool vmeas = zk > p.depth_eps;
      const int vnn = n[u] / p.W;
      const float un = (float)(n[u] - vnn * p.W), vn = (float)vnn;
      q0 = make_float4(xc, yc, zf, vmeas ? un : 0.0f);
      q1 = make_float4(vmeas ? vn : 0.0f, vmeas ? logf(zk) : 0.0f, vmeas ? 1.0f : 0.0f, sq);
    }
    const float4 z = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    r0[u] = act[u] ? q0 : z;
    r1[u] = act[u] ? q1 : z;
  }
#pragma unroll
  for (int u = 0; u < K; u++)
    if (act[u] && vm[u]) a.flags[i[u]] = 1;  // benign same-value races; popcounted by the fuse launch
}

__global__ void __launch_bounds__(256) track_setup_kernel(TrackArgs a, TrackParams p) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n == 0) track_state_init(a.state, a.T_WCf, a.T_WCk);
  int v_opt = 0, v_kf = 0;
  if (n < p.N) {
    float4 r0, r1;
    setup_point(a, p, n, r0, r1, v_opt, v_kf);
    float4* rec = reinterpret_cast<float4*>(a.rec) + 2 * (size_t)n;
    rec[0] = r0;
    rec[1] = r1;
  }
  // block-reduce the two counters into one packed 64-bit add on this block's XCD shard: one counter word
  // for all 1024 blocks serialises the adds (~11 ns each, MI355X_MICROARCH.md "fanin")
  __shared__ unsigned long long s_cnt[4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const unsigned long long bo = __ballot(v_opt), bk = __ballot(v_kf);
  if (lane == 0) s_cnt[wid] = ((unsigned long long)__popcll(bk) << 32) | (unsigned long long)__popcll(bo);
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long v = s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3];
    if (v) atomicAdd(&a.cnt[16 * (blockIdx.x % M3S_TRACK_SHARDS)], v);
  }
}

// the setup counters summed over the shards: low 32 bits n_valid_opt, high 32 bits n_valid_kf
__device__ __forceinline__ unsigned long long track_counts(const unsigned long long* cnt) {
  unsigned long long v = 0;
#pragma unroll
  for (int s = 0; s < M3S_TRACK_SHARDS; s++) v += cnt[16 * s];
  return v;
}

__device__ __forceinline__ bool track_skipped(unsigned n_valid_opt, const TrackParams& p) {
  return (float)n_valid_opt / (float)p.N < p.min_match_frac;  // tracker.py:67-70
}

// accumulate one whitened row (tracker.py:156-166): robust = si*sqrt(huber(si*r)); A = robust*J; b = robust*r.
// MASK: the row's structurally nonzero Jacobian entries (bit c; the calib rows of chain_row have constant
// -0 entries): their products add an exact +-0 to the fp64 sums and are skipped (a non-finite row still
// turns the structurally nonzero entries into NaN, so a failing solve still fails).
template <unsigned MASK = 0x7fu>
__device__ __forceinline__ void acc_row(double* acc, const float J[7], float r, float si, float k) {
  const float wr = si * r;
  const float ra = fabsf(wr);
  const float hub = ra < k ? 1.0f : k / ra;
  const float rob = si * sqrtf(hub);
  float A[7];
#pragma unroll
  for (int c = 0; c < 7; c++) A[c] = rob * J[c];
  const float b = rob * r;
  int l = 0;
#pragma unroll
  for (int c = 0; c < 7; c++) {
#pragma unroll
    for (int d = c; d < 7; d++) {
      if ((MASK >> c) & (MASK >> d) & 1u) acc[l] += (double)A[c] * (double)A[d];
      l++;
    }
  }
#pragma unroll
  for (int c = 0; c < 7; c++)
    if ((MASK >> c) & 1u) acc[28 + c] -= (double)A[c] * (double)b;  // g = -A^T b
  acc[35] += 0.5 * (double)b * (double)b;
}

// J = -(d h / d Y) [I, -[Y]x, Y]; dh is a 3-vector row of the measurement Jacobian
__device__ __forceinline__ void chain_row(const float dh[3], const float Y[3], float J[7]) {
  // S = -skew(Y) = [[0, z, -y], [-z, 0, x], [y, -x, 0]] (geometry.act_Sim3 dpC_dR)
  J[0] = -dh[0];
  J[1] = -dh[1];
  J[2] = -dh[2];
  J[3] = -(dh[1] * -Y[2] + dh[2] * Y[1]);
  J[4] = -(dh[0] * Y[2] + dh[2] * -Y[0]);
  J[5] = -(dh[0] * -Y[1] + dh[1] * Y[0]);
  J[6] = -(dh[0] * Y[0] + dh[1] * Y[1] + dh[2] * Y[2]);
}

// 7x7 Cholesky solve H tau = g in fp32 (torch.linalg.cholesky / cholesky_solve on the float32 H of
// tracker.py:168-169); false when H is not positive definite (torch raises). The normal equations
// themselves are accumulated in fp64; only this tiny serial tail runs in fp32, where div/sqrt are
// short instruction sequences (the fp64 ones dominated the single-lane tail).
__device__ bool chol7(const double Hd[7][7], const double gd[7], double tau[7]) {
  float L[7][7], Li[7];  // Li = 1 / L_jj (hardware rsq of the pivot: no divides on the chain)
  for (int j = 0; j < 7; j++) {
    float d = (float)Hd[j][j];
    for (int k = 0; k < j; k++) d -= L[j][k] * L[j][k];
    if (!(d > 0.0f)) return false;
    const float dinv = __builtin_amdgcn_rsqf(d);
    L[j][j] = d * dinv;
    Li[j] = dinv;
    for (int i = j + 1; i < 7; i++) {
      float s = (float)Hd[i][j];
      for (int k = 0; k < j; k++) s -= L[i][k] * L[j][k];
      L[i][j] = s * dinv;
    }
  }
  float y[7], t[7];
  for (int i = 0; i < 7; i++) {
    float s = (float)gd[i];
    for (int k = 0; k < i; k++) s -= L[i][k] * y[k];
    y[i] = s * Li[i];
  }
  for (int i = 6; i >= 0; i--) {
    float s = y[i];
    for (int k = i + 1; k < 7; k++) s -= L[k][i] * t[k];
    t[i] = s * Li[i];
  }
  for (int i = 0; i < 7; i++) tau[i] = t[i];
  return true;
}

// one thread: H, g, cost -> tau -> T update + convergence (tracker.py:156-171, 186-209). Pure: the solving
// block broadcasts the result (GnBcast) and block 0 writes the final state after the loop, so no state
// byte is written from several XCDs.
template <typename V>
__device__ __forceinline__ void wt(V* p, V v) {  // write-through (sc1) store
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

struct GnStep {
  float T[8];
  double cost;
  int iter, done, status;
};

__device__ GnStep gn_step(const TrackParams& p, const double* sum, const float* T, int iter, double old) {
  GnStep r;
  for (int c = 0; c < 8; c++) r.T[c] = T[c];
  double H[7][7], g[7], tau[7];
  int l = 0;
  for (int c = 0; c < 7; c++)
    for (int d = c; d < 7; d++) {
      H[c][d] = sum[l];
      H[d][c] = sum[l];
      l++;
    }
  for (int c = 0; c < 7; c++) g[c] = sum[28 + c];
  r.cost = sum[35];
  r.iter = iter;
  r.done = 1;
  r.status = M3S_TRACK_CHOLESKY_FAILED;
  if (!chol7(H, g, tau)) return r;
  float tf[7];
  float tn2 = 0.0f;
  for (int c = 0; c < 7; c++) {
    tf[c] = (float)tau[c];
    tn2 += tf[c] * tf[c];
  }
  float E[8];
  expSim3(tf, E);
  sim3_mul_norm(E, T, r.T);  // T_CkCf.retr(tau) = Exp(tau) * T_CkCf
  r.iter = iter + 1;
  // |(old - cost) / old| < rel_error without the divide; inf - x < inf * r is false on the first step,
  // like the reference's inf/inf = nan
  const bool conv = (fabs(old - r.cost) < (double)p.rel_error * fabs(old)) || (tn2 < p.delta_norm * p.delta_norm);
  r.done = conv || r.iter >= p.max_iters;
  r.status = conv ? M3S_TRACK_OK : (r.done ? M3S_TRACK_MAX_ITERS : M3S_TRACK_RUNNING);
  return r;
}

#ifdef M3S_GN_STAMPS  // (experiment builds only) s_memrealtime stamps of every block: [iteration][block][phase]
#define GN_NSTAMP (8 * 256 * 8)
__device__ unsigned long long g_gn_stamps[GN_NSTAMP];
#define GN_STAMP(k)                                                                                  \
  do {                                                                                               \
    if (threadIdx.x == 0 && iter0 < 8 && blockIdx.x < 256)                                           \
      g_gn_stamps[(iter0 * 256 + blockIdx.x) * 8 + (k)] = __builtin_amdgcn_s_memrealtime();          \
  } while (0)
#else
#define GN_STAMP(k) \
  do {              \
  } while (0)
#endif

typedef __attribute__((address_space(1))) double gdouble;
typedef __attribute__((address_space(1))) int gint;
typedef __attribute__((address_space(1))) unsigned gu32;
typedef __attribute__((address_space(1))) unsigned long long gull;

#ifndef GN_THREADS
#define GN_THREADS 256  // threads of a GN block (one block per CU)
#endif
#define GN_PPT (1024 / GN_THREADS)  // points per thread per round (1024 per block): record loads issued before any math
#ifndef GN_PAIR  // points in float2 pairs, fp32 product sums per thread (gn_pair) instead of fp64 FMAs per product
#define GN_PAIR 1
#endif
#define GN_MAX_BLOCKS 256           // partial rows per iteration slot

// ---- the 36 fp64 sums of a wave, reduce-scattered over its lanes (deterministic, no LDS) ----
// Six half-exchange steps: lanes l and l^32 (v_permlane32_swap: the two halves of a register pair trade places,
// no selects), l and l^16 (v_permlane16_swap), then within each 16-lane row l^8 (DPP row_ror:8), the 8-lane
// mirror pairs (row_half_mirror), l^2 and l^1 (quad_perm). At every step a lane keeps one half of its current
// sums and adds the partner's copy of that half. Afterwards lane gn_lane_of(c) holds the wave's total of sum c
// (the other 28 lanes hold padding zeros). Fixed order: identical in every block and every run.
__device__ __forceinline__ double dpp_f64(double v, int ctrl_sel) {
  int2 x = __builtin_bit_cast(int2, v);
  switch (ctrl_sel) {  // compile-time after unrolling
    case 0: x.x = __builtin_amdgcn_mov_dpp(x.x, 0x128, 0xF, 0xF, false); x.y = __builtin_amdgcn_mov_dpp(x.y, 0x128, 0xF, 0xF, false); break;
    case 1: x.x = __builtin_amdgcn_mov_dpp(x.x, 0x141, 0xF, 0xF, false); x.y = __builtin_amdgcn_mov_dpp(x.y, 0x141, 0xF, 0xF, false); break;
    case 2: x.x = __builtin_amdgcn_mov_dpp(x.x, 0x4E, 0xF, 0xF, false); x.y = __builtin_amdgcn_mov_dpp(x.y, 0x4E, 0xF, 0xF, false); break;
    default: x.x = __builtin_amdgcn_mov_dpp(x.x, 0xB1, 0xF, 0xF, false); x.y = __builtin_amdgcn_mov_dpp(x.y, 0xB1, 0xF, 0xF, false); break;
  }
  return __builtin_bit_cast(double, x);
}

// a and b trade their upper-32 / lower-32 lane halves (W = 32) or, within each 32-lane half, their upper-16 /
// lower-16 quarters (W = 16); returns a' + b': lanes of the lower part hold a + a(partner), the upper part b + b(partner)
template <int W>
__device__ __forceinline__ double swap_add(double a, double b) {
  const int2 xa = __builtin_bit_cast(int2, a), xb = __builtin_bit_cast(int2, b);
  int2 na, nb;
  if constexpr (W == 32) {
    const auto lo = __builtin_amdgcn_permlane32_swap(xa.x, xb.x, false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap(xa.y, xb.y, false, false);
    na = int2{(int)lo[0], (int)hi[0]};
    nb = int2{(int)lo[1], (int)hi[1]};
  } else {
    const auto lo = __builtin_amdgcn_permlane16_swap(xa.x, xb.x, false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap(xa.y, xb.y, false, false);
    na = int2{(int)lo[0], (int)hi[0]};
    nb = int2{(int)lo[1], (int)hi[1]};
  }
  return __builtin_bit_cast(double, na) + __builtin_bit_cast(double, nb);
}

// one DPP step: n live sums -> ceil(n/2); the lanes with `bit` set keep the upper half
template <int N, int SEL>
__device__ __forceinline__ void dpp_step(double* v, bool upper) {
  constexpr int H = (N + 1) / 2;
#pragma unroll
  for (int i = 0; i < H; i++) {
    const double lo = v[i], hi = i + H < N ? v[i + H] : 0.0;
    const double keep = upper ? hi : lo, give = upper ? lo : hi;
    v[i] = keep + dpp_f64(give, SEL);
  }
}

// lane holding sum c after wave_sum36 (c < 36)
__device__ __forceinline__ int gn_lane_of(int c) {
  const int r = c / 9, k = c - 9 * r;  // 16-lane row r, position k of {0,1,2,4,5,8,9,10,12}
  const int pos = (k < 3) ? k : (k < 5) ? k + 1 : (k < 8) ? k + 3 : 12;
  return 16 * r + pos;
}

__device__ __forceinline__ double wave_sum36(double (&v)[GN_NSUM], int lane) {
#pragma unroll
  for (int i = 0; i < 18; i++) v[i] = swap_add<32>(v[i], v[i + 18]);
#pragma unroll
  for (int i = 0; i < 9; i++) v[i] = swap_add<16>(v[i], v[i + 9]);
  dpp_step<9, 0>(v, lane & 8);
  dpp_step<5, 1>(v, lane & 4);
  dpp_step<3, 2>(v, lane & 2);
  dpp_step<2, 3>(v, lane & 1);
  return v[0];
}

__device__ __forceinline__ void gn_point(const TrackParams& p, const float* T, float4 r0, float4 r1, double* acc) {
  const float X[3] = {r0.x, r0.y, r0.z};
  float Y[3];
  actSim3(T, X, Y);
  const float sq = r1.w;
  if (p.mode == 0) {
    const float d = sqrtf(Y[0] * Y[0] + Y[1] * Y[1] + Y[2] * Y[2]);
    const float di = 1.0f / d;
    const float di2 = di * di;
    const float rr[3] = {di * Y[0], di * Y[1], di * Y[2]};
    const float res[4] = {r0.w - rr[0], r1.x - rr[1], r1.y - rr[2], r1.z - d};
    const float si_r = p.c_a * sq, si_d = p.c_b * sq;
#pragma unroll
    for (int k = 0; k < 3; k++) {
      float dh[3];
#pragma unroll
      for (int m = 0; m < 3; m++) dh[m] = di * ((k == m ? 1.0f : 0.0f) - di2 * (Y[k] * Y[m]));
      float J[7];
      chain_row(dh, Y, J);
      acc_row(acc, J, res[k], si_r, p.huber_k);
    }
    float J[7];
    chain_row(rr, Y, J);
    acc_row(acc, J, res[3], si_d, p.huber_k);
  } else {
    const float x = Y[0], y = Y[1], z = Y[2];
    const float pu = p.K[0] * x + p.K[1] * y + p.K[2] * z;
    const float pv = p.K[3] * x + p.K[4] * y + p.K[5] * z;
    const float pw = p.K[6] * x + p.K[7] * y + p.K[8] * z;
    const float u = pu / pw, v = pv / pw;
    const bool valid_z = z > p.depth_eps;
    const float logz = valid_z ? logf(z) : 0.0f;
    const bool valid = (u > p.pixel_border) && (u < (float)(p.W - 1) - p.pixel_border) &&
                       (v > p.pixel_border) && (v < (float)(p.H - 1) - p.pixel_border) && valid_z &&
                       (r1.z != 0.0f);
    const float vf = valid ? 1.0f : 0.0f;
    const float si_p = vf * (p.c_a * sq), si_z = vf * (p.c_b * sq);
    const float zi = 1.0f / z;
    const float res[3] = {r0.w - u, r1.x - v, r1.y - logz};
    float dh[3], J[7];
    dh[0] = p.K[0] * zi;
    dh[1] = 0.0f;
    dh[2] = (-p.K[0] * x * zi) * zi;
    chain_row(dh, Y, J);
    acc_row<0b1111101u>(acc, J, res[0], si_p, p.huber_k);  // J[1] = -dh[1] = -0
    dh[0] = 0.0f;
    dh[1] = p.K[4] * zi;
    dh[2] = (-p.K[4] * y * zi) * zi;
    chain_row(dh, Y, J);
    acc_row<0b1111110u>(acc, J, res[1], si_p, p.huber_k);  // J[0] = -0
    dh[0] = 0.0f;
    dh[1] = 0.0f;
    dh[2] = zi;
    chain_row(dh, Y, J);
    acc_row<0b1011100u>(acc, J, res[2], si_z, p.huber_k);  // J[0], J[1], J[5] = -0
  }
}

// All GN iterations in ONE launch (nparts <= 256 blocks, sized by the occupancy query so every block is
// resident). Per iteration:
//   1. every block accumulates its points' 36 fp64 sums, reduce-scatters them in each wave (wave_sum36) and
//      adds the 4 waves' totals in LDS (fixed order), publishes the block partial with write-through (sc1)
//      stores into the iteration's slot and takes a ticket on its XCD shard (blocks b and b + 8 share one);
//   2. the shard's last arriver loads its shard's partials with sc1 loads (no acquire fence: every partial byte
//      was stored sc1 and drained before its ticket, MI355X_MICROARCH.md "Valid forms" row 1), sums them in
//      block order and publishes the shard sum as 72 tagged 8-byte granules {32-bit half, iteration};
//   3. every block polls the 8 shard sums (one wave, sc1 loads), adds them in shard order and solves the 7x7
//      system, retracts and tests convergence itself: the same instructions on the same bytes, so every block
//      holds the same T bit for bit, and no broadcast hop or serial last-block tail sits on the chain.
// Spins are bounded: a stalled hand-off ends the frame with status STALLED (the host raises), never a hang.
// ---- two points per lane (float2 lanes), GN_PAIR builds: every per-point operation of gn_point, elementwise on
// the pair (so each point's rounding is gn_point's), with the row products accumulated in fp32 (packed FMAs, one
// rounding per product-sum) over the thread's points and added to the fp64 sums once per iteration (gn_flush):
// half the instructions of the fp64 product-sums at the GN launch's one wave per SIMD ----
typedef float gf2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ gf2 g2sqrt(gf2 x) { return gf2{sqrtf(x.x), sqrtf(x.y)}; }
__device__ __forceinline__ gf2 g2fma(gf2 a, gf2 b, gf2 c) { return __builtin_elementwise_fma(a, b, c); }

template <unsigned MASK = 0x7fu>
__device__ __forceinline__ void acc_row2(gf2* acc, const gf2 J[7], gf2 r, gf2 si, float k) {
  const gf2 wr = si * r;
  const gf2 ra = {fabsf(wr.x), fabsf(wr.y)};
  const gf2 hub = {ra.x < k ? 1.0f : k / ra.x, ra.y < k ? 1.0f : k / ra.y};
  const gf2 rob = si * g2sqrt(hub);
  gf2 A[7];
#pragma unroll
  for (int c = 0; c < 7; c++) A[c] = rob * J[c];
  const gf2 b = rob * r;
  int l = 0;
#pragma unroll
  for (int c = 0; c < 7; c++) {
#pragma unroll
    for (int d = c; d < 7; d++) {
      if ((MASK >> c) & (MASK >> d) & 1u) acc[l] = g2fma(A[c], A[d], acc[l]);
      l++;
    }
  }
#pragma unroll
  for (int c = 0; c < 7; c++)
    if ((MASK >> c) & 1u) acc[28 + c] = g2fma(-A[c], b, acc[28 + c]);  // g = -A^T b
  acc[35] = g2fma(0.5f * b, b, acc[35]);
}

__device__ __forceinline__ void chain_row2(const gf2 dh[3], const gf2 Y[3], gf2 J[7]) {
  J[0] = -dh[0];
  J[1] = -dh[1];
  J[2] = -dh[2];
  J[3] = -(dh[1] * -Y[2] + dh[2] * Y[1]);
  J[4] = -(dh[0] * Y[2] + dh[2] * -Y[0]);
  J[5] = -(dh[0] * -Y[1] + dh[1] * Y[0]);
  J[6] = -(dh[0] * Y[0] + dh[1] * Y[1] + dh[2] * Y[2]);
}

__device__ __forceinline__ void actSim3_2(const float* T, const gf2 X[3], gf2 Y[3]) {
  const float* q = &T[3];
  const gf2 uv0 = 2.0f * (q[1] * X[2] - q[2] * X[1]);
  const gf2 uv1 = 2.0f * (q[2] * X[0] - q[0] * X[2]);
  const gf2 uv2 = 2.0f * (q[0] * X[1] - q[1] * X[0]);
  const gf2 y0 = X[0] + q[3] * uv0 + (q[1] * uv2 - q[2] * uv1);
  const gf2 y1 = X[1] + q[3] * uv1 + (q[2] * uv0 - q[0] * uv2);
  const gf2 y2 = X[2] + q[3] * uv2 + (q[0] * uv1 - q[1] * uv0);
  Y[0] = y0 * T[7] + T[0];
  Y[1] = y1 * T[7] + T[1];
  Y[2] = y2 * T[7] + T[2];
}

// points a and b (b = a with weight 0 when the thread has no second point: exact zeros unless a's own row is
// non-finite, which poisons the sums anyway)
__device__ __forceinline__ void gn_pair(const TrackParams& p, const float* T, float4 a0, float4 a1, float4 b0,
                                        float4 b1, gf2* acc) {
  const gf2 X[3] = {gf2{a0.x, b0.x}, gf2{a0.y, b0.y}, gf2{a0.z, b0.z}};
  gf2 Y[3];
  actSim3_2(T, X, Y);
  const gf2 sq = {a1.w, b1.w};
  if (p.mode == 0) {
    const gf2 d = g2sqrt(Y[0] * Y[0] + Y[1] * Y[1] + Y[2] * Y[2]);
    const gf2 di = 1.0f / d;
    const gf2 di2 = di * di;
    const gf2 rr[3] = {di * Y[0], di * Y[1], di * Y[2]};
    const gf2 res[4] = {gf2{a0.w, b0.w} - rr[0], gf2{a1.x, b1.x} - rr[1], gf2{a1.y, b1.y} - rr[2],
                        gf2{a1.z, b1.z} - d};
    const gf2 si_r = p.c_a * sq, si_d = p.c_b * sq;
#pragma unroll
    for (int k = 0; k < 3; k++) {
      gf2 dh[3];
#pragma unroll
      for (int m = 0; m < 3; m++) dh[m] = di * ((k == m ? 1.0f : 0.0f) - di2 * (Y[k] * Y[m]));
      gf2 J[7];
      chain_row2(dh, Y, J);
      acc_row2(acc, J, res[k], si_r, p.huber_k);
    }
    gf2 J[7];
    chain_row2(rr, Y, J);
    acc_row2(acc, J, res[3], si_d, p.huber_k);
  } else {
    const gf2 x = Y[0], y = Y[1], z = Y[2];
    const gf2 pu = p.K[0] * x + p.K[1] * y + p.K[2] * z;
    const gf2 pv = p.K[3] * x + p.K[4] * y + p.K[5] * z;
    const gf2 pw = p.K[6] * x + p.K[7] * y + p.K[8] * z;
    const gf2 u = pu / pw, v = pv / pw;
    const bool vz0 = z.x > p.depth_eps, vz1 = z.y > p.depth_eps;
    const gf2 logz = {vz0 ? logf(z.x) : 0.0f, vz1 ? logf(z.y) : 0.0f};
    const float ub = p.pixel_border, uh = (float)(p.W - 1) - p.pixel_border, vh = (float)(p.H - 1) - p.pixel_border;
    const bool ok0 = (u.x > ub) && (u.x < uh) && (v.x > ub) && (v.x < vh) && vz0 && (a1.z != 0.0f);
    const bool ok1 = (u.y > ub) && (u.y < uh) && (v.y > ub) && (v.y < vh) && vz1 && (b1.z != 0.0f);
    const gf2 vf = {ok0 ? 1.0f : 0.0f, ok1 ? 1.0f : 0.0f};
    const gf2 si_p = vf * (p.c_a * sq), si_z = vf * (p.c_b * sq);
    const gf2 zi = 1.0f / z;
    const gf2 res[3] = {gf2{a0.w, b0.w} - u, gf2{a1.x, b1.x} - v, gf2{a1.y, b1.y} - logz};
    const gf2 z2 = {0.0f, 0.0f};
    gf2 dh[3], J[7];
    dh[0] = p.K[0] * zi;
    dh[1] = z2;
    dh[2] = (-p.K[0] * x * zi) * zi;
    chain_row2(dh, Y, J);
    acc_row2<0b1111101u>(acc, J, res[0], si_p, p.huber_k);
    dh[0] = z2;
    dh[1] = p.K[4] * zi;
    dh[2] = (-p.K[4] * y * zi) * zi;
    chain_row2(dh, Y, J);
    acc_row2<0b1111110u>(acc, J, res[1], si_p, p.huber_k);
    dh[0] = z2;
    dh[1] = z2;
    dh[2] = zi;
    chain_row2(dh, Y, J);
    acc_row2<0b1011100u>(acc, J, res[2], si_z, p.huber_k);
  }
}

// the thread's fp32 pair sums into its fp64 sums
__device__ __forceinline__ void gn_flush(double* acc, const gf2* a2) {
#pragma unroll
  for (int c = 0; c < GN_NSUM; c++) acc[c] += (double)a2[c].x + (double)a2[c].y;
}

//
// SETUP (folded setup, M3S_TRACK_FOLD_SETUP=1): no track_setup launch. Every block derives the initial T_CkCf
// itself (track_state_init's arithmetic), builds its points' records in the first iteration (setup_point: the
// first round into registers, later rounds also into the record buffer for the later iterations), and adds its
// valid counts to the shard counters before its iteration-0 ticket; the skip test (tracker.py:67-70) then reads the
// counters after the iteration-0 hand-off, before the first solve, and block 0 writes the whole final state.
template <bool SETUP>
__global__ void __launch_bounds__(GN_THREADS) gn_loop_kernel(TrackArgs a, TrackParams p) {
  TrackState* st = a.state;
  float T[8];
  double old;  // the convergence test's previous cost (inf before the first solve)
  unsigned long long counts = 0;
  if constexpr (SETUP) {
    float Tk[8], Tf[8], Ti[8];
#pragma unroll
    for (int c = 0; c < 8; c++) {
      Tk[c] = a.T_WCk[c];
      Tf[c] = a.T_WCf[c];
    }
    sim3_inv(Tk, Ti);
    sim3_mul_norm(Ti, Tf, T);
    old = __builtin_inf();
  } else {
    if (st->done) return;
    counts = track_counts(a.cnt);
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // for the host readback
      st->n_valid_opt = (int)(unsigned)counts;
      st->n_valid_kf = (int)(unsigned)(counts >> 32);
    }
    if (track_skipped((unsigned)counts, p)) {
      if (blockIdx.x == 0 && threadIdx.x == 0) {
        st->status = M3S_TRACK_SKIPPED;
        st->done = 1;
      }
      return;
    }
#pragma unroll
    for (int c = 0; c < 8; c++) T[c] = st->T[c];
    old = st->old_cost;
  }
  __shared__ double s_w[GN_THREADS / 64][64];  // per-wave totals (wave_sum36 lanes)
  __shared__ double s_sum[GN_NSUM];
  __shared__ double s_grp[7][GN_NSUM];
  __shared__ double s_shard[M3S_TRACK_SHARDS][GN_NSUM];
  __shared__ int s_last, s_stop, s_fin;
  __shared__ float s_T[8];
  __shared__ unsigned long long s_cnt[GN_THREADS / 64];  // SETUP: per-wave valid counts
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const unsigned nblk = gridDim.x;
  const int shard = blockIdx.x % M3S_TRACK_SHARDS;
  const int nsh = (int)min(nblk, (unsigned)M3S_TRACK_SHARDS);
  const unsigned per = (nblk - shard + M3S_TRACK_SHARDS - 1) / M3S_TRACK_SHARDS;  // blocks in this shard
  const float T0[8] = {T[0], T[1], T[2], T[3], T[4], T[5], T[6], T[7]};  // SETUP: a skipped frame keeps it
  int iters_done = 0, status = M3S_TRACK_RUNNING;
  double cost = 0.0;
  const float4* rec = reinterpret_cast<const float4*>(a.rec);
  const int stride = nblk * GN_THREADS;
  // the first round's records (every point at 512x512: 4 per thread) stay in registers for all iterations;
  // only the poses change between iterations
  const int n00 = blockIdx.x * GN_THREADS + threadIdx.x;
  float4 c0[GN_PPT], c1[GN_PPT];
  int v_opt = 0, v_kf = 0;  // SETUP: this thread's valid counts (iteration 0)
  if (SETUP && !p.direct) {  // the first round's records built in one batch (setup_points)
    int nn[GN_PPT];
#pragma unroll
    for (int u = 0; u < GN_PPT; u++) nn[u] = n00 + u * stride;
    setup_points<GN_PPT>(a, p, nn, c0, c1, v_opt, v_kf);
  } else {
#pragma unroll
    for (int u = 0; u < GN_PPT; u++) {
      if constexpr (SETUP) {
        const int n = n00 + u * stride;
        c0[u] = c1[u] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        if (n < p.N) {
          int vo = 0, vk = 0;
          setup_point(a, p, n, c0[u], c1[u], vo, vk);
          v_opt += vo;
          v_kf += vk;
        }
      } else {
        const int n = min(n00 + u * stride, p.N - 1);
        c0[u] = rec[2 * (size_t)n];
        c1[u] = rec[2 * (size_t)n + 1];
      }
    }
  }
  gu32* gran = (gu32*)(a.tick + M3S_TRACK_GRANULES);  // [2 parities][8 shards][72] x {half, tag}
  for (int it = 0; it < p.max_iters; it++) {
#ifdef M3S_GN_STAMPS
    const int iter0 = it;
#endif
    GN_STAMP(0);
    double acc[GN_NSUM];
#pragma unroll
    for (int c = 0; c < GN_NSUM; c++) acc[c] = 0.0;
#if GN_PAIR
    gf2 a2[GN_NSUM];
#pragma unroll
    for (int c = 0; c < GN_NSUM; c++) a2[c] = gf2{0.0f, 0.0f};
    auto pair = [&](int na, const float4& xa0, const float4& xa1, const float4& xb0, const float4& xb1) {
      if (na >= p.N) return;
      if (na + stride < p.N) {
        gn_pair(p, T, xa0, xa1, xb0, xb1, a2);
      } else {  // no second point: the first again with weight 0
        float4 z1 = xa1;
        z1.w = 0.0f;
        gn_pair(p, T, xa0, xa1, xa0, z1, a2);
      }
    };
#pragma unroll
    for (int u = 0; u < GN_PPT; u += 2) pair(n00 + u * stride, c0[u], c1[u], c0[u + 1], c1[u + 1]);
#else
#pragma unroll
    for (int u = 0; u < GN_PPT; u++)
      if (n00 + u * stride < p.N) gn_point(p, T, c0[u], c1[u], acc);
#endif
    for (int n0 = n00 + GN_PPT * stride; n0 < p.N; n0 += GN_PPT * stride) {
      float4 r0[GN_PPT], r1[GN_PPT];
#pragma unroll
      for (int u = 0; u < GN_PPT; u++) {
        const int n = min(n0 + u * stride, p.N - 1);
        if (SETUP && it == 0) {  // built here, stored for the later iterations (read back by this same thread)
          r0[u] = r1[u] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
          if (n0 + u * stride < p.N) {
            int vo = 0, vk = 0;
            setup_point(a, p, n, r0[u], r1[u], vo, vk);
            v_opt += vo;
            v_kf += vk;
            float4* w = reinterpret_cast<float4*>(a.rec) + 2 * (size_t)n;
            w[0] = r0[u];
            w[1] = r1[u];
          }
        } else {
          r0[u] = rec[2 * (size_t)n];
          r1[u] = rec[2 * (size_t)n + 1];
        }
      }
#if GN_PAIR
#pragma unroll
      for (int u = 0; u < GN_PPT; u += 2) pair(n0 + u * stride, r0[u], r1[u], r0[u + 1], r1[u + 1]);
#else
#pragma unroll
      for (int u = 0; u < GN_PPT; u++)
        if (n0 + u * stride < p.N) gn_point(p, T, r0[u], r1[u], acc);
#endif
    }
#if GN_PAIR
    gn_flush(acc, a2);
#endif
    GN_STAMP(1);
    s_w[wid][lane] = wave_sum36(acc, lane);
    if (SETUP && it == 0) {  // the wave's valid counts, packed (n_valid_kf << 32) | n_valid_opt like track_setup's
      unsigned long long c = ((unsigned long long)(unsigned)v_kf << 32) | (unsigned)v_opt;
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off, 64);
      if (lane == 0) s_cnt[wid] = c;
    }
    __syncthreads();
    if (SETUP && it == 0 && threadIdx.x == 0) {  // before this block's ticket (the vmcnt(0) below drains it)
      unsigned long long c = 0;
#pragma unroll
      for (int w = 0; w < GN_THREADS / 64; w++) c += s_cnt[w];
      if (c) __hip_atomic_fetch_add(&a.cnt[16 * shard], c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // the block partial: 36 threads add the 4 waves' totals, store it write-through into this iteration's slot
    const int slot = it % GN_SLOTS;
    gdouble* part = (gdouble*)(a.partials + (size_t)slot * GN_MAX_BLOCKS * GN_PSTRIDE);
    if (threadIdx.x < GN_NSUM) {
      const int l = gn_lane_of(threadIdx.x);
      double v = s_w[0][l];
#pragma unroll
      for (int w = 1; w < GN_THREADS / 64; w++) v += s_w[w][l];
      __hip_atomic_store(&part[(size_t)blockIdx.x * GN_PSTRIDE + threadIdx.x], v, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    GN_STAMP(2);
    if (threadIdx.x == 0) {  // the shard ticket (monotonic within the frame: it + 1 rounds of `per` arrivals)
      const unsigned t = __hip_atomic_fetch_add((gu32*)&a.tick[32 * shard], 1u, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
      s_last = t == (unsigned)(it + 1) * per - 1;
      s_stop = 0;
    }
    __syncthreads();
    const int par = it & 1;
    if (s_last) {
      GN_STAMP(3);
      // the shard's partial rows (blocks shard, shard + 8, ...), thread (c, g) walks column c over rows g, g + 7,
      // ... with sc1 loads, then the 7 group sums in order
      if (threadIdx.x < 7 * GN_NSUM) {  // <= 32 rows per shard: at most 5 per thread, all loads in flight at once
        const int c = threadIdx.x % GN_NSUM, g = threadIdx.x / GN_NSUM;
        double v[5];
#pragma unroll
        for (int k = 0; k < 5; k++) {
          const unsigned r = g + 7 * k;
          v[k] = r < per ? __hip_atomic_load(&part[(size_t)(shard + 8 * r) * GN_PSTRIDE + c], __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT)
                         : 0.0;
        }
        s_grp[g][c] = (((v[0] + v[1]) + v[2]) + v[3]) + v[4];
      }
      __syncthreads();
      if (threadIdx.x < 2 * GN_NSUM) {  // 72 granules: the lower / upper 32 bits of each shard sum, tagged it + 1
        const int c = threadIdx.x >> 1;
        const double v = (((((s_grp[0][c] + s_grp[1][c]) + s_grp[2][c]) + s_grp[3][c]) + s_grp[4][c]) + s_grp[5][c]) +
                         s_grp[6][c];
        const unsigned long long bits = __builtin_bit_cast(unsigned long long, v);
        const unsigned half = (threadIdx.x & 1) ? (unsigned)(bits >> 32) : (unsigned)bits;
        __hip_atomic_store((gull*)&gran[2 * ((par * M3S_TRACK_SHARDS + shard) * 2 * GN_NSUM + threadIdx.x)],
                           ((unsigned long long)(it + 1) << 32) | half, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      GN_STAMP(4);
    }
    if (threadIdx.x < 64) {
      // wave 0 polls every shard's 72 granules (lane l: granules l, l + 64, ... of the nsh x 72), until every tag
      // is this iteration's
      // (a poll round issues all of a lane's granule loads before it looks at any: one load, its wait and its tag
      // test at a time made each round nine dependent round trips)
      const int ng = nsh * 2 * GN_NSUM;
      constexpr int GPL = (M3S_TRACK_SHARDS * 2 * GN_NSUM + 63) / 64;  // granules per lane, at most
      unsigned spins = 0;
      for (;;) {
        bool ok = true;
        unsigned long long gv[GPL];
#pragma unroll
        for (int k = 0; k < GPL; k++)
          gv[k] = __hip_atomic_load((gull*)&gran[2 * (par * M3S_TRACK_SHARDS * 2 * GN_NSUM + min(lane + 64 * k, ng - 1))],
                                    __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
        for (int k = 0; k < GPL; k++) {
          const int g = lane + 64 * k;
          if (g < ng) {
            if ((unsigned)(gv[k] >> 32) != (unsigned)(it + 1)) {
              ok = false;
            } else {
              unsigned* w = reinterpret_cast<unsigned*>(&s_shard[0][0]);
              w[g] = (unsigned)gv[k];  // lo/hi words in place: granule g = shard g / 72, sum (g % 72) / 2, half g % 2
            }
          }
        }
        if (__all(ok)) break;
        __builtin_amdgcn_s_sleep(1);
        if (++spins > (1u << 22)) {  // a lost hand-off (~0.25 s): stop with status STALLED (the host raises)
          if (lane == 0) s_stop = 1;
          break;
        }
      }
    }
    __syncthreads();
    if (s_stop) {
      if (threadIdx.x == 0) {
        wt(&st->status, M3S_TRACK_STALLED);
        wt(&st->done, 1);
      }
      return;
    }
    GN_STAMP(5);
    if (threadIdx.x < GN_NSUM) {  // the frame's sums: the shard sums in shard order
      const int c = threadIdx.x;
      double v = s_shard[0][c];
      for (int k = 1; k < nsh; k++) v += s_shard[k][c];
      s_sum[c] = v;
    }
    if (SETUP && it == 0) {
      // every block's counts were added before its iteration-0 ticket, and every shard sum seen above follows all
      // of its shard's tickets: the counters are complete (device-scope loads)
      if (threadIdx.x == 0) {
        // the eight loads first, then the sum: written as c += load, the compiler kept each atomic load behind the
        // previous one's wait (eight dependent round trips before the first solve)
        unsigned long long cv[M3S_TRACK_SHARDS], c = 0;
#pragma unroll
        for (int k = 0; k < M3S_TRACK_SHARDS; k++)
          cv[k] = __hip_atomic_load(&a.cnt[16 * k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
        for (int k = 0; k < M3S_TRACK_SHARDS; k++) c += cv[k];
        s_cnt[0] = c;
      }
      __syncthreads();
      counts = s_cnt[0];
      if (track_skipped((unsigned)counts, p)) {
        status = M3S_TRACK_SKIPPED;
        break;
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      const GnStep r = gn_step(p, s_sum, T, it, old);
      for (int c = 0; c < 8; c++) s_T[c] = r.T[c];
      s_fin = r.done;
      old = r.cost;
      cost = r.cost;
      iters_done = r.iter;
      status = r.status;
    }
    __syncthreads();
    GN_STAMP(6);
#pragma unroll
    for (int c = 0; c < 8; c++) T[c] = s_T[c];
    const bool fin = s_fin != 0;
    __syncthreads();  // s_T / s_fin are rewritten in the next iteration
    if (fin) break;
  }
  // the final state, written by ONE block (plain stores of a single writer; the host and the fuse launch read it
  // after this launch); every block holds the same values
  if (SETUP && blockIdx.x == 0 && threadIdx.x == 0) {  // the whole state: track_state_init + the GN launch's writes
    TrackState v{};
#pragma unroll
    for (int c = 0; c < 8; c++) v.T_WCk[c] = a.T_WCk[c];
    v.n_valid_opt = (int)(unsigned)counts;
    v.n_valid_kf = (int)(unsigned)(counts >> 32);
    v.done = 1;
    v.status = status;
    if (status == M3S_TRACK_SKIPPED) {
#pragma unroll
      for (int c = 0; c < 8; c++) v.T[c] = T0[c];
      v.old_cost = __builtin_inf();
    } else {
      v.iter = iters_done;
      v.last_cost = cost;
      v.old_cost = cost;
#pragma unroll
      for (int c = 0; c < 8; c++) v.T[c] = T[c];
      if (status == M3S_TRACK_OK || status == M3S_TRACK_MAX_ITERS) {
        sim3_mul_norm(v.T_WCk, T, v.T_WCf);  // T_WCf = T_WCk * T_CkCf
        if (a.T_out != nullptr)
          for (int c = 0; c < 8; c++) {
            a.T_out[c] = v.T_WCf[c];
            a.T_out[8 + c] = T[c];
          }
      }
    }
    *st = v;
  }
  if (!SETUP && blockIdx.x == 0 && threadIdx.x == 0) {
    st->iter = iters_done;
    st->last_cost = cost;
    st->old_cost = cost;
    st->status = status;
    st->done = 1;
    st->done_chunk = 0;
    for (int c = 0; c < 8; c++) st->T[c] = T[c];
    if (status == M3S_TRACK_OK || status == M3S_TRACK_MAX_ITERS) {
      float Tk[8], Tw[8];
      for (int c = 0; c < 8; c++) Tk[c] = st->T_WCk[c];
      sim3_mul_norm(Tk, T, Tw);  // T_WCf = T_WCk * T_CkCf
      for (int c = 0; c < 8; c++) st->T_WCf[c] = Tw[c];
      if (a.T_out != nullptr)
        for (int c = 0; c < 8; c++) {
          a.T_out[c] = Tw[c];
          a.T_out[8 + c] = T[c];
        }
    }
  }
}

// keyframe.update_pointmap(T_CkCf.act(Xkf), Ckf), weighted_pointmap (frame.py:74-77). Runs only if the
// GN batch `chunk_id` finished with a pose (so it can be enqueued before the host reads the state
// back). Out of place like the reference (new X_canon / C tensors); X_out may alias X_in.
#define FUSE_COUNT_BLOCKS 32

// Thread 0 of each counting block arrives after its own n_unique add (the acq_rel ticket orders it); the
// last of the FUSE_COUNT_BLOCKS blocks to arrive copies the final state (n_unique now
// complete) to the host mirror and releases the call's generation at system scope.
__device__ void publish_state(const TrackState* st, TrackPublish pub) {
  if (__hip_atomic_fetch_add(pub.ticket, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) != FUSE_COUNT_BLOCKS - 1)
    return;
  TrackState v = *st;
  v.n_unique = __hip_atomic_load(&const_cast<TrackState*>(st)->n_unique, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
  pub.mirror->s = v;
  __hip_atomic_store(&pub.mirror->gen, pub.gen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(pub.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // every counting block arrived
}

// The counting blocks also leave the frame's scratch clean for the next frame on this workspace (the host then
// skips track_init): the unique-idx byte map (each entry zeroed by the thread that counted it), the setup
// counters, the GN shard tickets and granules (the publish ticket is re-armed by its last arriver).
__global__ void __launch_bounds__(256) fuse_kernel(const TrackState* __restrict__ st, int chunk_id, FuseArgs f,
                                                   int N, uint8_t* __restrict__ flags, int* __restrict__ n_unique,
                                                   TrackPublish pub, int clean_map, unsigned* __restrict__ tick,
                                                   unsigned long long* __restrict__ cnt_words) {
  const bool solved = st->done && st->done_chunk == chunk_id;
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (blockIdx.x < FUSE_COUNT_BLOCKS) {
    const int tcb = blockIdx.x * 256 + threadIdx.x;  // thread among the counting blocks
    for (int j = tcb; j < M3S_TRACK_TICK_WORDS; j += FUSE_COUNT_BLOCKS * 256)
      if (j < M3S_TRACK_PUBLISH_TICKET || j >= M3S_TRACK_GRANULES) tick[j] = 0u;
    if (tcb < M3S_TRACK_SHARDS * 16) cnt_words[tcb] = 0ull;
    const bool count = solved && n_unique != nullptr;
    if (count || clean_map) {
      // |unique(idx[valid])| (tracker.py:106-108): popcount of the byte map track_setup wrote (0/1 bytes,
      // 16-B padded), here after the solve instead of on the first GN iteration's critical path. A few
      // blocks reduce in LDS and add once each: one device-scope atomic per block, not per wave.
      __shared__ int s_cnt[4];
      uint4* fl = reinterpret_cast<uint4*>(flags);
      const int n16 = (N + 15) / 16;
      int cnt = 0;
      for (int i = tcb; i < n16; i += FUSE_COUNT_BLOCKS * 256) {
        const uint4 v = fl[i];
        cnt += __popc(v.x) + __popc(v.y) + __popc(v.z) + __popc(v.w);
        if (clean_map) fl[i] = make_uint4(0u, 0u, 0u, 0u);
      }
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off, 64);
      if ((threadIdx.x & 63) == 0) s_cnt[threadIdx.x >> 6] = cnt;
      __syncthreads();
      if (threadIdx.x == 0 && count) {
        const int tot = s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3];
        if (tot) atomicAdd(n_unique, tot);
      }
    }
    if (threadIdx.x == 0 && pub.mirror != nullptr) publish_state(st, pub);
  }
  if (!solved) return;
  if (f.X_in == nullptr || !(st->status == M3S_TRACK_OK || st->status == M3S_TRACK_MAX_ITERS)) return;
  if (n >= N) return;
  if (n == 0) {  // the store slot's counters (SharedKeyframes.__setitem__ of the fused record, frame.py:271-289)
    if (f.slot_N != nullptr) *f.slot_N = f.N_new;
    if (f.slot_N_updates != nullptr) *f.slot_N_updates = f.N_updates_new;
    if (f.slot_dirty != nullptr) *f.slot_dirty = 1;
  }
  float T[8];
#pragma unroll
  for (int c = 0; c < 8; c++) T[c] = st->T[c];
  const float X[3] = {f.Xkf[3 * (size_t)n], f.Xkf[3 * (size_t)n + 1], f.Xkf[3 * (size_t)n + 2]};
  float Y[3];
  actSim3(T, X, Y);
  const float c0 = f.C_in[n], c1 = f.Ckf[n];
  const float den = c0 + c1;
  float Xo[3];
#pragma unroll
  for (int k = 0; k < 3; k++) Xo[k] = (c0 * f.X_in[3 * (size_t)n + k] + c1 * Y[k]) / den;
#pragma unroll
  for (int k = 0; k < 3; k++) f.X_out[3 * (size_t)n + k] = Xo[k];
  f.C_out[n] = den;
  if (f.Ck_avg != nullptr) f.Ck_avg[n] = den / f.Nk_new;  // keyframe.get_average_conf()
  if (f.Cf_avg != nullptr) f.Cf_avg[n] = f.Cf[n] / f.Nf;  // frame.get_average_conf()
}

}  // namespace m3s

extern "C" hipError_t m3s_launch_track_init(const TrackArgs* a, const float* T_WCf, const float* T_WCk, int N,
                                            hipStream_t s) {
  const int n16 = (N + 15) / 16;  // the byte map is carved with a 16-B padded length
  (void)T_WCf;
  (void)T_WCk;  // read by track_setup (TrackArgs)
  hipLaunchKernelGGL(m3s::track_init_kernel, dim3((n16 + 255) / 256), dim3(256), 0, s,
                     reinterpret_cast<uint4*>(a->flags), n16, a->cnt, a->tick);
  return hipGetLastError();
}

extern "C" hipError_t m3s_launch_track_setup(const TrackArgs* a, const TrackParams* p, hipStream_t s) {
  hipLaunchKernelGGL(m3s::track_setup_kernel, dim3((p->N + 255) / 256), dim3(256), 0, s, *a, *p);
  return hipGetLastError();
}

// Blocks of gn_loop_kernel that can be resident at once on the current device (occupancy query x CUs,
// cached per device): the persistent launch's grid never exceeds it, so on an otherwise idle GPU every block
// is resident; work of other streams only delays blocks (finite kernels), and the bounded spin catches the rest.
extern "C" int m3s_track_max_parts(void) {
  static int cache[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 1;
  if (dev >= 0 && dev < 64 && cache[dev] > 0) return cache[dev];
  int per_cu = 0, per_cu_fold = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(m3s::gn_loop_kernel<false>),
                                                   GN_THREADS, 0) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu_fold,
                                                   reinterpret_cast<const void*>(m3s::gn_loop_kernel<true>),
                                                   GN_THREADS, 0) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 1;
  per_cu = per_cu_fold < per_cu ? per_cu_fold : per_cu;  // either variant's grid is fully resident
  const int n = per_cu * cus > 1 ? per_cu * cus : 1;
  if (dev >= 0 && dev < 64) cache[dev] = n;
  return n;
}

// one persistent launch runs every GN iteration (iters and chunk_id are kept for the call sites); fold: the setup
// runs inside it (gn_loop_kernel<true>, no track_setup launch before it)
extern "C" hipError_t m3s_launch_track_iters(const TrackArgs* a, const TrackParams* p, int nparts, int iters,
                                             int chunk_id, int fold, hipStream_t s) {
  (void)iters;
  (void)chunk_id;
  if (nparts < 1 || nparts > 256) return hipErrorInvalidValue;  // <= 32 blocks per XCD shard (the shard-last loads)
  if (fold)
    hipLaunchKernelGGL(m3s::gn_loop_kernel<true>, dim3(nparts), dim3(GN_THREADS), 0, s, *a, *p);
  else
    hipLaunchKernelGGL(m3s::gn_loop_kernel<false>, dim3(nparts), dim3(GN_THREADS), 0, s, *a, *p);
  return hipGetLastError();
}

// fusion (f->X_in non-null) and/or the unique-match count (count: the state's n_unique from the byte
// map) for the GN batch chunk_id that finished
extern "C" hipError_t m3s_launch_fuse(const TrackArgs* a, int chunk_id, const FuseArgs* f, int count, int N,
                                      const TrackPublish* pub, hipStream_t s) {
  const int grid = (N + 255) / 256 > FUSE_COUNT_BLOCKS ? (N + 255) / 256 : FUSE_COUNT_BLOCKS;  // every counting block publishes
  // count: the byte map was written by track_setup (fused path), so it is counted and cleared
  hipLaunchKernelGGL(m3s::fuse_kernel, dim3(grid), dim3(256), 0, s, a->state, chunk_id, *f, N, a->flags,
                     count ? &a->state->n_unique : nullptr, *pub, count, a->tick, a->cnt);
  return hipGetLastError();
}

#ifdef M3S_GN_STAMPS
extern "C" int m3s_debug_gn_stamps(unsigned long long* out) {
  (void)hipDeviceSynchronize();
  const int rc = hipMemcpyFromSymbol(out, HIP_SYMBOL(m3s::g_gn_stamps), sizeof(unsigned long long) * GN_NSTAMP) == hipSuccess ? 0 : -1;
  static unsigned long long z[GN_NSTAMP];  // zeros: cleared for the next frame (shard-last stamps are sparse)
  (void)hipMemcpyToSymbol(HIP_SYMBOL(m3s::g_gn_stamps), z, sizeof(z));
  return rc;
}
#endif
