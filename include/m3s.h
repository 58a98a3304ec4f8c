/*
 * m3s.h — C ABI of the MI355X-native MASt3R-SLAM tracking hot path (libm3s.so).
 *
 * Plain pointers and sizes only (no torch types). All array pointers are DEVICE pointers on the
 * current HIP device unless the comment says "host"; `stream` is a hipStream_t passed as void*
 * (NULL = default stream). Every entry point returns 0 on success or a negative M3S_E* code; the
 * message of the last failure on the calling thread is available from m3s_last_error().
 *
 * Each entry point replaces one operator of the reference's native extension
 * `mast3r_slam_backends` (bindings /root/reference/mast3r_slam/backend/src/gn.cpp:116-123,
 * declarations backend/include/gn.h) or fuses a stretch of the reference's Python glue
 * (mast3r_slam/matching.py, tracker.py). The Python module `mast3r_slam_backends` in
 * lightweight-mast3r-slam_amd/ binds these through ctypes.
 */
#ifndef M3S_H
#define M3S_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define M3S_ABI_VERSION 5

#define M3S_OK 0
#define M3S_EINVAL -1  /* bad shape / argument (reference: TORCH_CHECK -> RuntimeError) */
#define M3S_EHIP -2    /* HIP launch / runtime failure */
#define M3S_ESPACE -3  /* workspace too small */
#define M3S_ESTALL -4  /* global BA: a bounded dataflow hand-off wait of the factorisation timed out (a schedule
                        * fault, not a non-positive pivot): the GN loop stopped; reported by m3s_ba_iterations and
                        * m3s_gauss_newton. A non-positive pivot keeps the reference contract (dx = 0, no error). */

int m3s_abi_version(void);
const char* m3s_last_error(void);

/* Per-kernel HIP-event timing (no reference counterpart; the reference's profiler.py wraps regions
 * with torch.cuda.synchronize). When enabled, every launch group is bracketed by hipEvents on its
 * own stream under a name: prep_rays, proj_occlusion, refine_lin, track_setup, gn_iters,
 * ba_linearize, ba_solve. query synchronises the recorded events. */
void m3s_timing_enable(int on);
void m3s_timing_reset(void);
int m3s_timing_query(const char* name, double* total_ms, int* count);

/* ---------------------------------------------------------------------------------------------
 * Reference operators (drop-in for mast3r_slam_backends.*)
 * ------------------------------------------------------------------------------------------- */

/* iter_proj(rays_img_with_grad, pts_3d_norm, p_init, max_iter, lambda_init, cost_thresh)
 *   -> [p_new, converged]                                   gn.cpp:84-99, gn.h:89-95,
 *                                                           matching_kernels.cu:119-316
 * rays (B,H,W,C=9) f32, pts (B,N,3) f32, p_init (B,N,2) f32 -> p_new (B,N,2) f32, converged (B,N) u8 */
int m3s_iter_proj(const float* rays, const float* pts, const float* p_init, float* p_new, uint8_t* converged,
                  int B, int H, int W, int C, int N, int max_iter, float lambda_init, float cost_thresh,
                  void* stream);

/* refine_matches(D11, D21, p1, radius, dilation_max) -> [p1_new]
 *                                                           gn.cpp:101-114, gn.h:112-117,
 *                                                           matching_kernels.cu:25-116
 * dtype 0 = f16 (c10::Half step rounding), 1 = f32. D11 (B,H,W,F), D21 (B,N,F), p1 (B,N,2) i64
 * -> p1_new (B,N,2) i64 */
int m3s_refine_matches(int dtype, const void* D11, const void* D21, const int64_t* p1, int64_t* p1_new, int B,
                       int H, int W, int F, int N, int radius, int dilation_max, void* stream);

/* gauss_newton_{points,rays,calib}(Twc, Xs, Cs, [K,] ii, jj, idx_ii2jj, valid_match, Q, ...) -> [dx]
 *                                                           gn.cpp:3-82, gn.h:22-87,
 *                                                           gn_kernels.cu:725-811, 1140-1228, 1546-1637
 * Twc (Kp,8) f32 is updated IN PLACE (as the reference). Xs (Kp,N,3), Cs (Kp,N) f32; ii, jj (E) i64
 * global keyframe ids (remapped to dense ranks internally, gn_kernels.cu:161-170); idx (E,N) i64;
 * valid (E,N) u8; Q (E,N) f32. dx_out ((Kp-1),7) f32 receives the last step. iters_out (host,
 * nullable) receives the iteration count. The workspace must hold m3s_ba_workspace_size() bytes. */
typedef struct m3s_ba_config {
  int mode;          /* 0 points, 1 rays, 2 calib */
  float sigma_a;     /* sigma_point | sigma_ray | sigma_pixel */
  float sigma_b;     /* -           | sigma_dist | sigma_depth */
  float C_thresh, Q_thresh;
  float fx, fy, cx, cy; /* calib: K[0,0], K[1,1], K[0,2], K[1,2] (host values) */
  int height, width, pixel_border;
  float z_eps;
} m3s_ba_config;

/* Kp <= M3S_BA_MAX_POSES: the workspace is sized for the densest factor pattern of Kp poses (no edges are known
 * to the size query): nb (nb + 1) / 2 blocks of 512 B for nb = Kp - 1, 4.3 GB at the cap. */
#define M3S_BA_MAX_POSES 4096
size_t m3s_ba_workspace_size(int Kp, int N, int E);
int m3s_gauss_newton(const m3s_ba_config* cfg, float* Twc, const float* Xs, const float* Cs, int Kp, int N,
                     const int64_t* ii, const int64_t* jj, int E, const int64_t* idx, const uint8_t* valid,
                     const float* Q, int max_iter, float delta_thresh, float* dx_out, int* iters_out,
                     void* workspace, size_t workspace_bytes, void* stream);

/* Split BA for edge-sharded multi-GPU runs (no reference counterpart).
 * plan: rank remap + block-sparse assembly pattern for ALL E edges, shard = edges [e0, e1).
 * Per iteration: m3s_ba_linearize (this shard's rows of the (E,36) f64 edge-sum table), then the
 * caller all-reduces that table (offset/size from m3s_ba_edge_sums), then m3s_ba_solve. */
typedef struct m3s_ba_plan { unsigned char opaque[768]; } m3s_ba_plan;
int m3s_ba_make_plan(const m3s_ba_config* cfg, float* Twc, const float* Xs, const float* Cs, int Kp, int N,
                     const int64_t* ii, const int64_t* jj, int E, int e0, int e1, const int64_t* idx,
                     const uint8_t* valid, const float* Q, float delta_thresh, float* dx_out, void* workspace,
                     size_t workspace_bytes, m3s_ba_plan* plan, void* stream);
/* Zero-copy keyframe source: instead of the stacked Xs / Cs that
 * FactorGraph.get_poses_points builds with torch.stack (global_opt.py:114-121), the keyframes' own buffers.
 * Host arrays of Kp entries: X[k] -> that keyframe's (N,3) X_canon, C[k] -> its (N) confidence sum (device
 * pointers), N_avg[k] = its fusion count N; the average confidence is C * float32(1/N), exactly
 * Frame.get_average_conf (frame.py:93-94) on a torch device. Same plan and results as m3s_ba_make_plan. */
typedef struct m3s_ba_keyframes {
  const float* const* X;
  const float* const* C;
  const float* N_avg;
} m3s_ba_keyframes;
int m3s_ba_make_plan_kf(const m3s_ba_config* cfg, float* Twc, const m3s_ba_keyframes* kf, int Kp, int N,
                        const int64_t* ii, const int64_t* jj, int E, int e0, int e1, const int64_t* idx,
                        const uint8_t* valid, const float* Q, float delta_thresh, float* dx_out, void* workspace,
                        size_t workspace_bytes, m3s_ba_plan* plan, void* stream);
/* Record reuse across successive plans on ONE workspace (no reference counterpart; the reference backend calls
 * solve_GN once per new keyframe, main.py:150-155, and re-gathers every edge each time). Between two such calls
 * the edge set only grows and tracking changes only the keyframes it fuses into, so most edges' point records
 * (ba_pack: matched point or pixel + folded validity weight) are still valid in the workspace. With reuse ids a
 * plan packs only the edges that are new to the workspace or touch a keyframe whose points, confidences or
 * fusion count changed since the workspace's previous plan (an exact bit compare on the device against copies
 * the library keeps per keyframe); the other edges keep their records. Results are bit-identical to the plain
 * plan. edge_uid (E entries, host): a stable id per directed edge naming immutable match data (its idx / valid /
 * Q rows; FactorGraph uses 2u + direction for undirected edge u); kf_uid (Kp entries, host): a stable id per
 * pose rank (the keyframe's global index). Contract: between reuse plans the workspace holds nothing else (a
 * plain plan on it drops the cache); call m3s_ba_reuse_release(workspace) before freeing or repurposing it
 * (frees the keyframe copies, 16 B per keyframe point). */
typedef struct m3s_ba_reuse {
  const int64_t* edge_uid;
  const int64_t* kf_uid;
} m3s_ba_reuse;
int m3s_ba_make_plan_reuse(const m3s_ba_config* cfg, float* Twc, const float* Xs, const float* Cs, int Kp, int N,
                           const int64_t* ii, const int64_t* jj, int E, int e0, int e1, const int64_t* idx,
                           const uint8_t* valid, const float* Q, float delta_thresh, float* dx_out,
                           const m3s_ba_reuse* reuse, void* workspace, size_t workspace_bytes, m3s_ba_plan* plan,
                           void* stream);
int m3s_ba_make_plan_kf_reuse(const m3s_ba_config* cfg, float* Twc, const m3s_ba_keyframes* kf, int Kp, int N,
                              const int64_t* ii, const int64_t* jj, int E, int e0, int e1, const int64_t* idx,
                              const uint8_t* valid, const float* Q, float delta_thresh, float* dx_out,
                              const m3s_ba_reuse* reuse, void* workspace, size_t workspace_bytes, m3s_ba_plan* plan,
                              void* stream);
/* packed_edges: shard edges the plan's pack wrote; changed_keyframes: keyframes found changed (all without reuse) */
int m3s_ba_reuse_info(const m3s_ba_plan* plan, int* packed_edges, int* changed_keyframes);
int m3s_ba_reuse_release(const void* workspace);
/* The library keeps per-workspace host state for BA plans (the symbolic analysis a plan's solves use). Call
 * m3s_ba_plan_release(workspace) once no plan on `workspace` will be solved again and before freeing or repurposing
 * it (m3s_ba_reuse_release does it too); it joins a pending analysis and frees its tables. */
int m3s_ba_plan_release(const void* workspace);
/* Diagnostic: how many workspaces currently hold BA plan state (a leak check for callers that cache workspaces). */
int m3s_ba_plan_count(void);
int m3s_ba_edge_sums(const m3s_ba_plan* plan, size_t* byte_offset, size_t* byte_count);
int m3s_ba_linearize(const m3s_ba_plan* plan, void* stream);
int m3s_ba_solve(const m3s_ba_plan* plan, void* stream);
int m3s_ba_iterations(const m3s_ba_plan* plan, int* iters_out, void* stream); /* syncs the stream */
/* Host-only facts of a built plan (bench rooflines, tests): info[0] = linearisation chunks per edge,
 * [1] = factor blocks, [2] = elimination-tree levels, [3] = multi-workgroup factor steps, [4] = 1 if the dense
 * fallback factorisation is used, [5] = distinct target keyframes among the shard's edges, [6] = shard edges,
 * [7] = poses, [8..12] = 0 (round 5's opt-in solver phases, removed in round 6). info holds 13 ints. */
int m3s_ba_plan_info(const m3s_ba_plan* plan, int* info);
/* Host-only diagnostic of the symbolic factorisation the plan builds for these edges (host arrays):
 * stats[0] = factor blocks (7x7, diagonal included), [1] = elimination-tree levels, [2] = update groups
 * (source level, target column), [3] = update sources, [4] = source-map entries, [5] = groups run by
 * factor tasks. */
int m3s_ba_pattern_stats(const int64_t* ii, const int64_t* jj, int E, int Kp, int* stats);

/* ---------------------------------------------------------------------------------------------
 * Fused operators (replace stretches of the reference's Python glue)
 * ------------------------------------------------------------------------------------------- */

/* match(X11, X21, D11, D21, idx_init) -> (idx_1_to_2, valid_match2)     matching.py:8-90
 * X11, X21 (B,H,W,3) f32; D11, D21 (B,H,W,F) f32 (F % 8 == 0, F in {16,24,32}); idx_init (B,N) i64
 * or NULL (identity). idx_out (B,N) i64; valid_out (B,N) u8. Parameters = config `matching.*`. */
size_t m3s_match_workspace_size(int B, int H, int W, int F);
int m3s_match(const float* X11, const float* X21, const float* D11, const float* D21, const int64_t* idx_init,
              int64_t* idx_out, uint8_t* valid_out, int B, int H, int W, int F, int max_iter, float lambda_init,
              float cost_thresh, float dist_thresh, int radius, int dilation_max, void* workspace,
              size_t workspace_bytes, void* stream);

/* FrameTracker.track post-matching stretch (tracker.py:35-114): setup, Sim(3) GN to convergence
 * (rays: opt_pose_ray_dist_sim3 :173-214; calib: opt_pose_calib_sim3 :216-266), keyframe pointmap
 * fusion (frame.py:74-77) and the keyframe-selection statistics. */
#define M3S_TRACK_OK 1
#define M3S_TRACK_MAX_ITERS 2
#define M3S_TRACK_CHOLESKY_FAILED 3
#define M3S_TRACK_SKIPPED 4
/* The persistent GN launch's blocks did not all become resident within the bounded spin (e.g. the GPU
 * was shared with long-running persistent work): m3s_track then returns M3S_EHIP ("hand-off stalled")
 * instead of a result, never a silent relocalisation. */
#define M3S_TRACK_STALLED 5

typedef struct m3s_track_config {
  int mode;           /* 0 rays (use_calib False), 1 calib */
  int max_iters;      /* tracking.max_iters */
  float C_conf, Q_conf, min_match_frac;
  float sigma_a;      /* sigma_ray | sigma_pixel */
  float sigma_b;      /* sigma_dist | sigma_depth */
  float huber_k, rel_error, delta_norm;
  float pixel_border, depth_eps;
  float K[9];         /* calib intrinsics, row-major (host values) */
  int H, W;
} m3s_track_config;

typedef struct m3s_track_inputs {
  const int64_t* idx_f2k;      /* (N) */
  const uint8_t* valid_match;  /* (N) */
  const float* Xf;             /* (N,3) frame X_canon */
  const float* Cf;             /* (N)   frame C (sum) */
  float Nf;                    /* frame fusion count */
  const float* Qff;            /* (N) */
  const float* Xk;             /* (N,3) keyframe X_canon */
  const float* Ck;             /* (N)   keyframe C (sum) */
  float Nk;                    /* keyframe fusion count */
  const float* Qkf;            /* (N) */
  const float* T_WCf;          /* (8) device */
  const float* T_WCk;          /* (8) device */
  /* direct = 1: the opt_pose_* surface (tracker.py:173,216). idx_f2k is ignored (identity),
   * Qff holds Qk, valid_match holds valid_opt, Xf is already gathered (and constrained in calib
   * mode), meas_k (N,3) / valid_meas_k (N) are given; Cf, Ck, Qkf are unused. */
  int direct;
  const float* meas_k;
  const uint8_t* valid_meas_k;
} m3s_track_inputs;

typedef struct m3s_track_fuse_args {
  const float* Xk_canon; /* (N,3) keyframe X_canon; NULL = no fusion */
  const float* Ck_sum;   /* (N)   keyframe C */
  const float* Xkf;      /* (N,3) model output: keyframe points in the frame's camera */
  const float* Ckf;      /* (N) */
  float* Xk_out;         /* (N,3) fused X_canon (may alias Xk_canon: in place) */
  float* Ck_out;         /* (N)   fused C (may alias Ck_sum) */
  const float* Cf;       /* (N)   frame C (for Cf_avg_out; nullable) */
  float* Ck_avg_out;     /* (N)   fused C / Nk_new = keyframe.get_average_conf() (nullable) */
  float* Cf_avg_out;     /* (N)   Cf / Nf = frame.get_average_conf() (nullable) */
  float Nk_new, Nf;      /* keyframe N after this fusion, frame N (frame.py:83-84) */
  /* keyframe-store slot write-back (nullable; SharedKeyframes.__setitem__, frame.py:271-289, called at
   * tracker.py:101): with Xk_out / Ck_out pointing INTO the store's X[idx] / C[idx] rows, the fusion kernel also
   * stores the slot's fusion counters and dirty flag, on the device, when the frame tracked (the fusion's own
   * condition): slot_N = N_new, slot_N_updates = N_updates_new, slot_dirty = 1. Nothing else of the record changes
   * on a track (img, uimg, feat, pos, T_WC keep their values), so no full-record copy is needed. */
  int* slot_N;
  int* slot_N_updates;
  uint8_t* slot_dirty;
  int N_new, N_updates_new;
} m3s_track_fuse_args;

typedef struct m3s_track_result {
  float T_WCf[8];
  float T_CkCf[8];
  double cost;
  int iters, status, n_valid_opt, n_valid_kf, n_unique, N;
} m3s_track_result;

/* The track workspace's frame scratch (byte map, counters, tickets) persists across calls: each call's fusion launch
 * leaves it clean for the next frame, so only a fresh workspace is initialised. Call m3s_track_release(workspace)
 * before freeing or repurposing a workspace m3s_track used (a later workspace at the same address is then
 * initialised again); a workspace of another size at the same address is always initialised. */
size_t m3s_track_workspace_size(int N);
int m3s_track_release(const void* workspace);
int m3s_track(const m3s_track_inputs* in, const m3s_track_config* cfg, const m3s_track_fuse_args* fuse,
              int first_chunk, float* T_out_dev /* (16) nullable: T_WCf | T_CkCf on device */,
              m3s_track_result* result /* host */, void* workspace, size_t workspace_bytes, void* stream);

/* ---- retrieval codebook quantization ----
 * Replaces RetrievalDatabase.quantize_custom (mast3r_slam/retrieval_database.py:96-105):
 *   l2 = (|q|^2 + |c|^2) - 2 q c^T ; topk(l2, k, largest=False).indices, called from accumulate_scores (:119)
 *   and add_to_ivf_custom (:151-153) with the codebook `self.centroids` (:20-22).
 * m3s_codebook_prepare arranges the (C, D) fp32 centroids once (the reference moves them to the device once, in
 * __init__) into `codebook` (m3s_codebook_size bytes, device). m3s_quantize writes the (M, k) int64 indices of the
 * k nearest centroids of each of the M query rows (ascending distance; ties -> lower index), 1 <= k <= 8, k <= C.
 * Distances are computed with bf16 hi/lo split products on the matrix cores (fp32 accumulation): ~2^-16 relative
 * per product, tighter than the reference's TF32 GEMM (main.py:168). Everything is asynchronous on `stream`. */
size_t m3s_codebook_size(int C, int D);
int m3s_codebook_prepare(const float* centroids, int C, int D, void* codebook, size_t codebook_bytes, void* stream);
size_t m3s_quantize_workspace_size(int C, int D, int M, int k);
int m3s_quantize(const void* codebook, int C, int D, const float* qvecs, int M, int k, int64_t* topk_out,
                 void* workspace, size_t workspace_bytes, void* stream);

/* Measured-peak probe (no reference counterpart; bench.py's roofline context):
 * blocks x 256 lanes x iters x 8 chains of v_fma_f32 (2 flops each) on `stream`. */
int m3s_peak_fma_f32(float* out_dev, int blocks, int iters, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* M3S_H */
