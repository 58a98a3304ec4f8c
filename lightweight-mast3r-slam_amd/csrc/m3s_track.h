// Internal (non-ABI) structs shared by track.hip and abi.cpp. The public C ABI is include/m3s.h.
#pragma once
#include <stdint.h>

#define M3S_TRACK_RUNNING 0
#define M3S_TRACK_OK 1
#define M3S_TRACK_MAX_ITERS 2
#define M3S_TRACK_CHOLESKY_FAILED 3
#define M3S_TRACK_SKIPPED 4
#define M3S_TRACK_STALLED 5  // the persistent GN launch lost a hand-off (blocks not co-resident): an error, not a result

#define M3S_TRACK_SHARDS 8  // counter shards (one per XCD: blocks are dealt to XCDs round-robin)

// Device-resident GN state (one per tracked frame). Layout mirrored by m3s/_track.py (M3S_TRACK_STATE_*).
struct TrackState {
  float T[8];      // T_CkCf (current estimate)
  float T_WCk[8];  // keyframe pose
  float T_WCf[8];  // output: T_WCk * T_CkCf
  double old_cost;
  double last_cost;
  int iter;
  int done;
  int status;
  int n_valid_opt;
  int n_valid_kf;
  int n_unique;
  int done_chunk;  // host chunk id of the GN launch batch that finished (gates the fuse launch)
};

struct TrackParams {
  int N, H, W, mode;  // mode 0 = rays (opt_pose_ray_dist_sim3), 1 = calib (opt_pose_calib_sim3)
  float Nf, Nk;       // frame / keyframe fusion counts (get_average_conf divisors)
  float C_conf, Q_conf, min_match_frac;
  float c_a, c_b;     // float32(1/sigma_ray|pixel), float32(1/sigma_dist|depth)
  float huber_k, rel_error, delta_norm;
  int max_iters;
  float pixel_border, depth_eps;
  float fx, fy, cx, cy;
  float K[9];
  int direct;  // opt_pose_* surface: inputs already gathered / constrained (see m3s.h)
};

struct TrackArgs {
  const int64_t* idx;          // (N) idx_f2k
  const uint8_t* valid_match;  // (N)
  const float* Xf;             // (N,3) frame X_canon
  const float* Cf;             // (N) frame C (sum)
  const float* Qff;            // (N)
  const float* Xk;             // (N,3) keyframe X_canon
  const float* Ck;             // (N) keyframe C (sum)
  const float* Qkf;            // (N)
  const float* meas_k;         // (N,3) direct calib only
  const uint8_t* valid_meas;   // (N)   direct calib only
  float* rec;                 // (N,8) per-point GN record (workspace)
  uint8_t* flags;              // (N, padded to 16) unique(idx[valid]) byte map (workspace, zeroed per frame)
  double* partials;            // (nparts, 40) block partial sums (workspace)
  TrackState* state;
  unsigned long long* cnt;     // (8 x 16) setup counters, one 128-B line per XCD shard: (n_valid_kf << 32) | n_valid_opt
  unsigned* tick;              // (M3S_TRACK_TICK_WORDS) GN shard tickets, publish ticket, GN shard-sum granules
  float* T_out;                // (16) nullable: T_WCf | T_CkCf written by the solving block when done
  const float* T_WCf;          // (8) the frame's pose estimate (device), read by track_setup's state init
  const float* T_WCk;          // (8) the keyframe's pose (device)
};

// The tick region (zeroed per frame by track_init): one 128-B line per XCD shard ticket of the persistent GN
// launch (monotonic within the frame), the fuse kernel's publish ticket (one line), then the shard-sum granules
// of the GN launch: [2 iteration parities][8 shards][72] 8-byte {32-bit half of a shard sum, iteration + 1}.
#define M3S_TRACK_PUBLISH_TICKET (M3S_TRACK_SHARDS * 32)
#define M3S_TRACK_GRANULES ((M3S_TRACK_SHARDS + 1) * 32)
#define M3S_TRACK_TICK_WORDS (M3S_TRACK_GRANULES + 2 * M3S_TRACK_SHARDS * 72 * 2)

// The frame's result as the host reads it: a copy of the final TrackState in fine-grained (coherent)
// pinned host memory, written by the fuse launch once n_unique is complete and then released with the
// call's generation number; the host spins on gen instead of a D2H copy + hipStreamSynchronize.
struct TrackMirror {
  TrackState s;
  unsigned gen;
  unsigned pad[3];
};
struct TrackPublish {
  TrackMirror* mirror;  // host pointer (the same address on the device for hipHostMalloc memory)
  unsigned* ticket;     // tick + M3S_TRACK_PUBLISH_TICKET (zeroed by track_init)
  unsigned gen;
};

// keyframe fusion (weighted_pointmap) + the match_info average confidences (frame.py:74-77, 83-84)
struct FuseArgs {
  const float* X_in;  // (N,3) keyframe X_canon
  const float* C_in;  // (N)   keyframe C
  const float* Xkf;   // (N,3) keyframe points in the frame's camera
  const float* Ckf;   // (N)
  float* X_out;       // (N,3) may alias X_in
  float* C_out;       // (N)   may alias C_in
  const float* Cf;    // (N)   frame C (nullable)
  float* Ck_avg;      // (N)   C_out / Nk_new (nullable)
  float* Cf_avg;      // (N)   Cf / Nf (nullable)
  float Nk_new, Nf;
  int* slot_N;            // keyframe-store slot counters and dirty flag (nullable; m3s_track_fuse_args)
  int* slot_N_updates;
  uint8_t* slot_dirty;
  int N_new, N_updates_new;
};
