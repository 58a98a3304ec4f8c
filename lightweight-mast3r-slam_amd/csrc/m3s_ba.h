// Internal (non-ABI) structs shared by ba.hip and abi.cpp. The public C ABI is include/m3s.h.
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>

#define BA_MODE_POINTS 0
#define BA_MODE_RAYS 1
#define BA_MODE_CALIB 2

struct BaParams {
  int mode;
  int N;            // points per keyframe
  int chunks;       // point chunks per edge (blocks per edge)
  int edge_offset;  // first global edge row of this shard (edge_sums / idx / valid / Q row offset)
  float inv_a, inv_b;  // float(1/sigma_{point|ray|pixel}), float(1/sigma_{-|dist|depth}) (gn_kernels.cu:905-906)
  float C_thresh, Q_thresh;
  float fx, fy, cx, cy;
  int H, W, pixel_border;
  float z_eps;
};

struct BaArgs {
  float* Twc;            // (K,8) in/out
  const float* const* Xkf;  // (K) -> (N,3) keyframe points: rows of the stacked Xs, or each keyframe's X_canon
  const float* const* Ckf;  // (K) -> (N)   confidences: rows of the stacked Cs, or each keyframe's C sum
  const float* Cscale;      // (K) 1 (stacked Cs) or float32(1/N_k) (get_average_conf on a torch device: C * (1/N))
  const int* ii_rank;    // (E_local) dense rank of i (pin 0), shard-local
  const int* jj_rank;    // (E_local)
  const int64_t* idx;    // (E,N) global edge rows
  const uint8_t* valid;  // (E,N)
  const float* Q;        // (E,N)
  float4* rec;           // (E_local, N) per-call point records (ba_pack): {Xi | u_t, v_t, z_i ; sqrt-weight}
  double* partials;      // (E_local*chunks, 36)
  double* edge_sums;     // (E, 36) global edge rows; all-reduced across ranks in multi-GPU BA
  // assembly CSR (host-built once per call)
  const int* blk_row;  // (nblocks) block row (pose index, pin removed)
  const int* blk_col;  // (nblocks)
  const int* blk_ptr;  // (nblocks+1)
  const int* blk_ent;  // edge*2 + (sign<0)
  const int* rhs_ptr;  // (K-1+1)
  const int* rhs_ent;
  double* H;   // ((2n+1), n), n = 7(K-1); row n = rhs, rows n+1.. = carried identity (-> L^-T)
  double* x;   // (n)
  float* dx;   // (n) output, reference return value
  int* info;   // factorisation failure flag
  int* done;   // early-exit flag (|dx| < delta_thresh)
  int* iters;  // iterations executed
};
