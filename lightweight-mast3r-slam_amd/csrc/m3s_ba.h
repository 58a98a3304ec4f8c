// Internal (non-ABI) structs shared by ba.hip and abi.cpp. The public C ABI is include/m3s.h.
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>

#define BA_MODE_POINTS 0
#define BA_MODE_RAYS 1
#define BA_MODE_CALIB 2

#ifndef M3S_BA_SP_WAVES
#define M3S_BA_SP_WAVES 16  // waves of the one-workgroup sparse factorisation (ba.hip) and of its cost model (abi.cpp)
#endif

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

// record reuse (m3s_ba_make_plan_reuse): one keyframe's current buffers and the library's copy of them from the
// previous plan on the workspace ((3N + N) floats: X then C)
struct BaKfCopy {
  const float* X;
  const float* C;
  float* copy;
};

// bytes of one record slot: N 16-B records (calib uses 12 B of each), then N floats (rays: |Xi|) padded to 16 B. A slot's bytes sit at
// slot * ba_rec_slot_bytes(N) whatever the plan's edge count: record reuse keeps slots across the plans of a growing
// graph, and a region [all records | all |Xi|] would move its second part with the edge count
__host__ __device__ inline size_t ba_rec_slot_bytes(int N) { return (size_t)16 * N + (size_t)4 * ((N + 3) & ~3); }

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
  float4* rec;           // record slots (ba_rec_slot_bytes each): N point records {Xi | Xi/|Xi| (rays) ; sqrt-weight}
                         // (16 B) or {u_t | v_t << 16, log z_i, sqrt-weight} (calib, 12 B), then (rays) N floats |Xi|
  const int* rec_slot;   // (E_local) record slot of each shard edge (record reuse across plans), or null: slot = edge
  const int* pack_list;  // (n_pack) shard edges the pack writes, grouped by source keyframe (reuse: only the changed)
  double* partials;      // (E_local*chunks, 36)
  double* edge_sums;     // (E, 36) global edge rows; all-reduced across ranks in multi-GPU BA
  // block-sparse pose system (ba_pattern.h; analysed once per plan, factored on the device every iteration)
  int nb;                 // block columns = poses - 1 (pin)
  int nlev;               // elimination-tree levels
  int wide_steps;         // factor steps [0, wide_steps) run as multi-workgroup launches (ba_sparse_step_kernel)
  const int* perm;        // (nb) factor column -> pose index (pin removed)
  const int* col_ptr;     // (nb+1) factor blocks of each column, diagonal first
  const int* rowL;        // (nL) block row of each factor block
  const int* lev_ptr;     // (nlev+1) -> lev_col
  const int* lev_col;     // (nb) columns grouped by level
  const int* grp_ptr;     // (nlev+2) -> grp: the update groups of each step
  const int4* grp;        // {target column j, src begin, src end, 0}
  const int* pull_grp;    // (nb) the group a column's factor task runs first, or -1
  const int4* src;        // {block of L_jk, k, sidx offset, 0}
  const int* sidx;        // per group source, per block of column j: the source block of column k, or -1
  const int* sched;       // dataflow schedule of the one-workgroup part + back substitution (ba_pattern.h)
  int flow;               // sched present (else the level-synchronous loops)
  const int4* step_rec;   // per task of the wide steps, 2 x int4: {j, b0, b1, pull group or -1}, {src begin, end, 0, 0}
  const char* plan_lo;    // [plan_lo, plan_lo + plan_bytes): col_ptr .. sidx, sched, staged into LDS by the factor kernel
  int plan_bytes;
  const int* asm_ptr;     // (nL+1) assembly CSR: edge*2 + (sign<0), edge order
  const int* asm_ent;
  const int* rhs_ptr;     // (nb+1) per factor row
  const int* rhs_ent;
  const int* lin_tab;     // (E_local * chunks) linearisation block -> local edge * chunks + chunk
  double* L;   // (nL, 8, 8) factor blocks (7x7 used; diagonal blocks keep 1/L_mm in column 7)
  double* y;   // (nb, 8) rhs -> forward-substituted
  double* xs;  // (nb, 8) solution in factor order
  float* dx;   // (nb, 7) output in pose order, reference return value
  double* H;   // dense fallback ((2n+1), n), n = 7 nb: system, rhs row, carried identity (ba_dense.hip)
  int* info;   // factorisation failure flag
  int* done;   // early-exit flag (|dx| < delta_thresh)
  int* iters;  // iterations executed
  int* bad;    // non-positive pivot seen by a multi-workgroup factor step (cleared by the assembly)
  int* stalled;  // sticky: a dataflow / LDS hand-off wait timed out in some solve of this plan (M3S_ESTALL)
  int force_stall;  // tests only (M3S_BA_FORCE_STALL): the dataflow waits are never satisfied
};
// bits of the factor kernel's failure word
#define BA_BAD_LLT 1    // non-positive pivot: dx = 0 for this iteration (SimplicialLLT info != Success)
#define BA_BAD_STALL 2  // a bounded dataflow wait timed out
