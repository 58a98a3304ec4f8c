// Host-side symbolic analysis of the BA pose system (internal, not ABI).
//
// The reference assembles the pose system as Eigen triplets and factors it with SimplicialLLT
// (/root/reference/mast3r_slam/backend/src/gn_kernels.cu:57-159), re-analysing the pattern on every GN
// iteration. Here the pattern is analysed ONCE per plan, at 7x7-block granularity (one block per
// keyframe pose), and the numeric factorisation of every GN iteration runs on the device
// (ba_sparse_factor_kernel, ba.hip):
//   * ordering: minimum degree on the keyframe graph (ties to the lowest index), which keeps the fill of
//     the long chain + loop-closure graphs of SLAM small (K = 256 chess graph: 1922 factor blocks
//     instead of 32640 dense, elimination tree height 68 instead of 255);
//   * the factor's block columns, their levels in the elimination tree (a column's level is one more
//     than its highest child's), and the update work grouped per (source level, target column): one
//     wave owns each group (sources ascending), so every column's update order is fixed
//     (deterministic: identical on every rank); a column's children's-level group runs inside its own
//     factor task, right before it factors;
//   * the assembly CSR in factor-block order: the contributions (edge*2 + sign) of each block, in edge
//     order, and the rhs contributions per (new) block row.
#pragma once
#include <cstddef>
#include <vector>

struct BaPattern {
  int nb = 0;    // block columns (poses without the pinned one)
  int nL = 0;    // factor blocks (diagonal included)
  int nlev = 0;  // elimination-tree levels
  bool too_dense = false;  // the update source map outgrew max_sidx: the build stopped early (tables incomplete)
  std::vector<int> perm;      // (nb) new column -> old (pin-removed) pose index
  std::vector<int> col_ptr;   // (nb+1) factor blocks of column j: [col_ptr[j], col_ptr[j+1]), first = diagonal
  std::vector<int> rowL;      // (nL) block row (new index) of each factor block
  std::vector<int> lev_ptr;   // (nlev+1) into lev_col
  std::vector<int> lev_col;   // (nb) columns grouped by level, ascending within a level
  std::vector<int> grp_ptr;   // (nlev+2) into grp: the update groups of step s (sources at level s-1)
  std::vector<int> grp;       // int4 {target column j, src begin, src end, 0}; the factor tasks' own groups follow
  std::vector<int> pull_grp;  // (nb) group of column j's children's level, run by its factor task, or -1
  std::vector<int> src;       // int4 {block of L_jk in column k, k, sidx offset, 0}
  std::vector<int> sidx;      // per group source, per block b of column j: the block of column k at row rowL[b], or -1
  std::vector<int> asm_ptr;   // (nL+1) into asm_ent
  std::vector<int> asm_ent;   // edge*2 + (1 if the block takes -M)
  std::vector<int> rhs_ptr;   // (nb+1) per new block row, into rhs_ent
  std::vector<int> rhs_ent;   // edge*2 + (1 if the row takes -g)
};

// ri, rj: dense pose ranks (pin 0 = rank 0 is fixed) of the E directed edges; Kp poses. max_sidx bounds the
// update source map (the plan's table capacity, < INT_MAX): past it the build stops with too_dense set, before a
// dense large graph can exhaust host memory.
void ba_build_pattern(const int* ri, const int* rj, int E, int Kp, BaPattern* P, size_t max_sidx = (size_t)1 << 30);

// Dataflow schedule of the one-workgroup part of the numeric factorisation (steps [wide, nlev]) and of the whole
// back substitution: instead of a barrier per elimination-tree level, every wave of the workgroup walks its own
// task list and waits only on the tasks its inputs come from (flags in LDS). Lists come from a list-scheduling
// simulation over the task graph (estimated task costs, a penalty for a cross-wave hand-off), tasks in step order
// within every list, so the earliest unfinished task is always runnable (no deadlock). Per target column the
// update groups still apply in step order (a per-column counter), so the factor is bit-identical to the
// level-synchronous schedule. Layout (ints):
//   [wl_ptr waves+1] [bs_ptr waves+1] [fac_init nb] [wl_task 2 x ntask] [bs_col nb]
// wl_task = {code, q}: code >= 0 factors column code after q update groups landed on it; code < 0 runs update
// group -1 - code once q earlier groups landed on its target. fac_init[k] = 1 for columns factored by the
// multi-workgroup steps [0, wide). bs_col: back-substitution columns per wave, descending (parents first).
// bs_col entries carry BA_BS_NOWAIT when the wave's previous column is the parent (or the column is a root): struct(j)
// minus the parent lies in struct(parent), which the parent already waited for, so x_j needs no wait; the column is
// the low 24 bits.
#define BA_BS_NOWAIT (1 << 30)
#define BA_BS_COL 0xFFFFFF
// Returns the simulated finish time (us) of the factor part (the cost model's estimate).
double ba_flow_schedule(const BaPattern& P, int wide, int waves, std::vector<int>* sched);
