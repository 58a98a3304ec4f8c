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
// sub > 0 (subtree phase below, wide = 0): steps [0, sub) belong to the subtree launch except their update groups
// whose target column sits at level >= sub, which the one-workgroup schedule runs first (in step order per target).
// top > 0 (dense top phase, ba_top_plan): the columns at levels >= top are factored and solved by ba_dense_top_kernel
// between a factor-only and a back-substitution-only run of the one-workgroup kernel: their factor tasks, the update
// groups whose sources sit at levels >= top and their back-substitution tasks leave the lists; the pull groups of the
// columns at level `top` (sources below the cut) become update-group tasks.
// Returns the simulated finish time (us) of the factor part (the cost model's estimate).
double ba_flow_schedule(const BaPattern& P, int wide, int waves, std::vector<int>* sched, int sub = 0, int top = 0);

// Dense top phase (ba_dense_top_kernel, ba.hip): the columns at elimination-tree levels >= `top` (an ancestor-closed
// set: the root end of the tree, where the factor is nearly dense) as one dense (7T x 7T) fp64 Cholesky on the matrix
// cores in one workgroup. Layout (ints): [T, top, 0, 0] [top columns ascending (T)] [T x T: the factor block of
// L(row top_col[a], column top_col[b]) for a >= b, or -1 where the pattern has none]. Returns T (0: no top phase).
int ba_top_plan(const BaPattern& P, int top, std::vector<int>* tab);

// Subtree phase (ba_subtree_kernel, ba.hip): the columns below elimination-tree level `cut` fall into independent
// subtrees (a column belongs to its highest ancestor below the cut). One workgroup per subtree (small subtrees
// packed together, at most max_wg workgroups) runs steps [0, cut) of its columns level by level: their factor tasks
// (each with its pull group) and the update groups whose target is one of its columns; a barrier between steps.
// Every column's groups still apply in step order, with the same per-task arithmetic: the factor is bit-identical to
// the level-synchronous schedule. Layout (ints): per workgroup `cut` int4 step entries {first record, tasks, factor
// tasks (first), 0}, then 8-int task records {j, b0, b1, pull group or -1 (factor task) | group, src begin, src end,
// 0, 0}. Returns the number of workgroups; *cost_us = the estimated finish time of the slowest workgroup.
int ba_subtree_plan(const BaPattern& P, int cut, int waves, int max_wg, std::vector<int>* tab, double* cost_us);

// Frontal subtree phase (ba_front_kernel / ba_front_apply_kernel, ba.hip): the columns below elimination-tree level
// `cut` fall into independent subtrees; ONE launch runs one workgroup per subtree with the subtree's factor blocks,
// rhs rows and translated task tables resident in LDS (global -> LDS once, every step an LDS hand-off behind a
// workgroup barrier, LDS -> global once). The subtree's contributions to the columns above the cut are not applied as
// the level's update groups: each workgroup sums them per target column (its sources ascending) into a dense update
// column U_(W,j) laid out like column j's rows (rhs last) in a scratch region, and a second launch adds the U columns
// of every target (workgroups ascending) into L / y. The steps [cut, ...) then run without the groups whose sources
// lie below the cut (every step <= cut; the factor tasks of level `cut` pull nothing). Deterministic (fixed orders),
// but not bit-identical to the group schedules (the below-cut sums are associated per subtree).
// Layout of `tab` (ints): per workgroup an int4 {table offset, table ints (multiple of 4), 0, 0}, then the tables:
//   [16-int header: nslots, ncols, cut, 0, off_rec, off_src, off_sidx, off_slotgb, off_colj, 0...]
//   [cut + 1 int2 steps {first record, tasks}; entry `cut` = the U tasks]
//   [records 8 ints: {kind 0 factor | 1 group | 2 U, slot0, nblk, yslot, src begin, src end, U offset, 0}]
//   [sources int4 {slot of L_jk, yslot of k, sidx offset, 0}] [sidx: per source, per block of the target: slot or -1]
//   [slot -> global block] [yslot -> column]
// LDS image per workgroup: nslots blocks of 56 doubles (rows 0..6 of the 8x8 block), ncols rhs rows of 8 doubles,
// then the table; lds_bytes bounds it. `apply` (ints): napply 8-int entries {j, first block, nblk, list begin, list
// end, 0, 0, 0} (targets ascending), then the lists of U offsets (doubles into the scratch region). Returns the
// number of workgroups (0: the cut does not fit); *u_doubles = the scratch size, *napply = the apply entries.
int ba_front_plan(const BaPattern& P, int cut, size_t lds_bytes, std::vector<int>* tab, std::vector<int>* apply,
                  size_t* u_doubles, int* napply);

// Supernodal factorisation (ba_snode.hip, ba_snode.cpp): chains of consecutive etree columns as supernodes of at most
// `smax` columns, each a dense register panel of one group of 4 waves (7 rows per block row + the rhs row, at most
// `max_rows` rows), left-looking pulls from every descendant column, the supernodal tree cut at a height (cut_req >= 0
// forces it, -1 picks the estimate's best): the subtrees below in a multi-workgroup launch, the rest in one
// workgroup; `groups` groups per workgroup walk list-scheduled supernode lists. Layout (ints):
//   [16-int header: nsn, nwg (bottom workgroups), off_rec, off_pull, off_lists, cut height, groups, smax, max pairs,
//    tree height]
//   [records 8 ints per supernode: {s, R, rows offset, blk offset, pull begin, pull end, child begin, child end}]
//   per supernode: rows (R block rows: its columns, then the rows below), blk (s x R: factor block of L(row ib,
//   column t) or -1), children, per pull its map (R: block of L(row ib, k) or -1)
//   [pulls: 2 ints {k, map offset}]
//   [lists: (nwg + 1) x (groups + 1) item offsets: workgroup w < nwg bottom, w = nwg the top one] [items]
// Offsets are absolute (ints from the table start). Returns the number of supernodes (0: a panel does not fit or the
// pattern breaks the row-subset property: use another solver); *cost_us = the estimated makespan.
int ba_snode_plan(const BaPattern& P, int smax, int groups, int max_rows, int cut_req, std::vector<int>* tab,
                  int* nwg, double* cost_us);
