// Symbolic analysis of the BA pose system: ordering, factor pattern, level schedule, assembly CSR.
// See ba_pattern.h. Pure host C++ (runs once per BA plan).
#include "ba_pattern.h"

#include <algorithm>
#include <climits>
#include <cstdint>
#include <utility>

namespace {

struct int4_host {
  int x, y, z, w;
};
inline int4_host make_int4_host(int x, int y, int z) { return {x, y, z, 0}; }

inline int popcount_row(const uint64_t* r, int W) {
  int c = 0;
  for (int w = 0; w < W; w++) c += __builtin_popcountll(r[w]);
  return c;
}

}  // namespace

void ba_build_pattern(const int* ri, const int* rj, int E, int Kp, BaPattern* P, size_t max_sidx) {
  max_sidx = std::min<size_t>(max_sidx, (size_t)INT32_MAX / 2);
  const int nb = std::max(0, Kp - 1);
  P->nb = nb;
  const int W = (nb + 63) / 64;
  // adjacency of the pose graph (pin removed), as bitsets; the elimination graph grows in place
  std::vector<uint64_t> adj((size_t)nb * W, 0);
  auto row = [&](int v) { return adj.data() + (size_t)v * W; };
  for (int e = 0; e < E; e++) {
    const int a = ri[e] - 1, b = rj[e] - 1;
    if (a < 0 || b < 0 || a == b) continue;
    row(a)[b >> 6] |= 1ull << (b & 63);
    row(b)[a >> 6] |= 1ull << (a & 63);
  }
  // minimum-degree elimination (exact degrees on the elimination graph; ties to the lowest index)
  std::vector<int> deg(nb), pos(nb, -1), order(nb);
  std::vector<std::vector<int>> nbrs(nb);  // neighbours at elimination time (old indices) = factor column
  for (int v = 0; v < nb; v++) deg[v] = popcount_row(row(v), W);
  std::vector<char> alive(nb, 1);
  std::vector<uint64_t> nb_bits(W);
  for (int step = 0; step < nb; step++) {
    int v = -1;
    for (int u = 0; u < nb; u++)
      if (alive[u] && (v < 0 || deg[u] < deg[v])) v = u;
    order[step] = v;
    pos[v] = step;
    alive[v] = 0;
    const uint64_t* rv = row(v);
    std::copy(rv, rv + W, nb_bits.begin());
    std::vector<int>& nv = nbrs[v];
    for (int w = 0; w < W; w++)
      for (uint64_t m = nb_bits[w]; m; m &= m - 1) nv.push_back(w * 64 + __builtin_ctzll(m));
    for (int a : nv) {  // the neighbours of v become a clique; v leaves the graph
      uint64_t* ra = row(a);
      for (int w = 0; w < W; w++) ra[w] |= nb_bits[w];
      ra[a >> 6] &= ~(1ull << (a & 63));
      ra[v >> 6] &= ~(1ull << (v & 63));
      deg[a] = popcount_row(ra, W);
    }
  }
  // factor pattern in the new order: column j = order[j], rows = pos of its elimination neighbours
  P->perm = order;
  P->col_ptr.assign(nb + 1, 0);
  P->rowL.clear();
  std::vector<int> parent(nb, -1);
  for (int j = 0; j < nb; j++) {
    P->col_ptr[j] = (int)P->rowL.size();
    P->rowL.push_back(j);
    std::vector<int> rows;
    for (int a : nbrs[order[j]]) rows.push_back(pos[a]);
    std::sort(rows.begin(), rows.end());
    if (!rows.empty()) parent[j] = rows[0];
    P->rowL.insert(P->rowL.end(), rows.begin(), rows.end());
  }
  P->col_ptr[nb] = (int)P->rowL.size();
  P->nL = (int)P->rowL.size();
  // levels: leaves 0, a parent one above its highest child (parents come later in the order)
  std::vector<int> lev(nb, 0);
  int nlev = nb > 0 ? 1 : 0;
  for (int j = 0; j < nb; j++) {
    if (parent[j] >= 0) lev[parent[j]] = std::max(lev[parent[j]], lev[j] + 1);
    nlev = std::max(nlev, lev[j] + 1);
  }
  P->nlev = nlev;
  P->lev_ptr.assign(nlev + 1, 0);
  for (int j = 0; j < nb; j++) P->lev_ptr[lev[j] + 1]++;
  for (int l = 0; l < nlev; l++) P->lev_ptr[l + 1] += P->lev_ptr[l];
  P->lev_col.assign(nb, 0);
  {
    std::vector<int> fill(P->lev_ptr.begin(), P->lev_ptr.end() - 1);
    for (int j = 0; j < nb; j++) P->lev_col[fill[lev[j]]++] = j;
  }
  // Updates of column j by the columns k with j in struct(k) (all in lower levels), grouped by the
  // sources' level: one group per (level of k, j), sources ascending, so one wave owns each group and
  // every column's update order is fixed (deterministic: identical on every rank). The group of j's
  // children's level runs inside j's factor task (no barrier between them); the other groups run at the
  // step after their sources' level. Per group source, sidx maps each block b of column j to the block
  // of column k at row rowL[b] (-1 where struct(k) misses that row).
  P->grp_ptr.assign(nlev + 2, 0);
  P->grp.clear();
  P->src.clear();
  P->sidx.clear();
  P->pull_grp.assign(nb, -1);
  std::vector<std::vector<int>> by_tgt(nb);  // j -> sources k of the current level
  // slot[i] / stamp[i]: the block of the current source column k at row i, valid while stamp[i] == k + 1
  std::vector<int> touched, slot(nb, -1), stamp(nb, 0);
  std::vector<int4_host> pull_groups;  // groups run inside factor tasks, appended after the step groups
  P->src.reserve((size_t)4 * P->nL);
  P->sidx.reserve((size_t)8 * P->nL);
  auto emit = [&](int j, const std::vector<int>& ks, std::vector<int4_host>& out) {
    const int s0 = (int)P->src.size() / 4;
    for (int k : ks) {
      int bjk = -1;
      for (int q = P->col_ptr[k] + 1; q < P->col_ptr[k + 1]; q++) {
        slot[P->rowL[q]] = q;
        stamp[P->rowL[q]] = k + 1;
        if (P->rowL[q] == j) bjk = q;
      }
      P->src.push_back(bjk);
      P->src.push_back(k);
      P->src.push_back((int)P->sidx.size());
      P->src.push_back(0);
      for (int b = P->col_ptr[j]; b < P->col_ptr[j + 1]; b++) {
        const int i = P->rowL[b];
        P->sidx.push_back(stamp[i] == k + 1 ? slot[i] : -1);
      }
    }
    out.push_back(make_int4_host(j, s0, (int)P->src.size() / 4));
  };
  std::vector<int4_host> step_groups;
  for (int l = 0; l < nlev; l++) {  // sources at level l
    if (P->sidx.size() > max_sidx) {  // too dense for the plan tables: stop before host memory runs out
      P->too_dense = true;
      return;
    }
    touched.clear();
    for (int c = P->lev_ptr[l]; c < P->lev_ptr[l + 1]; c++) {
      const int k = P->lev_col[c];
      for (int b = P->col_ptr[k] + 1; b < P->col_ptr[k + 1]; b++) {
        const int j = P->rowL[b];
        if (by_tgt[j].empty()) touched.push_back(j);
        by_tgt[j].push_back(k);
      }
    }
    std::sort(touched.begin(), touched.end());
    step_groups.clear();
    for (int j : touched) {
      std::sort(by_tgt[j].begin(), by_tgt[j].end());
      if (lev[j] == l + 1) {
        P->pull_grp[j] = (int)pull_groups.size();
        emit(j, by_tgt[j], pull_groups);
      } else {
        emit(j, by_tgt[j], step_groups);
      }
      by_tgt[j].clear();
    }
    for (const int4_host& gq : step_groups) {
      P->grp.push_back(gq.x);
      P->grp.push_back(gq.y);
      P->grp.push_back(gq.z);
      P->grp.push_back(0);
    }
    P->grp_ptr[l + 2] = (int)P->grp.size() / 4;
  }
  P->grp_ptr[1] = P->grp_ptr[0];
  const int nstep = (int)P->grp.size() / 4;
  for (int j = 0; j < nb; j++)
    if (P->pull_grp[j] >= 0) P->pull_grp[j] += nstep;
  for (const int4_host& gq : pull_groups) {
    P->grp.push_back(gq.x);
    P->grp.push_back(gq.y);
    P->grp.push_back(gq.z);
    P->grp.push_back(0);
  }
  // assembly CSR (SparseBlock::update_lhs/rhs, gn_kernels.cu:71-113): per directed edge the blocks
  // (i,i) +M, (i,j) -M, (j,i) -M, (j,j) +M (M symmetric), lower blocks of the permuted system only,
  // contributions in edge order; rhs: row i takes -g, row j +g
  auto find_blk = [&](int r, int c) {  // new indices, r >= c
    const int* b = P->rowL.data() + P->col_ptr[c];
    const int* e = P->rowL.data() + P->col_ptr[c + 1];
    return (int)(std::lower_bound(b, e, r) - P->rowL.data());
  };
  std::vector<int> ent_blk;
  std::vector<int> ent_val;
  std::vector<int> cnt(P->nL + 1, 0), rcnt(nb + 1, 0);
  ent_blk.reserve((size_t)4 * E);
  ent_val.reserve((size_t)4 * E);
  std::vector<int> rrow, rval;
  rrow.reserve((size_t)2 * E);
  rval.reserve((size_t)2 * E);
  for (int e = 0; e < E; e++) {
    const int io = ri[e] - 1, jo = rj[e] - 1;
    const int rows[4] = {io, io, jo, jo}, cols[4] = {io, jo, io, jo};
    const int neg[4] = {0, 1, 1, 0};
    for (int k = 0; k < 4; k++) {
      if (rows[k] < 0 || cols[k] < 0) continue;
      int r = pos[rows[k]], c = pos[cols[k]];
      if (r < c) continue;  // the lower block of the permuted system: (j,i) and (i,j) are the same -M
      const int b = find_blk(r, c);
      ent_blk.push_back(b);
      ent_val.push_back(e * 2 + neg[k]);
      cnt[b + 1]++;
    }
    if (io >= 0) {
      rrow.push_back(pos[io]);
      rval.push_back(e * 2 + 1);
      rcnt[pos[io] + 1]++;
    }
    if (jo >= 0) {
      rrow.push_back(pos[jo]);
      rval.push_back(e * 2 + 0);
      rcnt[pos[jo] + 1]++;
    }
  }
  for (int b = 0; b < P->nL; b++) cnt[b + 1] += cnt[b];
  for (int j = 0; j < nb; j++) rcnt[j + 1] += rcnt[j];
  P->asm_ptr = cnt;
  P->asm_ent.assign(ent_val.size(), 0);
  {
    std::vector<int> fill(cnt.begin(), cnt.end() - 1);
    for (size_t t = 0; t < ent_val.size(); t++) P->asm_ent[fill[ent_blk[t]]++] = ent_val[t];
  }
  P->rhs_ptr = rcnt;
  P->rhs_ent.assign(rval.size(), 0);
  {
    std::vector<int> fill(rcnt.begin(), rcnt.end() - 1);
    for (size_t t = 0; t < rval.size(); t++) P->rhs_ent[fill[rrow[t]]++] = rval[t];
  }
}

namespace {

// greedy list scheduling: each task (in order) goes to the wave where it can start earliest, given its
// dependencies' finish times (+ hop when a dependency finished on another wave)
struct FlowSim {
  int waves;
  double hop;
  std::vector<double> avail, fin;
  std::vector<int> wave;
  FlowSim(int w, double h) : waves(w), hop(h), avail(w, 0.0) {}
  int place(const std::vector<int>& deps, double cost) {
    int best_w = 0;
    double best = 1e300;
    for (int w = 0; w < waves; w++) {
      double s = avail[w];
      for (int d : deps) s = std::max(s, fin[d] + (wave[d] != w ? hop : 0.0));
      if (s < best - 1e-12) {
        best = s;
        best_w = w;
      }
    }
    wave.push_back(best_w);
    fin.push_back(best + cost);
    avail[best_w] = best + cost;
    return best_w;
  }
};

}  // namespace

namespace {
std::vector<int> col_levels(const BaPattern& P) {
  std::vector<int> lev(P.nb, 0);
  for (int l = 0; l < P.nlev; l++)
    for (int c = P.lev_ptr[l]; c < P.lev_ptr[l + 1]; c++) lev[P.lev_col[c]] = l;
  return lev;
}
// estimated task costs (us) of the flow schedule: a factor task ~1.5 + its pull
// group, an update group ~0.8, ~0.3 per source and 64-row pass (one wave alone on its SIMD issues one fp64
// instruction per ~3.3 ns)
inline int col_passes(const BaPattern& P, int j) { return (7 * (P.col_ptr[j + 1] - P.col_ptr[j]) + 1 + 63) / 64; }
inline int grp_nsrc(const BaPattern& P, int g) { return P.grp[4 * (size_t)g + 2] - P.grp[4 * (size_t)g + 1]; }
inline double factor_cost(const BaPattern& P, int j) {
  const int g = P.pull_grp[j];
  return 1.5 + (g >= 0 ? 0.3 * grp_nsrc(P, g) * col_passes(P, j) : 0.0);
}
inline double group_cost(const BaPattern& P, int g) {
  return 0.8 + 0.3 * grp_nsrc(P, g) * col_passes(P, P.grp[4 * (size_t)g]);
}
}  // namespace

double ba_flow_schedule(const BaPattern& P, int wide, int waves, std::vector<int>* sched) {
  const int nb = P.nb, nlev = P.nlev;
  sched->clear();
  if (nb <= 0) return 0.0;
  const std::vector<int> lev = col_levels(P);
  const int done_below = std::max(wide, 0);  // columns factored before the one-workgroup kernel starts
  // estimated task costs (factor_cost / group_cost), hand-off ~0.15 us
  FlowSim F(waves, 0.15);
  std::vector<std::pair<int, int>> tasks;  // {code, q}
  std::vector<int> fac_task(nb, -1), last_grp(nb, -1), napplied(nb, 0), deps;
  auto src_deps = [&](int g) {
    for (int e = P.grp[4 * (size_t)g + 1]; e < P.grp[4 * (size_t)g + 2]; e++) {
      const int k = P.src[4 * (size_t)e + 1];
      if (fac_task[k] >= 0) deps.push_back(fac_task[k]);
    }
  };
  for (int l = std::max(0, wide); l <= nlev; l++) {
    if (l < nlev)
      for (int c = P.lev_ptr[l]; c < P.lev_ptr[l + 1]; c++) {
        const int j = P.lev_col[c], g = P.pull_grp[j];
        deps.clear();
        if (last_grp[j] >= 0) deps.push_back(last_grp[j]);
        if (g >= 0) src_deps(g);
        fac_task[j] = (int)tasks.size();
        tasks.push_back({j, napplied[j]});
        F.place(deps, factor_cost(P, j));
      }
    for (int t = P.grp_ptr[l]; t < P.grp_ptr[l + 1]; t++) {
      const int j = P.grp[4 * (size_t)t];
      deps.clear();
      if (last_grp[j] >= 0) deps.push_back(last_grp[j]);
      src_deps(t);
      last_grp[j] = (int)tasks.size();
      tasks.push_back({-1 - t, napplied[j]++});
      F.place(deps, group_cost(P, t));
    }
  }
  double makespan = 0.0;
  for (double f : F.fin) makespan = std::max(makespan, f);
  // back substitution: parents first (a parent has the higher index); x_j needs x of struct(j), which the parent's
  // own wait already covered (struct(j) \ {parent} lies in struct(parent))
  FlowSim B(waves, 0.15);
  std::vector<int> bcol, bwave(nb, -1), btask(nb, -1);
  for (int j = nb - 1; j >= 0; j--) {
    deps.clear();
    if (P.col_ptr[j + 1] - P.col_ptr[j] > 1 && btask[P.rowL[P.col_ptr[j] + 1]] >= 0)
      deps.push_back(btask[P.rowL[P.col_ptr[j] + 1]]);
    btask[j] = (int)bcol.size();
    bcol.push_back(j);
    bwave[j] = B.place(deps, 0.7 + 0.02 * (P.col_ptr[j + 1] - P.col_ptr[j]));
  }
  const int nt = (int)tasks.size();
  sched->assign(2 * (waves + 1) + nb + 2 * (size_t)nt + bcol.size(), 0);
  int* wl_ptr = sched->data();
  int* bs_ptr = wl_ptr + waves + 1;
  int* fac_init = bs_ptr + waves + 1;
  int* wl_task = fac_init + nb;
  int* bs_col = wl_task + 2 * (size_t)nt;
  for (int k = 0; k < nb; k++) fac_init[k] = lev[k] < done_below ? 1 : 0;
  for (int w = 0, o = 0, ob = 0; w < waves; w++) {
    wl_ptr[w] = o;
    for (int i = 0; i < nt; i++)
      if (F.wave[i] == w) {
        wl_task[2 * o] = tasks[i].first;
        wl_task[2 * o + 1] = tasks[i].second;
        o++;
      }
    wl_ptr[w + 1] = o;
    bs_ptr[w] = ob;
    int prev = -1;
    for (size_t i = 0; i < bcol.size(); i++)
      if (B.wave[i] == w) {
        const int j = bcol[i];
        const bool has_p = P.col_ptr[j + 1] - P.col_ptr[j] > 1;
        // the wave's previous column is j's parent (or j is a root): struct(j) is done, no wait
        const bool own = !has_p || P.rowL[P.col_ptr[j] + 1] == prev;
        bs_col[ob++] = j | (own ? BA_BS_NOWAIT : 0);
        prev = j;
      }
    bs_ptr[w + 1] = ob;
  }
  return makespan;
}

