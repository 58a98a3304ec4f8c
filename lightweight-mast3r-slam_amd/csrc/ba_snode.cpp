// Supernodal plan of the BA pose system's Cholesky factorisation (ba_snode.hip; ba_pattern.h ba_snode_plan).
//
// The reference factors the pose system with Eigen's SimplicialLLT (gn_kernels.cu:57-159): column by column. On the
// GPU a column-by-column schedule is a chain of ~70 dependent single-wave tasks (the elimination tree's height), each
// paying a global round trip and a cross-wave hand-off. Here columns that form a chain of the elimination tree (each
// the only child of the next) are grouped into supernodes of at most smax columns;
// a supernode is factored as one dense panel held in the registers of a group of 4 waves (one panel row per lane):
//   * its panel rows are its own columns followed by the rows below its top column (the etree row-subset property
//     puts every column's structure inside them), plus the right-hand side as one extra row (the forward
//     substitution rides along as the augmented row);
//   * it PULLS the updates of every descendant column k whose structure meets its columns (left-looking): rows of
//     L(:, k) times the 7x7 blocks L(c, k)^T, k ascending (a fixed order: every rank computes the same factor);
//   * then a dense 7x7-blocked right-looking Cholesky of the panel, two group barriers per column;
// The supernodal tree is cut at a height: the subtrees below run as ONE multi-workgroup launch (whole subtrees per
// workgroup, no cross-workgroup dependency), the part above in one workgroup; inside a workgroup, 4 groups walk
// list-scheduled supernode lists (children before parents) with LDS completion flags.
#include <algorithm>
#include <cstdio>
#include <numeric>
#include <vector>

#include "ba_pattern.h"

namespace {

struct Sn {
  std::vector<int> cols;  // ascending, a chain: cols[t + 1] = parent(cols[t])
  std::vector<int> rows;  // panel block rows: cols, then the rows below the top column (ascending)
  std::vector<int> blk;   // s x R: factor block of L(rows[ib], cols[t]) or -1
  std::vector<int> pulls;  // descendant columns k (ascending)
  std::vector<std::vector<int>> maps;  // per pull, R entries: block of L(rows[ib], k) or -1
  std::vector<int> child;  // child supernodes
  int parent = -1;
  int height = 0;
  int npairs = 0;  // sum over pulls of the columns hit
};

// estimated cost (us) of one supernode on a group of 4 waves: the panel's loads and the pull operands' L2 round
// trip, ~0.1 us per (pull column, hit column) pair of 49 FMAs + 28 loads on 3 waves, ~0.45 us per column of the dense
// panel factorisation (two group barriers + a lane-redundant 7x7 Cholesky + the trailing update), the stores
double sn_cost(const Sn& S) { return 1.2 + 0.1 * S.npairs + 0.45 * S.cols.size(); }

struct GroupSim {  // greedy list scheduling of supernodes (ascending) onto groups
  int groups;
  double hop;
  std::vector<double> avail;
  std::vector<double> fin;  // by supernode
  std::vector<int> grp;     // by supernode
  GroupSim(int g, double h, int nsn) : groups(g), hop(h), avail(g, 0.0), fin(nsn, 0.0), grp(nsn, -1) {}
  void place(int s, const std::vector<Sn>& sn, const std::vector<char>& here, double cost) {
    int best_g = 0;
    double best = 1e300;
    for (int g = 0; g < groups; g++) {
      double t = avail[g];
      for (int c : sn[s].child)
        if (here[c]) t = std::max(t, fin[c] + (grp[c] != g ? hop : 0.0));
      if (t < best - 1e-12) {
        best = t;
        best_g = g;
      }
    }
    grp[s] = best_g;
    fin[s] = best + cost;
    avail[best_g] = best + cost;
  }
};

}  // namespace

int ba_snode_plan(const BaPattern& P, int smax, int groups, int max_rows, int cut_req, std::vector<int>* tab,
                  int* nwg_out, double* cost_us) {
  tab->clear();
  *nwg_out = 0;
  *cost_us = 0.0;
  const int nb = P.nb;
  if (nb <= 0) return 0;
  std::vector<int> parent(nb, -1), nchild(nb, 0);
  for (int j = 0; j < nb; j++)
    if (P.col_ptr[j + 1] - P.col_ptr[j] > 1) {
      parent[j] = P.rowL[P.col_ptr[j] + 1];
      nchild[parent[j]]++;
    }
  auto nblk = [&](int j) { return P.col_ptr[j + 1] - P.col_ptr[j]; };
  // chain amalgamation: column j joins the supernode of its only child c when c is that supernode's top (the
  // columns need not be consecutive), capped at smax columns and max_rows panel rows. A child supernode starts at a
  // lower column than its parent's first, so supernode indices are a topological order (children first).
  std::vector<Sn> sn;
  std::vector<int> sn_of(nb, -1), only_child(nb, -1);
  for (int j = 0; j < nb; j++)
    if (parent[j] >= 0) only_child[parent[j]] = nchild[parent[j]] == 1 ? j : -1;
  for (int j = 0; j < nb; j++) {
    if (7 * nblk(j) + 1 > max_rows) return 0;  // one column alone does not fit a group's panel
    const int c = only_child[j];
    int S = -1;
    if (c >= 0) {
      const Sn& cur = sn[sn_of[c]];
      const int s = (int)cur.cols.size();
      if (cur.cols.back() == c && s < smax && 7 * (s + nblk(j)) + 1 <= max_rows) S = sn_of[c];
    }
    if (S < 0) {
      S = (int)sn.size();
      sn.emplace_back();
    }
    sn[S].cols.push_back(j);
    sn_of[j] = S;
  }
  const int nsn = (int)sn.size();
  std::vector<int> ib_of(nb, -1);
  for (int S = 0; S < nsn; S++) {
    Sn& X = sn[S];
    const int s = (int)X.cols.size(), top = X.cols.back();
    X.rows = X.cols;
    for (int b = P.col_ptr[top] + 1; b < P.col_ptr[top + 1]; b++) X.rows.push_back(P.rowL[b]);
    const int R = (int)X.rows.size();
    if (7 * R + 1 > max_rows) return 0;
    for (int ib = 0; ib < R; ib++) ib_of[X.rows[ib]] = ib;
    X.blk.assign((size_t)s * R, -1);
    for (int t = 0; t < s; t++)
      for (int b = P.col_ptr[X.cols[t]]; b < P.col_ptr[X.cols[t] + 1]; b++) {
        const int ib = ib_of[P.rowL[b]];
        if (ib < t) return 0;  // the etree row-subset property guarantees rows >= t inside the panel
        X.blk[(size_t)t * R + ib] = b;
      }
    for (int ib = 0; ib < R; ib++) ib_of[X.rows[ib]] = -1;
    X.parent = parent[top] >= 0 ? sn_of[parent[top]] : -1;
  }
  for (int S = 0; S < nsn; S++)
    if (sn[S].parent >= 0) sn[sn[S].parent].child.push_back(S);
  // pulls: descendant column k -> every supernode (other than its own) holding a column of struct(k)
  for (int k = 0; k < nb; k++)
    for (int b = P.col_ptr[k] + 1; b < P.col_ptr[k + 1]; b++) {
      const int S = sn_of[P.rowL[b]];
      if (S == sn_of[k]) continue;
      if (sn[S].pulls.empty() || sn[S].pulls.back() != k) sn[S].pulls.push_back(k);
    }
  for (int S = 0; S < nsn; S++) {
    Sn& X = sn[S];
    const int R = (int)X.rows.size(), s = (int)X.cols.size();
    for (int ib = 0; ib < R; ib++) ib_of[X.rows[ib]] = ib;
    for (int k : X.pulls) {
      std::vector<int> mp(R, -1);
      int first = -1;  // the lowest column of this supernode in struct(k)
      for (int b = P.col_ptr[k] + 1; b < P.col_ptr[k + 1] && first < 0; b++)
        if (sn_of[P.rowL[b]] == S) first = P.rowL[b];
      for (int b = P.col_ptr[k] + 1; b < P.col_ptr[k + 1]; b++) {
        const int i = P.rowL[b];
        if (i < first) continue;     // rows between k and this supernode: not its business
        if (ib_of[i] < 0) return 0;  // (row-subset property) every row >= the first hit lies in the panel
        mp[ib_of[i]] = b;
      }
      for (int t = 0; t < s; t++) X.npairs += mp[t] >= 0;
      X.maps.push_back(std::move(mp));
    }
    for (int ib = 0; ib < R; ib++) ib_of[X.rows[ib]] = -1;
  }
  int hmax = 0;
  for (int S = 0; S < nsn; S++) {  // children have lower indices
    for (int c : sn[S].child) sn[S].height = std::max(sn[S].height, sn[c].height + 1);
    hmax = std::max(hmax, sn[S].height);
  }
  std::vector<double> cost(nsn);
  for (int S = 0; S < nsn; S++) cost[S] = sn_cost(sn[S]);
  // the cut: supernodes of height < H run in the multi-workgroup launch (whole subtrees per workgroup), the rest in
  // the one-workgroup launch. Minimise the estimate: slowest bottom workgroup + a launch + the top makespan.
  const int max_wg = 128;
  auto evaluate = [&](int H, std::vector<int>* wg_of, int* nwg) {
    wg_of->assign(nsn, -1);
    std::vector<int> roots;
    for (int S = 0; S < nsn; S++)
      if (sn[S].height < H && (sn[S].parent < 0 || sn[sn[S].parent].height >= H)) roots.push_back(S);
    // subtree of each root: cost sum; LPT packing onto workgroups
    std::vector<int> root_of(nsn, -1);
    for (int S = nsn - 1; S >= 0; S--)
      if (sn[S].height < H) root_of[S] = (sn[S].parent >= 0 && sn[sn[S].parent].height < H) ? root_of[sn[S].parent] : S;
    std::vector<double> rc(nsn, 0.0);
    for (int S = 0; S < nsn; S++)
      if (root_of[S] >= 0) rc[root_of[S]] += cost[S];
    std::sort(roots.begin(), roots.end(), [&](int x, int y) { return rc[x] > rc[y] || (rc[x] == rc[y] && x < y); });
    *nwg = std::min((int)roots.size(), max_wg);
    std::vector<double> load(*nwg, 0.0);
    std::vector<int> wg_root(nsn, -1);
    for (int r : roots) {
      const int w = (int)(std::min_element(load.begin(), load.end()) - load.begin());
      load[w] += rc[r] / groups;
      wg_root[r] = w;
    }
    for (int S = 0; S < nsn; S++)
      if (root_of[S] >= 0) (*wg_of)[S] = wg_root[root_of[S]];
    // per workgroup list scheduling (bottom), then the top workgroup
    double bottom = 0.0;
    std::vector<char> here(nsn);
    for (int w = 0; w < *nwg; w++) {
      GroupSim G(groups, 0.3, nsn);
      for (int S = 0; S < nsn; S++) here[S] = (*wg_of)[S] == w;
      for (int S = 0; S < nsn; S++)
        if (here[S]) G.place(S, sn, here, cost[S]);
      for (double a : G.avail) bottom = std::max(bottom, a);
    }
    GroupSim G(groups, 0.3, nsn);
    for (int S = 0; S < nsn; S++) here[S] = (*wg_of)[S] < 0;
    for (int S = 0; S < nsn; S++)
      if (here[S]) G.place(S, sn, here, cost[S]);
    double top = 0.0;
    for (double a : G.avail) top = std::max(top, a);
    return (*nwg > 0 ? bottom + 2.0 : 0.0) + top;
  };
  int bestH = 0;
  double best = 1e300;
  std::vector<int> wg_of;
  int nwg = 0;
  for (int H = 0; H <= hmax + 1; H++) {
    if (cut_req >= 0 && H != std::min(cut_req, hmax + 1)) continue;
    const double c = evaluate(H, &wg_of, &nwg);
    if (c < best - 1e-9) {
      best = c;
      bestH = H;
    }
  }
  *cost_us = evaluate(bestH, &wg_of, &nwg);
  // per workgroup (nwg bottom ones, then the top one) and group: the supernode lists
  std::vector<std::vector<int>> lists((size_t)(nwg + 1) * groups);
  std::vector<char> here(nsn);
  for (int w = 0; w <= nwg; w++) {
    GroupSim G(groups, 0.3, nsn);
    for (int S = 0; S < nsn; S++) here[S] = (w < nwg) ? wg_of[S] == w : wg_of[S] < 0;
    for (int S = 0; S < nsn; S++)
      if (here[S]) {
        G.place(S, sn, here, cost[S]);
        lists[(size_t)w * groups + G.grp[S]].push_back(S);
      }
  }
  // the table (ints): header, records, then the variable sections
  std::vector<int>& T = *tab;
  T.assign(16, 0);
  auto put = [&](const std::vector<int>& v) {
    const int off = (int)T.size();
    T.insert(T.end(), v.begin(), v.end());
    return off;
  };
  T[0] = nsn;
  T[1] = nwg;
  T[2] = (int)T.size();
  T.resize(T.size() + 8 * (size_t)nsn, 0);
  std::vector<int> pull_ents;
  for (int S = 0; S < nsn; S++) {
    const Sn& X = sn[S];
    int* r = nullptr;
    const int ro = put(X.rows), bo = put(X.blk), co = put(X.child);
    const int pb = (int)pull_ents.size() / 2;
    for (size_t q = 0; q < X.pulls.size(); q++) {
      const int mo = put(X.maps[q]);
      pull_ents.push_back(X.pulls[q]);
      pull_ents.push_back(mo);
    }
    r = &T[T[2] + 8 * (size_t)S];
    r[0] = (int)X.cols.size();
    r[1] = (int)X.rows.size();
    r[2] = ro;
    r[3] = bo;
    r[4] = pb;
    r[5] = (int)pull_ents.size() / 2;
    r[6] = co;
    r[7] = co + (int)X.child.size();
  }
  T[3] = put(pull_ents);
  // lists: (nwg + 1) x (groups + 1) absolute item offsets, then the items
  const int lo = (int)T.size();
  T.resize(T.size() + (size_t)(nwg + 1) * (groups + 1), 0);
  T[4] = lo;
  for (int w = 0; w <= nwg; w++)
    for (int g = 0; g < groups; g++) {
      T[lo + w * (groups + 1) + g] = (int)T.size();
      const std::vector<int>& L = lists[(size_t)w * groups + g];
      T.insert(T.end(), L.begin(), L.end());
      T[lo + w * (groups + 1) + g + 1] = (int)T.size();
    }
  T[5] = bestH;
  T[6] = groups;
  T[7] = smax;
  int maxpairs = 0;
  for (const Sn& X : sn) maxpairs = std::max(maxpairs, X.npairs);
  T[8] = maxpairs;
  T[9] = hmax + 1;
  *nwg_out = nwg;
  return nsn;
}
