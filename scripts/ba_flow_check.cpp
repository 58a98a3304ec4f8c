// Host check of the BA dataflow schedule (ba_pattern.cpp ba_flow_schedule) against the device protocol of
// ba_sparse_factor_kernel's flow path (ba.hip): interprets every wave's task list with the kernel's wait
// conditions (update groups landed per column, source columns factored, x of struct(j) done) one task at a time,
// and fails on a deadlock (no wave can proceed), on an update group applied out of step order, on a factor task
// before all of its column's groups, or on a column left unfinished. Prints the schedule's simulated makespan.
// Graph: a chain of K poses plus `loops` random earlier co-visibility edges per keyframe (both directions), or
// "i j" pairs from a file. build: g++ -O2 -I../lightweight-mast3r-slam_amd/csrc ba_flow_check.cpp
// ../lightweight-mast3r-slam_amd/csrc/ba_pattern.cpp -o /tmp/ba_flow_check
// usage: ba_flow_check K loops seed wide [sub]   |   ba_flow_check -f edges.txt wide [sub]
// sub > 0 (with wide 0): the subtree phase (ba_subtree_plan, ba_subtree_kernel) runs steps [0, sub) first, step by
// step with its workgroups' tasks, under the same checks; sub = -1: the plan's cost-model cut (as abi.cpp).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "ba_pattern.h"

static int fail(const char* m, int a = -1, int b = -1) {
  printf("FAIL %s (%d, %d)\n", m, a, b);
  return 1;
}

int main(int argc, char** argv) {
  std::vector<int> ri, rj;
  int K = 0, wide = 0, sub = 0;
  if (argc >= 3 && !strcmp(argv[1], "-f")) {
    FILE* f = fopen(argv[2], "r");
    if (!f) return fail("cannot open edge file");
    int a, b;
    while (fscanf(f, "%d %d", &a, &b) == 2) {
      ri.push_back(a);
      rj.push_back(b);
      K = std::max(K, std::max(a, b) + 1);
    }
    fclose(f);
    wide = argc > 3 ? atoi(argv[3]) : 0;
    sub = argc > 4 ? atoi(argv[4]) : 0;
  } else if (argc >= 5) {
    K = atoi(argv[1]);
    const int loops = atoi(argv[2]);
    std::mt19937 rng(atoi(argv[3]));
    wide = atoi(argv[4]);
    sub = argc > 5 ? atoi(argv[5]) : 0;
    for (int k = 1; k < K; k++) {
      ri.push_back(k - 1), rj.push_back(k);
      ri.push_back(k), rj.push_back(k - 1);
      for (int l = 0; l < loops && k >= 3; l++) {
        const int o = (int)(rng() % (unsigned)(k - 1));
        ri.push_back(o), rj.push_back(k);
        ri.push_back(k), rj.push_back(o);
      }
    }
  } else {
    return fail("usage: ba_flow_check K loops seed wide | -f edges.txt wide");
  }
  BaPattern P;
  ba_build_pattern(ri.data(), rj.data(), (int)ri.size(), K, &P);
  const int nb = P.nb, W = 16;
  wide = std::min(wide, P.nlev + 1);
  if (sub < 0) {  // the cost-model cut of abi.cpp (subtree launch ~4 us + slowest workgroup + the flow makespan)
    double best = 1e300;
    std::vector<int> ts, tt;
    for (int c = 0; c < std::min(P.nlev + 1, 40); c++) {
      double su = 0.0;
      if (c > 0) ba_subtree_plan(P, c, 8, 128, &tt, &su);
      const double t = (c > 0 ? 4.0 + su : 0.0) + ba_flow_schedule(P, 0, W, &ts, c);
      if (t < best - 1e-9) best = t, sub = c;
    }
  }
  sub = std::min(sub, P.nlev);
  if (sub > 0) wide = 0;
  std::vector<int> S, T;
  ba_flow_schedule(P, wide, W, &S, sub);
  double sub_cost = 0.0;
  const int nwg = sub > 0 ? ba_subtree_plan(P, sub, 8, 128, &T, &sub_cost) : 0;
  if (sub > 0 && nwg <= 0 && P.nb > 0) return fail("subtree plan without workgroups", sub);
  if (nb == 0) {
    printf("OK empty\n");
    return 0;
  }
  const int* wl_ptr = S.data();
  const int* bs_ptr = wl_ptr + W + 1;
  const int* fac_init = bs_ptr + W + 1;
  const int nt = wl_ptr[W];
  const int* wl = fac_init + nb;
  const int* bs_col = wl + 2 * nt;
  if ((int)S.size() != 2 * (W + 1) + nb + 2 * nt + nb) return fail("schedule size");
  // level of each column; the expected group order per target = step order
  std::vector<int> lev(nb);
  for (int l = 0; l < P.nlev; l++)
    for (int c = P.lev_ptr[l]; c < P.lev_ptr[l + 1]; c++) lev[P.lev_col[c]] = l;
  int expect_tasks = 0;
  for (int l = wide; l <= P.nlev; l++) {
    if (l >= sub) expect_tasks += l < P.nlev ? P.lev_ptr[l + 1] - P.lev_ptr[l] : 0;
    for (int t = P.grp_ptr[l]; t < P.grp_ptr[l + 1]; t++) expect_tasks += (l >= sub || lev[P.grp[4 * t]] >= sub) ? 1 : 0;
  }
  if (nt != expect_tasks) return fail("task count", nt, expect_tasks);
  for (int j = 0; j < nb; j++)
    if (fac_init[j] != (lev[j] < std::max(wide, sub) ? 1 : 0)) return fail("fac_init", j);
  std::vector<int> app(nb, 0), fac(nb, 0), last_step(nb, -1), pos(W);
  for (int j = 0; j < nb; j++) fac[j] = (sub == 0 && fac_init[j]) ? 1 : 0;  // the launched wide steps: done
  auto step_of_group_ = [&](int g) {
    int l = 0;
    while (!(P.grp_ptr[l] <= g && g < P.grp_ptr[l + 1])) l++;
    return l;
  };
  auto srcs_done_ = [&](int g) {
    if (g < 0) return true;
    for (int e = P.grp[4 * g + 1]; e < P.grp[4 * g + 2]; e++)
      if (!fac[P.src[4 * e + 1]]) return false;
    return true;
  };
  // the subtree phase: step by step; within a step every task of every workgroup is independent (checked: a
  // factor task's groups all landed in earlier steps, a group's sources are factored and its target is not)
  std::vector<int> sub_app(nb, 0), owner(nb, -1);
  int sub_tasks = 0;
  for (int l = 0; l < sub; l++) {
    for (int w = 0; w < nwg; w++) {
      const int* e = T.data() + ((size_t)w * sub + l) * 4;
      const int* rec = T.data() + (size_t)nwg * sub * 4;
      for (int t = 0; t < e[1]; t++) {
        const int* r = rec + 8 * (size_t)(e[0] + t);
        const int j = r[0];
        if (r[1] != P.col_ptr[j] || r[2] != P.col_ptr[j + 1]) return fail("subtree record blocks", j);
        if (owner[j] >= 0 && owner[j] != w) return fail("column touched by two subtree workgroups", j);
        owner[j] = w;
        if (t < e[2]) {  // factor task
          if (lev[j] != l) return fail("subtree factor task at the wrong step", j, l);
          if (r[3] != P.pull_grp[j]) return fail("subtree factor task pull group", j);
          if (!srcs_done_(r[3])) return fail("subtree factor task before its sources", j);
          for (int g = P.grp_ptr[0]; g < P.grp_ptr[P.nlev + 1]; g++)
            if (P.grp[4 * g] == j && step_of_group_(g) < l && last_step[j] < step_of_group_(g))
              return fail("subtree factor before its update groups", j, g);
          if (fac[j]) return fail("column factored twice", j);
        } else {
          const int g = r[3];
          if (P.grp[4 * g] != j || step_of_group_(g) != l) return fail("subtree group record", j, g);
          if (lev[j] >= sub) return fail("subtree group with a target above the cut", j, g);
          if (!srcs_done_(g)) return fail("subtree group before its sources", j, g);
          if (fac[j]) return fail("subtree update after the target was factored", j, g);
          if (l <= last_step[j]) return fail("subtree groups out of step order", j, g);
        }
        sub_tasks++;
      }
    }
    // apply the step's effects after all its tasks were checked (they run concurrently)
    for (int w = 0; w < nwg; w++) {
      const int* e = T.data() + ((size_t)w * sub + l) * 4;
      const int* rec = T.data() + (size_t)nwg * sub * 4;
      for (int t = 0; t < e[1]; t++) {
        const int* r = rec + 8 * (size_t)(e[0] + t);
        if (t < e[2]) fac[r[0]] = 1;
        else last_step[r[0]] = l;
      }
    }
  }
  for (int j = 0; j < nb; j++)
    if (lev[j] < sub && !fac[j]) return fail("subtree column never factored", j);
  for (int w = 0; w < W; w++) pos[w] = wl_ptr[w];
  auto step_of_group = [&](int g) {
    int l = 0;
    while (!(P.grp_ptr[l] <= g && g < P.grp_ptr[l + 1])) l++;
    return l;
  };
  auto srcs_done = [&](int g) {
    if (g < 0) return true;
    for (int e = P.grp[4 * g + 1]; e < P.grp[4 * g + 2]; e++)
      if (!fac[P.src[4 * e + 1]]) return false;
    return true;
  };
  int done = 0;
  while (done < nt) {
    bool moved = false;
    for (int w = 0; w < W; w++) {
      if (pos[w] >= wl_ptr[w + 1]) continue;
      const int code = wl[2 * pos[w]], q = wl[2 * pos[w] + 1];
      if (code >= 0) {
        const int j = code, g = P.pull_grp[j];
        if (app[j] != q || !srcs_done(g)) continue;
        for (int t = P.grp_ptr[0]; t < P.grp_ptr[P.nlev + 1]; t++)  // every step group on j has landed
          if (P.grp[4 * t] == j && step_of_group(t) >= wide && last_step[j] < step_of_group(t))
            return fail("factor before its update groups", j, t);
        if (fac[j]) return fail("column factored twice", j);
        fac[j] = 1;
      } else {
        const int g = -1 - code, j = P.grp[4 * g];
        if (app[j] != q || !srcs_done(g)) continue;
        const int st = step_of_group(g);
        if (st <= last_step[j]) return fail("update groups out of step order", j, g);
        if (fac[j]) return fail("update after the target was factored", j, g);
        last_step[j] = st;
        app[j]++;
      }
      pos[w]++;
      done++;
      moved = true;
    }
    if (!moved) return fail("factor deadlock", done, nt);
  }
  for (int j = 0; j < nb; j++)
    if (!fac[j]) return fail("column never factored", j);
  // back substitution
  std::vector<int> xd(nb, 0), seen(nb, 0);
  for (int w = 0; w < W; w++) pos[w] = bs_ptr[w];
  int bdone = 0;
  if (bs_ptr[W] != nb) return fail("back-substitution list size", bs_ptr[W], nb);
  while (bdone < nb) {
    bool moved = false;
    for (int w = 0; w < W; w++) {
      if (pos[w] >= bs_ptr[w + 1]) continue;
      const int j = bs_col[pos[w]] & BA_BS_COL;
      bool ok = true;
      for (int b = P.col_ptr[j] + 1; b < P.col_ptr[j + 1]; b++) ok = ok && xd[P.rowL[b]];
      if (bs_col[pos[w]] & BA_BS_NOWAIT) {
        if (!ok) return fail("no-wait column whose struct is not done", j);
      } else if (!ok) {
        continue;
      }
      if (seen[j]++) return fail("column solved twice", j);
      xd[j] = 1;
      pos[w]++;
      bdone++;
      moved = true;
    }
    if (!moved) return fail("back-substitution deadlock", bdone, nb);
  }
  int longest = 0, busiest = 0, nowait = 0;
  for (int t = 0; t < nb; t++) nowait += (bs_col[t] & BA_BS_NOWAIT) ? 1 : 0;
  for (int w = 0; w < W; w++) {
    busiest = std::max(busiest, wl_ptr[w + 1] - wl_ptr[w]);
    longest = std::max(longest, bs_ptr[w + 1] - bs_ptr[w]);
  }
  printf("OK K %d E %d nlev %d wide %d sub %d (%d workgroups, %d tasks, est %.1f us) tasks %d (max %d per wave) back "
         "columns %d (max %d per wave, %d without a wait)\n",
         K, (int)ri.size(), P.nlev, wide, sub, nwg, sub_tasks, sub_cost, nt, busiest, nb, longest, nowait);
  return 0;
}
