// Host check of the BA dataflow schedule (ba_pattern.cpp ba_flow_schedule) against the device protocol of
// ba_sparse_factor_kernel's flow path (ba.hip): interprets every wave's task list with the kernel's wait
// conditions (update groups landed per column, source columns factored, x of struct(j) done) one task at a time,
// and fails on a deadlock (no wave can proceed), on an update group applied out of step order, on a factor task
// before all of its column's groups, or on a column left unfinished. Prints the schedule's simulated makespan.
// Graph: a chain of K poses plus `loops` random earlier co-visibility edges per keyframe (both directions), or
// "i j" pairs from a file. build: g++ -O2 -I../lightweight-mast3r-slam_amd/csrc ba_flow_check.cpp
// ../lightweight-mast3r-slam_amd/csrc/ba_pattern.cpp -o /tmp/ba_flow_check
// usage: ba_flow_check K loops seed wide   |   ba_flow_check -f edges.txt wide
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
  int K = 0, wide = 0;
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
  } else if (argc >= 5) {
    K = atoi(argv[1]);
    const int loops = atoi(argv[2]);
    std::mt19937 rng(atoi(argv[3]));
    wide = atoi(argv[4]);
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
  std::vector<int> S;
  ba_flow_schedule(P, wide, W, &S);
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
    expect_tasks += l < P.nlev ? P.lev_ptr[l + 1] - P.lev_ptr[l] : 0;
    expect_tasks += P.grp_ptr[l + 1] - P.grp_ptr[l];
  }
  if (nt != expect_tasks) return fail("task count", nt, expect_tasks);
  for (int j = 0; j < nb; j++)
    if (fac_init[j] != (lev[j] < wide ? 1 : 0)) return fail("fac_init", j);
  std::vector<int> app(nb, 0), fac(nb, 0), last_step(nb, -1), pos(W);
  for (int j = 0; j < nb; j++) fac[j] = fac_init[j] ? 1 : 0;  // the launched wide steps: done
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
  printf("OK K %d E %d nlev %d wide %d tasks %d (max %d per wave) back columns %d (max %d per wave, %d without a "
         "wait)\n",
         K, (int)ri.size(), P.nlev, wide, nt, busiest, nb, longest, nowait);
  return 0;
}
