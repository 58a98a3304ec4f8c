// CPU check of the supernodal plan (ba_snode.cpp, ba_pattern.h ba_snode_plan) with the kernel's semantics
// (ba_snode.hip): on a random SPD block system with a BA graph's pattern (random graphs, or an "i j" edge file), the
// table is interpreted exactly as the kernel does (per supernode: the panel rows' A entries, the pulls in table order,
// the 7x7-blocked right-looking panel Cholesky, the stores into the factor blocks / rhs rows), the workgroup lists are
// replayed with the kernel's wait rules (a group runs its next supernode once its children are done; every list must
// drain: no deadlock), and the factor and forward-substituted rhs are compared with a dense Cholesky of the same
// system. Exit status 0 when every case matches to 1e-9 (relative).
// build: g++ -O2 -I../lightweight-mast3r-slam_amd/csrc ba_snode_check.cpp ../lightweight-mast3r-slam_amd/csrc/ba_pattern.cpp
//        ../lightweight-mast3r-slam_amd/csrc/ba_snode.cpp -o /tmp/ba_snode_check
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "ba_pattern.h"

static int check(const std::vector<int>& ri, const std::vector<int>& rj, int Kp, int smax, int cut, unsigned seed,
                 const char* name, bool may_not_fit = false) {
  BaPattern P;
  ba_build_pattern(ri.data(), rj.data(), (int)ri.size(), Kp, &P);
  const int nb = P.nb, n = 7 * nb;
  std::vector<int> tab;
  int nwg = 0;
  double est = 0.0;
  const int ngr = getenv("SN_GROUPS") ? atoi(getenv("SN_GROUPS")) : 4;
  const int nsn = ba_snode_plan(P, smax, ngr, 256, cut, &tab, &nwg, &est);
  if (nsn <= 0) {  // a column or panel wider than a group's 256 lanes: the plan declines (the column solver runs)
    printf("%s: no supernodal plan%s\n", name, may_not_fit ? " (too dense: declined)" : "");
    return may_not_fit ? 0 : 1;
  }
  // random SPD system in factor order: A = sum over edges of [B; -B][B; -B]^T (7x7 B per edge) + diag
  std::mt19937 rng(seed);
  std::normal_distribution<double> nd(0.0, 1.0);
  std::vector<int> inv_perm(Kp, -1);  // pose rank -> factor column (rank 0 pinned)
  for (int j = 0; j < nb; j++) inv_perm[P.perm[j] + 1] = j;
  std::vector<double> A((size_t)n * n, 0.0), b(n);
  for (size_t e = 0; e < ri.size(); e++) {
    double B[49];
    for (double& x : B) x = nd(rng);
    const int ci = inv_perm[ri[e]], cj = inv_perm[rj[e]];
    const int cs[2] = {ci, cj};
    const double sg[2] = {1.0, -1.0};
    for (int u = 0; u < 2; u++)
      for (int v = 0; v < 2; v++) {
        if (cs[u] < 0 || cs[v] < 0) continue;
        for (int r = 0; r < 7; r++)
          for (int c = 0; c < 7; c++) {
            double s = 0.0;
            for (int k = 0; k < 7; k++) s += B[r * 7 + k] * B[c * 7 + k];
            A[(size_t)(7 * cs[u] + r) * n + 7 * cs[v] + c] += sg[u] * sg[v] * s;
          }
      }
  }
  for (int i = 0; i < n; i++) {
    A[(size_t)i * n + i] += 1.0;
    b[i] = nd(rng);
  }
  // block storage (8x8 per factor block) with A's lower blocks; y = b
  std::vector<double> L((size_t)P.nL * 64, 0.0), y((size_t)nb * 8, 0.0);
  for (int j = 0; j < nb; j++)
    for (int q = P.col_ptr[j]; q < P.col_ptr[j + 1]; q++) {
      const int i = P.rowL[q];
      for (int r = 0; r < 7; r++)
        for (int c = 0; c < 7; c++) L[(size_t)q * 64 + r * 8 + c] = A[(size_t)(7 * i + r) * n + 7 * j + c];
    }
  for (int j = 0; j < nb; j++)
    for (int c = 0; c < 7; c++) y[(size_t)j * 8 + c] = b[7 * j + c];
  // one supernode with the kernel's per-lane arithmetic
  const int* T = tab.data();
  auto factor_sn = [&](int S) {
    const int* rec = T + T[2] + 8 * S;
    const int s = rec[0], R = rec[1];
    const int* rows = T + rec[2];
    const int* blk = T + rec[3];
    const int nrow = 7 * R + 1;
    std::vector<double> v((size_t)nrow * 7 * s, 0.0), inv_own(nrow, 0.0);
    auto V = [&](int p, int t, int c) -> double& { return v[((size_t)p * s + t) * 7 + c]; };
    for (int p = 0; p < nrow; p++) {
      const bool rhs = p == 7 * R;
      const int ib = p / 7, m = p % 7;
      for (int t = 0; t < s; t++) {
        const double* src = nullptr;
        if (rhs) src = &y[(size_t)rows[t] * 8];
        else if (ib >= t && blk[t * R + ib] >= 0) src = &L[(size_t)blk[t * R + ib] * 64 + m * 8];
        for (int c = 0; c < 7; c++) V(p, t, c) = src ? src[c] : 0.0;
      }
    }
    const int* pl = T + T[3];
    for (int q = rec[4]; q < rec[5]; q++) {
      const int k = pl[2 * q];
      const int* map = T + pl[2 * q + 1];
      for (int p = 0; p < nrow; p++) {
        const bool rhs = p == 7 * R;
        const int ib = p / 7, m = p % 7;
        const double* src = rhs ? &y[(size_t)k * 8] : (map[ib] >= 0 ? &L[(size_t)map[ib] * 64 + m * 8] : nullptr);
        if (!src) continue;
        for (int t = 0; t < s; t++) {
          if (map[t] < 0) continue;
          const double* B = &L[(size_t)map[t] * 64];
          for (int c = 0; c < 7; c++) {
            double acc = 0.0;
            for (int mm = 0; mm < 7; mm++) acc = std::fma(src[mm], B[c * 8 + mm], acc);
            V(p, t, c) -= acc;
          }
        }
      }
    }
    for (int t = 0; t < s; t++) {
      double D[7][7], inv[7];
      for (int i = 0; i < 7; i++)
        for (int c = 0; c < 7; c++) D[i][c] = V(7 * t + i, t, c);
      for (int c = 0; c < 7; c++) {
        const double d = D[c][c];
        if (!(d > 0.0)) return false;
        inv[c] = 1.0 / std::sqrt(d);
        D[c][c] = d * inv[c];
        for (int i = c + 1; i < 7; i++) D[i][c] *= inv[c];
        for (int i = c + 1; i < 7; i++)
          for (int jj = c + 1; jj <= i; jj++) D[i][jj] = std::fma(-D[i][c], D[jj][c], D[i][jj]);
      }
      for (int p = 0; p < nrow; p++) {
        const bool rhs = p == 7 * R;
        const int ib = p / 7, m = p % 7;
        if (!rhs && ib == t) {
          for (int c = 0; c < 7; c++) V(p, t, c) = c <= m ? D[m][c] : 0.0;
          inv_own[p] = inv[m];
        } else if (rhs || ib > t) {
          for (int c = 0; c < 7; c++) {
            V(p, t, c) *= inv[c];
            for (int c2 = c + 1; c2 < 7; c2++) V(p, t, c2) = std::fma(-V(p, t, c), D[c2][c], V(p, t, c2));
          }
        }
      }
      for (int t2 = t + 1; t2 < s; t2++)
        for (int p = 0; p < nrow; p++) {
          const bool rhs = p == 7 * R;
          const int ib = p / 7;
          if (!(rhs || ib >= t2)) continue;
          for (int c = 0; c < 7; c++) {
            double acc = 0.0;
            for (int mm = 0; mm < 7; mm++) acc = std::fma(V(p, t, mm), V(7 * t2 + c, t, mm), acc);
            V(p, t2, c) -= acc;
          }
        }
    }
    for (int p = 0; p < nrow; p++) {
      const bool rhs = p == 7 * R;
      const int ib = p / 7, m = p % 7;
      for (int t = 0; t < s; t++) {
        if (rhs) {
          for (int c = 0; c < 7; c++) y[(size_t)rows[t] * 8 + c] = V(p, t, c);
        } else if (ib >= t && blk[t * R + ib] >= 0) {
          double* dst = &L[(size_t)blk[t * R + ib] * 64 + m * 8];
          for (int c = 0; c < 7; c++) dst[c] = V(p, t, c);
          if (ib == t) dst[7] = inv_own[p];
        }
      }
    }
    return true;
  };
  // replay the workgroup lists: bottom workgroups (any interleaving), then the top one; a group's head runs when its
  // children are done
  const int groups = T[6];
  std::vector<char> done(nsn, 0);
  int ran = 0;
  for (int w = 0; w <= nwg; w++) {
    const int* lp = T + T[4] + w * (groups + 1);
    std::vector<int> head(groups);
    for (int g = 0; g < groups; g++) head[g] = lp[g];
    bool progress = true;
    while (progress) {
      progress = false;
      for (int g = 0; g < groups; g++) {
        if (head[g] >= lp[g + 1]) continue;
        const int S = T[head[g]];
        const int* rec = T + T[2] + 8 * S;
        bool ready = true;
        for (int c = rec[6]; c < rec[7]; c++) ready = ready && done[T[c]];
        if (!ready) continue;
        if (!factor_sn(S)) {
          printf("%s: non-positive pivot\n", name);
          return 1;
        }
        done[S] = 1;
        ran++;
        head[g]++;
        progress = true;
      }
    }
    for (int g = 0; g < groups; g++)
      if (head[g] < lp[g + 1]) {
        printf("%s: workgroup %d group %d stalls at supernode %d\n", name, w, g, T[head[g]]);
        return 1;
      }
  }
  if (ran != nsn) {
    printf("%s: %d of %d supernodes ran\n", name, ran, nsn);
    return 1;
  }
  // dense Cholesky + forward substitution
  std::vector<double> D = A, z = b;
  for (int j = 0; j < n; j++) {
    double d = D[(size_t)j * n + j];
    for (int k = 0; k < j; k++) d -= D[(size_t)j * n + k] * D[(size_t)j * n + k];
    d = std::sqrt(d);
    D[(size_t)j * n + j] = d;
    for (int i = j + 1; i < n; i++) {
      double s = D[(size_t)i * n + j];
      for (int k = 0; k < j; k++) s -= D[(size_t)i * n + k] * D[(size_t)j * n + k];
      D[(size_t)i * n + j] = s / d;
    }
  }
  for (int i = 0; i < n; i++) {
    double s = z[i];
    for (int k = 0; k < i; k++) s -= D[(size_t)i * n + k] * z[k];
    z[i] = s / D[(size_t)i * n + i];
  }
  double err = 0.0, scale = 1e-300;
  for (int j = 0; j < nb; j++)
    for (int q = P.col_ptr[j]; q < P.col_ptr[j + 1]; q++) {
      const int i = P.rowL[q];
      for (int r = 0; r < 7; r++)
        for (int c = 0; c < 7; c++) {
          if (i == j && c > r) continue;
          const double want = D[(size_t)(7 * i + r) * n + 7 * j + c];
          err = std::max(err, std::fabs(L[(size_t)q * 64 + r * 8 + c] - want));
          scale = std::max(scale, std::fabs(want));
        }
    }
  for (int j = 0; j < nb; j++)
    for (int c = 0; c < 7; c++) {
      err = std::max(err, std::fabs(y[(size_t)j * 8 + c] - z[7 * j + c]));
      scale = std::max(scale, std::fabs(z[7 * j + c]));
    }
  const double rel = err / scale;
  int maxs = 0;
  for (int S = 0; S < nsn; S++) maxs = std::max(maxs, T[T[2] + 8 * S]);
  printf("%s: nb %d nL %d supernodes %d (max cols %d) bottom workgroups %d cut %d/%d est %.1f us: rel err %.2e\n", name,
         nb, P.nL, nsn, maxs, nwg, T[5], T[9], est, rel);
  return rel < 1e-9 ? 0 : 1;
}

int main(int argc, char** argv) {
  int bad = 0;
  if (argc > 1) {  // edge file
    FILE* f = fopen(argv[1], "r");
    if (!f) return 2;
    std::vector<int> ri, rj;
    int a, b, K = 0;
    while (fscanf(f, "%d %d", &a, &b) == 2) {
      ri.push_back(a);
      rj.push_back(b);
      K = std::max(K, std::max(a, b) + 1);
    }
    fclose(f);
    for (int cut : {-1, 0, 2, 5, 100}) bad |= check(ri, rj, K, 4, cut, 7, argv[1]);
    bad |= check(ri, rj, K, 1, -1, 8, argv[1]);
    bad |= check(ri, rj, K, 2, -1, 8, argv[1]);
    bad |= check(ri, rj, K, 6, -1, 9, argv[1]);
    return bad;
  }
  // random trajectory-like graphs: a chain plus loop edges
  std::mt19937 rng(3);
  for (int trial = 0; trial < 12; trial++) {
    const int K = 8 + (int)(rng() % 120);
    std::vector<int> ri, rj;
    for (int k = 1; k < K; k++) {
      ri.push_back(k - 1);
      rj.push_back(k);
      const int loops = rng() % 4;
      for (int l = 0; l < loops && k > 2; l++) {
        const int i = rng() % (k - 1);
        ri.push_back(i);
        rj.push_back(k);
      }
    }
    const int n0 = (int)ri.size();
    for (int e = 0; e < n0; e++) {  // both directions, as FactorGraph stores them
      ri.push_back(rj[e]);
      rj.push_back(ri[e]);
    }
    char name[64];
    snprintf(name, sizeof(name), "random K=%d", K);
    bad |= check(ri, rj, K, 1 + trial % 6, trial % 3 == 0 ? -1 : (int)(rng() % 6), 100 + trial, name, true);
  }
  return bad;
}
