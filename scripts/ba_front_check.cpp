// Host check of the BA frontal subtree phase (ba_pattern.cpp ba_front_plan) against the device semantics of
// ba_front_kernel / ba_front_apply_kernel and the steps after the cut (ba.hip): a random SPD pose system on the
// plan's pattern (7x7 edge blocks + a diagonal prior) is factored by an interpreter of the translated tables (LDS
// slots, rhs rows, update columns U), then the remaining steps [cut, nlev) without the groups whose sources lie below
// the cut, then the back substitution; x is compared with a dense Cholesky solve of the same system, and with the
// all-groups factorisation (cut 0). Prints the workgroups, the LDS image of the largest one, the scratch size and the
// relative errors; exits 1 on a table inconsistency or an error above 1e-9.
// build: g++ -O2 -std=c++17 -I../lightweight-mast3r-slam_amd/csrc ba_front_check.cpp
//        ../lightweight-mast3r-slam_amd/csrc/ba_pattern.cpp -o /tmp/ba_front_check
// usage: ba_front_check K loops seed cut [lds_kib]   |   ba_front_check -f edges.txt cut [lds_kib]
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "ba_pattern.h"

static int fail(const char* m, long a = -1, long b = -1) {
  printf("FAIL %s (%ld, %ld)\n", m, a, b);
  exit(1);
}

struct Sys {
  std::vector<double> L, y;  // nL x 64, nb x 8 (the device layout)
};

// v -= x L_jk^T, L_jk rows of stride `rs`
static void apply_src(double* v, const double* x, const double* bjk, int rs) {
  for (int c = 0; c < 7; c++) {
    double s = 0.0;
    for (int m = 0; m < 7; m++) s += x[m] * bjk[c * rs + m];
    v[c] -= s;
  }
}

// the factor of one column given its rows (nrow x 8), in place: rows 0..6 the diagonal block, the rest below it
static bool factor_rows(std::vector<double*>& rows) {
  bool ok = true;
  double lo[7][7] = {{0}}, inv[7];
  for (int m = 0; m < 7; m++) {
    double d = rows[m][m];
    if (!(d > 0.0)) {
      ok = false;
      d = 1.0;
    }
    inv[m] = 1.0 / std::sqrt(d);
    for (size_t p = 0; p < rows.size(); p++) {
      if ((int)p == m) continue;
      if (p < 7 && (int)p < m) continue;  // upper part of the diagonal block
      rows[p][m] *= inv[m];
    }
    rows[m][m] = d * inv[m];
    for (int c = m + 1; c < 7; c++) lo[c][m] = rows[c][m];
    for (size_t p = 0; p < rows.size(); p++) {
      if (p < 7 && (int)p <= m) continue;
      for (int c = m + 1; c < 7; c++) rows[p][c] -= rows[p][m] * lo[c][m];
    }
  }
  for (int m = 0; m < 7; m++) rows[m][7] = inv[m];
  return ok;
}

int main(int argc, char** argv) {
  std::vector<int> ri, rj;
  int K = 0, cut = 0, argi = 0;
  if (argc >= 4 && !strcmp(argv[1], "-f")) {
    FILE* f = fopen(argv[2], "r");
    if (!f) fail("cannot open edge file");
    int a, b;
    while (fscanf(f, "%d %d", &a, &b) == 2) {
      ri.push_back(a);
      rj.push_back(b);
      K = std::max(K, std::max(a, b) + 1);
    }
    fclose(f);
    cut = atoi(argv[3]);
    argi = 4;
  } else if (argc >= 5) {
    K = atoi(argv[1]);
    const int loops = atoi(argv[2]);
    std::mt19937 rng(atoi(argv[3]));
    cut = atoi(argv[4]);
    argi = 5;
    for (int k = 1; k < K; k++) {
      ri.push_back(k - 1), rj.push_back(k);
      for (int l = 0; l < loops && k >= 3; l++) {
        const int o = (int)(rng() % (unsigned)(k - 1));
        ri.push_back(o), rj.push_back(k);
      }
    }
  } else {
    fail("usage: ba_front_check K loops seed cut [lds_kib] | -f edges.txt cut [lds_kib]");
  }
  const size_t lds = (size_t)(argc > argi ? atoi(argv[argi]) : 152) * 1024;
  BaPattern P;
  ba_build_pattern(ri.data(), rj.data(), (int)ri.size(), K, &P);
  const int nb = P.nb, nL = P.nL;
  if (nb <= 0) {
    printf("OK nb 0\n");
    return 0;
  }
  // random SPD system on the pattern: per edge a PSD 7x7 block M (i,i)+M (j,j)+M (i,j)-M, a prior on the diagonal
  std::mt19937 rng(12345);
  std::normal_distribution<double> nd;
  const int n = 7 * nb;
  std::vector<double> A((size_t)n * n, 0.0), b(n);
  std::vector<int> pos(nb);
  for (int j = 0; j < nb; j++) pos[P.perm[j]] = j;
  auto add = [&](int r, int c, const double* M, double s) {
    for (int p = 0; p < 7; p++)
      for (int q = 0; q < 7; q++) A[(size_t)(7 * r + p) * n + 7 * c + q] += s * M[p * 7 + q];
  };
  for (size_t e = 0; e < ri.size(); e++) {
    const int io = ri[e] - 1, jo = rj[e] - 1;
    double B[49], M[49];
    for (double& v : B) v = nd(rng);
    for (int p = 0; p < 7; p++)
      for (int q = 0; q < 7; q++) {
        double s = 0;
        for (int t = 0; t < 7; t++) s += B[p * 7 + t] * B[q * 7 + t];
        M[p * 7 + q] = s;
      }
    if (io >= 0) add(pos[io], pos[io], M, 1.0);
    if (jo >= 0) add(pos[jo], pos[jo], M, 1.0);
    if (io >= 0 && jo >= 0) {
      add(pos[io], pos[jo], M, -1.0);
      add(pos[jo], pos[io], M, -1.0);
    }
  }
  for (int i = 0; i < n; i++) A[(size_t)i * n + i] += 1.0;
  for (double& v : b) v = nd(rng);
  // the device layout: lower blocks (row, col) of the permuted system, rhs rows
  auto load = [&](Sys& S) {
    S.L.assign((size_t)nL * 64, 0.0);
    S.y.assign((size_t)nb * 8, 0.0);
    for (int j = 0; j < nb; j++) {
      for (int q = P.col_ptr[j]; q < P.col_ptr[j + 1]; q++) {
        const int i = P.rowL[q];
        for (int p = 0; p < 7; p++)
          for (int c = 0; c < 7; c++) S.L[(size_t)q * 64 + p * 8 + c] = A[(size_t)(7 * i + p) * n + 7 * j + c];
      }
      for (int p = 0; p < 7; p++) S.y[(size_t)j * 8 + p] = b[7 * j + p];
    }
  };
  auto lev_of = [&]() {
    std::vector<int> lev(nb);
    for (int l = 0; l < P.nlev; l++)
      for (int c = P.lev_ptr[l]; c < P.lev_ptr[l + 1]; c++) lev[P.lev_col[c]] = l;
    return lev;
  };
  const std::vector<int> lev = lev_of();
  // global (group) tasks: the rows of column j, sources through P.src / P.sidx
  auto grow = [&](Sys& S, int j, int p) -> double* {
    const int nr = 7 * (P.col_ptr[j + 1] - P.col_ptr[j]);
    return p < nr ? &S.L[(size_t)(P.col_ptr[j] + p / 7) * 64 + (p % 7) * 8] : &S.y[(size_t)j * 8];
  };
  auto g_apply = [&](Sys& S, int j, int g) {
    const int nr = 7 * (P.col_ptr[j + 1] - P.col_ptr[j]) + 1;
    for (int e = P.grp[4 * g + 1]; e < P.grp[4 * g + 2]; e++) {
      const int bjk = P.src[4 * e], k = P.src[4 * e + 1], so = P.src[4 * e + 2];
      for (int p = 0; p < nr; p++) {
        const double* x;
        if (p == nr - 1)
          x = &S.y[(size_t)k * 8];
        else {
          const int sb = P.sidx[so + p / 7];
          if (sb < 0) continue;
          x = &S.L[(size_t)sb * 64 + (p % 7) * 8];
        }
        apply_src(grow(S, j, p), x, &S.L[(size_t)bjk * 64], 8);
      }
    }
  };
  auto g_factor = [&](Sys& S, int j, bool pull) {
    if (pull && P.pull_grp[j] >= 0) g_apply(S, j, P.pull_grp[j]);
    const int nr = 7 * (P.col_ptr[j + 1] - P.col_ptr[j]) + 1;
    std::vector<double*> rows(nr);
    for (int p = 0; p < nr; p++) rows[p] = grow(S, j, p);
    if (!factor_rows(rows)) fail("non-positive pivot", j);
  };
  // steps [from, nlev]: factor tasks (pull unless the column sits at level `cut` with a front phase), then the groups
  // of steps > skip
  auto rest = [&](Sys& S, int from, int skip) {
    for (int l = from; l <= P.nlev; l++) {
      if (l < P.nlev)
        for (int c = P.lev_ptr[l]; c < P.lev_ptr[l + 1]; c++) g_factor(S, P.lev_col[c], !(skip > 0 && l == skip));
      if (skip > 0 && l <= skip) continue;
      for (int t = P.grp_ptr[l]; t < P.grp_ptr[l + 1]; t++) g_apply(S, P.grp[4 * t], t);
    }
  };
  auto back = [&](Sys& S) {
    std::vector<double> x((size_t)nb * 8, 0.0);
    for (int j = nb - 1; j >= 0; j--) {
      double r[7];
      for (int m = 0; m < 7; m++) r[m] = S.y[(size_t)j * 8 + m];
      for (int q = P.col_ptr[j] + 1; q < P.col_ptr[j + 1]; q++) {
        const int i = P.rowL[q];
        for (int m = 0; m < 7; m++)
          for (int c = 0; c < 7; c++) r[m] -= S.L[(size_t)q * 64 + c * 8 + m] * x[(size_t)i * 8 + c];
      }
      const double* D = &S.L[(size_t)P.col_ptr[j] * 64];
      for (int m = 6; m >= 0; m--) {
        double s = r[m];
        for (int c = m + 1; c < 7; c++) s -= D[c * 8 + m] * x[(size_t)j * 8 + c];
        x[(size_t)j * 8 + m] = s * D[m * 8 + 7];
      }
    }
    return x;
  };
  // dense truth
  std::vector<double> C = A, z = b;
  for (int k = 0; k < n; k++) {
    const double d = std::sqrt(C[(size_t)k * n + k]);
    for (int i = k; i < n; i++) C[(size_t)i * n + k] /= d;
    for (int jj = k + 1; jj < n; jj++)
      for (int i = jj; i < n; i++) C[(size_t)i * n + jj] -= C[(size_t)i * n + k] * C[(size_t)jj * n + k];
  }
  for (int i = 0; i < n; i++) {
    double s = z[i];
    for (int k = 0; k < i; k++) s -= C[(size_t)i * n + k] * z[k];
    z[i] = s / C[(size_t)i * n + i];
  }
  for (int i = n - 1; i >= 0; i--) {
    double s = z[i];
    for (int k = i + 1; k < n; k++) s -= C[(size_t)k * n + i] * z[k];
    z[i] = s / C[(size_t)i * n + i];
  }
  auto err = [&](const std::vector<double>& x) {
    double num = 0, den = 0;
    for (int j = 0; j < nb; j++)
      for (int m = 0; m < 7; m++) {
        const double d = x[(size_t)j * 8 + m] - z[7 * j + m];
        num += d * d;
        den += z[7 * j + m] * z[7 * j + m];
      }
    return std::sqrt(num / den);
  };
  Sys G;
  load(G);
  rest(G, 0, 0);
  const double e_groups = err(back(G));
  // the front phase through its tables
  std::vector<int> tab, apl;
  size_t ud = 0;
  int napply = 0;
  const int nwg = ba_front_plan(P, cut, lds, &tab, &apl, &ud, &napply);
  if (nwg == 0) {
    printf("OK nwg 0 (cut %d does not fit) groups_err %.3g\n", cut, e_groups);
    return e_groups < 1e-9 ? 0 : 1;
  }
  Sys F;
  load(F);
  std::vector<double> U(ud, 0.0);
  size_t lds_max = 0;
  int cut_e = 0;
  for (int w = 0; w < nwg; w++) {
    const int* T = tab.data() + tab[4 * w];
    const int tlen = tab[4 * w + 1];
    if (tlen % 4) fail("table length not a multiple of 4", w, tlen);
    const int nslots = T[0], ncols = T[1];
    cut_e = T[2];
    const size_t need = (size_t)nslots * 448 + (size_t)ncols * 64 + (size_t)tlen * 4;
    if (need > lds_max && getenv("FRONT_VERBOSE"))
      printf("wg %d: slots %d cols %d table %d ints (rec %d src %d sidx %d)\n", w, nslots, ncols, tlen, T[5] - T[4],
             T[6] - T[5], T[7] - T[6]);
    lds_max = std::max(lds_max, need);
    std::vector<double> Ls((size_t)nslots * 56), Ys((size_t)ncols * 8);
    const int* slot_gb = T + T[7];
    const int* colj = T + T[8];
    for (int s = 0; s < nslots; s++) {
      if (slot_gb[s] < 0 || slot_gb[s] >= nL) fail("slot -> block", s, slot_gb[s]);
      for (int e = 0; e < 56; e++) Ls[(size_t)s * 56 + e] = F.L[(size_t)slot_gb[s] * 64 + e];
    }
    for (int c = 0; c < ncols; c++)
      for (int e = 0; e < 8; e++) Ys[(size_t)c * 8 + e] = F.y[(size_t)colj[c] * 8 + e];
    const int* rec = T + T[4];
    const int* src = T + T[5];
    const int* sx = T + T[6];
    auto row = [&](int slot0, int nblk, int ys, int p) -> double* {
      if (p < 7 * nblk) {
        if (slot0 + p / 7 >= nslots) fail("row slot", slot0, p);
        return &Ls[(size_t)(slot0 + p / 7) * 56 + (p % 7) * 8];
      }
      if (ys < 0 || ys >= ncols) fail("rhs slot", ys);
      return &Ys[(size_t)ys * 8];
    };
    auto sources = [&](int s0, int s1, int nblk, int p, double* v) {
      for (int e = s0; e < s1; e++) {
        const int* s = src + 4 * e;
        const double* x;
        if (p == 7 * nblk) {
          if (s[1] < 0 || s[1] >= ncols) fail("source rhs slot", s[1]);
          x = &Ys[(size_t)s[1] * 8];
        } else {
          const int sb = sx[s[2] + p / 7];
          if (sb < 0) continue;
          if (sb >= nslots) fail("source slot", sb);
          x = &Ls[(size_t)sb * 56 + (p % 7) * 8];
        }
        if (s[0] < 0 || s[0] >= nslots) fail("L_jk slot", s[0]);
        apply_src(v, x, &Ls[(size_t)s[0] * 56], 8);
      }
    };
    const int* steps = T + 16;
    for (int l = 0; l <= cut_e; l++) {
      for (int t = steps[2 * l]; t < steps[2 * l] + steps[2 * l + 1]; t++) {
        const int* r = rec + 8 * t;
        const int nrow = 7 * r[2] + 1;
        if (r[0] == 2) {
          for (int p = 0; p < nrow; p++) {
            double v[8] = {0};
            sources(r[4], r[5], r[2], p, v);
            for (int c = 0; c < 8; c++) U[(size_t)r[6] + (size_t)p * 8 + c] = v[c];
          }
          continue;
        }
        for (int p = 0; p < nrow; p++) sources(r[4], r[5], r[2], p, row(r[1], r[2], r[3], p));
        if (r[0] == 0) {
          std::vector<double*> rows(nrow);
          for (int p = 0; p < nrow; p++) rows[p] = row(r[1], r[2], r[3], p);
          if (!factor_rows(rows)) fail("non-positive pivot (front)", t);
        }
      }
    }
    for (int s = 0; s < nslots; s++)
      for (int e = 0; e < 56; e++) F.L[(size_t)slot_gb[s] * 64 + e] = Ls[(size_t)s * 56 + e];
    for (int c = 0; c < ncols; c++)
      for (int e = 0; e < 8; e++) F.y[(size_t)colj[c] * 8 + e] = Ys[(size_t)c * 8 + e];
  }
  // apply: L / y += U per target, workgroups ascending
  const int* lists = apl.data() + 8 * napply;
  for (int a = 0; a < napply; a++) {
    const int* e = apl.data() + 8 * a;
    const int j = e[0];
    if (lev[j] < cut_e) fail("apply target below the cut", j);
    if (e[1] != P.col_ptr[j] || e[2] != P.col_ptr[j + 1] - P.col_ptr[j]) fail("apply entry", j);
    for (int p = 0; p < 7 * e[2] + 1; p++) {
      double* v = grow(F, j, p);
      for (int u = e[3]; u < e[4]; u++)
        for (int c = 0; c < 8; c++) v[c] += U[(size_t)lists[u] + (size_t)p * 8 + c];
    }
  }
  rest(F, cut_e, cut_e);
  const double e_front = err(back(F));
  printf("%s nwg %d cut %d lds_max %zu B U %zu doubles napply %d err_front %.3g err_groups %.3g\n",
         e_front < 1e-9 && e_groups < 1e-9 ? "OK" : "FAIL", nwg, cut_e, lds_max, ud, napply, e_front, e_groups);
  return e_front < 1e-9 && e_groups < 1e-9 ? 0 : 1;
}
