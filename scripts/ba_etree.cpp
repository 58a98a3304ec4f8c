// Elimination-tree census of a BA pose graph under the library's symbolic analysis (ba_pattern.cpp):
// per level the columns and factor blocks, and for each cut level L the subtrees below it (roots at level <= L
// whose parent lies above L): their count, the largest one's columns / blocks / height. Input: "i j" per
// directed edge (pose ranks, 0 = pinned). build: g++ -O2 -I../lightweight-mast3r-slam_amd/csrc ba_etree.cpp
// ../lightweight-mast3r-slam_amd/csrc/ba_pattern.cpp -o /tmp/ba_etree
#include <algorithm>
#include <cstdio>
#include <vector>

#include "ba_pattern.h"

int main(int argc, char** argv) {
  FILE* f = fopen(argv[1], "r");
  std::vector<int> ri, rj;
  int a, b, K = 0;
  while (fscanf(f, "%d %d", &a, &b) == 2) {
    ri.push_back(a);
    rj.push_back(b);
    K = std::max(K, std::max(a, b) + 1);
  }
  BaPattern P;
  ba_build_pattern(ri.data(), rj.data(), (int)ri.size(), K, &P);
  const int nb = P.nb;
  std::vector<int> parent(nb, -1), lev(nb, 0), nblk(nb);
  for (int j = 0; j < nb; j++) {
    nblk[j] = P.col_ptr[j + 1] - P.col_ptr[j];
    if (nblk[j] > 1) parent[j] = P.rowL[P.col_ptr[j] + 1];
  }
  for (int l = 0; l < P.nlev; l++)
    for (int c = P.lev_ptr[l]; c < P.lev_ptr[l + 1]; c++) lev[P.lev_col[c]] = l;
  printf("nb %d nL %d nlev %d\nlevel: columns blocks\n", nb, P.nL, P.nlev);
  for (int l = 0; l < P.nlev; l++) {
    int bl = 0;
    for (int c = P.lev_ptr[l]; c < P.lev_ptr[l + 1]; c++) bl += nblk[P.lev_col[c]];
    printf("%d:%d/%d ", l, P.lev_ptr[l + 1] - P.lev_ptr[l], bl);
  }
  printf("\n");
  // subtree sizes (columns, blocks), children before parents in the order
  std::vector<int> scol(nb, 1), sblk(nblk);
  for (int j = 0; j < nb; j++)
    if (parent[j] >= 0) {
      scol[parent[j]] += scol[j];
      sblk[parent[j]] += sblk[j];
    }
  for (int L = 0; L < P.nlev; L += (L < 40 ? 2 : 8)) {
    int n = 0, mc = 0, mb = 0, tc = 0;
    for (int j = 0; j < nb; j++)
      if (lev[j] <= L && (parent[j] < 0 || lev[parent[j]] > L)) {
        n++;
        tc += scol[j];
        if (scol[j] > mc) {
          mc = scol[j];
          mb = sblk[j];
        }
      }
    printf("cut %2d: %3d subtrees, %3d columns below, largest %3d columns %4d blocks (%6.1f KB fp64)\n", L, n, tc, mc,
           mb, mb * 49 * 8 / 1024.0);
  }
  return 0;
}
