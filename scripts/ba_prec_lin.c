/* Precision experiment for the rays-mode BA linearisation: which fp32 stage of the HIP
 * build's rows (csrc/ba.hip ba_lin_kernel<BA_MODE_RAYS> + ba_edge_kernel) carries the coherent error that puts the
 * C4 EuRoC 320x512 K=256 graph 2.45e-5 from the fp64 truth. Not test or product code: scripts/ba_prec_exp.py drives it.
 *
 * Every stage is computed in double; a stage whose bit is set in `flags` rounds each of its operations to fp32
 * ((double)(float)x after every +,-,*,/,sqrt is exactly the fp32 operation: double has > 2*24+2 bits), so a build
 * with every bit set emulates the fp32 HIP arithmetic (up to its 1-ulp rsq/rcp estimates and the fma double
 * rounding) and flags = 0 is the fp64 truth's arithmetic. Reference rows: gn_kernels.cu:813-1138.
 *   bit 0 POSE  poses rounded to fp32 on entry (the HIP build stores Twc as float)
 *   bit 1 REL   relSim3 (T_ij = T_i^-1 T_j) in fp32
 *   bit 2 MAP   D = sR - I rounded to fp32, Y = X + fma(D, X, t) in fp32
 *   bit 3 REC   the record: r_i = X_i/|X_i|, |X_i| in fp32
 *   bit 4 NRM   |Y|^2, 1/|Y|, r_j = Y/|Y|, |Y| in fp32
 *   bit 5 ERR   residuals r_j - r_i, |Y| - |X_i| in fp32
 *   bit 6 JAC   Jacobian entries (n3, d_ab) in fp32
 *   bit 7 WGT   weights sqrt(q), huber in fp32
 *   bit 8 PROD  products w J J^T, w e J in fp32, summed in fp32 runs of 16 points per slot (512 slots per chunk)
 *   bit 9 ADJ   adjoint map A of T_i in fp32 (M = A L A^T in double)
 * build: gcc -O2 -fopenmp -fPIC -shared -ffp-contract=off scripts/ba_prec_lin.c -o /tmp/libbaprec.so -lm */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define B_POSE 1
#define B_REL 2
#define B_MAP 4
#define B_REC 8
#define B_NRM 16
#define B_ERR 32
#define B_JAC 64
#define B_WGT 128
#define B_PROD 256
#define B_ADJ 512

static inline double R(double x, int f) { return f ? (double)(float)x : x; }

static void quat_comp(const double* qi, const double* qj, double* o, int f) {
  o[0] = R(R(R(R(qi[3] * qj[0], f) + R(qi[0] * qj[3], f), f) + R(qi[1] * qj[2], f), f) - R(qi[2] * qj[1], f), f);
  o[1] = R(R(R(R(qi[3] * qj[1], f) - R(qi[0] * qj[2], f), f) + R(qi[1] * qj[3], f), f) + R(qi[2] * qj[0], f), f);
  o[2] = R(R(R(R(qi[3] * qj[2], f) + R(qi[0] * qj[1], f), f) - R(qi[1] * qj[0], f), f) + R(qi[2] * qj[3], f), f);
  o[3] = R(R(R(R(qi[3] * qj[3], f) - R(qi[0] * qj[0], f), f) - R(qi[1] * qj[1], f), f) - R(qi[2] * qj[2], f), f);
}

static void actSO3(const double* q, const double* X, double* Y, int f) {
  const double u0 = R(2.0 * R(R(q[1] * X[2], f) - R(q[2] * X[1], f), f), f);
  const double u1 = R(2.0 * R(R(q[2] * X[0], f) - R(q[0] * X[2], f), f), f);
  const double u2 = R(2.0 * R(R(q[0] * X[1], f) - R(q[1] * X[0], f), f), f);
  const double y0 = R(R(X[0] + R(q[3] * u0, f), f) + R(R(q[1] * u2, f) - R(q[2] * u1, f), f), f);
  const double y1 = R(R(X[1] + R(q[3] * u1, f), f) + R(R(q[2] * u0, f) - R(q[0] * u2, f), f), f);
  const double y2 = R(R(X[2] + R(q[3] * u2, f), f) + R(R(q[0] * u1, f) - R(q[1] * u0, f), f), f);
  Y[0] = y0;
  Y[1] = y1;
  Y[2] = y2;
}

static void relSim3(const double* Ti, const double* Tj, double* Tij, int f) {
  const double si_inv = R(1.0 / Ti[7], f);
  Tij[7] = R(si_inv * Tj[7], f);
  const double qi[4] = {-Ti[3], -Ti[4], -Ti[5], Ti[6]};
  quat_comp(qi, &Tj[3], &Tij[3], f);
  double t[3] = {R(Tj[0] - Ti[0], f), R(Tj[1] - Ti[1], f), R(Tj[2] - Ti[2], f)};
  actSO3(qi, t, t, f);
  for (int c = 0; c < 3; c++) Tij[c] = R(t[c] * si_inv, f);
}

static void adj_inv_row(const double* Ti, const double* X, double* Y, int f) {
  const double s_inv = R(1.0 / Ti[7], f);
  double Ra[3];
  actSO3(&Ti[3], &X[0], Ra, f);
  for (int c = 0; c < 3; c++) Y[c] = R(s_inv * Ra[c], f);
  actSO3(&Ti[3], &X[3], &Y[3], f);
  Y[3] = R(Y[3] + R(s_inv * R(R(Ti[1] * Ra[2], f) - R(Ti[2] * Ra[1], f), f), f), f);
  Y[4] = R(Y[4] + R(s_inv * R(R(Ti[2] * Ra[0], f) - R(Ti[0] * Ra[2], f), f), f), f);
  Y[5] = R(Y[5] + R(s_inv * R(R(Ti[0] * Ra[1], f) - R(Ti[1] * Ra[0], f), f), f), f);
  Y[6] = R(X[6] + R(s_inv * R(R(R(Ti[0] * Ra[0], f) + R(Ti[1] * Ra[1], f), f) + R(Ti[2] * Ra[2], f), f), f), f);
}

static inline double huber(double r, int f) {
  const double a = fabs(r);
  return a < 1.345 ? 1.0 : R(1.345 / a, f);
}

/* 35 local sums (28 L upper + 7 v) of one row */
static inline void row_sums(double* s, const double* J, double w, double e, int f) {
  int l = 0;
  for (int c = 0; c < 7; c++) {
    const double wj = R(w * J[c], f);
    for (int d = c; d < 7; d++, l++) s[l] = wj * J[d];
    s[28 + c] = wj * e;
  }
}

#define SLOTS 512
#define RUN 16

void prec_lin_rays(int flags, const double* Twc_in, const float* Xs, const float* Cs, int N, int E, int chunk,
                   const int64_t* ii_rank, const int64_t* jj_rank, const int64_t* idx, const uint8_t* valid,
                   const float* Q, double sigma_ray, double sigma_dist, double C_thresh, double Q_thresh,
                   double* Hs /* 4 x E x 49 */, double* gs /* 2 x E x 7 */) {
  const int fP = flags & B_POSE, fR = flags & B_REL, fM = flags & B_MAP, fC = flags & B_REC, fN = flags & B_NRM,
            fE = flags & B_ERR, fJ = flags & B_JAC, fW = flags & B_WGT, fS = flags & B_PROD, fA = flags & B_ADJ;
#pragma omp parallel
  {
    float* run = (float*)malloc(sizeof(float) * SLOTS * 35);
#pragma omp for schedule(dynamic, 1)
    for (int e = 0; e < E; e++) {
      const int ix = (int)ii_rank[e], jx = (int)jj_rank[e];
      double Ti[8], Tj[8], Tij[8];
      for (int c = 0; c < 8; c++) {
        Ti[c] = R(Twc_in[ix * 8 + c], fP);
        Tj[c] = R(Twc_in[jx * 8 + c], fP);
      }
      relSim3(Ti, Tj, Tij, fR);
      /* D = sR - I in double from T_ij, then rounded (MAP) */
      double D[9];
      {
        const double x = Tij[3], y = Tij[4], z = Tij[5], w = Tij[6], sc = Tij[7];
        const double Rm[9] = {1.0 - 2.0 * (y * y + z * z), 2.0 * (x * y - z * w),       2.0 * (x * z + y * w),
                              2.0 * (x * y + z * w),       1.0 - 2.0 * (x * x + z * z), 2.0 * (y * z - x * w),
                              2.0 * (x * z - y * w),       2.0 * (y * z + x * w),       1.0 - 2.0 * (x * x + y * y)};
        for (int c = 0; c < 9; c++) D[c] = R(sc * Rm[c] - ((c % 4 == 0) ? 1.0 : 0.0), fM);
      }
      const double t[3] = {R(Tij[0], fM), R(Tij[1], fM), R(Tij[2], fM)};
      const double sa_inv = 1.0 / sigma_ray, sb_inv = 1.0 / sigma_dist;
      double acc[35];
      memset(acc, 0, sizeof(acc));
      for (int k0 = 0; k0 < N; k0 += chunk) {
        const int k1 = k0 + chunk < N ? k0 + chunk : N;
        if (fS) memset(run, 0, sizeof(float) * SLOTS * 35);
        for (int k = k0; k < k1; k++) {
          const size_t g = (size_t)e * N + k;
          const int vm = valid[g] != 0;
          const int64_t ind = vm ? idx[g] : 0;
          const float* Xi = &Xs[((size_t)ix * N + ind) * 3];
          const float* Xj = &Xs[((size_t)jx * N + k) * 3];
          const float q = Q[g];
          const int ok = vm && (q > Q_thresh) && (Cs[(size_t)ix * N + ind] > C_thresh) &&
                         (Cs[(size_t)jx * N + k] > C_thresh);
          const double sq = ok ? R(sqrt((double)q), fW) : 0.0;
          /* record */
          const double n2i = R(R(R((double)Xi[0] * Xi[0], fC) + R((double)Xi[1] * Xi[1], fC), fC) +
                                   R((double)Xi[2] * Xi[2], fC), fC);
          const double invi = R(1.0 / sqrt(n2i), fC);
          const double n1i = R(n2i * invi, fC);
          const double ri[3] = {R(invi * Xi[0], fC), R(invi * Xi[1], fC), R(invi * Xi[2], fC)};
          /* map */
          double Y[3];
          for (int c = 0; c < 3; c++) {
            double a;
            if (fM) {
              a = (double)fmaf((float)D[3 * c + 2], Xj[2], (float)t[c]);
              a = (double)fmaf((float)D[3 * c + 1], Xj[1], (float)a);
              a = (double)fmaf((float)D[3 * c], Xj[0], (float)a);
              Y[c] = R(Xj[c] + a, 1);
            } else {
              Y[c] = Xj[c] + (D[3 * c] * Xj[0] + D[3 * c + 1] * Xj[1] + D[3 * c + 2] * Xj[2] + t[c]);
            }
          }
          const double n2j = R(R(R(Y[0] * Y[0], fN) + R(Y[1] * Y[1], fN), fN) + R(Y[2] * Y[2], fN), fN);
          const double inv = R(1.0 / sqrt(n2j), fN);
          const double n1j = R(n2j * inv, fN);
          const double rj[3] = {R(inv * Y[0], fN), R(inv * Y[1], fN), R(inv * Y[2], fN)};
          const double err[4] = {R(rj[0] - ri[0], fE), R(rj[1] - ri[1], fE), R(rj[2] - ri[2], fE), R(n1j - n1i, fE)};
          const double swr = R(sa_inv * sq, fW), swd = R(sb_inv * sq, fW);
          const double wr = R(swr * swr, fW), wd = R(swd * swd, fW);
          const double n3 = R(inv * R(1.0 / n2j, fJ), fJ);
          const double dxx = R(inv - R(R(Y[0] * Y[0], fJ) * n3, fJ), fJ);
          const double dyy = R(inv - R(R(Y[1] * Y[1], fJ) * n3, fJ), fJ);
          const double dzz = R(inv - R(R(Y[2] * Y[2], fJ) * n3, fJ), fJ);
          const double dxy = -R(R(Y[0] * Y[1], fJ) * n3, fJ);
          const double dxz = -R(R(Y[0] * Y[2], fJ) * n3, fJ);
          const double dyz = -R(R(Y[1] * Y[2], fJ) * n3, fJ);
          const double J[4][7] = {{dxx, dxy, dxz, 0, rj[2], -rj[1], 0},
                                  {dxy, dyy, dyz, -rj[2], 0, rj[0], 0},
                                  {dxz, dyz, dzz, rj[1], -rj[0], 0, 0},
                                  {rj[0], rj[1], rj[2], 0, 0, 0, n1j}};
          for (int r = 0; r < 4; r++) {
            const double sw = r < 3 ? swr : swd, w0 = r < 3 ? wr : wd;
            const double w = R(huber(R(sw * err[r], fW), fW) * w0, fW);
            if (w == 0.0) continue;
            double s[35];
            row_sums(s, J[r], w, err[r], fS);
            if (fS) {
              float* sl = run + (size_t)((k - k0) % SLOTS) * 35;
              for (int l = 0; l < 35; l++) {
                /* fp32 fma of the rounded w*J[c] (row_sums) and J[d] into the slot's run */
                sl[l] = (float)((double)sl[l] + s[l]);
              }
            } else {
              for (int l = 0; l < 35; l++) acc[l] += s[l];
            }
          }
          if (fS && ((k - k0) % (SLOTS * RUN)) == SLOTS * RUN - 1) {
            for (int l = 0; l < SLOTS * 35; l++) {
              acc[l % 35] += (double)run[l];
              run[l] = 0.0f;
            }
          }
        }
        if (fS) {
          for (int l = 0; l < SLOTS * 35; l++) {
            acc[l % 35] += (double)run[l];
            run[l] = 0.0f;
          }
        }
      }
      /* M = A L A^T, g = A v with A = adj_inv_row(T_i) columns */
      double L[7][7], v[7], A[7][7];
      {
        int l = 0;
        for (int c = 0; c < 7; c++)
          for (int d = c; d < 7; d++, l++) L[c][d] = L[d][c] = acc[l];
        for (int c = 0; c < 7; c++) v[c] = acc[28 + c];
      }
      double TiA[8];
      for (int c = 0; c < 8; c++) TiA[c] = R(Ti[c], fA);
      for (int c = 0; c < 7; c++) {
        double X[7] = {0, 0, 0, 0, 0, 0, 0}, Yc[7];
        X[c] = 1.0;
        adj_inv_row(TiA, X, Yc, fA);
        for (int r = 0; r < 7; r++) A[r][c] = Yc[r];
      }
      double AL[7][7], M[7][7], gv[7];
      for (int r = 0; r < 7; r++)
        for (int c = 0; c < 7; c++) {
          double s = 0;
          for (int k = 0; k < 7; k++) s += A[r][k] * L[k][c];
          AL[r][c] = s;
        }
      for (int r = 0; r < 7; r++) {
        for (int c = 0; c < 7; c++) {
          double s = 0;
          for (int k = 0; k < 7; k++) s += AL[r][k] * A[c][k];
          M[r][c] = s;
        }
        double s = 0;
        for (int k = 0; k < 7; k++) s += A[r][k] * v[k];
        gv[r] = s;
      }
      for (int r = 0; r < 7; r++) {
        for (int c = 0; c < 7; c++) {
          Hs[((size_t)0 * E + e) * 49 + r * 7 + c] = M[r][c];
          Hs[((size_t)1 * E + e) * 49 + r * 7 + c] = -M[r][c];
          Hs[((size_t)2 * E + e) * 49 + r * 7 + c] = -M[r][c];
          Hs[((size_t)3 * E + e) * 49 + r * 7 + c] = M[r][c];
        }
        gs[(size_t)e * 7 + r] = -gv[r];
        gs[((size_t)E + e) * 7 + r] = gv[r];
      }
    }
    free(run);
  }
}
