// Shared device helpers for the MI355X (gfx950) kernels of the tracking hot path.
//
// Sim(3) math follows the reference's device restatement of lietorch
// (/root/reference/mast3r_slam/backend/src/gn_kernels.cu:172-413) with pose layout
// [t(3), q(4, xyzw), s] and tangent layout [tau(3), phi(3), sigma]. Double-typed literals of the
// reference are kept in double where they change the float result.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define M3S_WAVE 64

namespace m3s {

__device__ __forceinline__ void quat_comp(const float* qi, const float* qj, float* out) {
  out[0] = qi[3] * qj[0] + qi[0] * qj[3] + qi[1] * qj[2] - qi[2] * qj[1];
  out[1] = qi[3] * qj[1] - qi[0] * qj[2] + qi[1] * qj[3] + qi[2] * qj[0];
  out[2] = qi[3] * qj[2] + qi[0] * qj[1] - qi[1] * qj[0] + qi[2] * qj[3];
  out[3] = qi[3] * qj[3] - qi[0] * qj[0] - qi[1] * qj[1] - qi[2] * qj[2];
}

__device__ __forceinline__ void actSO3(const float* q, const float* X, float* Y) {
  float uv0 = 2.0f * (q[1] * X[2] - q[2] * X[1]);  // 2.0*(float) in double == exact doubling
  float uv1 = 2.0f * (q[2] * X[0] - q[0] * X[2]);
  float uv2 = 2.0f * (q[0] * X[1] - q[1] * X[0]);
  float y0 = X[0] + q[3] * uv0 + (q[1] * uv2 - q[2] * uv1);
  float y1 = X[1] + q[3] * uv1 + (q[2] * uv0 - q[0] * uv2);
  float y2 = X[2] + q[3] * uv2 + (q[0] * uv1 - q[1] * uv0);
  Y[0] = y0;
  Y[1] = y1;
  Y[2] = y2;
}

__device__ __forceinline__ void actSim3(const float* T, const float* X, float* Y) {
  actSO3(&T[3], X, Y);
  Y[0] = Y[0] * T[7] + T[0];
  Y[1] = Y[1] * T[7] + T[1];
  Y[2] = Y[2] * T[7] + T[2];
}

// T_ij = T_i^-1 T_j   (gn_kernels.cu:252-272)
__device__ __forceinline__ void relSim3(const float* Ti, const float* Tj, float* Tij) {
  const float si_inv = 1.0f / Ti[7];
  Tij[7] = si_inv * Tj[7];
  const float qi_inv[4] = {-Ti[3], -Ti[4], -Ti[5], Ti[6]};
  quat_comp(qi_inv, &Tj[3], &Tij[3]);
  float t[3] = {Tj[0] - Ti[0], Tj[1] - Ti[1], Tj[2] - Ti[2]};
  actSO3(qi_inv, t, t);
  Tij[0] = t[0] * si_inv;
  Tij[1] = t[1] * si_inv;
  Tij[2] = t[2] * si_inv;
}

// Row-vector adjoint-inverse map of a local Jacobian row (gn_kernels.cu:277-297).
__device__ __forceinline__ void adj_inv_row(const float* Ti, const float* X, float* Y) {
  const float s_inv = 1.0f / Ti[7];
  float Ra[3];
  actSO3(&Ti[3], &X[0], Ra);
  Y[0] = s_inv * Ra[0];
  Y[1] = s_inv * Ra[1];
  Y[2] = s_inv * Ra[2];
  actSO3(&Ti[3], &X[3], &Y[3]);
  Y[3] += s_inv * (Ti[1] * Ra[2] - Ti[2] * Ra[1]);
  Y[4] += s_inv * (Ti[2] * Ra[0] - Ti[0] * Ra[2]);
  Y[5] += s_inv * (Ti[0] * Ra[1] - Ti[1] * Ra[0]);
  Y[6] = X[6] + (s_inv * (Ti[0] * Ra[0] + Ti[1] * Ra[1] + Ti[2] * Ra[2]));
}

// expSim3 (gn_kernels.cu:299-390), float with the reference's double literals.
__device__ __forceinline__ void expSim3(const float* xi, float* T) {
  const float tau[3] = {xi[0], xi[1], xi[2]};
  const float phi[3] = {xi[3], xi[4], xi[5]};
  const float sigma = xi[6];
  const float scale = expf(sigma);
  const float theta_sq = phi[0] * phi[0] + phi[1] * phi[1] + phi[2] * phi[2];
  float imag, real;
  if ((double)theta_sq < 1e-6) {
    const float theta_p4 = theta_sq * theta_sq;
    imag = (float)(0.5 - (1.0 / 48.0) * theta_sq + (1.0 / 3840.0) * theta_p4);
    real = (float)(1.0 - (1.0 / 8.0) * theta_sq + (1.0 / 384.0) * theta_p4);
  } else {
    const float theta = sqrtf(theta_sq);
    imag = sinf(0.5f * theta) / theta;  // 0.5*theta in double == exact halving
    real = cosf(0.5f * theta);
  }
  T[3] = imag * phi[0];
  T[4] = imag * phi[1];
  T[5] = imag * phi[2];
  T[6] = real;
  T[7] = scale;
  const float theta = sqrtf(theta_sq);
  float A, B, C;
  if (fabs((double)sigma) < 1e-6) {
    C = 1.0f;
    if (fabs((double)theta) < 1e-6) {
      A = 0.5f;
      B = (float)(1.0 / 6.0);
    } else {
      A = (1.0f - cosf(theta)) / theta_sq;
      B = (theta - sinf(theta)) / (theta_sq * theta);
    }
  } else {
    C = (scale - 1.0f) / sigma;
    if (fabs((double)theta) < 1e-6) {
      const float sigma_sq = sigma * sigma;
      A = ((sigma - 1.0f) * scale + 1.0f) / sigma_sq;
      B = (scale * 0.5f * sigma_sq + scale - 1.0f - sigma * scale) / (sigma_sq * sigma);
    } else {
      const float a = scale * sinf(theta);
      const float b = scale * cosf(theta);
      const float c = theta_sq + sigma * sigma;
      A = (a * sigma + (1.0f - b) * theta) / (theta * c);
      B = (C - ((b - 1.0f) * sigma + a * theta) / c) / theta_sq;
    }
  }
  float t0 = C * tau[0], t1 = C * tau[1], t2 = C * tau[2];
  float c0 = phi[1] * tau[2] - phi[2] * tau[1];
  float c1 = phi[2] * tau[0] - phi[0] * tau[2];
  float c2 = phi[0] * tau[1] - phi[1] * tau[0];
  t0 += A * c0;
  t1 += A * c1;
  t2 += A * c2;
  float d0 = phi[1] * c2 - phi[2] * c1;
  float d1 = phi[2] * c0 - phi[0] * c2;
  float d2 = phi[0] * c1 - phi[1] * c0;
  T[0] = t0 + B * d0;
  T[1] = t1 + B * d1;
  T[2] = t2 + B * d2;
}

// T <- Exp(xi) * T  (gn_kernels.cu:392-413; no quaternion re-normalisation, as the reference)
__device__ __forceinline__ void retrSim3(const float* xi, float* T) {
  float D[8];
  expSim3(xi, D);
  float q1[4];
  quat_comp(&D[3], &T[3], q1);
  float t1[3];
  actSO3(&D[3], &T[0], t1);
  T[0] = t1[0] * D[7] + D[0];
  T[1] = t1[1] * D[7] + D[1];
  T[2] = t1[2] * D[7] + D[2];
  T[3] = q1[0];
  T[4] = q1[1];
  T[5] = q1[2];
  T[6] = q1[3];
  T[7] = D[7] * T[7];
}

// ---- fp64 forms of the global-BA pose math. The BA poses stay float (the reference's Twc), but
// the two per-edge / per-pose steps whose fp32 rounding is coherent over a whole edge or pose run in double:
//  * expSim3's series coefficients cancel catastrophically in fp32 for the small steps of a converging BA
//    (C = (e^s - 1)/s, A = (1 - cos t)/t^2, B = (t - sin t)/t^3: relative errors up to O(1) at |phi| ~ 1e-2), and
//  * relSim3's translation t_j - t_i rounds at |t_i| (metres), coherent over every point of the edge.
// On the C4 EuRoC 320x512 K=256 rays graph (scripts/ba_prec_exp.py, an fp32-stage emulation of the HIP rows) the fp32
// retraction alone put the poses 2.0e-5 from the fp64 truth; a double retraction 2.6e-6; plus a double relSim3 5e-7.
// Same formulas and thresholds as the reference's float code (gn_kernels.cu:252-272, 299-413), evaluated in double
// (what the fp64 truth, oracle/liboracle_m3s_f64.so, computes).
__device__ __forceinline__ void quat_comp_d(const double* qi, const double* qj, double* out) {
  out[0] = qi[3] * qj[0] + qi[0] * qj[3] + qi[1] * qj[2] - qi[2] * qj[1];
  out[1] = qi[3] * qj[1] - qi[0] * qj[2] + qi[1] * qj[3] + qi[2] * qj[0];
  out[2] = qi[3] * qj[2] + qi[0] * qj[1] - qi[1] * qj[0] + qi[2] * qj[3];
  out[3] = qi[3] * qj[3] - qi[0] * qj[0] - qi[1] * qj[1] - qi[2] * qj[2];
}

__device__ __forceinline__ void actSO3_d(const double* q, const double* X, double* Y) {
  const double uv0 = 2.0 * (q[1] * X[2] - q[2] * X[1]);
  const double uv1 = 2.0 * (q[2] * X[0] - q[0] * X[2]);
  const double uv2 = 2.0 * (q[0] * X[1] - q[1] * X[0]);
  const double y0 = X[0] + q[3] * uv0 + (q[1] * uv2 - q[2] * uv1);
  const double y1 = X[1] + q[3] * uv1 + (q[2] * uv0 - q[0] * uv2);
  const double y2 = X[2] + q[3] * uv2 + (q[0] * uv1 - q[1] * uv0);
  Y[0] = y0;
  Y[1] = y1;
  Y[2] = y2;
}

// T_ij = T_i^-1 T_j of two float poses, in double
__device__ __forceinline__ void relSim3_d(const float* Ti, const float* Tj, double* Tij) {
  const double si_inv = 1.0 / (double)Ti[7];
  Tij[7] = si_inv * (double)Tj[7];
  const double qi_inv[4] = {-(double)Ti[3], -(double)Ti[4], -(double)Ti[5], (double)Ti[6]};
  const double qj[4] = {Tj[3], Tj[4], Tj[5], Tj[6]};
  quat_comp_d(qi_inv, qj, &Tij[3]);
  double t[3] = {(double)Tj[0] - (double)Ti[0], (double)Tj[1] - (double)Ti[1], (double)Tj[2] - (double)Ti[2]};
  actSO3_d(qi_inv, t, t);
  Tij[0] = t[0] * si_inv;
  Tij[1] = t[1] * si_inv;
  Tij[2] = t[2] * si_inv;
}

__device__ __forceinline__ void expSim3_d(const double* xi, double* T) {
  const double tau[3] = {xi[0], xi[1], xi[2]};
  const double phi[3] = {xi[3], xi[4], xi[5]};
  const double sigma = xi[6];
  const double scale = exp(sigma);
  const double theta_sq = phi[0] * phi[0] + phi[1] * phi[1] + phi[2] * phi[2];
  double imag, real;
  if (theta_sq < 1e-6) {
    const double theta_p4 = theta_sq * theta_sq;
    imag = 0.5 - (1.0 / 48.0) * theta_sq + (1.0 / 3840.0) * theta_p4;
    real = 1.0 - (1.0 / 8.0) * theta_sq + (1.0 / 384.0) * theta_p4;
  } else {
    const double theta = sqrt(theta_sq);
    imag = sin(0.5 * theta) / theta;
    real = cos(0.5 * theta);
  }
  T[3] = imag * phi[0];
  T[4] = imag * phi[1];
  T[5] = imag * phi[2];
  T[6] = real;
  T[7] = scale;
  const double theta = sqrt(theta_sq);
  double A, B, C;
  if (fabs(sigma) < 1e-6) {
    C = 1.0;
    if (fabs(theta) < 1e-6) {
      A = 0.5;
      B = 1.0 / 6.0;
    } else {
      A = (1.0 - cos(theta)) / theta_sq;
      B = (theta - sin(theta)) / (theta_sq * theta);
    }
  } else {
    C = (scale - 1.0) / sigma;
    if (fabs(theta) < 1e-6) {
      const double sigma_sq = sigma * sigma;
      A = ((sigma - 1.0) * scale + 1.0) / sigma_sq;
      B = (scale * 0.5 * sigma_sq + scale - 1.0 - sigma * scale) / (sigma_sq * sigma);
    } else {
      const double a = scale * sin(theta);
      const double b = scale * cos(theta);
      const double c = theta_sq + sigma * sigma;
      A = (a * sigma + (1.0 - b) * theta) / (theta * c);
      B = (C - ((b - 1.0) * sigma + a * theta) / c) / theta_sq;
    }
  }
  const double c0 = phi[1] * tau[2] - phi[2] * tau[1];
  const double c1 = phi[2] * tau[0] - phi[0] * tau[2];
  const double c2 = phi[0] * tau[1] - phi[1] * tau[0];
  const double d0 = phi[1] * c2 - phi[2] * c1;
  const double d1 = phi[2] * c0 - phi[0] * c2;
  const double d2 = phi[0] * c1 - phi[1] * c0;
  T[0] = C * tau[0] + A * c0 + B * d0;
  T[1] = C * tau[1] + A * c1 + B * d1;
  T[2] = C * tau[2] + A * c2 + B * d2;
}

// T <- Exp(xi) * T of a float pose and a float step, in double, rounded back to float once
__device__ __forceinline__ void retrSim3_d(const float* xi, float* T) {
  double x[7], D[8], Td[8];
  for (int c = 0; c < 7; c++) x[c] = xi[c];
  for (int c = 0; c < 8; c++) Td[c] = T[c];
  expSim3_d(x, D);
  double q1[4], t1[3];
  quat_comp_d(&D[3], &Td[3], q1);
  actSO3_d(&D[3], &Td[0], t1);
  for (int c = 0; c < 3; c++) T[c] = (float)(t1[c] * D[7] + D[c]);
  for (int c = 0; c < 4; c++) T[3 + c] = (float)q1[c];
  T[7] = (float)(D[7] * Td[7]);
}

// ---- wave64 reductions (DPP/permute through __shfl_xor; no warp-synchronous assumptions) ----
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Bijective block remap (cdna guide §5 "XCD swizzle"): hardware deals block b to XCD b % 8; this
// returns the logical block so that each XCD gets one contiguous run of logical blocks.
__device__ __forceinline__ int xcd_remap(int b, int nb) {
  const int q = nb / 8, r = nb % 8, x = b % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

}  // namespace m3s
