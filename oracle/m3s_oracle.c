/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C CPU restatement of the reference's native hot path
 * (/root/reference/mast3r_slam/backend/src/{matching,gn}_kernels.cu).  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library, and only as the checker / CPU baseline.
 * The product path (lightweight-mast3r-slam_amd/) never links or calls it.
 *
 * What is restated, line-faithfully (float arithmetic with the reference's double-typed literals
 * kept double, c10::Half step rounding in refine):
 *   - iter_proj_kernel        matching_kernels.cu:119-275
 *   - refine_matches_kernel   matching_kernels.cu:25-81  (f16 and f32 instantiations)
 *   - Sim3 device math        gn_kernels.cu:172-413
 *   - point_align_kernel      gn_kernels.cu:455-723
 *   - ray_align_kernel        gn_kernels.cu:813-1138
 *   - calib_proj_kernel       gn_kernels.cu:1231-1543
 *   - pose_retr_kernel        gn_kernels.cu:415-453
 *   - gauss_newton_*_cuda host loops gn_kernels.cu:725-811, 1140-1228, 1546-1637, including the
 *     unique/searchsorted rank remap (:161-170) and the SparseBlock assembly (:71-113).
 *
 * Deliberate deviations ("truth mode"): per-edge H/g sums are accumulated in fp64 (the reference
 * block-reduces fp32 partials, :36-55), and Eigen's SimplicialLLT (:132-153, third-party,
 * submodule not vendored) is replaced by a dense fp64 Cholesky, which gives the same solution to
 * rounding; a non-positive pivot yields dx = 0 exactly like the reference's failure branch (:147-150).
 *
 * Parity status: the CUDA sources cannot be compiled in this image (no nvcc, Eigen submodule
 * absent), so these kernel restatements are pinned against the reference's importable Python glue
 * where the math overlaps (tests/golden/make_golden.py) and otherwise "parity unpinned" — see
 * DESIGN.md §Oracle.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <float.h>
#include <omp.h>

#define M3O_EPS 1e-6 /* gn_kernels.cu:34 */

/* ------------------------------------------------------------------------------------------ */
/* IEEE binary16 <-> binary32, round-to-nearest-even (c10::Half semantics, Half.h fp16_ieee_*). */
/* ------------------------------------------------------------------------------------------ */
static inline float m3o_h2f(uint16_t h) {
  uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
  uint32_t exp = (h >> 10) & 0x1fu;
  uint32_t man = h & 0x3ffu;
  uint32_t bits;
  if (exp == 0) {
    if (man == 0) {
      bits = sign;
    } else { /* subnormal: normalise */
      int e = -1;
      do { e++; man <<= 1; } while ((man & 0x400u) == 0);
      man &= 0x3ffu;
      bits = sign | ((uint32_t)(127 - 15 - e) << 23) | (man << 13);
    }
  } else if (exp == 31) {
    bits = sign | 0x7f800000u | (man << 13);
  } else {
    bits = sign | ((exp + 127 - 15) << 23) | (man << 13);
  }
  float f;
  memcpy(&f, &bits, 4);
  return f;
}

static inline uint16_t m3o_f2h(float f) {
  uint32_t x;
  memcpy(&x, &f, 4);
  uint32_t sign = (x >> 16) & 0x8000u;
  uint32_t absx = x & 0x7fffffffu;
  if (absx >= 0x7f800000u) { /* inf or nan */
    return (uint16_t)(sign | (absx > 0x7f800000u ? 0x7e00u : 0x7c00u));
  }
  if (absx >= 0x477ff000u) { /* rounds to >= 65520 -> inf */
    return (uint16_t)(sign | 0x7c00u);
  }
  int32_t e = (int32_t)(absx >> 23) - 127;
  if (e < -14) { /* result is subnormal (or zero) in half */
    if (e < -25) return (uint16_t)sign; /* < 2^-25: rounds to 0 (2^-25 exactly is a tie -> 0) */
    uint32_t man = (absx & 0x7fffffu) | 0x800000u; /* 24 bits */
    int shift = -14 - e + 13;                      /* bits to drop */
    uint32_t q = man >> shift;
    uint32_t rem = man & ((1u << shift) - 1u);
    uint32_t half = 1u << (shift - 1);
    if (rem > half || (rem == half && (q & 1u))) q++;
    return (uint16_t)(sign | q);
  }
  uint32_t man = absx & 0x7fffffu;
  uint32_t q = ((uint32_t)(e + 15) << 10) | (man >> 13);
  uint32_t rem = man & 0x1fffu;
  if (rem > 0x1000u || (rem == 0x1000u && (q & 1u))) q++;
  return (uint16_t)(sign | q);
}

/* host threads of the OpenMP loops (bench.py's cpu_baseline times 1 thread and all cores) */
void m3o_set_threads(int n) { omp_set_num_threads(n > 0 ? n : 1); }

/* BA sums in the reference's own order (gn_kernels.cu:531-723, 890-1138, 1326-1543): per edge THREADS = 256
 * float accumulators, point k into thread k % 256 (each thread walks k = tid, tid + 256, ...), every product-sum
 * contracted to an FMA as nvcc does by default (hij += w * Jn * Jm -> fmaf(w * Jn, Jm, hij)), then the float
 * blockReduce tree (:45-55: +128, +64, +32, ..., +1). 0 (default): per-point fp32 products summed in fp64. */
static int g_ref_order = 0;
void m3o_set_ref_order(int on) { g_ref_order = on; }

void m3o_f32_to_f16(const float* in, uint16_t* out, int64_t n) {
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; i++) out[i] = m3o_f2h(in[i]);
}

void m3o_f16_to_f32(const uint16_t* in, float* out, int64_t n) {
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; i++) out[i] = m3o_h2f(in[i]);
}

/* ------------------------------------------------------------------------------------------ */
/* iter_proj  (matching_kernels.cu:119-275)                                                    */
/* ------------------------------------------------------------------------------------------ */
static inline void m3o_clamp(float* x, float lo, float hi) { *x = fminf(fmaxf(*x, lo), hi); } /* :21-23 */

static inline void m3o_bilinear_weights(float u, float v, int* u11, int* v11, float w[4]) {
  *u11 = (int)floorf(u);
  *v11 = (int)floorf(v);
  float du = u - (float)(*u11);
  float dv = v - (float)(*v11);
  w[0] = du * dv;                                  /* w11 */
  w[1] = (float)((1.0 - (double)du) * (double)dv); /* w12: (1.0-du)*dv in double */
  w[2] = (float)((double)du * (1.0 - (double)dv)); /* w21 */
  w[3] = (float)((1.0 - (double)du) * (1.0 - (double)dv)); /* w22 */
}

/* ------------------------------------------------------------------------------------------ */
/* prep_for_iter_proj's torch glue (matching.py:25-49, image.py:5-38) in the reference's own fp32 */
/* arithmetic. Pinned against the reference run (tests/golden/matching_48x64.npz rays / pts, bit  */
/* for bit; tests/test_oracle.py): torch's CPU vector_norm of a 3-vector is the FMA chain          */
/* sqrt(fma(z, z, fma(y, y, x * x))), F.normalize divides by max(norm, eps), and the depthwise     */
/* conv2d of the reflect-padded image is a row-major FMA chain over all 9 taps, zero taps included */
/* (acc = w00 * v00, then acc = fma(w, v, acc)).                                                   */
/* ------------------------------------------------------------------------------------------ */
static inline float m3o_norm3f(float x, float y, float z) { return sqrtf(fmaf(z, z, fmaf(y, y, x * x))); }

void m3o_norm3(const float* x, float* out, int64_t n) {
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; i++) out[i] = m3o_norm3f(x[3 * i], x[3 * i + 1], x[3 * i + 2]);
}

void m3o_normalize3(const float* x, float* out, int64_t n) {
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; i++) {
    const float nr = fmaxf(m3o_norm3f(x[3 * i], x[3 * i + 1], x[3 * i + 2]), 1e-12f);
    for (int c = 0; c < 3; c++) out[3 * i + c] = x[3 * i + c] / nr;
  }
}

/* img (B,H,W,3) -> gx, gy (B,H,W,3); F.pad(mode="reflect") by 1, kernel (1/32) [[-3,0,3],[-10,0,10],[-3,0,3]] and
 * its transpose (image.py:10-24: the weights are (1/32) * integer, exact in fp32) */
void m3o_img_gradient(const float* img, float* gx, float* gy, int B, int H, int W) {
  static const float kx[3][3] = {{-0.09375f, 0.0f, 0.09375f}, {-0.3125f, 0.0f, 0.3125f}, {-0.09375f, 0.0f, 0.09375f}};
#pragma omp parallel for collapse(2) schedule(static)
  for (int b = 0; b < B; b++) {
    for (int y = 0; y < H; y++) {
      for (int x = 0; x < W; x++) {
        for (int c = 0; c < 3; c++) {
          float ax = 0.0f, ay = 0.0f;
          for (int t = 0; t < 9; t++) {
            const int dy = t / 3 - 1, dx = t % 3 - 1;
            int yy = y + dy, xx = x + dx;
            yy = yy < 0 ? -yy : (yy >= H ? 2 * H - 2 - yy : yy);
            xx = xx < 0 ? -xx : (xx >= W ? 2 * W - 2 - xx : xx);
            const float v = img[(((size_t)b * H + yy) * W + xx) * 3 + c];
            const float wx = kx[t / 3][t % 3], wy = kx[t % 3][t / 3];
            if (t == 0) {
              ax = wx * v;
              ay = wy * v;
            } else {
              ax = fmaf(wx, v, ax);
              ay = fmaf(wy, v, ay);
            }
          }
          gx[(((size_t)b * H + y) * W + x) * 3 + c] = ax;
          gy[(((size_t)b * H + y) * W + x) * 3 + c] = ay;
        }
      }
    }
  }
}

/* diag (optional, test infrastructure for the fused match's mismatch census): per pixel
 *   [0] the smallest LM accept margin over the iterations, |new_cost - cost| / (sqrt(cost) + sqrt(new_cost)): a
 *       rounding-level difference in either cost (each is a sum of squares of err = r - p, err's rounding ~ ulp(|r|))
 *       can flip the accept / reject branch only when this is of the order of that rounding;
 *   [1] the last iteration's convergence margin, |c - cost_thresh| / (sqrt(c) + sqrt(cost_thresh)) for the cost c the
 *       converged flag was decided on. */
static void iter_proj_impl(const float* rays, const float* pts, const float* p_init, float* p_new,
                           uint8_t* converged, int B, int H, int W, int N, int max_iter, float lambda_init,
                           float cost_thresh, float* diag) {
#pragma omp parallel for collapse(2) schedule(static)
  for (int b = 0; b < B; b++) {
    for (int n = 0; n < N; n++) {
      const float* img = rays + (size_t)b * H * W * 9;
      const float* p = pts + ((size_t)b * N + n) * 3;
      float u = p_init[((size_t)b * N + n) * 2 + 0];
      float v = p_init[((size_t)b * N + n) * 2 + 1];
      m3o_clamp(&u, 1.0f, (float)(W - 2));
      m3o_clamp(&v, 1.0f, (float)(H - 2));
      uint8_t conv = 0;
      float lambda = lambda_init;
      double acc_margin = INFINITY, conv_margin = INFINITY;
      for (int it = 0; it < max_iter; it++) {
        int u11, v11;
        float w[4];
        m3o_bilinear_weights(u, v, &u11, &v11, w);
        const float* r11 = img + ((size_t)(v11 + 1) * W + (u11 + 1)) * 9;
        const float* r12 = img + ((size_t)(v11 + 1) * W + u11) * 9;
        const float* r21 = img + ((size_t)v11 * W + (u11 + 1)) * 9;
        const float* r22 = img + ((size_t)v11 * W + u11) * 9;
        float r[3], gx[3], gy[3], err[3];
        for (int j = 0; j < 3; j++) r[j] = w[0] * r11[j] + w[1] * r12[j] + w[2] * r21[j] + w[3] * r22[j];
        for (int j = 3; j < 6; j++) gx[j - 3] = w[0] * r11[j] + w[1] * r12[j] + w[2] * r21[j] + w[3] * r22[j];
        for (int j = 6; j < 9; j++) gy[j - 6] = w[0] * r11[j] + w[1] * r12[j] + w[2] * r21[j] + w[3] * r22[j];
        float r_norm = sqrtf(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
        float r_norm_inv = (float)(1.0 / (double)r_norm);
        for (int j = 0; j < 3; j++) r[j] *= r_norm_inv;
        for (int j = 0; j < 3; j++) err[j] = r[j] - p[j];
        float cost = err[0] * err[0] + err[1] * err[1] + err[2] * err[2];
        float A00 = gx[0] * gx[0] + gx[1] * gx[1] + gx[2] * gx[2];
        float A01 = gx[0] * gy[0] + gx[1] * gy[1] + gx[2] * gy[2];
        float A11 = gy[0] * gy[0] + gy[1] * gy[1] + gy[2] * gy[2];
        float b0 = -(err[0] * gx[0] + err[1] * gx[1] + err[2] * gx[2]);
        float b1 = -(err[0] * gy[0] + err[1] * gy[1] + err[2] * gy[2]);
        A00 += lambda;
        A11 += lambda;
        float det_inv = (float)(1.0 / (double)(A00 * A11 - A01 * A01));
        float delta_u = det_inv * (A11 * b0 - A01 * b1);
        float delta_v = det_inv * (-A01 * b0 + A00 * b1);
        float u_new = u + delta_u;
        float v_new = v + delta_v;
        m3o_clamp(&u_new, 1.0f, (float)(W - 2));
        m3o_clamp(&v_new, 1.0f, (float)(H - 2));
        m3o_bilinear_weights(u_new, v_new, &u11, &v11, w);
        r11 = img + ((size_t)(v11 + 1) * W + (u11 + 1)) * 9;
        r12 = img + ((size_t)(v11 + 1) * W + u11) * 9;
        r21 = img + ((size_t)v11 * W + (u11 + 1)) * 9;
        r22 = img + ((size_t)v11 * W + u11) * 9;
        for (int j = 0; j < 3; j++) r[j] = w[0] * r11[j] + w[1] * r12[j] + w[2] * r21[j] + w[3] * r22[j];
        r_norm = sqrtf(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
        r_norm_inv = (float)(1.0 / (double)r_norm);
        for (int j = 0; j < 3; j++) r[j] *= r_norm_inv;
        for (int j = 0; j < 3; j++) err[j] = r[j] - p[j];
        float new_cost = err[0] * err[0] + err[1] * err[1] + err[2] * err[2];
        /* a step that rounds to no move (u_new == u, v_new == v) compares a cost with itself: no rounding can flip it */
        if (diag && (u_new != u || v_new != v)) {
          const double m = fabs((double)new_cost - (double)cost) / (sqrt((double)cost) + sqrt((double)new_cost) + 1e-30);
          if (m < acc_margin) acc_margin = m;
        }
        const float decided = new_cost < cost ? new_cost : cost;
        if (new_cost < cost) {
          u = u_new;
          v = v_new;
          lambda = (float)((double)lambda * 0.1);
          conv = new_cost < cost_thresh;
        } else {
          lambda = (float)((double)lambda * 10.0);
          conv = cost < cost_thresh;
        }
        if (diag)
          conv_margin = fabs((double)decided - (double)cost_thresh) /
                        (sqrt((double)decided) + sqrt((double)cost_thresh) + 1e-30);
      }
      p_new[((size_t)b * N + n) * 2 + 0] = u;
      p_new[((size_t)b * N + n) * 2 + 1] = v;
      converged[(size_t)b * N + n] = conv;
      if (diag) {
        diag[((size_t)b * N + n) * 2 + 0] = (float)acc_margin;
        diag[((size_t)b * N + n) * 2 + 1] = (float)conv_margin;
      }
    }
  }
}

void m3o_iter_proj(const float* rays, const float* pts, const float* p_init, float* p_new,
                   uint8_t* converged, int B, int H, int W, int N, int max_iter, float lambda_init,
                   float cost_thresh) {
  iter_proj_impl(rays, pts, p_init, p_new, converged, B, H, W, N, max_iter, lambda_init, cost_thresh, NULL);
}

void m3o_iter_proj_diag(const float* rays, const float* pts, const float* p_init, float* p_new,
                        uint8_t* converged, int B, int H, int W, int N, int max_iter, float lambda_init,
                        float cost_thresh, float* diag) {
  iter_proj_impl(rays, pts, p_init, p_new, converged, B, H, W, N, max_iter, lambda_init, cost_thresh, diag);
}

/* ------------------------------------------------------------------------------------------ */
/* refine_matches (matching_kernels.cu:25-81)                                                  */
/* ------------------------------------------------------------------------------------------ */
static inline int m3o_inside(int u, int v, int W, int H) { return v >= 0 && v < H && u >= 0 && u < W; }

/* scalar_t = c10::Half: every '*' and '+=' rounds to half (Half.h operator* / operator+ / +=);
 * max_score starts at cuda::std::numeric_limits<c10::Half>::min() = Half() = +0. */
void m3o_refine_matches_f16(const uint16_t* D11, const uint16_t* D21, const int64_t* p1,
                            int64_t* p1_new, int B, int H, int W, int F, int N, int radius,
                            int dilation_max) {
#pragma omp parallel for collapse(2) schedule(dynamic, 256)
  for (int b = 0; b < B; b++) {
    for (int n = 0; n < N; n++) {
      const uint16_t* q = D21 + ((size_t)b * N + n) * F;
      const uint16_t* img = D11 + (size_t)b * H * W * F;
      int64_t u0 = p1[((size_t)b * N + n) * 2 + 0];
      int64_t v0 = p1[((size_t)b * N + n) * 2 + 1];
      uint16_t max_score = 0;
      int64_t u_new = u0, v_new = v0;
      for (int d = dilation_max; d > 0; d--) {
        const int rd = radius * d;
        const int diam = 2 * rd + 1;
        for (int i = 0; i < diam; i += d) {
          for (int j = 0; j < diam; j += d) {
            const int64_t u = u0 - rd + i;
            const int64_t v = v0 - rd + j;
            if (m3o_inside((int)u, (int)v, W, H)) {
              const uint16_t* c = img + ((size_t)v * W + u) * F;
              uint16_t score = 0;
              for (int k = 0; k < F; k++) {
                uint16_t prod = m3o_f2h(m3o_h2f(q[k]) * m3o_h2f(c[k]));
                score = m3o_f2h(m3o_h2f(score) + m3o_h2f(prod));
              }
              if (m3o_h2f(score) > m3o_h2f(max_score)) {
                max_score = score;
                u_new = u;
                v_new = v;
              }
            }
          }
        }
        u0 = u_new;
        v0 = v_new;
      }
      p1_new[((size_t)b * N + n) * 2 + 0] = u_new;
      p1_new[((size_t)b * N + n) * 2 + 1] = v_new;
    }
  }
}

/* scalar_t = float: plain fp32 MACs, max_score starts at FLT_MIN (libcu++ numeric_limits<float>). */
void m3o_refine_matches_f32(const float* D11, const float* D21, const int64_t* p1, int64_t* p1_new,
                            int B, int H, int W, int F, int N, int radius, int dilation_max) {
#pragma omp parallel for collapse(2) schedule(dynamic, 256)
  for (int b = 0; b < B; b++) {
    for (int n = 0; n < N; n++) {
      const float* q = D21 + ((size_t)b * N + n) * F;
      const float* img = D11 + (size_t)b * H * W * F;
      int64_t u0 = p1[((size_t)b * N + n) * 2 + 0];
      int64_t v0 = p1[((size_t)b * N + n) * 2 + 1];
      float max_score = FLT_MIN;
      int64_t u_new = u0, v_new = v0;
      for (int d = dilation_max; d > 0; d--) {
        const int rd = radius * d;
        const int diam = 2 * rd + 1;
        for (int i = 0; i < diam; i += d) {
          for (int j = 0; j < diam; j += d) {
            const int64_t u = u0 - rd + i;
            const int64_t v = v0 - rd + j;
            if (m3o_inside((int)u, (int)v, W, H)) {
              const float* c = img + ((size_t)v * W + u) * F;
              float score = 0.0f;
              for (int k = 0; k < F; k++) score += q[k] * c[k];
              if (score > max_score) {
                max_score = score;
                u_new = u;
                v_new = v;
              }
            }
          }
        }
        u0 = u_new;
        v0 = v_new;
      }
      p1_new[((size_t)b * N + n) * 2 + 0] = u_new;
      p1_new[((size_t)b * N + n) * 2 + 1] = v_new;
    }
  }
}

/* ------------------------------------------------------------------------------------------ */
/* Sim3 device math (gn_kernels.cu:172-413). Pose layout [t(3), q(4, xyzw), s].                */
/* ------------------------------------------------------------------------------------------ */
static inline float m3o_huber(float r) { /* :172-175 */
  const float r_abs = fabsf(r);
  return (double)r_abs < 1.345 ? 1.0f : (float)(1.345 / (double)r_abs);
}

static void m3o_quat_comp(const float* qi, const float* qj, float* out) { /* :178-184 */
  out[0] = qi[3] * qj[0] + qi[0] * qj[3] + qi[1] * qj[2] - qi[2] * qj[1];
  out[1] = qi[3] * qj[1] - qi[0] * qj[2] + qi[1] * qj[3] + qi[2] * qj[0];
  out[2] = qi[3] * qj[2] + qi[0] * qj[1] - qi[1] * qj[0] + qi[2] * qj[3];
  out[3] = qi[3] * qj[3] - qi[0] * qj[0] - qi[1] * qj[1] - qi[2] * qj[2];
}

static void m3o_quat_inv(const float* q, float* out) { /* :187-193 */
  out[0] = -q[0];
  out[1] = -q[1];
  out[2] = -q[2];
  out[3] = q[3];
}

static void m3o_actSO3(const float* q, const float* X, float* Y) { /* :195-205 */
  float uv[3];
  uv[0] = (float)(2.0 * (double)(q[1] * X[2] - q[2] * X[1]));
  uv[1] = (float)(2.0 * (double)(q[2] * X[0] - q[0] * X[2]));
  uv[2] = (float)(2.0 * (double)(q[0] * X[1] - q[1] * X[0]));
  float y0 = X[0] + q[3] * uv[0] + (q[1] * uv[2] - q[2] * uv[1]);
  float y1 = X[1] + q[3] * uv[1] + (q[2] * uv[0] - q[0] * uv[2]);
  float y2 = X[2] + q[3] * uv[2] + (q[0] * uv[1] - q[1] * uv[0]);
  Y[0] = y0;
  Y[1] = y1;
  Y[2] = y2;
}

static void m3o_actSim3(const float* t, const float* q, const float* s, const float* X, float* Y) {
  m3o_actSO3(q, X, Y); /* :207-219 */
  Y[0] *= s[0];
  Y[1] *= s[0];
  Y[2] *= s[0];
  Y[0] += t[0];
  Y[1] += t[1];
  Y[2] += t[2];
}

static inline float m3o_dot3(const float* t, const float* s) { return t[0] * s[0] + t[1] * s[1] + t[2] * s[2]; }

static void m3o_relSim3(const float* ti, const float* qi, const float* si, const float* tj,
                        const float* qj, const float* sj, float* tij, float* qij, float* sij) {
  float si_inv = (float)(1.0 / (double)si[0]); /* :252-272 */
  sij[0] = si_inv * sj[0];
  float qi_inv[4];
  m3o_quat_inv(qi, qi_inv);
  m3o_quat_comp(qi_inv, qj, qij);
  tij[0] = tj[0] - ti[0];
  tij[1] = tj[1] - ti[1];
  tij[2] = tj[2] - ti[2];
  m3o_actSO3(qi_inv, tij, tij);
  tij[0] *= si_inv;
  tij[1] *= si_inv;
  tij[2] *= si_inv;
}

static void m3o_apply_Sim3_adj_inv(const float* t, const float* q, const float* s, const float* X,
                                   float* Y) { /* :277-297 */
  const float s_inv = (float)(1.0 / (double)s[0]);
  float Ra[3];
  m3o_actSO3(q, &X[0], Ra);
  Y[0] = s_inv * Ra[0];
  Y[1] = s_inv * Ra[1];
  Y[2] = s_inv * Ra[2];
  m3o_actSO3(q, &X[3], &Y[3]);
  Y[3] += s_inv * (t[1] * Ra[2] - t[2] * Ra[1]);
  Y[4] += s_inv * (t[2] * Ra[0] - t[0] * Ra[2]);
  Y[5] += s_inv * (t[0] * Ra[1] - t[1] * Ra[0]);
  Y[6] = X[6] + (s_inv * m3o_dot3(t, Ra));
}

static void m3o_expSO3(const float* phi, float* q) { /* :299-321 */
  float theta_sq = phi[0] * phi[0] + phi[1] * phi[1] + phi[2] * phi[2];
  float imag, real;
  if ((double)theta_sq < M3O_EPS) {
    float theta_p4 = theta_sq * theta_sq;
    imag = (float)(0.5 - (1.0 / 48.0) * theta_sq + (1.0 / 3840.0) * theta_p4);
    real = (float)(1.0 - (1.0 / 8.0) * theta_sq + (1.0 / 384.0) * theta_p4);
  } else {
    float theta = sqrtf(theta_sq);
    imag = sinf((float)(0.5 * theta)) / theta;
    real = cosf((float)(0.5 * theta));
  }
  q[0] = imag * phi[0];
  q[1] = imag * phi[1];
  q[2] = imag * phi[2];
  q[3] = real;
}

static void m3o_cross_inplace(const float* a, float* b) {
  float x0 = a[1] * b[2] - a[2] * b[1];
  float x1 = a[2] * b[0] - a[0] * b[2];
  float x2 = a[0] * b[1] - a[1] * b[0];
  b[0] = x0;
  b[1] = x1;
  b[2] = x2;
}

static void m3o_expSim3(const float* xi, float* t, float* q, float* s) { /* :323-390 */
  float tau[3] = {xi[0], xi[1], xi[2]};
  float phi[3] = {xi[3], xi[4], xi[5]};
  float sigma = xi[6];
  float scale = expf(sigma);
  m3o_expSO3(phi, q);
  s[0] = scale;
  float theta_sq = phi[0] * phi[0] + phi[1] * phi[1] + phi[2] * phi[2];
  float theta = sqrtf(theta_sq);
  float A, B, C;
  const float one = 1.0f, half = 0.5f;
  if (fabs((double)sigma) < M3O_EPS) {
    C = one;
    if (fabs((double)theta) < M3O_EPS) {
      A = half;
      B = (float)(1.0 / 6.0);
    } else {
      A = (one - cosf(theta)) / theta_sq;
      B = (theta - sinf(theta)) / (theta_sq * theta);
    }
  } else {
    C = (scale - one) / sigma;
    if (fabs((double)theta) < M3O_EPS) {
      float sigma_sq = sigma * sigma;
      A = ((sigma - one) * scale + one) / sigma_sq;
      B = (scale * half * sigma_sq + scale - one - sigma * scale) / (sigma_sq * sigma);
    } else {
      float a = scale * sinf(theta);
      float b = scale * cosf(theta);
      float c = theta_sq + sigma * sigma;
      A = (a * sigma + (one - b) * theta) / (theta * c);
      B = (C - ((b - one) * sigma + a * theta) / (c)) / (theta_sq);
    }
  }
  t[0] = C * tau[0];
  t[1] = C * tau[1];
  t[2] = C * tau[2];
  m3o_cross_inplace(phi, tau);
  t[0] += A * tau[0];
  t[1] += A * tau[1];
  t[2] += A * tau[2];
  m3o_cross_inplace(phi, tau);
  t[0] += B * tau[0];
  t[1] += B * tau[1];
  t[2] += B * tau[2];
}

static void m3o_retrSim3(const float* xi, const float* t, const float* q, const float* s, float* t1,
                         float* q1, float* s1) { /* :392-413 */
  float dt[3] = {0, 0, 0};
  float dq[4] = {0, 0, 0, 1};
  float ds[1] = {0};
  m3o_expSim3(xi, dt, dq, ds);
  m3o_quat_comp(dq, q, q1);
  m3o_actSO3(dq, t, t1);
  t1[0] *= ds[0];
  t1[1] *= ds[0];
  t1[2] *= ds[0];
  t1[0] += dt[0];
  t1[1] += dt[1];
  t1[2] += dt[2];
  s1[0] = ds[0] * s[0];
}

/* pose_retr_kernel (:415-453): poses[k] <- retr(dx[k-num_fix], poses[k]) for k >= num_fix. */
void m3o_pose_retr(float* poses, const float* dx, int num_poses, int num_fix) {
  for (int k = num_fix; k < num_poses; k++) {
    float* P = poses + (size_t)k * 8;
    float t1[3], q1[4], s1[1];
    m3o_retrSim3(dx + (size_t)(k - num_fix) * 7, &P[0], &P[3], &P[7], t1, q1, s1);
    P[0] = t1[0];
    P[1] = t1[1];
    P[2] = t1[2];
    P[3] = q1[0];
    P[4] = q1[1];
    P[5] = q1[2];
    P[6] = q1[3];
    P[7] = s1[0];
  }
}

/* exported single-pose helpers, used by the tests to pin the product's Sim3 device math */
void m3o_exp_sim3(const float* xi, float* out8) { m3o_expSim3(xi, &out8[0], &out8[3], &out8[7]); }
void m3o_act_sim3(const float* T8, const float* X, float* Y) { m3o_actSim3(&T8[0], &T8[3], &T8[7], X, Y); }
void m3o_rel_sim3(const float* Ti, const float* Tj, float* Tij) {
  m3o_relSim3(&Ti[0], &Ti[3], &Ti[7], &Tj[0], &Tj[3], &Tj[7], &Tij[0], &Tij[3], &Tij[7]);
}

/* ------------------------------------------------------------------------------------------ */
/* BA edge linearisation: one call per edge, H(14x14 upper) and g accumulated in fp64.          */
/* mode 0 = points (:455-723), 1 = rays (:813-1138), 2 = calib (:1231-1543)                    */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
  int mode;
  float sigma_a;  /* point / ray / pixel */
  float sigma_b;  /* - / dist / depth */
  float C_thresh, Q_thresh;
  /* calib */
  float fx, fy, cx, cy;
  int height, width, pixel_border;
  float z_eps;
} m3o_ba_params;

static void m3o_accum_row(double* hij, double* vi, double* vj, const float* Jx, float w, float err) {
  int l = 0;
  for (int n = 0; n < 14; n++)
    for (int m = 0; m <= n; m++) hij[l++] += (double)(w * Jx[n] * Jx[m]);
  for (int n = 0; n < 7; n++) {
    vi[n] += (double)(w * err * Jx[n]);
    vj[n] += (double)(w * err * Jx[7 + n]);
  }
}

static void m3o_accum_row_f(float* hij, float* vi, float* vj, const float* Jx, float w, float err) {
  int l = 0;
  for (int n = 0; n < 14; n++)
    for (int m = 0; m <= n; m++, l++) hij[l] = fmaf(w * Jx[n], Jx[m], hij[l]);
  for (int n = 0; n < 7; n++) {
    vi[n] = fmaf(w * err, Jx[n], vi[n]);
    vj[n] = fmaf(w * err, Jx[7 + n], vj[n]);
  }
}

/* blockReduce (gn_kernels.cu:36-55) of 256 float slots with stride `st` (slot t at v[t * st]) -> v[0] */
static float m3o_block_reduce(float* v, int st) {
  for (int h = 128; h >= 1; h >>= 1)
    for (int t = 0; t < h; t++) v[t * st] += v[(t + h) * st];
  return v[0];
}

static void m3o_row(const float* Ji_local, const float* ti, const float* qi, const float* si, float* Jx) {
  float Jl[7];
  memcpy(Jl, Ji_local, sizeof(Jl));
  m3o_apply_Sim3_adj_inv(ti, qi, si, Jl, &Jx[7]);
  for (int n = 0; n < 7; n++) Jx[n] = -Jx[7 + n];
}

static void m3o_linearize_edge(const m3o_ba_params* P, const float* Twc, const float* Xs,
                               const float* Cs, int N, int ix, int jx, const int64_t* idx,
                               const uint8_t* valid_match, const float* Q, double* Hout /*4x7x7*/,
                               double* gout /*2x7*/) {
  const float *ti = &Twc[ix * 8], *qi = &Twc[ix * 8 + 3], *si = &Twc[ix * 8 + 7];
  const float *tj = &Twc[jx * 8], *qj = &Twc[jx * 8 + 3], *sj = &Twc[jx * 8 + 7];
  float tij[3], qij[4], sij[1];
  m3o_relSim3(ti, qi, si, tj, qj, sj, tij, qij, sij);
  double hij[105];
  double vi[7], vj[7];
  memset(hij, 0, sizeof(hij));
  memset(vi, 0, sizeof(vi));
  memset(vj, 0, sizeof(vj));
  /* reference order: per thread slot t (0..255) 105 + 7 + 7 floats */
  float* rf = g_ref_order ? (float*)calloc((size_t)256 * 119, sizeof(float)) : NULL;
#define M3O_ACC(Jx_, w_, e_)                                                                      \
  do {                                                                                            \
    if (rf) {                                                                                     \
      float* sl = rf + (size_t)(k % 256) * 119;                                                   \
      m3o_accum_row_f(sl, sl + 105, sl + 112, Jx_, w_, e_);                                       \
    } else {                                                                                      \
      m3o_accum_row(hij, vi, vj, Jx_, w_, e_);                                                    \
    }                                                                                             \
  } while (0)
  const float sa_inv = (float)(1.0 / (double)P->sigma_a);
  const float sb_inv = P->mode == 0 ? 0.0f : (float)(1.0 / (double)P->sigma_b);
  for (int k = 0; k < N; k++) {
    const int vm = valid_match[k] != 0;
    const int64_t ind = vm ? idx[k] : 0;
    const float* Xi = &Xs[((size_t)ix * N + ind) * 3];
    const float* Xj = &Xs[((size_t)jx * N + k) * 3];
    float Xj_Ci[3];
    m3o_actSim3(tij, qij, sij, Xj, Xj_Ci);
    const float q = Q[k];
    const float ci = Cs[(size_t)ix * N + ind];
    const float cj = Cs[(size_t)jx * N + k];
    int valid = vm & (q > P->Q_thresh) & (ci > P->C_thresh) & (cj > P->C_thresh);
    float Jl[7], Jx[14];
    if (P->mode == 0) {
      float err[3] = {Xj_Ci[0] - Xi[0], Xj_Ci[1] - Xi[1], Xj_Ci[2] - Xi[2]};
      const float sw = valid ? sa_inv * sqrtf(q) : 0.0f;
      float w[3];
      for (int r = 0; r < 3; r++) w[r] = m3o_huber(sw * err[r]) * (sw * sw);
      const float J0[7] = {1, 0, 0, 0, Xj_Ci[2], -Xj_Ci[1], Xj_Ci[0]};
      const float J1[7] = {0, 1, 0, -Xj_Ci[2], 0, Xj_Ci[0], Xj_Ci[1]};
      const float J2[7] = {0, 0, 1, Xj_Ci[1], -Xj_Ci[0], 0, Xj_Ci[2]};
      m3o_row(J0, ti, qi, si, Jx);
      M3O_ACC(Jx, w[0], err[0]);
      m3o_row(J1, ti, qi, si, Jx);
      M3O_ACC(Jx, w[1], err[1]);
      m3o_row(J2, ti, qi, si, Jx);
      M3O_ACC(Jx, w[2], err[2]);
    } else if (P->mode == 1) {
      const float norm2_i = Xi[0] * Xi[0] + Xi[1] * Xi[1] + Xi[2] * Xi[2];
      const float norm1_i = sqrtf(norm2_i);
      const float norm1_i_inv = (float)(1.0 / (double)norm1_i);
      float ri[3] = {norm1_i_inv * Xi[0], norm1_i_inv * Xi[1], norm1_i_inv * Xi[2]};
      const float norm2_j = Xj_Ci[0] * Xj_Ci[0] + Xj_Ci[1] * Xj_Ci[1] + Xj_Ci[2] * Xj_Ci[2];
      const float norm1_j = sqrtf(norm2_j);
      const float norm1_j_inv = (float)(1.0 / (double)norm1_j);
      float rj[3] = {norm1_j_inv * Xj_Ci[0], norm1_j_inv * Xj_Ci[1], norm1_j_inv * Xj_Ci[2]};
      float err[4] = {rj[0] - ri[0], rj[1] - ri[1], rj[2] - ri[2], norm1_j - norm1_i};
      const float swr = valid ? sa_inv * sqrtf(q) : 0.0f;
      const float swd = valid ? sb_inv * sqrtf(q) : 0.0f;
      float w[4];
      w[0] = m3o_huber(swr * err[0]) * (swr * swr);
      w[1] = m3o_huber(swr * err[1]) * (swr * swr);
      w[2] = m3o_huber(swr * err[2]) * (swr * swr);
      w[3] = m3o_huber(swd * err[3]) * (swd * swd);
      const float n3 = norm1_j_inv / norm2_j;
      const float dxx = norm1_j_inv - Xj_Ci[0] * Xj_Ci[0] * n3;
      const float dyy = norm1_j_inv - Xj_Ci[1] * Xj_Ci[1] * n3;
      const float dzz = norm1_j_inv - Xj_Ci[2] * Xj_Ci[2] * n3;
      const float dxy = -Xj_Ci[0] * Xj_Ci[1] * n3;
      const float dxz = -Xj_Ci[0] * Xj_Ci[2] * n3;
      const float dyz = -Xj_Ci[1] * Xj_Ci[2] * n3;
      const float J0[7] = {dxx, dxy, dxz, 0.0f, rj[2], -rj[1], 0.0f};
      const float J1[7] = {dxy, dyy, dyz, -rj[2], 0.0f, rj[0], 0.0f};
      const float J2[7] = {dxz, dyz, dzz, rj[1], -rj[0], 0.0f, 0.0f};
      const float J3[7] = {rj[0], rj[1], rj[2], 0.0f, 0.0f, 0.0f, norm1_j};
      m3o_row(J0, ti, qi, si, Jx);
      M3O_ACC(Jx, w[0], err[0]);
      m3o_row(J1, ti, qi, si, Jx);
      M3O_ACC(Jx, w[1], err[1]);
      m3o_row(J2, ti, qi, si, Jx);
      M3O_ACC(Jx, w[2], err[2]);
      m3o_row(J3, ti, qi, si, Jx);
      M3O_ACC(Jx, w[3], err[3]);
    } else {
      const int u_target = (int)(ind % P->width);
      const int v_target = (int)(ind / P->width);
      const int valid_z = (Xj_Ci[2] > P->z_eps) && (Xi[2] > P->z_eps);
      const float zj_inv = valid_z ? (float)(1.0 / (double)Xj_Ci[2]) : 0.0f;
      const float zj_log = valid_z ? logf(Xj_Ci[2]) : 0.0f;
      const float zi_log = valid_z ? logf(Xi[2]) : 0.0f;
      const float x_div_z = Xj_Ci[0] * zj_inv;
      const float y_div_z = Xj_Ci[1] * zj_inv;
      const float u = P->fx * x_div_z + P->cx;
      const float v = P->fy * y_div_z + P->cy;
      const int valid_u = (u > (float)P->pixel_border) && (u < (float)(P->width - 1 - P->pixel_border));
      const int valid_v = (v > (float)P->pixel_border) && (v < (float)(P->height - 1 - P->pixel_border));
      float err[3] = {u - (float)u_target, v - (float)v_target, zj_log - zi_log};
      valid = valid & valid_u & valid_v & valid_z;
      const float swp = valid ? sa_inv * sqrtf(q) : 0.0f;
      const float swd = valid ? sb_inv * sqrtf(q) : 0.0f;
      float w[3];
      w[0] = m3o_huber(swp * err[0]) * (swp * swp);
      w[1] = m3o_huber(swp * err[1]) * (swp * swp);
      w[2] = m3o_huber(swd * err[2]) * (swd * swd);
      const float fx = P->fx, fy = P->fy;
      const float J0[7] = {fx * zj_inv, 0.0f, -fx * x_div_z * zj_inv, -fx * x_div_z * y_div_z,
                           fx * (1 + x_div_z * x_div_z), -fx * y_div_z, 0.0f};
      const float J1[7] = {0.0f, fy * zj_inv, -fy * y_div_z * zj_inv, -fy * (1 + y_div_z * y_div_z),
                           fy * x_div_z * y_div_z, fy * x_div_z, 0.0f};
      const float J2[7] = {0.0f, 0.0f, zj_inv, y_div_z, -x_div_z, 0.0f, 1.0f};
      m3o_row(J0, ti, qi, si, Jx);
      M3O_ACC(Jx, w[0], err[0]);
      m3o_row(J1, ti, qi, si, Jx);
      M3O_ACC(Jx, w[1], err[1]);
      m3o_row(J2, ti, qi, si, Jx);
      M3O_ACC(Jx, w[2], err[2]);
    }
    (void)Jl;
  }
#undef M3O_ACC
  if (rf) {  /* the float block reductions, in the reference's order (gs first, then hij) */
    for (int n = 0; n < 7; n++) {
      vi[n] = (double)m3o_block_reduce(rf + 105 + n, 119);
      vj[n] = (double)m3o_block_reduce(rf + 112 + n, 119);
    }
    for (int l = 0; l < 105; l++) hij[l] = (double)m3o_block_reduce(rf + l, 119);
    free(rf);
  }
  for (int n = 0; n < 7; n++) {
    gout[n] = vi[n];
    gout[7 + n] = vj[n];
  }
  int l = 0; /* block placement :699-722 */
  for (int n = 0; n < 14; n++) {
    for (int m = 0; m <= n; m++) {
      const double s = hij[l++];
      if (n < 7 && m < 7) {
        Hout[0 * 49 + n * 7 + m] = s;
        Hout[0 * 49 + m * 7 + n] = s;
      } else if (n >= 7 && m < 7) {
        Hout[1 * 49 + m * 7 + (n - 7)] = s;
        Hout[2 * 49 + (n - 7) * 7 + m] = s;
      } else {
        Hout[3 * 49 + (n - 7) * 7 + (m - 7)] = s;
        Hout[3 * 49 + (m - 7) * 7 + (n - 7)] = s;
      }
    }
  }
}

/* Linearise every edge; Hs (4,E,7,7) and gs (2,E,7) fp64, reference layout (:757-758).
 * ii/jj here are already dense ranks into Twc/Xs (the kernel's ii_edge/jj_edge). */
void m3o_ba_linearize(int mode, const float* Twc, const float* Xs, const float* Cs, int N, int E,
                      const int64_t* ii_rank, const int64_t* jj_rank, const int64_t* idx,
                      const uint8_t* valid_match, const float* Q, const float* params /*12*/,
                      double* Hs, double* gs) {
  m3o_ba_params P;
  P.mode = mode;
  P.sigma_a = params[0];
  P.sigma_b = params[1];
  P.C_thresh = params[2];
  P.Q_thresh = params[3];
  P.fx = params[4];
  P.fy = params[5];
  P.cx = params[6];
  P.cy = params[7];
  P.height = (int)params[8];
  P.width = (int)params[9];
  P.pixel_border = (int)params[10];
  P.z_eps = params[11];
#pragma omp parallel for schedule(dynamic, 1)
  for (int e = 0; e < E; e++) {
    double H4[196], g2[14];
    m3o_linearize_edge(&P, Twc, Xs, Cs, N, (int)ii_rank[e], (int)jj_rank[e], idx + (size_t)e * N,
                       valid_match + (size_t)e * N, Q + (size_t)e * N, H4, g2);
    for (int b = 0; b < 4; b++)
      memcpy(&Hs[((size_t)b * E + e) * 49], &H4[b * 49], 49 * sizeof(double));
    for (int b = 0; b < 2; b++) memcpy(&gs[((size_t)b * E + e) * 7], &g2[b * 7], 7 * sizeof(double));
  }
}

/* Dense fp64 Cholesky solve of A x = b in place (A n x n row-major, lower factor).
 * Returns 0 on success, -1 when a pivot is not positive (SimplicialLLT NumericalIssue). */
int m3o_cholesky_solve(double* A, double* b, int n) {
  for (int j = 0; j < n; j++) {
    double d = A[(size_t)j * n + j];
    for (int k = 0; k < j; k++) d -= A[(size_t)j * n + k] * A[(size_t)j * n + k];
    if (!(d > 0.0)) return -1;
    d = sqrt(d);
    A[(size_t)j * n + j] = d;
#pragma omp parallel for schedule(static) if (n > 256)
    for (int i = j + 1; i < n; i++) {
      double s = A[(size_t)i * n + j];
      for (int k = 0; k < j; k++) s -= A[(size_t)i * n + k] * A[(size_t)j * n + k];
      A[(size_t)i * n + j] = s / d;
    }
  }
  for (int i = 0; i < n; i++) { /* L y = b */
    double s = b[i];
    for (int k = 0; k < i; k++) s -= A[(size_t)i * n + k] * b[k];
    b[i] = s / A[(size_t)i * n + i];
  }
  for (int i = n - 1; i >= 0; i--) { /* L^T x = y */
    double s = b[i];
    for (int k = i + 1; k < n; k++) s -= A[(size_t)k * n + i] * b[k];
    b[i] = s / A[(size_t)i * n + i];
  }
  return 0;
}

static int m3o_cmp_i64(const void* a, const void* b) {
  int64_t x = *(const int64_t*)a, y = *(const int64_t*)b;
  return (x > y) - (x < y);
}

static int64_t m3o_searchsorted(const int64_t* u, int64_t n, int64_t key) {
  int64_t lo = 0, hi = n; /* torch.searchsorted left */
  while (lo < hi) {
    int64_t mid = (lo + hi) / 2;
    if (u[mid] < key) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

/* gauss_newton_{points,rays,calib}_cuda host loop (:725-811 / :1140-1228 / :1546-1637).
 * Twc (K,8) updated in place; dx_out ((K-1),7). Returns the number of iterations run, or -1 on a
 * bad remap (more unique ids than poses). */
int m3o_gauss_newton(int mode, float* Twc, const float* Xs, const float* Cs, int K, int N, int E,
                     const int64_t* ii, const int64_t* jj, const int64_t* idx,
                     const uint8_t* valid_match, const float* Q, const float* params, int max_iter,
                     float delta_thresh, float* dx_out) {
  const int num_fix = 1;
  int64_t* u = (int64_t*)malloc(sizeof(int64_t) * 2 * (size_t)(E > 0 ? E : 1));
  memcpy(u, ii, sizeof(int64_t) * E);
  memcpy(u + E, jj, sizeof(int64_t) * E);
  qsort(u, 2 * (size_t)E, sizeof(int64_t), m3o_cmp_i64);
  int64_t nu = 0;
  for (int64_t k = 0; k < 2 * (int64_t)E; k++)
    if (nu == 0 || u[k] != u[nu - 1]) u[nu++] = u[k];
  if (nu > K) {
    free(u);
    return -1;
  }
  int64_t* ie = (int64_t*)malloc(sizeof(int64_t) * (E > 0 ? E : 1));
  int64_t* je = (int64_t*)malloc(sizeof(int64_t) * (E > 0 ? E : 1));
  for (int e = 0; e < E; e++) {
    ie[e] = m3o_searchsorted(u, nu, ii[e]);
    je[e] = m3o_searchsorted(u, nu, jj[e]);
  }
  const int nopt = K - num_fix;
  const int n = nopt * 7;
  double* Hs = (double*)malloc(sizeof(double) * 4 * 49 * (size_t)(E > 0 ? E : 1));
  double* gs = (double*)malloc(sizeof(double) * 2 * 7 * (size_t)(E > 0 ? E : 1));
  double* A = (double*)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1) * (n > 0 ? n : 1));
  double* b = (double*)malloc(sizeof(double) * (n > 0 ? n : 1));
  int it;
  for (it = 0; it < max_iter; it++) {
    m3o_ba_linearize(mode, Twc, Xs, Cs, N, E, ie, je, idx, valid_match, Q, params, Hs, gs);
    memset(A, 0, sizeof(double) * (size_t)n * n);
    memset(b, 0, sizeof(double) * n);
    for (int e = 0; e < E; e++) {
      const int64_t io = ie[e] - num_fix, jo = je[e] - num_fix;
      const int64_t rows[4] = {io, io, jo, jo}, cols[4] = {io, jo, io, jo};
      for (int blk = 0; blk < 4; blk++) {
        if (rows[blk] < 0 || cols[blk] < 0) continue;
        const double* h = &Hs[((size_t)blk * E + e) * 49];
        for (int r = 0; r < 7; r++)
          for (int c = 0; c < 7; c++) A[(size_t)(rows[blk] * 7 + r) * n + cols[blk] * 7 + c] += h[r * 7 + c];
      }
      if (io >= 0)
        for (int r = 0; r < 7; r++) b[io * 7 + r] += gs[(size_t)e * 7 + r];
      if (jo >= 0)
        for (int r = 0; r < 7; r++) b[jo * 7 + r] += gs[((size_t)E + e) * 7 + r];
    }
    int ok = n > 0 ? m3o_cholesky_solve(A, b, n) : -1;
    for (int r = 0; r < n; r++) dx_out[r] = ok == 0 ? (float)(-b[r]) : 0.0f; /* dx = -A.solve() */
    m3o_pose_retr(Twc, dx_out, K, num_fix);
    double nrm = 0.0;
    for (int r = 0; r < n; r++) nrm += (double)dx_out[r] * (double)dx_out[r];
    if ((float)sqrt(nrm) < delta_thresh) {
      it++;
      break;
    }
  }
  free(u);
  free(ie);
  free(je);
  free(Hs);
  free(gs);
  free(A);
  free(b);
  return it;
}
