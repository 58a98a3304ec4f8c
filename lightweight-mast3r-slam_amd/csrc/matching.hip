// Dense projective matching for MI355X (gfx950): prep (ray image + gradients), iterative
// projection (LM over a bilinear ray image), occlusion test and coarse-to-fine descriptor refine.
//
// Reference semantics:
//   prep_for_iter_proj + img_gradient   /root/reference/mast3r_slam/matching.py:25-49, image.py:5-38
//   iter_proj_kernel                    backend/src/matching_kernels.cu:119-275
//   occlusion check                     matching.py:68-76
//   refine_matches_kernel (c10::Half)   backend/src/matching_kernels.cu:25-81
//   pixel_to_lin                        matching.py:13-15
//
// This file is compiled with -ffp-contract=off: the refine score must round every half product and
// every half add separately (c10::Half operator* / operator+), which a contracted v_fma_f16 breaks.
#include "m3s_half.hpp"

extern "C" hipError_t m3s_launch_refine_tile(const void*, const void*, const void*, void*, int, int, int, int, int,
                                             int, int, void*, int*, const float*, hipStream_t);
extern "C" int m3s_refine_tile_ok(int, int, int, int, int, int);

namespace m3s {

// Refine tile path: D11 (B,H,W,24) f32 -> f16 (RNE, == torch .half()) of pixel n into image b's three chunk planes
// (H,W,8) (one 16-B store per plane: lanes store consecutive pixels); returns the sum of squares of its f16 values
// (the refine screen's norm bound, refine.hip; 0 past the image). The loads are split from the conversion so the
// prep kernel issues them first, under the ray halo's loads and stencil (desc_load, then desc_planar).
// (unconditional: a pixel past the image loads pixel N - 1 and stores nothing, so no branch join waits on the loads)
__device__ __forceinline__ void desc_load(const float* __restrict__ D11, int b, int n, int N, float4 v[6]) {
  const float4* src = reinterpret_cast<const float4*>(D11 + ((size_t)b * N + min(n, N - 1)) * 24);
#pragma unroll
  for (int k = 0; k < 6; k++) v[k] = src[k];
}

__device__ __forceinline__ float desc_planar(const float4 v[6], h1* __restrict__ D11h, int b, int n, int N) {
  float ss = 0.0f;
  if (n < N) {
    const size_t plane = (size_t)N * 8;
    h1* dst = D11h + (size_t)b * 3 * plane + (size_t)n * 8;
#pragma unroll
    for (int c = 0; c < 3; c++) {
      const float4 v0 = v[2 * c], v1 = v[2 * c + 1];
      h1 r[8] = {(h1)v0.x, (h1)v0.y, (h1)v0.z, (h1)v0.w, (h1)v1.x, (h1)v1.y, (h1)v1.z, (h1)v1.w};
      *reinterpret_cast<uint4*>(dst + c * plane) = *reinterpret_cast<uint4*>(r);
#pragma unroll
      for (int k = 0; k < 8; k++) ss += (float)r[k] * (float)r[k];
    }
  }
  return ss;
}

// ------------------------------------------------------------------------------------------
// prep: rays = X/max(|X|,1e-12); gx, gy = Scharr/32 with reflect padding; out (B,H,W,9).
// One 16x16 tile per 256-thread block, normalised rays of an 18x18 halo staged in LDS.
// Also converts D11 (B,H,W,F) f32 -> f16 (RNE, == torch .half()) for the same pixels: planar (refine tile path, one
// pixel per thread) with the tile's descriptor-norm partial max |D11h[pixel]|_2 into cnorm_part (nullable), else in
// the (B,H,W,F) layout of the per-pixel refine kernels.
// ------------------------------------------------------------------------------------------
// torch.linalg.vector_norm / F.normalize of an fp32 3-vector in the reference's rounding: sqrt(fma(z, z, fma(y, y,
// x * x))) (pinned bit for bit against the reference run's golden rays / pts; oracle m3o_norm3)
__device__ __forceinline__ float norm3_ref(float x, float y, float z) {
  return sqrtf(__builtin_fmaf(z, z, __builtin_fmaf(y, y, x * x)));
}

#define PREP_T 16
// DMODE: 0 no descriptors, 1 planar (refine tile path), 2 the (B,H,W,F) row layout; a template argument so the
// planar path's descriptor loads, issued first, cross no branch join (a runtime `if` made the compiler convert them,
// and so wait for them, right behind the loads)
template <int DMODE>
__global__ void __launch_bounds__(256) prep_rays_kernel(const float* __restrict__ X11, float* __restrict__ rays9,
                                                        const float* __restrict__ D11, h1* __restrict__ D11h, int H,
                                                        int W, int F, int planar, float* __restrict__ cnorm_part) {
  __shared__ float tile[(PREP_T + 2) * (PREP_T + 2) * 3];
  const int b = blockIdx.z;
  const int u0 = blockIdx.x * PREP_T, v0 = blockIdx.y * PREP_T;
  const float* Xb = X11 + (size_t)b * H * W * 3;
  const int lx = threadIdx.x % PREP_T, ly = threadIdx.x / PREP_T;
  const int x = u0 + lx, y = v0 + ly;
  constexpr bool planar_d = DMODE == 1;
  const int dn = (x < W && y < H) ? y * W + x : H * W;
  // the 18x18 halo: 324 pixels, two per thread at most (256 threads); both loads issued before either is used
  constexpr int HALO = (PREP_T + 2) * (PREP_T + 2);
  static_assert(HALO <= 2 * 256, "prep halo: two pixels per thread");
  float hv[2][3];
#pragma unroll
  for (int r = 0; r < 2; r++) {
    const int t = min((int)threadIdx.x + 256 * r, HALO - 1);
    const int hy = t / (PREP_T + 2), hx = t % (PREP_T + 2);
    int yy = v0 + hy - 1, xx = u0 + hx - 1;
    // reflect padding (F.pad mode="reflect"): -1 -> 1, H -> H-2
    yy = yy < 0 ? -yy : (yy >= H ? 2 * H - 2 - yy : yy);
    xx = xx < 0 ? -xx : (xx >= W ? 2 * W - 2 - xx : xx);
    yy = min(max(yy, 0), H - 1);
    xx = min(max(xx, 0), W - 1);
    const float* p = Xb + ((size_t)yy * W + xx) * 3;
    hv[r][0] = p[0];
    hv[r][1] = p[1];
    hv[r][2] = p[2];
  }
  // then the pixel's descriptor loads (vmcnt retires in order: behind the halo's, so the stencil waits only for those)
  float4 dv[6];
  if constexpr (planar_d) desc_load(D11, b, dn, H * W, dv);
#pragma unroll
  for (int r = 0; r < 2; r++) {
    const int t = threadIdx.x + 256 * r;
    if (t < HALO) {
      const float a = hv[r][0], c = hv[r][1], d = hv[r][2];
      const float n = fmaxf(norm3_ref(a, c, d), 1e-12f);
      tile[t * 3 + 0] = a / n;
      tile[t * 3 + 1] = c / n;
      tile[t * 3 + 2] = d / n;
    }
  }
  __syncthreads();
  if (x < W && y < H) {
    float* o = rays9 + (((size_t)b * H + y) * W + x) * 9;
#define T3(dy, dx, c) tile[(((ly + 1 + (dy)) * (PREP_T + 2)) + (lx + 1 + (dx))) * 3 + (c)]
#pragma unroll
    for (int c = 0; c < 3; c++) {
      o[c] = T3(0, 0, c);
      // gx kernel (1/32)[[-3,0,3],[-10,0,10],[-3,0,3]]; gy its transpose (image.py:10-24), in the reference's
      // depthwise conv2d order: a row-major FMA chain over all 9 taps, zero taps included (bit-exact against the
      // reference run's rays: tests/golden/matching_48x64.npz, oracle m3o_img_gradient)
      const float t00 = T3(-1, -1, c), t01 = T3(-1, 0, c), t02 = T3(-1, 1, c), t10 = T3(0, -1, c), t11 = T3(0, 0, c),
                  t12 = T3(0, 1, c), t20 = T3(1, -1, c), t21 = T3(1, 0, c), t22 = T3(1, 1, c);
      float gx = -0.09375f * t00;
      gx = __builtin_fmaf(0.0f, t01, gx);
      gx = __builtin_fmaf(0.09375f, t02, gx);
      gx = __builtin_fmaf(-0.3125f, t10, gx);
      gx = __builtin_fmaf(0.0f, t11, gx);
      gx = __builtin_fmaf(0.3125f, t12, gx);
      gx = __builtin_fmaf(-0.09375f, t20, gx);
      gx = __builtin_fmaf(0.0f, t21, gx);
      gx = __builtin_fmaf(0.09375f, t22, gx);
      float gy = -0.09375f * t00;
      gy = __builtin_fmaf(-0.3125f, t01, gy);
      gy = __builtin_fmaf(-0.09375f, t02, gy);
      gy = __builtin_fmaf(0.0f, t10, gy);
      gy = __builtin_fmaf(0.0f, t11, gy);
      gy = __builtin_fmaf(0.0f, t12, gy);
      gy = __builtin_fmaf(0.09375f, t20, gy);
      gy = __builtin_fmaf(0.3125f, t21, gy);
      gy = __builtin_fmaf(0.09375f, t22, gy);
      o[3 + c] = gx;
      o[6 + c] = gy;
    }
#undef T3
  }
  if constexpr (planar_d) {
    const float ss = desc_planar(dv, D11h, b, dn, H * W);
    if (cnorm_part != nullptr) {
      // the tile's max |D11h[pixel]|_2, one partial per block (proj_occlusion reduces them before refine reads the
      // bound); NaN / inf descriptors give a NaN / inf partial, which switches the screen off for every lane
      __shared__ float s_max[4];
      float nmax = sqrtf(ss);
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) nmax = fmaxf_nan(nmax, __shfl_xor(nmax, off, 64));
      if ((threadIdx.x & 63) == 0) s_max[threadIdx.x >> 6] = nmax;
      __syncthreads();
      if (threadIdx.x == 0)
        cnorm_part[((size_t)b * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x] =
            fmaxf_nan(fmaxf_nan(s_max[0], s_max[1]), fmaxf_nan(s_max[2], s_max[3]));
    }
  } else if constexpr (DMODE == 2) {
    // f32 -> f16 of this tile's descriptor rows (B,H,W,F), 4 channels per lane-step (the per-pixel kernels'
    // layout; the refine tile path's planar layout is written by the proj launch, desc_planar above)
    for (int t = threadIdx.x; t < PREP_T * PREP_T * (F / 4); t += blockDim.x) {
      const int pix = t / (F / 4), q = t % (F / 4);
      const int xx = u0 + pix % PREP_T, yy = v0 + pix / PREP_T;
      if (xx < W && yy < H) {
        const size_t off = (((size_t)b * H + yy) * W + xx) * F + q * 4;
        const float4 v = *reinterpret_cast<const float4*>(D11 + off);
        h1 r[4] = {(h1)v.x, (h1)v.y, (h1)v.z, (h1)v.w};
        *reinterpret_cast<uint2*>(D11h + off) = *reinterpret_cast<uint2*>(r);
      }
    }
  }
}

// max of the prep partials into cmax[0] (the refine screen's descriptor-norm bound), by the first wave of one block
// of the launch between prep and refine (proj_occlusion)
// (16 loads per lane in flight at once: one at a time, the 1024 partials of a 512x512 image were 16 dependent
// round trips in front of block 0's own pixels, and the launch ends with its last block; the max is
// order-independent, NaN included, so the result is the same)
__device__ __forceinline__ void reduce_cnorm(const float* __restrict__ part, int nparts, float* __restrict__ cmax) {
  const int lane = threadIdx.x & 63;
  float m = 0.0f;
  for (int base = lane; base < nparts; base += 64 * 16) {
    float v[16];
#pragma unroll
    for (int k = 0; k < 16; k++) v[k] = part[min(base + 64 * k, nparts - 1)];
#pragma unroll
    for (int k = 0; k < 16; k++) m = fmaxf_nan(m, v[k]);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) m = fmaxf_nan(m, __shfl_xor(m, off, 64));
  if (lane == 0) *cmax = m;
}

// ------------------------------------------------------------------------------------------
// iter_proj core (matching_kernels.cu:139-273), one point per lane.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void bilin_w(float u, float v, int& u11, int& v11, float w[4]) {
  u11 = (int)floorf(u);
  v11 = (int)floorf(v);
  const float du = u - (float)u11;
  const float dv = v - (float)v11;
  // (1.0-du)*dv etc. are evaluated in double by the reference (:161-164). u, v >= 1 after clamping,
  // so du, dv are multiples of ulp(u) >= 2^-23 and 1-du, 1-dv are exact in float; the double
  // product of two exact floats is then rounded once to float — the same value as this float
  // product (no fp64 needed, bit-identical).
  const float cu = 1.0f - du, cv = 1.0f - dv;
  w[0] = du * dv;
  w[1] = cu * dv;
  w[2] = du * cv;
  w[3] = cu * cv;
}

// The four corners' 9 channels: channels 0..7 as four packed fp32 pairs (each element rounds as the scalar
// expression w0 r11 + w1 r12 + w2 r21 + w3 r22 does: -ffp-contract=off, no fma; the loads land in even-aligned
// register pairs and the weights broadcast by op_sel, so no moves), channel 8 scalar
__device__ __forceinline__ void bilin_sample9(const float* __restrict__ img, int W, int u11, int v11, const float w[4],
                                              float* out) {
  typedef float wf2 __attribute__((ext_vector_type(2)));
  // two 18-float runs, (v11, u11 .. u11 + 1) and the row below, from one 32-bit offset each (u11, v11 lie inside the
  // image and the launchers require 9 H W < 2^31): the corners are immediate offsets of the two run pointers
  const unsigned o = (unsigned)(v11 * W + u11) * 9u;
  const float* r22 = img + o;
  const float* r21 = r22 + 9;
  const float* r12 = img + (o + 9u * (unsigned)W);
  const float* r11 = r12 + 9;
  const wf2 w0 = {w[0], w[0]}, w1 = {w[1], w[1]}, w2 = {w[2], w[2]}, w3 = {w[3], w[3]};
  auto ld2 = [](const float* q) {
    wf2 r;
    r.x = q[0];
    r.y = q[1];
    return r;
  };
#pragma unroll
  for (int j = 0; j < 8; j += 2) {
    const wf2 o = w0 * ld2(r11 + j) + w1 * ld2(r12 + j) + w2 * ld2(r21 + j) + w3 * ld2(r22 + j);
    out[j] = o.x;
    out[j + 1] = o.y;
  }
  out[8] = w[0] * r11[8] + w[1] * r12[8] + w[2] * r21[8] + w[3] * r22[8];
}

// One LM iteration (matching_kernels.cu:185-270 loop body) on the carried state. LAST (the fused kernel's final
// iteration): the occlusion test's X11 gather at both possible final pixels, the accepted step's and the kept one's,
// is issued beside the iteration's own sample, so its round trip is not one more link after the loop; xo gets the
// one the accept / reject picks (matching.py:68-76 reads X11 at the final .long() pixel).
struct LmState {
  float u, v, lambda, cost, e0, e1, e2;
  float s[9];
  bool conv;
};

template <bool LAST>
__device__ __forceinline__ void lm_iter(LmState& m, const float* __restrict__ img, int H, int W, const float p[3],
                                        float cost_thresh, const float* __restrict__ X11b, float* xo) {
  const float* s = m.s;
  float A00 = s[3] * s[3] + s[4] * s[4] + s[5] * s[5];
  const float A01 = s[3] * s[6] + s[4] * s[7] + s[5] * s[8];
  float A11 = s[6] * s[6] + s[7] * s[7] + s[8] * s[8];
  const float b0 = -(m.e0 * s[3] + m.e1 * s[4] + m.e2 * s[5]);
  const float b1 = -(m.e0 * s[6] + m.e1 * s[7] + m.e2 * s[8]);
  A00 += m.lambda;
  A11 += m.lambda;
  const float det_inv = 1.0f / (A00 * A11 - A01 * A01);
  float u_new = m.u + det_inv * (A11 * b0 - A01 * b1);
  float v_new = m.v + det_inv * (-A01 * b0 + A00 * b1);
  u_new = fminf(fmaxf(u_new, 1.0f), (float)(W - 2));
  v_new = fminf(fmaxf(v_new, 1.0f), (float)(H - 2));
  float xa[3], xb[3];
  if constexpr (LAST) {
    const float* qa = X11b + ((size_t)(int)v_new * W + (int)u_new) * 3;  // .long() truncation; u, v >= 1
    const float* qb = X11b + ((size_t)(int)m.v * W + (int)m.u) * 3;
#pragma unroll
    for (int c = 0; c < 3; c++) {
      xa[c] = qa[c];
      xb[c] = qb[c];
    }
  }
  int u11, v11;
  float w[4], t[9];
  bilin_w(u_new, v_new, u11, v11, w);
  bilin_sample9(img, W, u11, v11, w, t);
  const float r_norm_inv = 1.0f / sqrtf(t[0] * t[0] + t[1] * t[1] + t[2] * t[2]);
  const float f0 = t[0] * r_norm_inv - p[0];
  const float f1 = t[1] * r_norm_inv - p[1];
  const float f2 = t[2] * r_norm_inv - p[2];
  const float new_cost = f0 * f0 + f1 * f1 + f2 * f2;
  if (new_cost < m.cost) {
    m.u = u_new;
    m.v = v_new;
#pragma unroll
    for (int k = 0; k < 9; k++) m.s[k] = t[k];
    m.e0 = f0;
    m.e1 = f1;
    m.e2 = f2;
    m.conv = new_cost < cost_thresh;
    m.cost = new_cost;
    m.lambda = (float)((double)m.lambda * 0.1);
    if constexpr (LAST) {
#pragma unroll
      for (int c = 0; c < 3; c++) xo[c] = xa[c];
    }
  } else {
    m.lambda = (float)((double)m.lambda * 10.0);
    m.conv = m.cost < cost_thresh;
    if constexpr (LAST) {
#pragma unroll
      for (int c = 0; c < 3; c++) xo[c] = xb[c];
    }
  }
}

// OCC: X11b non-null, xo gets X11 at the final (.long()) pixel, gathered during the last iteration (lm_iter<true>)
template <bool OCC>
__device__ __forceinline__ void iter_proj_point(const float* __restrict__ img, int H, int W, const float p[3],
                                                float& u, float& v, bool& conv, int max_iter, float lambda_init,
                                                float cost_thresh, const float* __restrict__ X11b = nullptr,
                                                float* xo = nullptr) {
  LmState m;
  m.u = fminf(fmaxf(u, 1.0f), (float)(W - 2));
  m.v = fminf(fmaxf(v, 1.0f), (float)(H - 2));
  m.lambda = lambda_init;
  m.conv = conv;
  // The reference samples (u, v) at the top of every iteration and (u_new, v_new) for the new cost.
  // The top-of-loop sample always equals the previous iteration's accepted sample (u_new) or its own
  // previous value (rejected), so the 9-channel sample is carried instead of refetched: one
  // dependent gather per iteration instead of two, identical values.
  int u11, v11;
  float w[4];
  if constexpr (OCC) {
    if (max_iter <= 0) {  // no iteration: the occlusion pixel is the clamped start, gathered beside its sample
      const float* q = X11b + ((size_t)(int)m.v * W + (int)m.u) * 3;
#pragma unroll
      for (int c = 0; c < 3; c++) xo[c] = q[c];
    }
  }
  bilin_w(m.u, m.v, u11, v11, w);
  bilin_sample9(img, W, u11, v11, w, m.s);
  // The residual e and cost of the carried sample are carried too: an accepted step's (f, new_cost)
  // are exactly what the next iteration would recompute from the same sample (bit-identical).
  // 1.0/r_norm in double then float == IEEE float division (53 >= 2*24+2, innocuous double rounding)
  const float r_norm_inv = 1.0f / sqrtf(m.s[0] * m.s[0] + m.s[1] * m.s[1] + m.s[2] * m.s[2]);
  m.e0 = m.s[0] * r_norm_inv - p[0];
  m.e1 = m.s[1] * r_norm_inv - p[1];
  m.e2 = m.s[2] * r_norm_inv - p[2];
  m.cost = m.e0 * m.e0 + m.e1 * m.e1 + m.e2 * m.e2;
  if constexpr (OCC) {
    for (int i = 0; i < max_iter - 1; i++) lm_iter<false>(m, img, H, W, p, cost_thresh, nullptr, nullptr);
    if (max_iter > 0) lm_iter<true>(m, img, H, W, p, cost_thresh, X11b, xo);
  } else {
    for (int i = 0; i < max_iter; i++) lm_iter<false>(m, img, H, W, p, cost_thresh, nullptr, nullptr);
  }
  u = m.u;
  v = m.v;
  conv = m.conv;
}

// lin_to_pixel (matching.py:18-22) with Python floor semantics for any i0 sign; 32-bit division for the indices
// inside [0, 2^31) (the same quotient and remainder)
__device__ __forceinline__ void lin_to_pixel_f(int64_t i0, int W, float& u, float& v) {
  if (i0 >= 0 && i0 <= 0x7fffffff) {
    const unsigned q = (unsigned)i0 / (unsigned)W;
    u = (float)((unsigned)i0 - q * (unsigned)W);
    v = (float)q;
    return;
  }
  int64_t vq = i0 / W, uq = i0 % W;
  if (uq < 0) {
    uq += W;
    vq -= 1;
  }
  u = (float)uq;
  v = (float)vq;
}

// Reference-signature kernel: rays (B,H,W,9), pts (B,N,3) normalised, p_init (B,N,2) f32.
__global__ void __launch_bounds__(256) iter_proj_kernel(const float* __restrict__ rays, const float* __restrict__ pts,
                                                        const float* __restrict__ p_init, float* __restrict__ p_new,
                                                        uint8_t* __restrict__ converged, int H, int W, int N,
                                                        int max_iter, float lambda_init, float cost_thresh) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (n >= N) return;
  const size_t bn = (size_t)b * N + n;
  const float p[3] = {pts[bn * 3 + 0], pts[bn * 3 + 1], pts[bn * 3 + 2]};
  float u = p_init[bn * 2 + 0], v = p_init[bn * 2 + 1];
  bool conv = false;
  iter_proj_point<false>(rays + (size_t)b * H * W * 9, H, W, p, u, v, conv, max_iter, lambda_init, cost_thresh);
  p_new[bn * 2 + 0] = u;
  p_new[bn * 2 + 1] = v;
  converged[bn] = conv;
}

// Fused: normalise X21 on the fly, p_init from idx_init (or identity), LM projection, .long()
// truncation, occlusion test against raw X11 (matching.py:68-76). Writes p1 (B,N,2) int32 and
// valid (B,N) u8.
__global__ void __launch_bounds__(256) proj_occlusion_kernel(
    const float* __restrict__ rays, const float* __restrict__ X11, const float* __restrict__ X21,
    const int64_t* __restrict__ idx_init, int* __restrict__ p1, uint8_t* __restrict__ valid, int H, int W,
    int max_iter, float lambda_init, float cost_thresh, float dist_thresh, int* zero_counter,
    const float* __restrict__ cnorm_part, int nparts, float* __restrict__ cmax) {
  const int N = H * W;
  if (cmax != nullptr && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x < 64) reduce_cnorm(cnorm_part, nparts, cmax);
  // contiguous pixel runs per XCD: each XCD's L2 then holds the rays rows its LM gathers touch
  const int n = xcd_remap(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (zero_counter != nullptr && n == 0 && b == 0) *zero_counter = 0;  // refine's outlier list (next launch)
  if (n >= N) return;
  const size_t bn = (size_t)b * N + n;
  const float x = X21[bn * 3 + 0], y = X21[bn * 3 + 1], z = X21[bn * 3 + 2];
  const float nrm = fmaxf(norm3_ref(x, y, z), 1e-12f);  // F.normalize (matching.py:44)
  const float p[3] = {x / nrm, y / nrm, z / nrm};
  float u, v;
  lin_to_pixel_f(idx_init != nullptr ? idx_init[bn] : (int64_t)n, W, u, v);
  bool conv = false;
  float Xg[3];  // X11 at the final pixel, gathered during the last LM iteration
  iter_proj_point<true>(rays + (size_t)b * H * W * 9, H, W, p, u, v, conv, max_iter, lambda_init, cost_thresh,
                        X11 + (size_t)b * H * W * 3, Xg);
  const int pu = (int)u, pv = (int)v;  // .long() truncation; u,v >= 1 after clamping
  const float dx = Xg[0] - x, dy = Xg[1] - y, dz = Xg[2] - z;
  const float d = norm3_ref(dx, dy, dz);  // torch.linalg.norm (matching.py:71-73)
  p1[bn * 2 + 0] = pu;
  p1[bn * 2 + 1] = pv;
  valid[bn] = conv && (d < dist_thresh);
}

// ------------------------------------------------------------------------------------------
// refine (matching_kernels.cu:36-80) with c10::Half step rounding: each product and each
// partial sum rounds to binary16 (v_pk_mul_f16 / v_add_f16 are correctly rounded, == Half ops).
// ------------------------------------------------------------------------------------------
template <int F>
__device__ __forceinline__ h1 score_f16(const h2* q, const h1* __restrict__ c) {
  h2 cv[F / 2];
  const uint4* c4 = reinterpret_cast<const uint4*>(c);
#pragma unroll
  for (int k = 0; k < F / 8; k++) {
    const uint4 t = c4[k];
    cv[4 * k + 0] = *reinterpret_cast<const h2*>(&t.x);
    cv[4 * k + 1] = *reinterpret_cast<const h2*>(&t.y);
    cv[4 * k + 2] = *reinterpret_cast<const h2*>(&t.z);
    cv[4 * k + 3] = *reinterpret_cast<const h2*>(&t.w);
  }
  h1 s = (h1)0.0f;
#pragma unroll
  for (int k = 0; k < F / 2; k++) {
    const h2 pr = q[k] * cv[k];
    s = s + pr.x;
    s = s + pr.y;
  }
  return s;
}

template <int F>
__device__ __forceinline__ void refine_point(const h1* __restrict__ img, int H, int W, const h2* q, int radius,
                                             int dilation_max, int& u0, int& v0) {
  h1 max_score = (h1)0.0f;  // cuda::std::numeric_limits<c10::Half>::min() == Half() == +0
  int u_new = u0, v_new = v0;
  for (int d = dilation_max; d > 0; d--) {
    const int rd = radius * d;
    const int diam = 2 * rd + 1;
    for (int i = 0; i < diam; i += d) {
      const int u = u0 - rd + i;
      for (int j = 0; j < diam; j += d) {
        const int v = v0 - rd + j;
        if (v >= 0 && v < H && u >= 0 && u < W) {
          const h1 s = score_f16<F>(q, img + ((size_t)v * W + u) * F);
          if (s > max_score) {
            max_score = s;
            u_new = u;
            v_new = v;
          }
        }
      }
    }
    u0 = u_new;
    v0 = v_new;
  }
}

// Reference signature: D11 (B,H,W,F) f16, D21 (B,N,F) f16, p1 (B,N,2) i64 -> p1_new (B,N,2) i64.
template <int F>
__global__ void __launch_bounds__(256) refine_f16_kernel(const h1* __restrict__ D11, const h1* __restrict__ D21,
                                                         const int64_t* __restrict__ p1, int64_t* __restrict__ p1_new,
                                                         int H, int W, int N, int radius, int dilation_max) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (n >= N) return;
  const size_t bn = (size_t)b * N + n;
  h2 q[F / 2];
  load_query<F, false>(D21, bn, q);
  int u0 = (int)p1[bn * 2 + 0], v0 = (int)p1[bn * 2 + 1];
  refine_point<F>(D11 + (size_t)b * H * W * F, H, W, q, radius, dilation_max, u0, v0);
  p1_new[bn * 2 + 0] = u0;
  p1_new[bn * 2 + 1] = v0;
}

// Fused tail: D21 f32 converted in-register, p1 int32 from proj_occlusion, writes idx = u + W*v.
template <int F>
__global__ void __launch_bounds__(256) refine_lin_kernel(const h1* __restrict__ D11h, const float* __restrict__ D21,
                                                         const int* __restrict__ p1, int64_t* __restrict__ idx_out,
                                                         int H, int W, int radius, int dilation_max) {
  const int N = H * W;
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (n >= N) return;
  const size_t bn = (size_t)b * N + n;
  h2 q[F / 2];
  load_query<F, true>(D21, bn, q);
  int u0 = p1[bn * 2 + 0], v0 = p1[bn * 2 + 1];
  refine_point<F>(D11h + (size_t)b * H * W * F, H, W, q, radius, dilation_max, u0, v0);
  idx_out[bn] = (int64_t)u0 + (int64_t)W * v0;
}

// fp32 instantiation of the reference kernel (AT_DISPATCH float): fp32 MACs, max starts at FLT_MIN.
__global__ void __launch_bounds__(256) refine_f32_kernel(const float* __restrict__ D11, const float* __restrict__ D21,
                                                         const int64_t* __restrict__ p1, int64_t* __restrict__ p1_new,
                                                         int H, int W, int F, int N, int radius, int dilation_max) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (n >= N) return;
  const size_t bn = (size_t)b * N + n;
  const float* q = D21 + bn * F;
  const float* img = D11 + (size_t)b * H * W * F;
  int u0 = (int)p1[bn * 2 + 0], v0 = (int)p1[bn * 2 + 1];
  float max_score = 1.17549435e-38f;  // FLT_MIN
  int u_new = u0, v_new = v0;
  for (int d = dilation_max; d > 0; d--) {
    const int rd = radius * d, diam = 2 * rd + 1;
    for (int i = 0; i < diam; i += d) {
      for (int j = 0; j < diam; j += d) {
        const int u = u0 - rd + i, v = v0 - rd + j;
        if (v >= 0 && v < H && u >= 0 && u < W) {
          const float* c = img + ((size_t)v * W + u) * F;
          float s = 0.0f;
          for (int k = 0; k < F; k++) s += q[k] * c[k];
          if (s > max_score) {
            max_score = s;
            u_new = u;
            v_new = v;
          }
        }
      }
    }
    u0 = u_new;
    v0 = v_new;
  }
  p1_new[bn * 2 + 0] = u0;
  p1_new[bn * 2 + 1] = v0;
}

}  // namespace m3s

// ------------------------------------------------------------------------------------------
// launchers (called from abi.cpp)
// ------------------------------------------------------------------------------------------
// D11 (nullable): convert the descriptors too, planar (refine tile path, F = 24; cnorm_part nullable: the tile
// partials of the screen's norm bound, B * tiles floats) or in the (B,H,W,F) layout (per-pixel refine kernels)
extern "C" hipError_t m3s_launch_prep(const float* X11, float* rays9, const float* D11, void* D11h, int B, int H,
                                      int W, int F, int planar, float* cnorm_part, hipStream_t s) {
  dim3 grid((W + PREP_T - 1) / PREP_T, (H + PREP_T - 1) / PREP_T, B);
  auto k = D11 == nullptr ? m3s::prep_rays_kernel<0> : planar ? m3s::prep_rays_kernel<1> : m3s::prep_rays_kernel<2>;
  hipLaunchKernelGGL(k, grid, dim3(256), 0, s, X11, rays9, D11, reinterpret_cast<m3s::h1*>(D11h), H, W, F, planar,
                     cnorm_part);
  return hipGetLastError();
}

extern "C" int m3s_prep_parts(int B, int H, int W) {
  return B * ((W + PREP_T - 1) / PREP_T) * ((H + PREP_T - 1) / PREP_T);
}

extern "C" hipError_t m3s_launch_iter_proj(const float* rays, const float* pts, const float* p_init, float* p_new,
                                           uint8_t* conv, int B, int H, int W, int N, int max_iter, float lambda_init,
                                           float cost_thresh, hipStream_t s) {
  if ((size_t)9 * H * W >= ((size_t)1 << 31)) return hipErrorInvalidValue;  // bilin_sample9's 32-bit offsets
  dim3 grid((N + 255) / 256, B);
  hipLaunchKernelGGL(m3s::iter_proj_kernel, grid, dim3(256), 0, s, rays, pts, p_init, p_new, conv, H, W, N,
                     max_iter, lambda_init, cost_thresh);
  return hipGetLastError();
}

extern "C" hipError_t m3s_launch_proj_occlusion(const float* rays, const float* X11, const float* X21,
                                                const int64_t* idx_init, int* p1, uint8_t* valid, int B, int H, int W,
                                                int max_iter, float lambda_init, float cost_thresh, float dist_thresh,
                                                int* zero_counter, const float* cnorm_part, int nparts, float* cmax,
                                                hipStream_t s) {
  if ((size_t)9 * H * W >= ((size_t)1 << 31)) return hipErrorInvalidValue;  // bilin_sample9's 32-bit offsets
  // cmax (nullable): one wave reduces prep's tile partials into the refine screen's bound
  dim3 grid((H * W + 255) / 256, B);
  hipLaunchKernelGGL(m3s::proj_occlusion_kernel, grid, dim3(256), 0, s, rays, X11, X21, idx_init, p1, valid, H, W,
                     max_iter, lambda_init, cost_thresh, dist_thresh, zero_counter, cnorm_part, nparts, cmax);
  return hipGetLastError();
}

extern "C" hipError_t m3s_launch_refine_f16(const void* D11, const void* D21, const int64_t* p1, int64_t* p1_new, int B,
                                            int H, int W, int F, int N, int radius, int dilation_max, hipStream_t s) {
  dim3 grid((N + 255) / 256, B);
  const m3s::h1* a = reinterpret_cast<const m3s::h1*>(D11);
  const m3s::h1* q = reinterpret_cast<const m3s::h1*>(D21);
  if (N == H * W &&
      m3s_launch_refine_tile(D11, D21, p1, p1_new, B, H, W, F, radius, dilation_max, 0, nullptr, nullptr, nullptr, s) ==
          hipSuccess)
    return hipSuccess;  // tiled LDS path (query n is pixel n of the grid)
  switch (F) {
    case 24:
      hipLaunchKernelGGL(m3s::refine_f16_kernel<24>, grid, dim3(256), 0, s, a, q, p1, p1_new, H, W, N, radius,
                         dilation_max);
      break;
    case 16:
      hipLaunchKernelGGL(m3s::refine_f16_kernel<16>, grid, dim3(256), 0, s, a, q, p1, p1_new, H, W, N, radius,
                         dilation_max);
      break;
    case 32:
      hipLaunchKernelGGL(m3s::refine_f16_kernel<32>, grid, dim3(256), 0, s, a, q, p1, p1_new, H, W, N, radius,
                         dilation_max);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

extern "C" hipError_t m3s_launch_refine_f32(const float* D11, const float* D21, const int64_t* p1, int64_t* p1_new,
                                            int B, int H, int W, int F, int N, int radius, int dilation_max,
                                            hipStream_t s) {
  dim3 grid((N + 255) / 256, B);
  hipLaunchKernelGGL(m3s::refine_f32_kernel, grid, dim3(256), 0, s, D11, D21, p1, p1_new, H, W, F, N, radius,
                     dilation_max);
  return hipGetLastError();
}

// olist/ocount: deferred-outlier list (B*H*W int4) + counter, zeroed by proj_occlusion_kernel
extern "C" hipError_t m3s_launch_refine_lin(const void* D11h, const float* D21, const int* p1, int64_t* idx_out, int B,
                                            int H, int W, int F, int radius, int dilation_max, void* olist,
                                            int* ocount, const float* cmax, hipStream_t s) {
  dim3 grid((H * W + 255) / 256, B);
  const m3s::h1* a = reinterpret_cast<const m3s::h1*>(D11h);
  // tiled LDS path exactly when m3s_refine_tile_ok (prep wrote the PLANAR D11h then)
  if (radius > 0 && m3s_refine_tile_ok(B, H, W, F, radius, dilation_max))
    return m3s_launch_refine_tile(D11h, D21, p1, idx_out, B, H, W, F, radius, dilation_max, 1, olist, ocount, cmax, s);
  switch (F) {
    case 24:
      hipLaunchKernelGGL(m3s::refine_lin_kernel<24>, grid, dim3(256), 0, s, a, D21, p1, idx_out, H, W, radius,
                         dilation_max);
      break;
    case 16:
      hipLaunchKernelGGL(m3s::refine_lin_kernel<16>, grid, dim3(256), 0, s, a, D21, p1, idx_out, H, W, radius,
                         dilation_max);
      break;
    case 32:
      hipLaunchKernelGGL(m3s::refine_lin_kernel<32>, grid, dim3(256), 0, s, a, D21, p1, idx_out, H, W, radius,
                         dilation_max);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}
