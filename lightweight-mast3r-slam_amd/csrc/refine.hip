// LDS-tiled coarse-to-fine descriptor refine for MI355X (gfx950), F = 24, radius 3.
//
// Reference semantics: refine_matches_kernel<c10::Half>, /root/reference/mast3r_slam/backend/src/
// matching_kernels.cu:25-81 — per query pixel, dilation d = dmax..1, a 7x7 grid of stride d around
// the current centre (u outer, v inner), score = sequential c10::Half sum over 24 channels of
// half(q_k * c_k), strict '>' against a running max that starts at +0 and is never reset, re-centre
// after each level.
//
// MI355X design: one 32x8 pixel tile per 256-lane block (4 blocks / CU, 40 KiB LDS each).
//   * Per level the block estimates the tile's flow (mean centre displacement), takes the bbox of
//     the centres within 16 px of it, places a 64-column x 40-row window over bbox +- 3d and streams
//     D11 (f16) into LDS in three 8-channel chunks (16 B / px) with global_load_lds — one
//     wave-instruction per window row. Four resident blocks per CU hide each other's fill latency
//     (measured faster than double-buffering at two blocks per CU: RT_NBUF).
//   * Levels are specialised on d, so every candidate read is one ds_read_b128 with an immediate
//     offset from a single per-lane base; the 49 running half sums live in registers across the
//     three chunks (the sum stays sequential over k = 0..23: c10::Half step rounding unchanged).
//   * Lanes whose 49 candidates do not all fall inside the window (outlier centres, a clipped
//     window) are scored cooperatively by their wave straight from global memory: 49 lanes, one
//     candidate each, then a first-maximum wave arg-max (same result as the sequential scan).
//   * Tiles are dealt to XCDs in contiguous runs (bijective remap) so each XCD's 4 MiB L2 holds
//     its slab of D11.
// Compiled with -ffp-contract=off.
#include "m3s_half.hpp"

namespace m3s {

#define RT_TW 32
#define RT_TH 8
#define RT_COLS 64
#define RT_ROWS 40
#ifndef RT_NBUF
#define RT_NBUF 1  // 1: 40 KiB, 4 blocks/CU (measured faster); 2: 80 KiB, double-buffered chunks, 2 blocks/CU
#endif

typedef __attribute__((address_space(1))) const void* gvoid_t;
typedef __attribute__((address_space(3))) void* lvoid_t;

__device__ __forceinline__ int xcd_remap(int b, int nb) {  // bijective (cdna guide §5 "XCD swizzle")
  const int q = nb / 8, r = nb % 8, x = b % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

// Lanes whose level does not fit the window: the wave takes them one at a time, 49 lanes score the
// 49 candidates of that pixel from global memory (three 16-B loads each, all in flight at once) and
// a wave arg-max picks the first candidate in scan order holding the maximum -- the same result as
// the reference's sequential strict-'>' scan, since the running max only grows from +0.
#ifdef M3S_COOP_NOINLINE
#define M3S_COOP_ATTR __attribute__((noinline))
#else
#define M3S_COOP_ATTR __forceinline__  // a call would spill the caller's live VGPRs to scratch
#endif
template <int D>
__device__ M3S_COOP_ATTR void refine_level_coop(const h1* __restrict__ img, int H, int W, const h2* q,
                                                             int& cu, int& cv, h1& max_score, bool need, int lane) {
  constexpr int R = 3, RD = R * D, F = 24, G = 2 * R + 1;
  uint64_t m = __ballot(need);
  const int ci = lane / G, cj = lane % G;
  while (m) {
    const int src = __ffsll((long long)m) - 1;
    m &= m - 1;
    const int scu = __shfl(cu, src, 64), scv = __shfl(cv, src, 64);
    h2 sq[F / 2];
#pragma unroll
    for (int k = 0; k < F / 2; k++) {
      const int t = __shfl(*reinterpret_cast<const int*>(&q[k]), src, 64);
      sq[k] = *reinterpret_cast<const h2*>(&t);
    }
    const int u = scu - RD + ci * D, v = scv - RD + cj * D;
    const bool ok = lane < G * G && u >= 0 && u < W && v >= 0 && v < H;
    const uint4* p = reinterpret_cast<const uint4*>(img + ((size_t)min(max(v, 0), H - 1) * W + min(max(u, 0), W - 1)) * F);
    const uint4 c0 = p[0], c1 = p[1], c2 = p[2];
    h1 sc = (h1)0.0f;
    add8(sc, &sq[0], c0);
    add8(sc, &sq[4], c1);
    add8(sc, &sq[8], c2);
    const float sf = (ok && sc == sc) ? (float)sc : -INFINITY;  // NaN never wins a strict '>'
    float vmax = sf;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) vmax = fmaxf(vmax, __shfl_xor(vmax, off, 64));
    const uint64_t hit = __ballot(sf == vmax);
    const int first = __ffsll((long long)hit) - 1;
    if (lane == src && vmax > (float)max_score) {
      max_score = (h1)vmax;
      cu = scu - RD + (first / G) * D;
      cv = scv - RD + (first % G) * D;
    }
  }
}

// 49 candidates x one 8-channel chunk from the LDS window; base = candidate (0,0) of this lane
#ifdef M3S_REFINE_STATS
__device__ unsigned long long g_refine_stats[32];
#endif

template <int D>
__device__ __forceinline__ void score_chunk(const uint4* base, const h2* q4, h1* s) {
  constexpr int G = 7;
#pragma unroll
  for (int i = 0; i < G; i++) {
#pragma unroll
    for (int j = 0; j < G; j++) add8(s[i * G + j], q4, base[j * D * RT_COLS + i * D]);
    // bound the live candidate loads to one column (7 x 16 B) to keep the VGPR budget
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <int D>
__device__ __forceinline__ void refine_level(const h1* __restrict__ img, int H, int W, bool active, const h2* q,
                                             int& cu, int& cv, h1& max_score, uint4 (*lds)[RT_ROWS * RT_COLS],
                                             int (*s_red)[4], int lane, int wid, int u_pix, int v_pix) {
  constexpr int R = 3, G = 2 * R + 1, F = 24, RD = R * D;
  // 1) tile flow estimate: mean centre displacement (cu - u_pix) over active lanes
  int su = active ? cu - u_pix : 0, sv = active ? cv - v_pix : 0, na = active ? 1 : 0;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    su += __shfl_xor(su, off, 64);
    sv += __shfl_xor(sv, off, 64);
    na += __shfl_xor(na, off, 64);
  }
  __syncthreads();  // previous level's readers of s_red / lds are done
  if (lane == 0) {
    s_red[wid][0] = su;
    s_red[wid][1] = sv;
    s_red[wid][2] = na;
  }
  __syncthreads();
  const int nall = max(1, s_red[0][2] + s_red[1][2] + s_red[2][2] + s_red[3][2]);
  const int fu = (s_red[0][0] + s_red[1][0] + s_red[2][0] + s_red[3][0]) / nall;
  const int fv = (s_red[0][1] + s_red[1][1] + s_red[2][1] + s_red[3][1]) / nall;
  // 2) bbox of the inlier centres (within 16 px of pixel + tile flow); outliers take the global path
  const bool inl = active && abs(cu - u_pix - fu) <= 16 && abs(cv - v_pix - fv) <= 16;
  int mnu = inl ? cu : INT_MAX, mxu = inl ? cu : INT_MIN;
  int mnv = inl ? cv : INT_MAX, mxv = inl ? cv : INT_MIN;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    mnu = min(mnu, __shfl_xor(mnu, off, 64));
    mxu = max(mxu, __shfl_xor(mxu, off, 64));
    mnv = min(mnv, __shfl_xor(mnv, off, 64));
    mxv = max(mxv, __shfl_xor(mxv, off, 64));
  }
  __syncthreads();
  if (lane == 0) {
    s_red[wid][0] = mnu;
    s_red[wid][1] = mxu;
    s_red[wid][2] = mnv;
    s_red[wid][3] = mxv;
  }
  __syncthreads();
  mnu = min(min(s_red[0][0], s_red[1][0]), min(s_red[2][0], s_red[3][0]));
  mxu = max(max(s_red[0][1], s_red[1][1]), max(s_red[2][1], s_red[3][1]));
  mnv = min(min(s_red[0][2], s_red[1][2]), min(s_red[2][2], s_red[3][2]));
  mxv = max(max(s_red[0][3], s_red[1][3]), max(s_red[2][3], s_red[3][3]));
  if (mnu > mxu) {  // no inlier: any window (every active lane goes global)
    mnu = mxu = 0;
    mnv = mxv = 0;
  }
  // window placement: exact bbox cover when it fits, else centred on the bbox
  const int x_lo = mnu - RD, x_hi = mxu + RD, y_lo = mnv - RD, y_hi = mxv + RD;
  const int wx0 = (x_hi - x_lo + 1 <= RT_COLS) ? x_lo : ((x_lo + x_hi) >> 1) - RT_COLS / 2;
  const int wy0 = (y_hi - y_lo + 1 <= RT_ROWS) ? y_lo : ((y_lo + y_hi) >> 1) - RT_ROWS / 2;
  const int nrows = min(RT_ROWS, y_hi - wy0 + 1);
  const int gx = min(max(wx0 + lane, 0), W - 1);
  const int u_lo = cu - RD, v_lo = cv - RD;
  const int bx = u_lo - wx0, by = v_lo - wy0;  // window coordinates of candidate (0, 0)
  const bool lane_in = active && bx >= 0 && bx + 2 * RD < RT_COLS && by >= 0 && by + 2 * RD < nrows;
#ifdef M3S_REFINE_STATS  // (experiment builds only) per-level outlier lanes / waves
  {
    const uint64_t bm = __ballot(active && !lane_in);
    if (lane == 0 && bm) {
      atomicAdd(&g_refine_stats[2 * D], (unsigned long long)__popcll(bm));
      atomicAdd(&g_refine_stats[2 * D + 1], 1ull);
    }
  }
#endif
#ifndef M3S_NO_COOP  // (timing experiment only: skips the outlier lanes)
  if (__ballot(active && !lane_in)) refine_level_coop<D>(img, H, W, q, cu, cv, max_score, active && !lane_in, lane);
#endif
  h1 s[G * G];
#pragma unroll
  for (int c = 0; c < G * G; c++) s[c] = (h1)0.0f;
#if RT_NBUF == 2
#pragma unroll
  for (int chunk = 0; chunk < F / 8; chunk++) {
    if (chunk == 0) {  // the first chunk of a level cannot be prefetched: its window needs the bbox
      for (int y = wid; y < nrows; y += 4) {
        const int gy = min(max(wy0 + y, 0), H - 1);
        __builtin_amdgcn_global_load_lds((gvoid_t)(img + ((size_t)gy * W + gx) * F), (lvoid_t)&lds[0][y * RT_COLS],
                                         16, 0, 0);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
    if (chunk + 1 < F / 8) {  // one global_load_lds (64 lanes x 16 B) per window row, next chunk
      for (int y = wid; y < nrows; y += 4) {
        const int gy = min(max(wy0 + y, 0), H - 1);
        __builtin_amdgcn_global_load_lds((gvoid_t)(img + ((size_t)gy * W + gx) * F + (chunk + 1) * 8),
                                         (lvoid_t)&lds[(chunk + 1) & 1][y * RT_COLS], 16, 0, 0);
      }
    }
    if (lane_in) score_chunk<D>(&lds[chunk & 1][by * RT_COLS + bx], &q[chunk * 4], s);
    if (chunk + 1 < F / 8) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  }
#else
  __syncthreads();  // the reduction scratch aliases the window: its readers are done
#pragma unroll
  for (int chunk = 0; chunk < F / 8; chunk++) {
    if (chunk) __syncthreads();  // previous chunk's readers are done
    for (int y = wid; y < nrows; y += 4) {
      const int gy = min(max(wy0 + y, 0), H - 1);
      __builtin_amdgcn_global_load_lds((gvoid_t)(img + ((size_t)gy * W + gx) * F + chunk * 8),
                                       (lvoid_t)&lds[0][y * RT_COLS], 16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (lane_in) score_chunk<D>(&lds[0][by * RT_COLS + bx], &q[chunk * 4], s);
  }
#endif
  if (lane_in) {  // scan-order arg-max: u outer, v inner, strict '>' (matching_kernels.cu:54-71)
    int bu = cu, bvv = cv;
#pragma unroll
    for (int i = 0; i < G; i++) {
      const bool uok = u_lo + i * D >= 0 && u_lo + i * D < W;
#pragma unroll
      for (int j = 0; j < G; j++) {
        const bool vok = v_lo + j * D >= 0 && v_lo + j * D < H;
        if (uok && vok && s[i * G + j] > max_score) {
          max_score = s[i * G + j];
          bu = u_lo + i * D;
          bvv = v_lo + j * D;
        }
      }
    }
    cu = bu;
    cv = bvv;
  }
}

// P1_I64: p1 given as (B,N,2) int64 (reference op) else int32 (fused); LIN_OUT: write idx = u + W v.
template <bool D21_F32, bool P1_I64, bool LIN_OUT>
__global__ void __launch_bounds__(256, 2 * (3 - RT_NBUF)) refine_tile_kernel(const h1* __restrict__ D11h, const void* __restrict__ D21,
                                                             const void* __restrict__ p1v, void* __restrict__ outv,
                                                             int H, int W, int dilation_max, int tiles_x,
                                                             int tiles_per_img, int nblocks) {
  constexpr int F = 24;
  __shared__ uint4 lds[RT_NBUF][RT_ROWS * RT_COLS];
  // level-start reductions run while buffer 1 is idle (its last readers passed a barrier, its next
  // fill is issued after the chunk-0 barrier)
  int(*s_red)[4] = reinterpret_cast<int(*)[4]>(&lds[RT_NBUF - 1][0]);
  const int lb = xcd_remap(blockIdx.x, nblocks);
  const int b = lb / tiles_per_img, t = lb % tiles_per_img;
  const int tx = t % tiles_x, ty = t / tiles_x;
  const int lx = threadIdx.x % RT_TW, ly = threadIdx.x / RT_TW;
  const int u_pix = tx * RT_TW + lx, v_pix = ty * RT_TH + ly;
  const bool active = u_pix < W && v_pix < H;
  const int N = H * W;
  const size_t bn = (size_t)b * N + (size_t)v_pix * W + u_pix;
  const h1* img = D11h + (size_t)b * N * F;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  h2 q[F / 2];
  int cu = 0, cv = 0;
  if (active) {
    load_query<F, D21_F32>(D21, bn, q);
    if constexpr (P1_I64) {
      cu = (int)reinterpret_cast<const int64_t*>(p1v)[bn * 2];
      cv = (int)reinterpret_cast<const int64_t*>(p1v)[bn * 2 + 1];
    } else {
      cu = reinterpret_cast<const int*>(p1v)[bn * 2];
      cv = reinterpret_cast<const int*>(p1v)[bn * 2 + 1];
    }
  } else {
#pragma unroll
    for (int k = 0; k < F / 2; k++) q[k] = h2{(h1)0.0f, (h1)0.0f};
  }
  h1 max_score = (h1)0.0f;  // numeric_limits<c10::Half>::min() == +0, never reset between levels
  for (int d = dilation_max; d > 0; d--) {
    switch (d) {
      case 8: refine_level<8>(img, H, W, active, q, cu, cv, max_score, lds, s_red, lane, wid, u_pix, v_pix); break;
      case 7: refine_level<7>(img, H, W, active, q, cu, cv, max_score, lds, s_red, lane, wid, u_pix, v_pix); break;
      case 6: refine_level<6>(img, H, W, active, q, cu, cv, max_score, lds, s_red, lane, wid, u_pix, v_pix); break;
      case 5: refine_level<5>(img, H, W, active, q, cu, cv, max_score, lds, s_red, lane, wid, u_pix, v_pix); break;
      case 4: refine_level<4>(img, H, W, active, q, cu, cv, max_score, lds, s_red, lane, wid, u_pix, v_pix); break;
      case 3: refine_level<3>(img, H, W, active, q, cu, cv, max_score, lds, s_red, lane, wid, u_pix, v_pix); break;
      case 2: refine_level<2>(img, H, W, active, q, cu, cv, max_score, lds, s_red, lane, wid, u_pix, v_pix); break;
      default: refine_level<1>(img, H, W, active, q, cu, cv, max_score, lds, s_red, lane, wid, u_pix, v_pix); break;
    }
  }
  if (active) {
    if constexpr (LIN_OUT) {
      reinterpret_cast<int64_t*>(outv)[bn] = (int64_t)cu + (int64_t)W * cv;
    } else {
      reinterpret_cast<int64_t*>(outv)[bn * 2] = cu;
      reinterpret_cast<int64_t*>(outv)[bn * 2 + 1] = cv;
    }
  }
}

}  // namespace m3s

// D21 f32 + p1 int32 -> idx (fused path) or D21 f16 + p1 int64 -> p1_new (reference op).
// Returns hipErrorNotSupported when the shape is not eligible (caller falls back to per-pixel).
extern "C" hipError_t m3s_launch_refine_tile(const void* D11h, const void* D21, const void* p1, void* out, int B,
                                             int H, int W, int F, int radius, int dilation_max, int fused,
                                             hipStream_t s) {
  if (F != 24 || radius != 3 || dilation_max < 1 || dilation_max > 8) return hipErrorNotSupported;
  const int tx = (W + RT_TW - 1) / RT_TW, ty = (H + RT_TH - 1) / RT_TH, nb = tx * ty * B;
  const m3s::h1* a = reinterpret_cast<const m3s::h1*>(D11h);
  if (fused)
    hipLaunchKernelGGL((m3s::refine_tile_kernel<true, false, true>), dim3(nb), dim3(256), 0, s, a, D21, p1, out, H, W,
                       dilation_max, tx, tx * ty, nb);
  else
    hipLaunchKernelGGL((m3s::refine_tile_kernel<false, true, false>), dim3(nb), dim3(256), 0, s, a, D21, p1, out, H,
                       W, dilation_max, tx, tx * ty, nb);
  return hipGetLastError();
}

#ifdef M3S_REFINE_STATS
extern "C" int m3s_debug_refine_stats(unsigned long long* out, int reset) {
  (void)hipDeviceSynchronize();
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(m3s::g_refine_stats), sizeof(unsigned long long) * 32) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[32] = {0};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(m3s::g_refine_stats), z, sizeof(z));
  }
  return 0;
}
#endif
