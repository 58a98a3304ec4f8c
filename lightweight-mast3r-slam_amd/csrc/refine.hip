// LDS-tiled coarse-to-fine descriptor refine for MI355X (gfx950), F = 24, radius 3.
//
// Reference semantics: refine_matches_kernel<c10::Half>, /root/reference/mast3r_slam/backend/src/
// matching_kernels.cu:25-81 — per query pixel, dilation d = dmax..1, a 7x7 grid of stride d around
// the current centre (u outer, v inner), score = sequential c10::Half sum over 24 channels of
// half(q_k * c_k), strict '>' against a running max that starts at +0 and is never reset, re-centre
// after each level.
//
// MI355X design: one 32x8 pixel tile per 256-lane block (4 blocks / CU, 40 KiB LDS each).
//   * Once per tile the block estimates the tile's flow (mean initial centre displacement); per level
//     it takes the bbox of the centres within 16 px of it, places a 64-column x 40-row window over
//     bbox +- 3d and streams D11 (f16) into LDS in three 8-channel chunks (16 B / px) with
//     global_load_lds — one wave-instruction per window row, only the cover's columns. Four resident blocks per CU
//     hide each other's fill latency (measured: faster than double-buffering at two blocks per CU). The fine levels'
//     covers are small enough for other layouts of the same 40 KiB (bound-screened path): at d = 2 two 26 x 48
//     chunk buffers (chunk c + 1 streams in while chunk c is screened), at d = 1 all three chunk planes of a 17 x 48
//     window in one fill, the survivors then rescored from LDS.
//   * Levels are specialised on d, so every candidate read is one ds_read_b128 with an immediate
//     offset from a single per-lane base; the 49 running half sums live in registers across the
//     three chunks (the sum stays sequential over k = 0..23: c10::Half step rounding unchanged).
//   * A lane whose 49 candidates do not fit the window (an outlier centre, a clipped window) is
//     DEFERRED: its state (pixel, centre, running max, level) is appended to a list and the lane
//     leaves the tile (it no longer widens the window of later levels). refine_outlier_kernel then
//     finishes every deferred pixel with one wave per pixel: 49 lanes score the 49 candidates from
//     global memory (all loads in flight at once) and a first-maximum wave arg-max reproduces the
//     sequential strict-'>' scan (the running max only grows from +0). Without a list (reference
//     op path, no workspace) the wave scores its outliers in place, one at a time (wave_level).
//   * Tiles are dealt to XCDs in contiguous runs (bijective remap) so each XCD's 4 MiB L2 holds
//     its slab of D11.
// Compiled with -ffp-contract=off and -fno-slp-vectorize: each candidate's half sum stays a scalar chain (VOP2
// v_add_f16 for the even channel, SDWA v_add_f16 for the odd one) instead of the SLP vectoriser pairing two
// candidates per v_pk_add_f16 behind v_perm / v_pack transposes. Measured issue costs on gfx950 at 4 waves/SIMD
// (scripts/micro/fma_rates, profiles/r03_valu_issue_rates.txt): VOP2 f16 add 1.18 ns, SDWA / VOP3P / v_perm
// 2.03-2.09 ns per wave-instruction, so 2.67 ns per channel-candidate against 3.1 ns paired: 125 -> 116 us.
#include "m3s_half.hpp"

namespace m3s {

// Tile geometry (RT_WAVES waves per block, two pixel rows per wave). The shipped build: 32 x 8 tiles, 4 waves, a
// 40-row window (40 KiB, four blocks per CU). RT_TALL (experiment): 32 x 16 tiles, 8 waves, a 56-row window (56 KiB,
// two blocks per CU: the same 16 waves per CU), so the +-3d halo of a level's window is shared by twice the pixels.
#ifndef RT_TALL
#define RT_TALL 0
#endif
#define RT_TW 32
#define RT_COLS 64
#define RT_PCOLS 48
#if RT_TALL
#define RT_WAVES 8
#define RT_TH 16
#define RT_ROWS 56
#define RT_PROWS 24
#define RT_DROWS 36
#else
#define RT_WAVES 4
#define RT_TH 8
#define RT_ROWS 40  // 40 x 64 x 16 B = 40 KiB per block: four blocks per CU
// packed window (SCREEN, d = 1): all three chunk planes resident at once, 3 x 17 rows x 48 columns x 16 B = 38.25 KiB
// (the d = 1 cover is 16 x 39-40 on 97 % of the synthetic 512x512 tiles, scripts/refine_window_stats.py)
#define RT_PROWS 17
// double-buffered window (SCREEN, d = 2): two 26-row x 48-column chunk buffers (2 x 19.5 KiB), chunk c + 1 streams in
// while chunk c is screened (the d = 2 cover is 23 x 45-47 on 97.6 % of the synthetic 512x512 tiles)
#define RT_DROWS 26
#endif
static_assert(RT_TH == 2 * RT_WAVES, "two pixel rows per wave");
static_assert(3 * RT_PROWS * RT_PCOLS <= RT_ROWS * RT_COLS && 2 * RT_DROWS * RT_PCOLS <= RT_ROWS * RT_COLS,
              "the packed and double-buffered windows share the block's window");
#define RT_THREADS (64 * RT_WAVES)
#define RT_PPLANE (RT_PROWS * RT_PCOLS)
#define RT_DBUF (RT_DROWS * RT_PCOLS)
#ifndef RT_INPLACE_MAX  // window outliers a wave scores in place at one level (more: deferred to the list)
#define RT_INPLACE_MAX 8
#endif

typedef __attribute__((address_space(1))) const void* gvoid_t;
typedef __attribute__((address_space(3))) void* lvoid_t;

#ifdef M3S_REFINE_STATS  // (experiment builds only) per-level deferred lanes / waves
__device__ unsigned long long g_refine_stats[64];
#endif
#ifdef M3S_REFINE_BSTAMPS  // (experiment builds only) per-block start / end s_memrealtime, hardware id, active lanes
__device__ unsigned long long g_refine_bstamps[8192 * 4];
#endif

// One level of one pixel by the whole wave (cu, cv, max_score, sq wave-uniform): lane c < 49 scores
// candidate (c / 7, c % 7) from global memory; the first candidate in scan order holding the wave
// maximum wins if it beats the running max — the sequential strict-'>' scan's result.
// D11h layouts: PLANAR (fused path, written by prep_rays_kernel) = per image three chunk planes (H,W,8) f16, so a
// window row of one chunk is one contiguous 16 B-per-pixel run; otherwise the caller's (H,W,24) f16.
template <bool PLANAR>
__device__ __forceinline__ const h1* pix_ptr(const h1* img, size_t pix) {
  return img + pix * (PLANAR ? 8 : 24);
}
template <bool PLANAR>
__device__ __forceinline__ void load_chunks(const h1* p, size_t N, uint4& c0, uint4& c1, uint4& c2) {
  const size_t cs = PLANAR ? N * 8 : 8;  // chunk stride in halves
  c0 = *reinterpret_cast<const uint4*>(p);
  c1 = *reinterpret_cast<const uint4*>(p + cs);
  c2 = *reinterpret_cast<const uint4*>(p + 2 * cs);
}

template <int D, bool PLANAR>
__device__ __forceinline__ void wave_level(const h1* __restrict__ img, int H, int W, const h2* sq, int& cu, int& cv,
                                           h1& max_score, int lane) {
  constexpr int R = 3, RD = R * D, G = 2 * R + 1;
  const int ci = lane / G, cj = lane % G;
  const int u = cu - RD + ci * D, v = cv - RD + cj * D;
  const bool ok = lane < G * G && u >= 0 && u < W && v >= 0 && v < H;
  uint4 c0, c1, c2;
  load_chunks<PLANAR>(pix_ptr<PLANAR>(img, (size_t)min(max(v, 0), H - 1) * W + min(max(u, 0), W - 1)),
                      (size_t)H * W, c0, c1, c2);
  h1 sc = (h1)0.0f;
  add8(sc, &sq[0], c0);
  add8(sc, &sq[4], c1);
  add8(sc, &sq[8], c2);
  const float sf = (ok && sc == sc) ? (float)sc : -INFINITY;  // NaN never wins a strict '>'
  float vmax = sf;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) vmax = fmaxf(vmax, __shfl_xor(vmax, off, 64));
  const int first = __ffsll((long long)__ballot(sf == vmax)) - 1;
  if (vmax > (float)max_score) {
    max_score = (h1)vmax;
    cu = cu - RD + (first / G) * D;
    cv = cv - RD + (first % G) * D;
  }
}

// 49 candidates x one 8-channel chunk from the LDS window; base = candidate (0,0) of this lane
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

// Bound-screened refine (SCREEN): the level's 49 candidates are first scored by an fp32 dot of the same half operands
// (v_dot2c_f32_f16: 12 per candidate instead of 24 half products + 24 half adds), then only candidates whose screen
// score lies within the rounding bound of the level's best are scored by the exact c10::Half chain, in scan order.
// The result is the sequential scan's, bit for bit:
//   * |S_half - S_real| <= 24 u P + 24 * 2^-25 for the c10::Half chain (u = 2^-11: 24 product roundings, 23 add
//     roundings, each <= u times a partial sum <= (1 + 0.013) P), where P = sum |q_k c_k| <= |q|_2 |c|_2, and
//     |S_dot2 - S_real| <= 12 (3 * 2^-24 P + 2^-36) (measured on gfx950, scripts/micro/dot2_exact.hip: at most
//     3 fp32 roundings of |a0 b0| + |a1 b1| + |acc| per instruction, 2^-36 absolute with subnormal halves);
//     so B = 0.0125 |q| cmax + 2^-18 bounds |S_half - S_dot2| (24 u = 0.01172), cmax = max |D11h[pixel]|_2
//     over the image (prep_rays_kernel).
//   * The winner w (first candidate in scan order with S_half[w] = M = max S_half, when M beats the running max)
//     has S_dot2[w] >= M - B >= Lmax - 2B, where Lmax = max over in-image candidates of S_dot2 (M >= S_half[c] >=
//     S_dot2[c] - B), and S_dot2[w] > max_score - B. A candidate failing either cannot win nor tie the winner,
//     so the scan over the survivors alone (ascending order, strict '>') returns the full scan's result.
//   * After the first level the centre candidate (3,3) is the last winner (its score IS the running max) or the
//     start pixel that did not beat +0: it never wins a strict '>' and is dropped from the survivors.
//   * |q| cmax > 16384 (overflow range) or non-finite: every in-image candidate survives (exact for all).
template <int D, int STRIDE = RT_COLS>
__device__ __forceinline__ void screen_chunk(const uint4* base, const h2* q4, float* a) {
  constexpr int G = 7;
#pragma unroll
  for (int i = 0; i < G; i++) {
    // the column's candidate reads in flight together (RT_COLBATCH of them: one LDS latency per batch, not per
    // candidate)
#ifndef RT_COLBATCH
#define RT_COLBATCH 7
#endif
#pragma unroll
    for (int j0 = 0; j0 < G; j0 += RT_COLBATCH) {
      uint4 c[RT_COLBATCH];
#pragma unroll
      for (int j = j0; j < min(G, j0 + RT_COLBATCH); j++) c[j - j0] = base[j * D * STRIDE + i * D];
#pragma unroll
      for (int j = j0; j < min(G, j0 + RT_COLBATCH); j++) {
        const h2* cv = reinterpret_cast<const h2*>(&c[j - j0]);
        float t = a[i * G + j];
#pragma unroll
        for (int k = 0; k < 4; k++) t = __builtin_amdgcn_fdot2(q4[k], cv[k], t, false);
        a[i * G + j] = t;
      }
    }
    // pin the column's dot products here: otherwise the last chunk's are sunk into the survivor code and all 49
    // candidate loads stay live across it (1000+ spilled VGPRs)
    float* ac = &a[i * G];
    asm volatile("" : "+v"(ac[0]), "+v"(ac[1]), "+v"(ac[2]), "+v"(ac[3]), "+v"(ac[4]), "+v"(ac[5]), "+v"(ac[6]));
    __builtin_amdgcn_sched_barrier(0);
  }
}

// bit c set where a[c] >= T (c < 49; NaN never), two VALU per candidate: the compare's lane mask (an SGPR pair) shifted
// into the mask word by an add-with-carry (m = m + m + carry), candidates in descending order so candidate c lands on
// bit c. The compiler's select / or / 64-bit shift form took about four per candidate. Each instruction is its own asm
// statement and the compares run two candidates ahead of the adds: gfx950 needs two wait states between a VALU write
// of an SGPR and a VALU read of it (the compiler pads v_cmp -> v_cndmask with s_nop 1), and the interleave provides
// them without nops; the compiler sees every operand, so it pads wherever the distance is short (the last two adds).
__device__ __forceinline__ uint64_t screen_mask(const float* a, float T) {
  constexpr int C = 49;
  unsigned lo = 0u, hi = 0u;
  unsigned long long s[C];
#pragma unroll
  for (int k = 0; k < C + 2; k++) {
    if (k < C) asm volatile("v_cmp_ge_f32_e64 %0, %1, %2" : "=s"(s[k]) : "v"(a[C - 1 - k]), "v"(T));
    if (k >= 2) {
      unsigned long long co;  // the carry-out (dead)
      if (C - 1 - (k - 2) >= 32)
        asm volatile("v_addc_co_u32_e64 %0, %1, %0, %0, %2" : "+v"(hi), "=s"(co) : "s"(s[k - 2]));
      else
        asm volatile("v_addc_co_u32_e64 %0, %1, %0, %0, %2" : "+v"(lo), "=s"(co) : "s"(s[k - 2]));
    }
  }
  return ((uint64_t)hi << 32) | lo;
}

// exact c10::Half chains of the survivor mask m in ascending scan order, read from D11h (L2); strict '>'. Two
// survivors per trip: both candidates' loads are in flight before the first chain (one L2 round trip per pair)
template <int D, bool PLANAR>
__device__ __forceinline__ void exact_survivors(const h1* __restrict__ img, int H, int W, const h2* q, int u_lo,
                                                int v_lo, uint64_t m, h1& max_score, int& bi) {
  while (__ballot(m != 0)) {  // wave-uniform trip count: the lane with the most survivors
    const int ca = m != 0 ? __ffsll((long long)m) - 1 : -1;
    m &= m - 1;
    const int cb = m != 0 ? __ffsll((long long)m) - 1 : -1;
    m &= m - 1;
    uint4 a0, a1, a2, b0, b1, b2;
    if (ca >= 0) {
      const int i = ca / 7, j = ca - 7 * i;
      load_chunks<PLANAR>(pix_ptr<PLANAR>(img, (size_t)(v_lo + j * D) * W + (u_lo + i * D)), (size_t)H * W, a0, a1,
                          a2);
    }
    if (cb >= 0) {
      const int i = cb / 7, j = cb - 7 * i;
      load_chunks<PLANAR>(pix_ptr<PLANAR>(img, (size_t)(v_lo + j * D) * W + (u_lo + i * D)), (size_t)H * W, b0, b1,
                          b2);
    }
    if (ca >= 0) {
      h1 sc = (h1)0.0f;
      add8(sc, &q[0], a0);
      add8(sc, &q[4], a1);
      add8(sc, &q[8], a2);
      if (sc > max_score) {
        max_score = sc;
        bi = ca;
      }
    }
    if (cb >= 0) {
      h1 sc = (h1)0.0f;
      add8(sc, &q[0], b0);
      add8(sc, &q[4], b1);
      add8(sc, &q[8], b2);
      if (sc > max_score) {
        max_score = sc;
        bi = cb;
      }
    }
  }
}

// LDS DMA of one window row (64 lanes x 16 B) by inline asm, for the double-buffered window: the compiler treats a
// global_load_lds as an LDS store of unknown extent and drains it (vmcnt(0)) before the next ds_read, which would
// serialise the fill of chunk c + 1 behind the screen of chunk c; the explicit vmcnt(0) + barrier order it instead.
// One wait state between the M0 write and the DMA (the compiler's own sequences keep one there too).
// lds_addr: the row's LDS byte address (wave-uniform)
__device__ __forceinline__ void lds_dma_row(const h1* g, unsigned lds_addr) {
  const unsigned m0 = __builtin_amdgcn_readfirstlane(lds_addr);
  // M0 is an operand ({m0}): the compiler writes it itself right before the asm and knows its value (it also sets M0
  // for its own global_load_lds); the s_nop is the wait state between that M0 write and the DMA that reads it
  asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "{m0}"(m0) : "memory");
}

// the packed window's variant: the survivors' three chunks are read from the resident LDS planes (base = candidate
// (0,0) of this lane in plane 0), no L2 round trip; same ascending order, same strict '>'
template <int D>
__device__ __forceinline__ void exact_survivors_lds(const uint4* base, const h2* q, uint64_t m, h1& max_score,
                                                    int& bi) {
  while (m != 0) {
    const int c = __ffsll((long long)m) - 1;
    m &= m - 1;
    const int i = c / 7, j = c - 7 * i;
    const uint4* p = base + j * D * RT_PCOLS + i * D;
    const uint4 c0 = p[0], c1 = p[RT_PPLANE], c2 = p[2 * RT_PPLANE];
    h1 sc = (h1)0.0f;
    add8(sc, &q[0], c0);
    add8(sc, &q[4], c1);
    add8(sc, &q[8], c2);
    if (sc > max_score) {
      max_score = sc;
      bi = c;
    }
  }
}

struct TileCtx {
  const h1* img;
  int H, W, lane, wid, u_pix, v_pix;
  int fu, fv;   // tile flow estimate: mean initial centre displacement (fixed for all levels)
  int tcu, tcv; // tile centre + flow estimate: the window's centre when the centres' cover does not fit
  int bn;       // batch * N + pixel
  int4* olist;  // deferred-pixel list (nullable: score outliers in place)
  int* ocount;
  unsigned lds_addr;  // LDS byte address of the window (the block's __shared__ array)
  float bq;      // SCREEN: this lane's bound B (0.0125 |q| cmax + 2^-18)
  bool sok;      // SCREEN: the bound is usable (|q| cmax <= 16384 and finite)
};

template <int D, bool SCREEN, bool PLANAR>
__device__ __forceinline__ void refine_level(const TileCtx& t, bool& active, const h2* q, int& cu, int& cv,
                                             h1& max_score, uint4* lds, int (*s_red)[4], bool first) {
  constexpr int R = 3, G = 2 * R + 1, F = 24, RD = R * D;
  const int lane = t.lane, wid = t.wid, H = t.H, W = t.W;
  // bbox of the inlier centres (within 16 px of pixel + the tile's flow estimate t.fu/t.fv)
  const bool inl = active && abs(cu - t.u_pix - t.fu) <= 16 && abs(cv - t.v_pix - t.fv) <= 16;
  int mnu = inl ? cu : INT_MAX, mxu = inl ? cu : INT_MIN;
  int mnv = inl ? cv : INT_MAX, mxv = inl ? cv : INT_MIN;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    mnu = min(mnu, __shfl_xor(mnu, off, 64));
    mxu = max(mxu, __shfl_xor(mxu, off, 64));
    mnv = min(mnv, __shfl_xor(mnv, off, 64));
    mxv = max(mxv, __shfl_xor(mxv, off, 64));
  }
  __syncthreads();  // previous level's readers of s_red / lds are done
  if (lane == 0) {
    s_red[wid][0] = mnu;
    s_red[wid][1] = mxu;
    s_red[wid][2] = mnv;
    s_red[wid][3] = mxv;
  }
  __syncthreads();
  mnu = s_red[0][0];
  mxu = s_red[0][1];
  mnv = s_red[0][2];
  mxv = s_red[0][3];
#pragma unroll
  for (int w = 1; w < RT_WAVES; w++) {
    mnu = min(mnu, s_red[w][0]);
    mxu = max(mxu, s_red[w][1]);
    mnv = min(mnv, s_red[w][2]);
    mxv = max(mxv, s_red[w][3]);
  }
  if (mnu > mxu) {  // no inlier: any window (every active lane is an outlier)
    mnu = mxu = 0;
    mnv = mxv = 0;
  }
  // window placement: exact bbox cover when it fits, else centred on the tile's centre displaced by its flow
  // estimate. A cover that does not fit is mostly a tight cluster plus a few far centres at one end: centring on the
  // bbox middle deferred the cluster itself (d = 4 on the synthetic 512x512 pair: 1502 deferred lanes against 54,
  // scripts/refine_window_stats.py)
  const int x_lo = mnu - RD, x_hi = mxu + RD, y_lo = mnv - RD, y_hi = mxv + RD;
  bool packed = false, dbuf = false;  // block-uniform: every input is
  if constexpr (SCREEN && D == 1) packed = x_hi - x_lo + 1 <= RT_PCOLS && y_hi - y_lo + 1 <= RT_PROWS;
  if constexpr (SCREEN && D == 2) dbuf = x_hi - x_lo + 1 <= RT_PCOLS && y_hi - y_lo + 1 <= RT_DROWS;
  const int wc = (packed || dbuf) ? RT_PCOLS : RT_COLS, wr = packed ? RT_PROWS : (dbuf ? RT_DROWS : RT_ROWS);
  const int wx0 = (x_hi - x_lo + 1 <= wc) ? x_lo : t.tcu - wc / 2;
  const int wy0 = (y_hi - y_lo + 1 <= wr) ? y_lo : t.tcv - wr / 2;
  // rows and columns actually filled: the bbox cover, clipped to the window (a fine level's cover is ~40 of the 64
  // columns: the fill, bound by L2 -> LDS bandwidth, moves only those)
  const int nrows = min(wr, y_hi - wy0 + 1), ncols = min(wc, x_hi - wx0 + 1);
  const bool col_in = lane < ncols;
  const int gx = min(max(wx0 + lane, 0), W - 1);
  const int u_lo = cu - RD, v_lo = cv - RD;
  const int bx = u_lo - wx0, by = v_lo - wy0;  // window coordinates of candidate (0, 0)
  const bool lane_in = active && bx >= 0 && bx + 2 * RD < ncols && by >= 0 && by + 2 * RD < nrows;
  const bool outl = active && !lane_in;
  const uint64_t om = __ballot(outl);
#ifdef M3S_REFINE_STATS
  if (lane == 0 && om) {
    atomicAdd(&g_refine_stats[2 * D], (unsigned long long)__popcll(om));
    atomicAdd(&g_refine_stats[2 * D + 1], 1ull);
  }
#endif
  if (om) {
    // a wave with a few window outliers scores them in place (one wave-level each, while the rest of the tile waits
    // at the next barrier); more than RT_INPLACE_MAX go to the deferred list (one wave per pixel in
    // refine_outlier_kernel), which keeps pathological inputs (scattered warm starts: every lane an outlier) parallel
    if (t.olist != nullptr && __popcll(om) > RT_INPLACE_MAX) {
      // defer: one atomic per wave reserves the slots, lanes write {pixel, centre, max bits, level}
      const int leader = __ffsll((long long)om) - 1;
      int base = 0;
      if (lane == leader) base = atomicAdd(t.ocount, __popcll(om));
      base = __shfl(base, leader, 64);
      if (outl) {
        const int rank = __popcll(om & ((1ull << lane) - 1ull));
        const unsigned short mb = *reinterpret_cast<const unsigned short*>(&max_score);
        t.olist[base + rank] = make_int4(t.bn, (cu & 0xffff) | (cv << 16), (int)mb | (D << 16), 0);
        active = false;
      }
    } else {
      // in place: the wave takes its outliers one at a time
      uint64_t m = om;
      while (m) {
        const int src = __ffsll((long long)m) - 1;
        m &= m - 1;
        int scu = __shfl(cu, src, 64), scv = __shfl(cv, src, 64);
        const unsigned short mb0 = (unsigned short)__shfl((int)*reinterpret_cast<const unsigned short*>(&max_score),
                                                          src, 64);
        h1 smax = *reinterpret_cast<const h1*>(&mb0);
        h2 sq[F / 2];
#pragma unroll
        for (int k = 0; k < F / 2; k++) {
          const int v = __shfl(*reinterpret_cast<const int*>(&q[k]), src, 64);
          sq[k] = *reinterpret_cast<const h2*>(&v);
        }
        wave_level<D, PLANAR>(t.img, H, W, sq, scu, scv, smax, lane);
        if (lane == src) {
          cu = scu;
          cv = scv;
          max_score = smax;
        }
      }
    }
  }
  // per-lane column offset; the row base (and the chunk plane) is wave-uniform (scalar)
  const int lane_off = gx * (PLANAR ? 8 : F);
  const size_t cstride = PLANAR ? (size_t)H * W * 8 : 8, rstride = (size_t)W * (PLANAR ? 8 : F);
  if constexpr (SCREEN) {
    float a[G * G];
#pragma unroll
    for (int c = 0; c < G * G; c++) a[c] = 0.0f;
    __syncthreads();  // the reduction scratch aliases the window: its readers are done
    if (packed) {  // (d = 1 only) the three chunk planes in one fill
#ifndef RT_NOLOAD
      for (int r = wid; r < 3 * nrows; r += RT_WAVES) {
        const int chunk = r >= 2 * nrows ? 2 : (r >= nrows ? 1 : 0), y = r - chunk * nrows;
        const int gy = min(max(wy0 + y, 0), H - 1);
        const h1* rowp = t.img + (size_t)gy * rstride + chunk * cstride;
        if (col_in)
          __builtin_amdgcn_global_load_lds((gvoid_t)(rowp + lane_off),
                                           (lvoid_t)&lds[chunk * RT_PPLANE + y * RT_PCOLS], 16, 0, 0);
      }
#endif
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
#ifndef RT_NOCOMP
      if (lane_in) {
        const int b0 = by * RT_PCOLS + bx;
        screen_chunk<D, RT_PCOLS>(&lds[b0], &q[0], a);
        screen_chunk<D, RT_PCOLS>(&lds[RT_PPLANE + b0], &q[4], a);
        screen_chunk<D, RT_PCOLS>(&lds[2 * RT_PPLANE + b0], &q[8], a);
      }
#endif
    } else if (dbuf) {  // (d = 2 only) chunk c + 1 lands in the other buffer while chunk c is screened
      auto fill = [&](int chunk, int buf) {
#ifndef RT_NOLOAD
        for (int y = wid; y < nrows; y += RT_WAVES) {
          const int gy = min(max(wy0 + y, 0), H - 1);
          const h1* rowp = t.img + (size_t)gy * rstride + chunk * cstride;
          if (col_in) lds_dma_row(rowp + lane_off, t.lds_addr + (unsigned)(buf + y * RT_PCOLS) * 16u);
        }
#endif
      };
      const int b0 = by * RT_PCOLS + bx;
      fill(0, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      // the same wait as a builtin: the compiler's wait model (blind to the asm) learns that none of its own loads
      // (a previous level's survivor loads, spill reloads) is still in flight, so it places no vmcnt(0) of its own
      // after fill(1), which would drain the DMA with them
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) expcnt(7) lgkmcnt(15)
      __syncthreads();
      fill(1, RT_DBUF);
#ifndef RT_NOCOMP
      if (lane_in) screen_chunk<D, RT_PCOLS>(&lds[b0], &q[0], a);
#endif
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();  // chunk 1 landed; every wave is done with buffer 0
      fill(2, 0);
#ifndef RT_NOCOMP
      if (lane_in) screen_chunk<D, RT_PCOLS>(&lds[RT_DBUF + b0], &q[4], a);
#endif
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
#ifndef RT_NOCOMP
      if (lane_in) screen_chunk<D, RT_PCOLS>(&lds[b0], &q[8], a);
#endif
    } else {
#pragma unroll
      for (int chunk = 0; chunk < F / 8; chunk++) {
        if (chunk) __syncthreads();
#ifndef RT_NOLOAD
        for (int y = wid; y < nrows; y += RT_WAVES) {
          const int gy = min(max(wy0 + y, 0), H - 1);
          const h1* rowp = t.img + (size_t)gy * rstride + chunk * cstride;
          if (col_in)
            __builtin_amdgcn_global_load_lds((gvoid_t)(rowp + lane_off), (lvoid_t)&lds[y * RT_COLS], 16, 0, 0);
        }
#endif
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
#ifndef RT_NOCOMP
        if (lane_in) screen_chunk<D>(&lds[by * RT_COLS + bx], &q[chunk * 4], a);
#endif
      }
    }
    if (lane_in) {
      uint64_t vm = (1ull << (G * G)) - 1ull;  // in-image candidates
      if (__ballot(lane_in && !(u_lo >= 0 && u_lo + 6 * D < W && v_lo >= 0 && v_lo + 6 * D < H)) != 0) {
        uint64_t jm = 0;
#pragma unroll
        for (int j = 0; j < G; j++) jm |= (v_lo + j * D >= 0 && v_lo + j * D < H) ? (1ull << j) : 0ull;
        vm = 0;
#pragma unroll
        for (int i = 0; i < G; i++) vm |= (u_lo + i * D >= 0 && u_lo + i * D < W) ? (jm << (i * G)) : 0ull;
        // out-of-image candidates scored clamped window pixels: they take no part in the level's best (nor survive)
#pragma unroll
        for (int c = 0; c < G * G; c++) a[c] = ((vm >> c) & 1ull) ? a[c] : -INFINITY;
      }
      float lmax = a[0];
#pragma unroll
      for (int c = 1; c < G * G; c++) lmax = fmaxf(lmax, a[c]);
      const float T = fmaxf((float)max_score - t.bq, lmax - 2.0f * t.bq);
      uint64_t m = screen_mask(a, T);
      if (!t.sok) m = ~0ull;
      m &= vm;
      if (!first) m &= ~(1ull << (G * G / 2));
#ifdef M3S_REFINE_STATS  // survivors per level: lanes' sum [32 + 2D], per-wave maximum summed [33 + 2D]
      {
        int ns = __popcll(m), mx = ns;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) mx = max(mx, __shfl_xor(mx, off, 64));
        int sm = ns;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) sm += __shfl_xor(sm, off, 64);
        if (lane == __ffsll((long long)__ballot(1)) - 1) {
          atomicAdd(&g_refine_stats[32 + 2 * D], (unsigned long long)sm);
          atomicAdd(&g_refine_stats[33 + 2 * D], (unsigned long long)mx);
        }
      }
#endif
#ifdef RT_NOSURV
      m = 0;
#endif
      int bi = -1;
      if (packed)
        exact_survivors_lds<D>(&lds[by * RT_PCOLS + bx], q, m, max_score, bi);
      else
        exact_survivors<D, PLANAR>(t.img, H, W, q, u_lo, v_lo, m, max_score, bi);
      if (bi >= 0) {
        cu = u_lo + (bi / G) * D;
        cv = v_lo + (bi % G) * D;
      }
    }
    return;
  }
  h1 s[G * G];
#pragma unroll
  for (int c = 0; c < G * G; c++) s[c] = (h1)0.0f;
  __syncthreads();  // the reduction scratch aliases the window: its readers are done
#pragma unroll
  for (int chunk = 0; chunk < F / 8; chunk++) {
    if (chunk) __syncthreads();  // previous chunk's readers are done
#ifndef RT_NOLOAD
    for (int y = wid; y < nrows; y += RT_WAVES) {  // one global_load_lds (64 lanes x 16 B) per window row
      const int gy = min(max(wy0 + y, 0), H - 1);
      const h1* rowp = t.img + (size_t)gy * rstride + chunk * cstride;
      if (col_in) __builtin_amdgcn_global_load_lds((gvoid_t)(rowp + lane_off), (lvoid_t)&lds[y * RT_COLS], 16, 0, 0);
    }
#endif
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
#ifndef RT_NOCOMP
    if (lane_in) score_chunk<D>(&lds[by * RT_COLS + bx], &q[chunk * 4], s);
#endif
  }
  if (lane_in) {  // scan-order arg-max: u outer, v inner, strict '>' (matching_kernels.cu:54-71)
    int bi = -1;
    if (__ballot(lane_in && !(u_lo >= 0 && u_lo + 6 * D < W && v_lo >= 0 && v_lo + 6 * D < H)) == 0) {
      // every candidate grid of the wave lies inside the image: index-only tracking
#pragma unroll
      for (int c = 0; c < G * G; c++) {
        const bool gt = s[c] > max_score;
        max_score = gt ? s[c] : max_score;
        bi = gt ? c : bi;
      }
    } else {
#pragma unroll
      for (int i = 0; i < G; i++) {
        const bool uok = u_lo + i * D >= 0 && u_lo + i * D < W;
#pragma unroll
        for (int j = 0; j < G; j++) {
          const bool vok = v_lo + j * D >= 0 && v_lo + j * D < H;
          const bool gt = uok && vok && s[i * G + j] > max_score;
          max_score = gt ? s[i * G + j] : max_score;
          bi = gt ? i * G + j : bi;
        }
      }
    }
    if (bi >= 0) {
      cu = u_lo + (bi / G) * D;
      cv = v_lo + (bi % G) * D;
    }
  }
}

template <bool P1_I64>
__device__ __forceinline__ void load_p1(const void* p1v, size_t bn, int& cu, int& cv) {
  if constexpr (P1_I64) {
    cu = (int)reinterpret_cast<const int64_t*>(p1v)[bn * 2];
    cv = (int)reinterpret_cast<const int64_t*>(p1v)[bn * 2 + 1];
  } else {
    cu = reinterpret_cast<const int*>(p1v)[bn * 2];
    cv = reinterpret_cast<const int*>(p1v)[bn * 2 + 1];
  }
}

template <bool LIN_OUT>
__device__ __forceinline__ void store_out(void* outv, size_t bn, int W, int cu, int cv) {
  if constexpr (LIN_OUT) {
    reinterpret_cast<int64_t*>(outv)[bn] = (int64_t)cu + (int64_t)W * cv;
  } else {
    reinterpret_cast<int64_t*>(outv)[bn * 2] = cu;
    reinterpret_cast<int64_t*>(outv)[bn * 2 + 1] = cv;
  }
}

// P1_I64: p1 given as (B,N,2) int64 (reference op) else int32 (fused); LIN_OUT: write idx = u + W v.
// SCREEN: bound-screened scoring (cmaxp = the descriptor-norm bound written by prep / proj_occlusion).
// LIN_OUT (fused path) reads the PLANAR D11h of prep_rays_kernel.
#ifndef RT_MIN_BLOCKS  // blocks per CU the register budget is sized for (16 waves: 128 VGPRs, the LDS limit too)
#define RT_MIN_BLOCKS (16 / RT_WAVES)
#endif
template <bool D21_F32, bool P1_I64, bool LIN_OUT, bool SCREEN>
__global__ void __launch_bounds__(RT_THREADS, RT_MIN_BLOCKS) refine_tile_kernel(const h1* __restrict__ D11h, const void* __restrict__ D21,
                                                             const void* __restrict__ p1v, void* __restrict__ outv,
                                                             int H, int W, int dilation_max, int tiles_x,
                                                             int tiles_per_img, int nblocks, int4* olist,
                                                             int* ocount, const float* __restrict__ cmaxp) {
  constexpr int F = 24;
  __shared__ uint4 lds[RT_ROWS * RT_COLS];
  int(*s_red)[4] = reinterpret_cast<int(*)[4]>(&lds[0]);  // level-start reductions alias the window
  const int lb = xcd_remap(blockIdx.x, nblocks);
  const int b = lb / tiles_per_img, tt = lb % tiles_per_img;
  const int tx = tt % tiles_x, ty = tt / tiles_x;
  TileCtx t;
  t.H = H;
  t.W = W;
  t.lane = threadIdx.x & 63;
  t.wid = threadIdx.x >> 6;
  {  // pixel of this lane: each ds_read_b128 lane group (16 lanes, one LDS cycle when conflict-free) takes 16
     // CONTIGUOUS pixels of one row, so lanes whose centres are displaced alike hit 16 distinct bank quads; the
     // row-major lane order put pixels 17 px apart into one group, which collide on a 1-px displacement change
    const int l = t.lane & 31;
    const int g = (l < 4 || (l >= 12 && l < 16) || (l >= 20 && l < 28)) ? 0 : 1;
    const int r = g == 0 ? (l < 4 ? l : l < 16 ? l - 8 : l - 12) : (l < 12 ? l - 4 : l < 20 ? l - 8 : l - 16);
    t.u_pix = tx * RT_TW + g * 16 + r;
    t.v_pix = ty * RT_TH + 2 * t.wid + (t.lane >> 5);
  }
  t.olist = olist;
  t.ocount = ocount;
  t.lds_addr = (unsigned)(uintptr_t)(lvoid_t)lds;
  bool active = t.u_pix < W && t.v_pix < H;
  const int N = H * W;
  const size_t bn = (size_t)b * N + (size_t)t.v_pix * W + t.u_pix;
  t.bn = (int)bn;
  t.img = D11h + (size_t)b * N * F;
  h2 q[F / 2];
  int cu = 0, cv = 0;
  if (active) {
    load_query<F, D21_F32>(D21, bn, q);
    load_p1<P1_I64>(p1v, bn, cu, cv);
  } else {
#pragma unroll
    for (int k = 0; k < F / 2; k++) q[k] = h2{(h1)0.0f, (h1)0.0f};
  }
  {  // tile flow estimate, once per tile: the centres move by at most 3d per level, well inside the
     // +-16 px inlier band, so the initial mean serves every level (saves a block reduction per level)
    int su = active ? cu - t.u_pix : 0, sv = active ? cv - t.v_pix : 0, na = active ? 1 : 0;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      su += __shfl_xor(su, off, 64);
      sv += __shfl_xor(sv, off, 64);
      na += __shfl_xor(na, off, 64);
    }
    if (t.lane == 0) {
      s_red[t.wid][0] = su;
      s_red[t.wid][1] = sv;
      s_red[t.wid][2] = na;
    }
    __syncthreads();
    // block-uniform: SGPRs (readfirstlane), not VGPRs live across every level
    int tu = 0, tv = 0, tn = 0;
#pragma unroll
    for (int w = 0; w < RT_WAVES; w++) {
      tu += s_red[w][0];
      tv += s_red[w][1];
      tn += s_red[w][2];
    }
    const int nall = max(1, tn);
    t.fu = __builtin_amdgcn_readfirstlane(tu / nall);
    t.fv = __builtin_amdgcn_readfirstlane(tv / nall);
    t.tcu = tx * RT_TW + RT_TW / 2 + t.fu;
    t.tcv = ty * RT_TH + RT_TH / 2 + t.fv;
  }
  t.bq = 0.0f;
  t.sok = false;
  if constexpr (SCREEN) {
    float qq = 0.0f;
#pragma unroll
    for (int k = 0; k < F / 2; k++) qq = __builtin_amdgcn_fdot2(q[k], q[k], qq, false);
    const float pq = sqrtf(qq) * *cmaxp * 1.001f;  // |q|_2 |c|_2 bound, rounded up
    t.sok = pq <= 16384.0f;                         // false for NaN / inf
    t.bq = t.sok ? 0.0125f * pq + 0x1p-18f : 0.0f;
  }
  const bool mine = active;  // deferred pixels are written by refine_outlier_kernel
#ifdef M3S_REFINE_BSTAMPS
  if (threadIdx.x == 0 && blockIdx.x < 8192) g_refine_bstamps[blockIdx.x * 4 + 0] = __builtin_amdgcn_s_memrealtime();
#endif
  h1 max_score = (h1)0.0f;   // numeric_limits<c10::Half>::min() == +0, never reset between levels
  // the levels as straight-line code (d = dilation_max .. 1) instead of a loop over a switch of the eight inlined level
  // bodies: across that loop's back edge the register allocator made ~800 copies and spilled 19 VGPRs (80 B of scratch
  // per lane, ~18 MB of scratch writes per frame); straight-line, the screened kernel takes 118 VGPRs and spills none
  // (csrc/Makefile checks it: scripts/isa_check_spills.py)
#define RT_LEVEL(DD)                                                                                        \
  if (dilation_max >= DD)                                                                                   \
    refine_level<DD, SCREEN, LIN_OUT>(t, active, q, cu, cv, max_score, lds, s_red, dilation_max == DD);
  RT_LEVEL(8)
  RT_LEVEL(7)
  RT_LEVEL(6)
  RT_LEVEL(5)
  RT_LEVEL(4)
  RT_LEVEL(3)
  RT_LEVEL(2)
  RT_LEVEL(1)
#undef RT_LEVEL
  if (mine && active) store_out<LIN_OUT>(outv, bn, W, cu, cv);
#ifdef M3S_REFINE_BSTAMPS
  const unsigned long long nact = __popcll(__ballot(active));
  // aliases the window (done with): a separate __shared__ array would push the block past 40 KiB of LDS and
  // change the occupancy being measured (4 -> 3 blocks per CU)
  unsigned long long* s_act = reinterpret_cast<unsigned long long*>(&lds[0]);
  __syncthreads();
  if (t.lane == 0) s_act[t.wid] = nact;
  __syncthreads();
  if (threadIdx.x == 0 && blockIdx.x < 8192) {
    unsigned hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    g_refine_bstamps[blockIdx.x * 4 + 1] = __builtin_amdgcn_s_memrealtime();
    g_refine_bstamps[blockIdx.x * 4 + 2] = hw;
    unsigned long long na = 0;
    for (int w = 0; w < RT_WAVES; w++) na += s_act[w];
    g_refine_bstamps[blockIdx.x * 4 + 3] = na;
  }
#endif
}

// Finishes the deferred pixels: one wave per pixel, levels d0..1 by wave_level (grid-stride over
// the list; the count is read on the device, so the launch needs no host sync).
template <bool D21_F32, bool LIN_OUT>
__global__ void __launch_bounds__(256) refine_outlier_kernel(const h1* __restrict__ D11h,
                                                             const void* __restrict__ D21, void* __restrict__ outv,
                                                             int H, int W, const int4* __restrict__ olist,
                                                             const int* __restrict__ ocount) {
  constexpr int F = 24;
  const int lane = threadIdx.x & 63;
  const int nwaves = gridDim.x * (blockDim.x >> 6);
  const int count = *ocount;
  const int N = H * W;
  for (int o = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); o < count; o += nwaves) {
    const int4 r = olist[o];
    const size_t bn = (size_t)r.x;
    int cu = (int)(short)(r.y & 0xffff), cv = r.y >> 16;
    const unsigned short mb = (unsigned short)(r.z & 0xffff);
    h1 max_score = *reinterpret_cast<const h1*>(&mb);
    const int d0 = r.z >> 16;
    const h1* img = D11h + (bn / N) * (size_t)N * F;
    h2 q[F / 2];
    load_query<F, D21_F32>(D21, bn, q);
    for (int d = d0; d > 0; d--) {
      switch (d) {
        case 8: wave_level<8, LIN_OUT>(img, H, W, q, cu, cv, max_score, lane); break;
        case 7: wave_level<7, LIN_OUT>(img, H, W, q, cu, cv, max_score, lane); break;
        case 6: wave_level<6, LIN_OUT>(img, H, W, q, cu, cv, max_score, lane); break;
        case 5: wave_level<5, LIN_OUT>(img, H, W, q, cu, cv, max_score, lane); break;
        case 4: wave_level<4, LIN_OUT>(img, H, W, q, cu, cv, max_score, lane); break;
        case 3: wave_level<3, LIN_OUT>(img, H, W, q, cu, cv, max_score, lane); break;
        case 2: wave_level<2, LIN_OUT>(img, H, W, q, cu, cv, max_score, lane); break;
        default: wave_level<1, LIN_OUT>(img, H, W, q, cu, cv, max_score, lane); break;
      }
    }
    if (lane == 0) store_out<LIN_OUT>(outv, bn, W, cu, cv);
  }
}

}  // namespace m3s

// shapes the tile kernel takes (else the per-pixel kernels of matching.hip); the fused path's prep writes the
// PLANAR D11h exactly when this holds
extern "C" int m3s_refine_tile_ok(int B, int H, int W, int F, int radius, int dilation_max) {
  if (F != 24 || radius != 3 || dilation_max < 1 || dilation_max > 8) return 0;
  if ((long long)B * H * W >= (1ll << 31) || H >= 32768 || W >= 32768) return 0;
  return 1;
}

// D21 f32 + p1 int32 -> idx (fused path) or D21 f16 + p1 int64 -> p1_new (reference op).
// olist/ocount (nullable): deferred-outlier list of >= B*H*W int4 and its counter, zeroed on the
// stream before this launch. Returns hipErrorNotSupported when the shape is not eligible (the
// caller falls back to the per-pixel kernels).
extern "C" hipError_t m3s_launch_refine_tile(const void* D11h, const void* D21, const void* p1, void* out, int B,
                                             int H, int W, int F, int radius, int dilation_max, int fused,
                                             void* olist, int* ocount, const float* cmax, hipStream_t s) {
  if (!m3s_refine_tile_ok(B, H, W, F, radius, dilation_max)) return hipErrorNotSupported;
  const int tx = (W + RT_TW - 1) / RT_TW, ty = (H + RT_TH - 1) / RT_TH, nb = tx * ty * B;
  const m3s::h1* a = reinterpret_cast<const m3s::h1*>(D11h);
  int4* ol = reinterpret_cast<int4*>(olist);
  if (ol == nullptr) ocount = nullptr;
  if (fused && cmax != nullptr)
    hipLaunchKernelGGL((m3s::refine_tile_kernel<true, false, true, true>), dim3(nb), dim3(RT_THREADS), 0, s, a, D21, p1,
                       out, H, W, dilation_max, tx, tx * ty, nb, ol, ocount, cmax);
  else if (fused)
    hipLaunchKernelGGL((m3s::refine_tile_kernel<true, false, true, false>), dim3(nb), dim3(RT_THREADS), 0, s, a, D21, p1,
                       out, H, W, dilation_max, tx, tx * ty, nb, ol, ocount, nullptr);
  else
    hipLaunchKernelGGL((m3s::refine_tile_kernel<false, true, false, false>), dim3(nb), dim3(RT_THREADS), 0, s, a, D21,
                       p1, out, H, W, dilation_max, tx, tx * ty, nb, ol, ocount, nullptr);
  if (ol != nullptr) {
    // 1024 waves: the list is empty or short once waves score up to RT_INPLACE_MAX outliers in place (a smaller
    // grid launches and drains faster); pathological inputs (every lane an outlier) take several passes
    const int ob = 256;
    if (fused)
      hipLaunchKernelGGL((m3s::refine_outlier_kernel<true, true>), dim3(ob), dim3(256), 0, s, a, D21, out, H, W, ol,
                         ocount);
    else
      hipLaunchKernelGGL((m3s::refine_outlier_kernel<false, false>), dim3(ob), dim3(256), 0, s, a, D21, out, H, W,
                         ol, ocount);
  }
  return hipGetLastError();
}

#ifdef M3S_REFINE_BSTAMPS
extern "C" int m3s_debug_refine_bstamps(unsigned long long* out) {
  (void)hipDeviceSynchronize();
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(m3s::g_refine_bstamps), sizeof(unsigned long long) * 8192 * 4) == hipSuccess
             ? 0 : -1;
}
#endif
#ifdef M3S_REFINE_STATS
extern "C" int m3s_debug_refine_stats(unsigned long long* out, int reset) {
  (void)hipDeviceSynchronize();
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(m3s::g_refine_stats), sizeof(unsigned long long) * 64) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[64] = {0};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(m3s::g_refine_stats), z, sizeof(z));
  }
  return 0;
}
#endif
