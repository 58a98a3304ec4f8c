// C ABI of libm3s.so (include/m3s.h): argument validation, workspace carving, host-side planning
// (rank remap, assembly pattern) and launch sequencing. Kernels live in matching.hip, track.hip
// and ba.hip. No torch types anywhere below this line.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <future>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/m3s.h"
#include "m3s_ba.h"
#include "ba_pattern.h"
#include "m3s_track.h"

extern "C" {
hipError_t m3s_launch_prep(const float*, float*, const float*, void*, int, int, int, int, int, float*, hipStream_t);
int m3s_prep_parts(int, int, int);
int m3s_refine_tile_ok(int, int, int, int, int, int);
hipError_t m3s_launch_iter_proj(const float*, const float*, const float*, float*, uint8_t*, int, int, int, int, int,
                                float, float, hipStream_t);
hipError_t m3s_launch_proj_occlusion(const float*, const float*, const float*, const int64_t*, int*, uint8_t*, int, int,
                                     int, int, float, float, float, int*, const float*, int, float*, hipStream_t);
hipError_t m3s_launch_refine_f16(const void*, const void*, const int64_t*, int64_t*, int, int, int, int, int, int, int,
                                 hipStream_t);
hipError_t m3s_launch_refine_f32(const float*, const float*, const int64_t*, int64_t*, int, int, int, int, int, int,
                                 int, hipStream_t);
hipError_t m3s_launch_refine_lin(const void*, const float*, const int*, int64_t*, int, int, int, int, int, int,
                                 void*, int*, const float*, hipStream_t);
hipError_t m3s_launch_track_setup(const TrackArgs*, const TrackParams*, hipStream_t);
hipError_t m3s_launch_track_iters(const TrackArgs*, const TrackParams*, int, int, int, int, hipStream_t);
hipError_t m3s_launch_fuse(const TrackArgs*, int, const FuseArgs*, int, int, const TrackPublish*, hipStream_t);
hipError_t m3s_launch_track_init(const TrackArgs*, const float*, const float*, int, hipStream_t);
int m3s_track_max_parts(void);
hipError_t m3s_launch_ba_lin(const BaArgs*, const BaParams*, int, int, hipStream_t);
hipError_t m3s_launch_ba_pack(const BaArgs*, const BaParams*, int, hipStream_t);
hipError_t m3s_launch_ba_kf_compare(const BaKfCopy*, int, int, uint8_t*, hipStream_t);
hipError_t m3s_launch_ba_solve(const BaArgs*, int, int, float, const int*, const int*, const int*, hipStream_t);
hipError_t m3s_launch_ba_solve_dense(const BaArgs*, int, int, float, hipStream_t);
hipError_t m3s_launch_peak_fma_f32(float*, int, int, hipStream_t);
hipError_t m3s_launch_rq_prep(const float*, int, int, int, int, int, uint4*, int, float, float*, hipStream_t);
hipError_t m3s_launch_rq_topk(const uint4*, const float*, const uint4*, const float*, int, int, int, int, int,
                              unsigned long long*, int64_t*, hipStream_t);
}

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

int hip_fail(hipError_t e, const char* where) {
  return fail(M3S_EHIP, std::string(where) + ": " + hipGetErrorString(e));
}

inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

struct Carver {
  char* base;
  size_t off = 0;
  explicit Carver(void* b) : base(static_cast<char*>(b)) {}
  template <typename T>
  T* take(size_t count) {
    T* p = reinterpret_cast<T*>(base ? base + off : nullptr);
    off += align256(sizeof(T) * (count > 0 ? count : 1));
    return p;
  }
};

#define M3S_CHECK(cond, msg)                 \
  do {                                       \
    if (!(cond)) return fail(M3S_EINVAL, msg); \
  } while (0)

#define HIP_TRY(expr, where)                \
  do {                                      \
    hipError_t _e = (expr);                 \
    if (_e != hipSuccess) return hip_fail(_e, where); \
  } while (0)

// ---- per-kernel HIP-event timing (bench.py reads it; off by default, zero cost when off) ----
// Events come from a pool that is created once and recycled by m3s_timing_reset: creating events
// per launch costs host time inside the measured loop.
struct TimedSpan {
  hipEvent_t a, b;
};
std::map<std::string, std::vector<TimedSpan>> g_spans;
std::vector<hipEvent_t> g_event_pool;  // free events
bool g_timing = false;

hipEvent_t pool_event() {
  if (g_event_pool.empty()) {
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
  }
  hipEvent_t e = g_event_pool.back();
  g_event_pool.pop_back();
  return e;
}

struct Span {
  hipStream_t s;
  hipEvent_t a = nullptr, b = nullptr;
  const char* name;
  Span(const char* n, hipStream_t st) : s(st), name(n) {
    if (!g_timing) return;
    a = pool_event();
    b = pool_event();
    if (a == nullptr || b == nullptr) {
      a = b = nullptr;
      return;
    }
    (void)hipEventRecord(a, s);
  }
  ~Span() {
    if (!g_timing || a == nullptr) return;
    (void)hipEventRecord(b, s);
    g_spans[name].push_back({a, b});
  }
};

}  // namespace

extern "C" void m3s_timing_enable(int on) {
  g_timing = on != 0;
  while (g_timing && g_event_pool.size() < 1024) {  // pre-create outside any timed loop
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) break;
    g_event_pool.push_back(e);
  }
}

extern "C" void m3s_timing_reset(void) {
  for (auto& kv : g_spans)
    for (auto& sp : kv.second) {
      g_event_pool.push_back(sp.a);
      g_event_pool.push_back(sp.b);
    }
  g_spans.clear();
}

// total milliseconds and span count recorded under `name` (synchronises the recorded events)
extern "C" int m3s_timing_query(const char* name, double* total_ms, int* count) {
  *total_ms = 0.0;
  *count = 0;
  auto it = g_spans.find(name);
  if (it == g_spans.end()) return M3S_OK;
  for (auto& sp : it->second) {
    HIP_TRY(hipEventSynchronize(sp.b), "timing sync");
    float ms = 0.0f;
    HIP_TRY(hipEventElapsedTime(&ms, sp.a, sp.b), "timing elapsed");
    *total_ms += ms;
    *count += 1;
  }
  return M3S_OK;
}

extern "C" int m3s_abi_version(void) { return M3S_ABI_VERSION; }
extern "C" const char* m3s_last_error(void) { return g_err.c_str(); }

// ------------------------------------------------------------------------------------------
// reference operators
// ------------------------------------------------------------------------------------------
extern "C" int m3s_iter_proj(const float* rays, const float* pts, const float* p_init, float* p_new,
                             uint8_t* converged, int B, int H, int W, int C, int N, int max_iter, float lambda_init,
                             float cost_thresh, void* stream) {
  M3S_CHECK(B >= 0 && N >= 0 && H >= 3 && W >= 3, "iter_proj: image must be at least 3x3");
  M3S_CHECK(C == 9, "iter_proj: rays_img_with_grad must have 9 channels (ray, gx, gy)");
  M3S_CHECK(max_iter >= 0, "iter_proj: max_iter must be >= 0");
  if (B == 0 || N == 0) return M3S_OK;
  M3S_CHECK(rays && pts && p_init && p_new && converged, "iter_proj: null pointer");
  HIP_TRY(m3s_launch_iter_proj(rays, pts, p_init, p_new, converged, B, H, W, N, max_iter, lambda_init, cost_thresh,
                               (hipStream_t)stream),
          "iter_proj launch");
  return M3S_OK;
}

extern "C" int m3s_refine_matches(int dtype, const void* D11, const void* D21, const int64_t* p1, int64_t* p1_new,
                                  int B, int H, int W, int F, int N, int radius, int dilation_max, void* stream) {
  M3S_CHECK(B >= 0 && N >= 0 && H >= 1 && W >= 1, "refine_matches: bad shape");
  M3S_CHECK(radius >= 0 && dilation_max >= 0, "refine_matches: radius/dilation_max must be >= 0");
  if (B == 0 || N == 0) return M3S_OK;
  M3S_CHECK(D11 && D21 && p1 && p1_new, "refine_matches: null pointer");
  if (dtype == 0) {
    M3S_CHECK(F == 16 || F == 24 || F == 32, "refine_matches: f16 path supports F in {16,24,32}");
    HIP_TRY(m3s_launch_refine_f16(D11, D21, p1, p1_new, B, H, W, F, N, radius, dilation_max, (hipStream_t)stream),
            "refine_matches launch");
  } else if (dtype == 1) {
    M3S_CHECK(F >= 1, "refine_matches: F must be >= 1");
    HIP_TRY(m3s_launch_refine_f32((const float*)D11, (const float*)D21, p1, p1_new, B, H, W, F, N, radius,
                                  dilation_max, (hipStream_t)stream),
            "refine_matches launch");
  } else {
    return fail(M3S_EINVAL, "refine_matches: dtype must be 0 (f16) or 1 (f32)");
  }
  return M3S_OK;
}

// ------------------------------------------------------------------------------------------
// fused match
// ------------------------------------------------------------------------------------------
struct MatchWs {
  float* rays9;   // (B,H,W,9) rays + gradients
  void* D11h;     // f16: (B,3,H,W,8) chunk planes on the refine tile path, else (B,H,W,F)
  int* p1;        // (B,N,2) int32
  int4* olist;    // (B*N) refine deferred-outlier records
  int* ocount;    // refine deferred-outlier count
  float* cpart;   // the refine screen's norm bound, prep's tile partials (m3s_prep_parts)
  float* cmax;    // ... reduced by the proj launch (refine.hip SCREEN)
};

static size_t match_carve(Carver& c, int B, int H, int W, int F, MatchWs* w) {
  w->rays9 = c.take<float>((size_t)B * H * W * 9);
  w->D11h = c.take<uint16_t>((size_t)B * H * W * F);
  w->p1 = c.take<int>((size_t)B * H * W * 2);
  w->olist = c.take<int4>((size_t)B * H * W);
  w->ocount = c.take<int>(1);
  w->cpart = c.take<float>((size_t)m3s_prep_parts(B, H, W));
  w->cmax = c.take<float>(1);
  return c.off;
}

extern "C" size_t m3s_match_workspace_size(int B, int H, int W, int F) {
  Carver c(nullptr);
  MatchWs w;
  return match_carve(c, B, H, W, F, &w);
}

extern "C" int m3s_match(const float* X11, const float* X21, const float* D11, const float* D21,
                         const int64_t* idx_init, int64_t* idx_out, uint8_t* valid_out, int B, int H, int W, int F,
                         int max_iter, float lambda_init, float cost_thresh, float dist_thresh, int radius,
                         int dilation_max, void* workspace, size_t workspace_bytes, void* stream) {
  M3S_CHECK(B >= 1 && H >= 3 && W >= 3, "match: image must be at least 3x3");
  M3S_CHECK(F == 16 || F == 24 || F == 32, "match: descriptor dim must be 16, 24 or 32");
  M3S_CHECK(X11 && X21 && D11 && D21 && idx_out && valid_out, "match: null pointer");
  M3S_CHECK(max_iter >= 0 && radius >= 0 && dilation_max >= 0, "match: negative parameter");
  if (workspace_bytes < m3s_match_workspace_size(B, H, W, F)) return fail(M3S_ESPACE, "match: workspace too small");
  Carver c(workspace);
  MatchWs w;
  match_carve(c, B, H, W, F, &w);
  float* rays9 = w.rays9;
  void* D11h = w.D11h;
  int* p1 = w.p1;
  hipStream_t s = (hipStream_t)stream;
  // bound-screened refine (refine.hip): prep publishes the descriptor-norm bound; M3S_REFINE_SCREEN=0 scores every
  // candidate with the exact chain instead (same results, bit for bit; read per call so tests can compare both)
  const char* screen_env = getenv("M3S_REFINE_SCREEN");
  // the refine tile kernel reads prep's chunk-planar D11h (refine.hip); the per-pixel fallback the (H,W,F) one
  const int planar = radius > 0 && m3s_refine_tile_ok(B, H, W, F, radius, dilation_max);
  const bool screen = (screen_env == nullptr || atoi(screen_env) != 0) && planar;
  {
    Span sp("prep_rays", s);
    // the f16 descriptors: the tile path's chunk planes (+ the screen's tile partials) or the (B,H,W,F) layout
    HIP_TRY(m3s_launch_prep(X11, rays9, radius > 0 ? D11 : nullptr, D11h, B, H, W, F, planar,
                            screen ? w.cpart : nullptr, s),
            "match prep launch");
  }
  {
    Span sp("proj_occlusion", s);
    HIP_TRY(m3s_launch_proj_occlusion(rays9, X11, X21, idx_init, p1, valid_out, B, H, W, max_iter, lambda_init,
                                      cost_thresh, dist_thresh, w.ocount, w.cpart, m3s_prep_parts(B, H, W),
                                      screen ? w.cmax : nullptr, s),
            "match proj launch");
  }
  // radius == 0: the refine loop is empty and the kernel only writes idx = pixel_to_lin(p1)
  // (matching.py:78-88); D11h is never read then.
  {
    Span sp("refine_lin", s);
    // every wave scores its window outliers in place (no deferred list, no refine_outlier_kernel launch: on coherent
    // inputs the list is empty and the launch alone cost ~2 us per frame; a scattered warm start, every lane an
    // outlier, costs its waves 64 pixels x 5 levels serially). M3S_REFINE_INPLACE=0: waves with more than
    // RT_INPLACE_MAX outliers defer them to the list and the outlier launch
    const char* inplace_env = getenv("M3S_REFINE_INPLACE");
    const bool inplace = !(inplace_env != nullptr && inplace_env[0] == '0');
    HIP_TRY(m3s_launch_refine_lin(D11h, D21, p1, idx_out, B, H, W, F, radius, radius > 0 ? dilation_max : 0,
                                  inplace ? nullptr : w.olist,
                                  w.ocount, screen ? w.cmax : nullptr, s),
            "match refine launch");
  }
  return M3S_OK;
}

// ------------------------------------------------------------------------------------------
// tracking
// ------------------------------------------------------------------------------------------
// GN blocks: 2 points per lane at 512x512 (512 blocks = 2 per CU), at most 512 partials to reduce
// pinned host copy of the device state: the one per-frame readback is a direct DMA, not a staged copy
// Per host thread: the frame result mirror in fine-grained pinned memory (the fuse launch writes it).
static TrackMirror* pinned_mirror() {
  static thread_local TrackMirror* h = nullptr;
  if (h == nullptr) {
    void* p = nullptr;
    if (hipHostMalloc(&p, sizeof(TrackMirror), hipHostMallocCoherent | hipHostMallocPortable) != hipSuccess)
      return nullptr;
    h = static_cast<TrackMirror*>(p);
    memset(h, 0, sizeof(TrackMirror));
  }
  return h;
}

// Wait for generation `gen` in the mirror: a spin on the host-coherent word (no interrupt wake-up, no
// D2H copy kernel), with a stream query every 1024 polls so a failed or drained stream ends the wait.
static int wait_published(const TrackMirror* m, unsigned gen, hipStream_t s) {
  for (unsigned spin = 1;; spin++) {
    if (__atomic_load_n(&m->gen, __ATOMIC_ACQUIRE) == gen) return M3S_OK;
    if ((spin & 1023u) == 0) {
      const hipError_t q = hipStreamQuery(s);
      if (q == hipSuccess) {
        if (__atomic_load_n(&m->gen, __ATOMIC_ACQUIRE) == gen) return M3S_OK;
        return fail(M3S_EHIP, "track: stream drained without publishing the frame state");
      }
      if (q != hipErrorNotReady) return fail(M3S_EHIP, std::string("track sync: ") + hipGetErrorString(q));
    }
    __builtin_ia32_pause();
  }
}

// workspaces whose frame scratch the last fuse launch cleared: workspace -> {the workspace's size, the image size N
// of that frame}. The scratch layout (track_carve) depends on N: a frame of another size wrote its records and
// partials where this size's byte map lies (a 48x64 frame left 5540 stale map entries under a following 512x512
// frame's unique-match count), so the record holds only for the same N. Dropped by m3s_track_release (the caller
// frees or repurposes the workspace).
struct TrackClean {
  size_t bytes;
  int N;
};
static std::mutex g_track_clean_mu;
static std::map<const void*, TrackClean> g_track_clean;

extern "C" int m3s_track_release(const void* workspace) {
  std::lock_guard<std::mutex> lock(g_track_clean_mu);
  g_track_clean.erase(workspace);
  return M3S_OK;
}

static int track_nparts(int N) { return std::max(1, std::min(256, (N + 1023) / 1024)); }  // <= 1 block per CU

static size_t track_carve(Carver& c, int N, TrackState** st, uint8_t** flags, double** partials, float** rec,
                          unsigned long long** cnt, unsigned** tick) {
  *st = c.take<TrackState>(1);
  *cnt = c.take<unsigned long long>(M3S_TRACK_SHARDS * 16);
  *tick = c.take<unsigned>(M3S_TRACK_TICK_WORDS);
  *flags = c.take<uint8_t>(((size_t)N + 15) / 16 * 16);
  *partials = c.take<double>((size_t)64 * 256 * 40);  // GN_SLOTS iterations x up to 256 blocks x GN_PSTRIDE
  *rec = c.take<float>((size_t)N * 8);
  return c.off;
}

extern "C" size_t m3s_track_workspace_size(int N) {
  Carver c(nullptr);
  TrackState* st;
  uint8_t* bm;
  double* pa;
  float* rec;
  unsigned long long* cnt;
  unsigned* tick;
  return track_carve(c, N, &st, &bm, &pa, &rec, &cnt, &tick);
}

extern "C" int m3s_track(const m3s_track_inputs* in, const m3s_track_config* cfg, const m3s_track_fuse_args* fuse,
                         int first_chunk, float* T_out_dev, m3s_track_result* result, void* workspace,
                         size_t workspace_bytes, void* stream) {
  M3S_CHECK(in && cfg && result, "track: null argument");
  const int N = cfg->H * cfg->W;
  M3S_CHECK(cfg->H >= 1 && cfg->W >= 1, "track: bad image size");
  M3S_CHECK(cfg->mode == 0 || cfg->mode == 1, "track: mode must be 0 (rays) or 1 (calib)");
  M3S_CHECK(cfg->max_iters >= 1, "track: max_iters must be >= 1");
  if (in->direct) {
    M3S_CHECK(in->valid_match && in->Xf && in->Qff && in->T_WCf && in->T_WCk, "track: null input pointer");
    M3S_CHECK(cfg->mode == 0 ? in->Xk != nullptr : (in->meas_k && in->valid_meas_k),
              "track direct: rays needs Xk, calib needs meas_k/valid_meas_k");
  } else {
    M3S_CHECK(in->idx_f2k && in->valid_match && in->Xf && in->Cf && in->Qff && in->Xk && in->Ck && in->Qkf &&
                  in->T_WCf && in->T_WCk,
              "track: null input pointer");
    M3S_CHECK(in->Nf > 0 && in->Nk > 0, "track: fusion counts must be positive");
  }
  if (workspace_bytes < m3s_track_workspace_size(N)) return fail(M3S_ESPACE, "track: workspace too small");
  Carver c(workspace);
  TrackArgs a;
  TrackState* st;
  track_carve(c, N, &st, &a.flags, &a.partials, &a.rec, &a.cnt, &a.tick);
  a.state = st;
  a.idx = in->idx_f2k;
  a.valid_match = in->valid_match;
  a.Xf = in->Xf;
  a.Cf = in->Cf;
  a.Qff = in->Qff;
  a.Xk = in->Xk;
  a.Ck = in->Ck;
  a.Qkf = in->Qkf;
  a.meas_k = in->meas_k;
  a.valid_meas = in->valid_meas_k;
  TrackParams p;
  memset(&p, 0, sizeof(p));
  p.N = N;
  p.H = cfg->H;
  p.W = cfg->W;
  p.mode = cfg->mode;
  p.Nf = in->direct ? 1.0f : in->Nf;
  p.Nk = in->direct ? 1.0f : in->Nk;
  p.direct = in->direct != 0;
  p.C_conf = cfg->C_conf;
  p.Q_conf = cfg->Q_conf;
  p.min_match_frac = in->direct ? -1.0f : cfg->min_match_frac;  // opt_pose_* never skips
  p.c_a = (float)(1.0 / (double)cfg->sigma_a);  // tracker.py:175-176: python 1/sigma cast to float32
  p.c_b = (float)(1.0 / (double)cfg->sigma_b);
  p.huber_k = cfg->huber_k;
  p.rel_error = cfg->rel_error;
  p.delta_norm = cfg->delta_norm;
  p.max_iters = cfg->max_iters;
  p.pixel_border = cfg->pixel_border;
  p.depth_eps = cfg->depth_eps;
  for (int i = 0; i < 9; i++) p.K[i] = cfg->K[i];
  p.fx = cfg->K[0];
  p.fy = cfg->K[4];
  p.cx = cfg->K[2];
  p.cy = cfg->K[5];
  if (p.mode == 1) M3S_CHECK(p.fx != 0.0f && p.fy != 0.0f, "track: calib mode needs K");
  hipStream_t s = (hipStream_t)stream;
  a.T_out = T_out_dev;
  a.T_WCf = in->T_WCf;
  a.T_WCk = in->T_WCk;
  const bool do_fuse = fuse && fuse->Xk_canon;
  FuseArgs fa{};
  if (do_fuse) {
    M3S_CHECK(fuse->Ck_sum && fuse->Xkf && fuse->Ckf, "track: fusion needs Ck_sum, Xkf, Ckf");
    M3S_CHECK(!fuse->Ck_avg_out || fuse->Nk_new > 0.0f, "track: Ck_avg_out needs Nk_new > 0");
    M3S_CHECK(!fuse->Cf_avg_out || (fuse->Cf && fuse->Nf > 0.0f), "track: Cf_avg_out needs Cf and Nf > 0");
    fa.X_in = fuse->Xk_canon;
    fa.C_in = fuse->Ck_sum;
    fa.Xkf = fuse->Xkf;
    fa.Ckf = fuse->Ckf;
    fa.X_out = fuse->Xk_out ? fuse->Xk_out : const_cast<float*>(fuse->Xk_canon);
    fa.C_out = fuse->Ck_out ? fuse->Ck_out : const_cast<float*>(fuse->Ck_sum);
    fa.Cf = fuse->Cf;
    fa.Ck_avg = fuse->Ck_avg_out;
    fa.Cf_avg = fuse->Cf_avg_out;
    fa.Nk_new = fuse->Nk_new;
    fa.Nf = fuse->Nf;
    fa.slot_N = fuse->slot_N;
    fa.slot_N_updates = fuse->slot_N_updates;
    fa.slot_dirty = fuse->slot_dirty;
    fa.N_new = fuse->N_new;
    fa.N_updates_new = fuse->N_updates_new;
  }
  // the previous frame's fuse launch left this workspace's scratch clean (byte map of n16 entries, counters,
  // tickets): track_init runs only for a fresh / grown / failed workspace
  bool clean = false;
  {
    std::lock_guard<std::mutex> lock(g_track_clean_mu);
    auto it = g_track_clean.find(workspace);
    clean = it != g_track_clean.end() && it->second.bytes == workspace_bytes && it->second.N == N;
    g_track_clean.erase(workspace);  // dirty until this call has published
  }
  if (!clean) HIP_TRY(m3s_launch_track_init(&a, in->T_WCf, in->T_WCk, N, s), "track init launch");
  // the per-point setup runs inside the GN launch's first iteration (gn_loop_kernel<true>: no track_setup launch);
  // M3S_TRACK_FOLD_SETUP=0 keeps the separate track_setup launch (A/B)
  const char* fold_env = getenv("M3S_TRACK_FOLD_SETUP");
  const int fold = !(fold_env != nullptr && fold_env[0] == '0');
  if (!fold) {
    Span sp("track_setup", s);
    HIP_TRY(m3s_launch_track_setup(&a, &p, s), "track setup launch");
  }
  (void)first_chunk;  // every GN iteration runs inside one persistent launch (gn_loop_kernel)
  const int nparts = std::min(track_nparts(N), m3s_track_max_parts());  // every block co-resident
  TrackMirror* mirror = pinned_mirror();
  if (mirror == nullptr) return fail(M3S_EHIP, "track: pinned result mirror allocation failed");
  static thread_local unsigned gen = 0;
  TrackPublish pub{mirror, a.tick + M3S_TRACK_PUBLISH_TICKET, ++gen};
  {
    Span sp("gn_iters", s);
    HIP_TRY(m3s_launch_track_iters(&a, &p, nparts, p.max_iters, 0, fold, s), "track iterate launch");
  }
  // keyframe.update_pointmap(T_CkCf.act(Xkf), Ckf) after a successful solve (tracker.py:91-101): enqueued
  // before the readback, it runs only if the solve finished with a pose
  // The same launch publishes the result to the host mirror; the call returns once it has (the fusion
  // blocks may still be running: later work on this stream is ordered after them).
  HIP_TRY(m3s_launch_fuse(&a, 0, &fa, p.direct ? 0 : 1, N, &pub, s), "track fuse launch");
  if (int rc = wait_published(mirror, pub.gen, s)) return rc;
  {
    std::lock_guard<std::mutex> lock(g_track_clean_mu);
    g_track_clean[workspace] = {workspace_bytes, N};  // the fuse launch cleared what this frame dirtied
  }
  const TrackState& hs = mirror->s;
  if (hs.status == M3S_TRACK_STALLED)
    return fail(M3S_EHIP, "track: the persistent GN launch's hand-off stalled (its blocks were not co-resident); "
                          "no pose for this frame");
  memcpy(result->T_WCf, hs.T_WCf, sizeof(result->T_WCf));
  memcpy(result->T_CkCf, hs.T, sizeof(result->T_CkCf));
  result->cost = hs.last_cost;
  result->iters = hs.iter;
  result->status = hs.status;
  result->n_valid_opt = hs.n_valid_opt;
  result->n_valid_kf = hs.n_valid_kf;
  result->n_unique = hs.n_unique;
  result->N = N;
  return M3S_OK;
}

// ------------------------------------------------------------------------------------------
// bundle adjustment
// ------------------------------------------------------------------------------------------
namespace {

constexpr int BA_MAX_WIDE_STEPS = 40;

struct BaPlanImpl {
  BaArgs a;
  BaParams p;
  int Kp, N, E, e0, e1;
  int n_targets;  // distinct target keyframes j among this shard's edges (their X_j slabs are streamed per iteration)
  float delta_thresh;
  size_t edge_sums_off, edge_sums_bytes;
  void* ws;
  unsigned long long sym_gen;  // the PlanSym (symbolic half) this plan owns, by generation
  int n_packed, n_dirty;       // edges the pack wrote, keyframes found changed (record reuse; all without it)
};
static_assert(sizeof(BaPlanImpl) <= sizeof(m3s_ba_plan), "m3s_ba_plan too small");

// points of one keyframe per linearisation block: 24576 x 12 B = 295 KB of X_j, so the ~100 blocks an XCD
// runs at once (the edges of a few target keyframes, same chunk) share their X_j slabs in its 4 MiB L2. Small
// graphs (the early-sequence global optimisations) would leave most CUs idle at that length: their chunks
// shrink (down to 4096 points, 8 rounds per lane) until E x chunks reaches 512 blocks. A function of the
// FULL edge count, so every rank of a sharded solve cuts its edges exactly like the unsharded one.
// M3S_BA_CHUNK_POINTS (tests): a fixed chunk length instead.
constexpr int BA_CHUNK_POINTS = 24576, BA_CHUNK_MIN_POINTS = 4096, BA_LIN_MIN_BLOCKS = 512;
int ba_chunks(int N, int E) {
  const int base = std::max(1, (N + BA_CHUNK_POINTS - 1) / BA_CHUNK_POINTS);
  if (const char* f = getenv("M3S_BA_CHUNK_POINTS")) {
    const int len = std::max(256, atoi(f));
    return std::max(1, (N + len - 1) / len);
  }
  if ((int64_t)E * base >= BA_LIN_MIN_BLOCKS || E <= 0) return base;
  const int most = std::max(1, (N + BA_CHUNK_MIN_POINTS - 1) / BA_CHUNK_MIN_POINTS);
  return std::max(base, std::min(most, (BA_LIN_MIN_BLOCKS + E - 1) / E));
}

constexpr int BA_DENSE_MAX_POSES = 1025;  // dense fallback workspace: (2n+1) n doubles, ~0.8 GB at this size

// factor blocks of the densest possible pattern (every pose coupled to every other)
inline size_t ba_max_blocks(int Kp) {
  const size_t nb = (size_t)std::max(0, Kp - 1);
  return nb * (nb + 1) / 2;
}

// the plan's host-built tables, uploaded in ONE copy: rank arrays, keyframe pointer tables and the
// symbolic factorisation (ba_pattern.h), packed at their actual sizes into a region sized for the worst case
constexpr int BA_SYM_SECTIONS = 16;  // the symbolic half's sections (build_symbolic)
constexpr int BA_SP_PLAN_BYTES = 144 * 1024;  // ba.hip SP_PLAN_BYTES: LDS of the one-workgroup factor kernel
constexpr int BA_BLOB_SECTIONS = 8 + BA_SYM_SECTIONS;
// update pairs (source block row -> target block) the plan can hold: every pattern up to K ~ 600, and the
// sparse patterns of larger graphs
inline size_t ba_max_pairs(int Kp) {
  const size_t nb = (size_t)std::max(0, Kp - 1);
  return std::min(nb * nb * nb / 6 + nb * nb + 64, 32 * ba_max_blocks(Kp) + 64);
}
size_t ba_blob_capacity(int Kp, int E, int chunks) {
  const size_t nb = (size_t)std::max(0, Kp - 1), nLm = ba_max_blocks(Kp);
  // ranks, perm, col_ptr, rowL, lev_ptr, lev_col, grp_ptr, grp, pull_grp, src, sidx, asm CSR, rhs CSR
  const size_t ints = 2 * (size_t)E + nb + (nb + 1) + nLm + (nb + 1) + nb + (nb + 2) + 4 * nLm + nb + 4 * nLm +
                      ba_max_pairs(Kp) + (nLm + 1) + 4 * (size_t)E + (nb + 1) + 2 * (size_t)E +
                      (size_t)E * chunks +  // + the linearisation block table
                      2 * (size_t)E +       // + record slots and the pack list (record reuse)
                      8 * 2 * nb * (size_t)std::min<size_t>(BA_MAX_WIDE_STEPS, nb + 1) +  // + wide-step task records
                      2 * (M3S_BA_SP_WAVES + 1) + 2 * nb + 2 * (nb + nLm);  // + the dataflow schedule
  return ints * 4 + (size_t)Kp * (8 + 8 + 4) + BA_BLOB_SECTIONS * 16;
}

size_t ba_carve(Carver& c, int Kp, int N, int E, int chunks, BaArgs* a, size_t* es_off, void** blob) {
  const int nb = std::max(0, Kp - 1);
  // record slots (worst case: a shard packs only its own edges), each N records + the rays' N |Xi|
  a->rec = c.take<float4>((size_t)E * ba_rec_slot_bytes(N) / 16);
  a->partials = c.take<double>((size_t)E * chunks * 36);
  *es_off = c.off;
  a->edge_sums = c.take<double>((size_t)E * 36);
  a->L = c.take<double>(std::max<size_t>(ba_max_blocks(Kp), 1) * 64);
  a->y = c.take<double>((size_t)std::max(nb, 1) * 8);
  a->xs = c.take<double>((size_t)std::max(nb, 1) * 8);
  a->dx = c.take<float>((size_t)std::max(nb, 1) * 7);
  // the dense fallback's system (graphs up to BA_DENSE_MAX_POSES poses)
  const size_t n = (size_t)nb * 7;
  a->H = Kp <= BA_DENSE_MAX_POSES ? c.take<double>(std::max<size_t>((2 * n + 1) * n, 1)) : nullptr;
  a->info = c.take<int>(8);
  a->done = a->info + 1;
  a->iters = a->info + 2;
  *blob = c.take<char>(ba_blob_capacity(Kp, E, chunks));
  return c.off;
}

// pinned staging for the plan upload; reused across plans once the previous upload has landed
struct PlanStage {
  std::mutex mu;
  char* buf = nullptr;
  size_t cap = 0;
  hipEvent_t landed = nullptr;
  bool pending = false;
};
// one staging buffer + event per device: an event recorded on another device's stream would fail, and plans
// for different GPUs need not serialise on one mutex
PlanStage& plan_stage() {
  static std::mutex map_mu;
  static std::map<int, PlanStage> stages;
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> lock(map_mu);
  return stages[dev];  // std::map nodes never move
}

// Record reuse across plans on one workspace (m3s_ba_make_plan_reuse). The backend solves once per new keyframe
// (main.py:150-155): the edge set only grows and tracking changes only the keyframes it fuses into, so most edges'
// point records are still valid in the workspace. Per workspace: the record slot of every directed edge (by the
// caller's edge uid), a copy of every keyframe's points and confidences as last packed (by keyframe uid) for the
// next plan's exact compare, and the parameters the records depend on besides those.
struct RecCache {
  bool valid = false;
  int N = 0, mode = -1, W = 0;
  float Q_thresh = 0.0f, C_thresh = 0.0f, z_eps = 0.0f;
  std::unordered_map<int64_t, int> slot_of;  // edge uid -> record slot (shard-local)
  std::unordered_map<int64_t, int> copy_of;  // keyframe uid -> copy index
  std::vector<uint32_t> scale;               // per copy: bits of the Cscale its records were packed with
  std::vector<char> primed;                  // per copy: compared (and so filled) at least once
  float* copies = nullptr;                   // device: cap x 4N floats (X then C)
  int cap = 0, used = 0;
  BaKfCopy* table = nullptr;                 // device: tcap entries
  BaKfCopy* table_h = nullptr;               // pinned host staging of the table
  uint8_t* dirty = nullptr;                  // device: tcap flags
  uint8_t* dirty_h = nullptr;                // pinned host: tcap flags
  int tcap = 0;
  void reset_maps() {
    slot_of.clear();
    copy_of.clear();
    scale.clear();
    primed.clear();
    used = 0;
  }
  void free_all() {
    if (copies) (void)hipFree(copies);
    if (table) (void)hipFree(table);
    if (dirty) (void)hipFree(dirty);
    if (table_h) (void)hipHostFree(table_h);
    if (dirty_h) (void)hipHostFree(dirty_h);
    copies = nullptr;
    table = nullptr;
    dirty = nullptr;
    table_h = nullptr;
    dirty_h = nullptr;
    cap = tcap = 0;
    reset_maps();
    valid = false;
  }
};
std::mutex g_rec_mu;
std::map<const void*, RecCache> g_rec;  // by workspace (map nodes never move)

}  // namespace

extern "C" size_t m3s_ba_workspace_size(int Kp, int N, int E) {
  Carver c(nullptr);
  BaArgs a;
  size_t off;
  void* blob;
  return ba_carve(c, Kp, N, E, ba_chunks(N, E), &a, &off, &blob);
}

extern "C" int m3s_ba_pattern_stats(const int64_t* ii, const int64_t* jj, int E, int Kp, int* stats) {
  M3S_CHECK(ii && jj && stats && E >= 0 && Kp >= 1, "ba pattern: bad arguments");
  std::vector<int64_t> u(ii, ii + E);
  u.insert(u.end(), jj, jj + E);
  std::sort(u.begin(), u.end());
  u.erase(std::unique(u.begin(), u.end()), u.end());
  M3S_CHECK((int)u.size() <= Kp, "ba pattern: more unique keyframe ids than poses");
  std::vector<int> ri(E), rj(E);
  for (int e = 0; e < E; e++) {
    ri[e] = (int)(std::lower_bound(u.begin(), u.end(), ii[e]) - u.begin());
    rj[e] = (int)(std::lower_bound(u.begin(), u.end(), jj[e]) - u.begin());
  }
  BaPattern P;
  M3S_CHECK(Kp <= M3S_BA_MAX_POSES, "ba pattern: at most 4096 poses (M3S_BA_MAX_POSES)");
  ba_build_pattern(ri.data(), rj.data(), E, Kp, &P, ba_max_pairs(Kp));
  if (P.too_dense) return fail(M3S_EINVAL, "ba pattern: too dense for the plan tables");
  stats[0] = P.nL;
  stats[1] = P.nlev;
  stats[2] = (int)P.grp.size() / 4;
  stats[3] = (int)P.src.size() / 4;
  stats[4] = (int)P.sidx.size();
  stats[5] = (int)std::count_if(P.pull_grp.begin(), P.pull_grp.end(), [](int g) { return g >= 0; });
  return M3S_OK;
}

namespace {
// The symbolic half of a plan (ordering, factor pattern, levels, update groups, assembly CSR; ba_pattern.h) and
// the solve schedule derived from it. It is needed only from the first m3s_ba_solve on, so it is built on a host
// worker thread while the device packs the point records and runs the first linearisation: the host analysis
// (~0.6 ms at K = 256) leaves the replicated, unsharded part of a multi-GPU solve. m3s_ba_solve (or
// m3s_ba_plan_info) joins it once and uploads its tables. One per workspace (a new plan on the same workspace
// first joins the previous one); `gen` ties a plan to it.
struct PlanSym {
  unsigned long long gen = 0;
  std::future<int> fut;
  bool joined = false, uploaded = false;
  int rc = M3S_OK;
  std::string err;
  // worker output (read by the main thread only after the join)
  std::vector<char> image;  // the tables, packed at 16-B aligned offsets, as uploaded
  size_t off[BA_SYM_SECTIONS] = {0};
  int nb = 0, nlev = 0, nL = 0, wide_steps = 0, dense = 0, flow = 0, plan_lo_off = 0, plan_bytes = 0;
  bool pack_deferred = false;    // the plan's pack runs inside its first linearisation (set at plan time, under g_sym_mu)
  int step_tasks[BA_MAX_WIDE_STEPS] = {0};
  int step_base[BA_MAX_WIDE_STEPS] = {0};  // first task record of each wide step
  int step_na[BA_MAX_WIDE_STEPS] = {0};    // its factor tasks (update groups follow)
  char* dst = nullptr;  // device destination (the blob region after the plan's own tables)
};
std::mutex g_sym_mu;
std::map<const void*, std::unique_ptr<PlanSym>> g_sym;  // by workspace
unsigned long long g_sym_gen = 0;

// worker: ranks ri / rj (all E edges) -> the packed symbolic tables and the factor schedule
int build_symbolic(PlanSym* Y, std::vector<int> ri, std::vector<int> rj, int E, int Kp, bool has_dense,
                   size_t capacity) {
  BaPattern S;
  ba_build_pattern(ri.data(), rj.data(), E, Kp, &S, ba_max_pairs(Kp));
  if (S.too_dense || S.sidx.size() > ba_max_pairs(Kp)) {
    Y->err = "ba: factor pattern too dense for the plan tables";
    return M3S_EINVAL;
  }
  // sparse or dense factorisation: measured on MI355X (scripts/ba_exp.py), the one-workgroup sparse
  // factorisation costs ~3.8 us per elimination-tree level plus ~0.03 us per source-map entry (its
  // update volume); the dense one ~2.7 us per pose (its pivot chain)
  Y->dense = has_dense && 3.8 * S.nlev + 0.03 * (double)S.sidx.size() > 2.7 * S.nb;
  const char* solver = getenv("M3S_BA_SOLVER");
  if (solver) {  // tests and experiments: force one factorisation
    if (!strcmp(solver, "sparse")) Y->dense = 0;
    if (!strcmp(solver, "dense") && has_dense) Y->dense = 1;
  }
  // the leaf end of the elimination tree as multi-workgroup launches (steps [0, wide_steps)), the root end in the
  // one-workgroup kernel, minimising the measured step costs (MI355X, C5/C4 graphs): a launch ~5.8 us per step, a
  // step inside the workgroup ~3.7 us per round of M3S_BA_SP_WAVES waves (one wave per task). M3S_BA_WIDE=t (tests,
  // experiments): every step up to the last one with more than t tasks. (Round 5's opt-in alternatives for this
  // split, the subtree, frontal, supernodal and dense-top phases, measured slower or no faster and were removed in
  // round 6; they are kept at git tag ba-solver-experiments-r5, DESIGN.md §4 BA.)
  std::vector<int> tasks(S.nlev + 1);
  for (int l = 0; l <= S.nlev; l++) {
    const int na = l < S.nlev ? S.lev_ptr[l + 1] - S.lev_ptr[l] : 0;
    tasks[l] = na + S.grp_ptr[l + 1] - S.grp_ptr[l];
    if (l < BA_MAX_WIDE_STEPS) Y->step_tasks[l] = tasks[l];
  }
  const int lmax = std::min(S.nlev + 1, BA_MAX_WIDE_STEPS);
  const char* fenv = getenv("M3S_BA_FLOW");
  const bool flow_on = !(fenv && !strcmp(fenv, "0"));  // M3S_BA_FLOW=0 (A/B experiments): level-synchronous loops
  std::vector<int> sched;
  // bytes the one-workgroup dataflow kernel stages in LDS for a schedule (m3s_launch_ba_solve's test): the loop
  // tables col_ptr .. sidx (sections 1-9, 16-B aligned as packed below) + the schedule, x (8 doubles per column) and
  // 3 flags per column. A plan whose dataflow schedule does not fit runs level-synchronously.
  size_t table_bytes = 0;
  {
    const std::vector<int>* t[9] = {&S.col_ptr, &S.lev_ptr, &S.lev_col, &S.grp_ptr, &S.grp, &S.pull_grp, &S.src,
                                    &S.sidx, &S.rowL};
    for (const std::vector<int>* v : t) table_bytes += (sizeof(int) * v->size() + 15) & ~(size_t)15;
  }
  auto flow_fits = [&](const std::vector<int>& sc) {
    const size_t plan = table_bytes + sizeof(int) * sc.size();
    return ((plan + 15) & ~(size_t)15) + (size_t)S.nb * 64 + (size_t)S.nb * 12 <= (size_t)BA_SP_PLAN_BYTES;
  };
  auto legacy_split = [&]() {  // launched wide steps: minimise the measured step costs
    constexpr double kLaunchUs = 5.8, kRoundUs = 3.7;
    std::vector<double> suffix(lmax + 1, 0.0);  // cost of steps [L, lmax) inside the workgroup
    for (int l = lmax - 1; l >= 0; l--)
      suffix[l] = suffix[l + 1] + kRoundUs * ((tasks[l] + M3S_BA_SP_WAVES - 1) / M3S_BA_SP_WAVES);
    int best_L = 0;
    double best = suffix[0];
    for (int L = 1; L <= lmax; L++) {
      const double c = kLaunchUs * L + suffix[L];
      if (c < best) {
        best = c;
        best_L = L;
      }
    }
    return best_L;
  };
  if (const char* w = getenv("M3S_BA_WIDE")) {
    const int thr = atoi(w);
    int last = -1;
    for (int l = 0; l <= S.nlev; l++)
      if (tasks[l] > thr) last = l;
    Y->wide_steps = std::min(last + 1, BA_MAX_WIDE_STEPS);
  } else {
    Y->wide_steps = legacy_split();
  }
  // the wide steps' task records (ba_sparse_step_kernel): per task {j, b0, b1, pull group or -1} and its group's
  // source range, so a launched task starts with its column's own loads
  std::vector<int> step_rec;
  {
    auto put = [&](int j, int g) {
      const int* gq = g >= 0 ? &S.grp[4 * (size_t)g] : nullptr;
      const int r[8] = {j, S.col_ptr[j], S.col_ptr[j + 1], g, gq ? gq[1] : 0, gq ? gq[2] : 0, 0, 0};
      step_rec.insert(step_rec.end(), r, r + 8);
    };
    for (int l = 0; l < lmax; l++) {
      Y->step_base[l] = (int)step_rec.size() / 8;
      Y->step_na[l] = l < S.nlev ? S.lev_ptr[l + 1] - S.lev_ptr[l] : 0;
      for (int c = l < S.nlev ? S.lev_ptr[l] : 0; c < (l < S.nlev ? S.lev_ptr[l + 1] : 0); c++)
        put(S.lev_col[c], S.pull_grp[S.lev_col[c]]);
      for (int t = S.grp_ptr[l]; t < S.grp_ptr[l + 1]; t++) put(S.grp[4 * (size_t)t], t);  // (none at step 0)
      Y->step_tasks[l] = (int)step_rec.size() / 8 - Y->step_base[l];
    }
  }
  // dataflow schedule of the one-workgroup part and the back substitution (ba_pattern.h)
  if (flow_on) ba_flow_schedule(S, Y->wide_steps, M3S_BA_SP_WAVES, &sched);
  Y->flow = sched.empty() ? 0 : 1;
  if (Y->flow && !flow_fits(sched)) {  // the kernel would run level-synchronously: drop the schedule (and say so)
    Y->flow = 0;
    sched.clear();
  }
  const std::vector<int>* secs[BA_SYM_SECTIONS] = {&S.perm,    &S.col_ptr,  &S.rowL,    &S.lev_ptr,  &S.lev_col,
                                                   &S.grp_ptr, &S.grp,      &S.pull_grp, &S.src,     &S.sidx,
                                                   &sched,     &S.asm_ptr,  &S.asm_ent, &S.rhs_ptr, &S.rhs_ent,
                                                   &step_rec};
  size_t total = 0;
  for (int k = 0; k < BA_SYM_SECTIONS; k++) {
    Y->off[k] = total;
    total += (sizeof(int) * secs[k]->size() + 15) & ~(size_t)15;
  }
  if (total > capacity) {
    Y->err = "ba: factor pattern too dense for the plan tables";
    return M3S_EINVAL;
  }
  Y->image.assign(total, 0);
  for (int k = 0; k < BA_SYM_SECTIONS; k++)
    if (!secs[k]->empty()) memcpy(Y->image.data() + Y->off[k], secs[k]->data(), sizeof(int) * secs[k]->size());
  Y->nb = S.nb;
  Y->nlev = S.nlev;
  Y->nL = S.nL;
  Y->plan_lo_off = (int)Y->off[1];  // col_ptr .. sidx and the dataflow schedule, staged into LDS by the factor kernel
  Y->plan_bytes = (int)(Y->off[10] + sched.size() * sizeof(int) - Y->off[1]);
  return M3S_OK;
}

// the plan's PlanSym, joined (with `upload`, its tables enqueued on `s` the first time); nullptr + g_err on failure
PlanSym* plan_symbolic(const BaPlanImpl* P, hipStream_t s, bool upload, int* rc) {
  std::lock_guard<std::mutex> lock(g_sym_mu);
  auto it = g_sym.find(P->ws);
  if (it == g_sym.end() || it->second->gen != P->sym_gen) {
    *rc = fail(M3S_EINVAL, "ba: this plan was superseded by a newer plan on the same workspace");
    return nullptr;
  }
  PlanSym* Y = it->second.get();
  if (!Y->joined) {
    Y->rc = Y->fut.get();
    Y->joined = true;
  }
  if (upload && !Y->uploaded && Y->rc == M3S_OK) {
    Y->uploaded = true;
    if (!Y->image.empty()) {
      PlanStage& st = plan_stage();
      std::lock_guard<std::mutex> sl(st.mu);
      hipError_t e = hipSuccess;
      if (st.pending) e = hipEventSynchronize(st.landed);
      st.pending = false;
      if (e == hipSuccess && !st.landed) e = hipEventCreateWithFlags(&st.landed, hipEventDisableTiming);
      if (e == hipSuccess && st.cap < Y->image.size()) {
        if (st.buf) (void)hipHostFree(st.buf);
        st.buf = nullptr;
        st.cap = 0;
        const size_t want = std::max(Y->image.size(), (size_t)1 << 20);
        e = hipHostMalloc((void**)&st.buf, want, hipHostMallocDefault);
        if (e == hipSuccess) st.cap = want;
      }
      if (e == hipSuccess) {
        memcpy(st.buf, Y->image.data(), Y->image.size());
        e = hipMemcpyAsync(Y->dst, st.buf, Y->image.size(), hipMemcpyHostToDevice, s);
      }
      if (e == hipSuccess) e = hipEventRecord(st.landed, s);
      if (e != hipSuccess) {
        Y->rc = M3S_EHIP;
        Y->err = std::string("ba symbolic upload: ") + hipGetErrorString(e);
      } else {
        st.pending = true;
      }
      std::vector<char>().swap(Y->image);
    }
  }
  if (Y->rc != M3S_OK) {
    *rc = fail(Y->rc, Y->err);
    return nullptr;
  }
  *rc = M3S_OK;
  return Y;
}

// P->a with the symbolic tables of Y
BaArgs with_symbolic(const BaPlanImpl* P, const PlanSym* Y) {
  BaArgs a = P->a;
  const char* d = Y->dst;
  const void** dst[BA_SYM_SECTIONS] = {
      (const void**)&a.perm,    (const void**)&a.col_ptr, (const void**)&a.rowL,    (const void**)&a.lev_ptr,
      (const void**)&a.lev_col, (const void**)&a.grp_ptr, (const void**)&a.grp,     (const void**)&a.pull_grp,
      (const void**)&a.src,     (const void**)&a.sidx,    (const void**)&a.sched,   (const void**)&a.asm_ptr,
      (const void**)&a.asm_ent, (const void**)&a.rhs_ptr, (const void**)&a.rhs_ent, (const void**)&a.step_rec};
  for (int k = 0; k < BA_SYM_SECTIONS; k++) *dst[k] = d + Y->off[k];
  a.plan_lo = d + Y->plan_lo_off;
  a.plan_bytes = Y->plan_bytes;
  a.nb = Y->nb;
  a.nlev = Y->nlev;
  a.wide_steps = Y->wide_steps;
  a.flow = Y->flow;
  return a;
}

// Keyframe sources (host arrays of Kp entries) -> the plan's device tables.
int ba_make_plan_impl(const m3s_ba_config* cfg, float* Twc, const float* const* Xh, const float* const* Ch,
                      const float* scale_h, int Kp, int N, const int64_t* ii, const int64_t* jj, int E, int e0, int e1,
                      const int64_t* idx, const uint8_t* valid, const float* Q, float delta_thresh, float* dx_out,
                      const int64_t* edge_uid, const int64_t* kf_uid, void* workspace, size_t workspace_bytes,
                      m3s_ba_plan* plan, void* stream) {
  M3S_CHECK(cfg && plan, "ba: null argument");
  M3S_CHECK(cfg->mode >= 0 && cfg->mode <= 2, "ba: mode must be 0 (points), 1 (rays) or 2 (calib)");
  M3S_CHECK(Kp >= 1 && N >= 1 && E >= 0, "ba: bad sizes");
  M3S_CHECK(0 <= e0 && e0 <= e1 && e1 <= E, "ba: bad shard range");
  // the workspace reserves the factor and plan tables of the densest pattern (m3s_ba_workspace_size knows no
  // edges): nb(nb+1)/2 blocks of 512 B, 4.3 GB at this cap
  M3S_CHECK(Kp <= M3S_BA_MAX_POSES, "ba: at most 4096 poses (M3S_BA_MAX_POSES)");
  if (cfg->mode == 2) M3S_CHECK(cfg->width > 0 && cfg->height > 0 && (int64_t)cfg->width * cfg->height == N,
                                "ba calib: height*width must equal the points per keyframe");
  if (cfg->mode == 2)  // the 12-B calib record holds the matched pixel as u | v << 16 (ba.hip pack_record)
    M3S_CHECK(cfg->width < 65536 && cfg->height < 65536, "ba calib: width and height must be below 65536");
  if (workspace_bytes < m3s_ba_workspace_size(Kp, N, E)) return fail(M3S_ESPACE, "ba: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  BaPlanImpl P;
  memset(&P, 0, sizeof(P));
  const int chunks = ba_chunks(N, E);
  Carver c(workspace);
  void* blob;
  ba_carve(c, Kp, N, E, chunks, &P.a, &P.edge_sums_off, &blob);
  P.edge_sums_bytes = (size_t)E * 36 * sizeof(double);
  // a previous plan on this workspace: its worker must be done before the workspace is rewritten
  PlanSym* Y = nullptr;
  {
    std::lock_guard<std::mutex> lock(g_sym_mu);
    auto& slot = g_sym[workspace];
    if (slot && !slot->joined && slot->fut.valid()) slot->fut.wait();
    slot.reset(new PlanSym());
    Y = slot.get();
    Y->gen = ++g_sym_gen;
    P.sym_gen = Y->gen;
  }
  // record reuse: which keyframes changed since the workspace's previous plan (exact device compare, after the rank
  // remap below: only the keyframes this shard's edges touch are compared)
  RecCache* RC = nullptr;
  std::vector<uint8_t> kdirty(Kp, 1);
  std::vector<int> rc_ci;  // record reuse: copy index of each keyframe
  {
    std::lock_guard<std::mutex> lock(g_rec_mu);
    if (edge_uid && kf_uid) {
      RC = &g_rec[workspace];
    } else {
      auto it = g_rec.find(workspace);  // a plain plan repacks every slot: whatever was cached there is gone
      if (it != g_rec.end()) it->second.valid = false;
    }
  }
  if (RC) {
    const bool same = RC->valid && RC->N == N && RC->mode == cfg->mode && RC->Q_thresh == cfg->Q_thresh &&
                      RC->C_thresh == cfg->C_thresh &&
                      (cfg->mode != 2 || (RC->W == cfg->width && RC->z_eps == cfg->z_eps));
    if (!same) {
      RC->reset_maps();
      RC->N = N;
      RC->mode = cfg->mode;
      RC->Q_thresh = cfg->Q_thresh;
      RC->C_thresh = cfg->C_thresh;
      RC->W = cfg->width;
      RC->z_eps = cfg->z_eps;  // calib records hold log z_i, or NaN where z_i <= z_eps
    }
    RC->valid = false;  // until this plan is complete
    std::vector<int> ci(Kp, -1);
    int fresh = 0;
    for (int k = 0; k < Kp; k++) fresh += RC->copy_of.count(kf_uid[k]) ? 0 : 1;
    const size_t per = (size_t)4 * N;  // floats per keyframe copy
    if (RC->used + fresh > RC->cap) {  // grow the copies (geometric), keeping the ones in use
      const int cap = std::max(RC->used + fresh, RC->cap + RC->cap / 2 + 8);
      float* nc = nullptr;
      HIP_TRY(hipStreamSynchronize(s), "ba sync");
      HIP_TRY(hipMalloc((void**)&nc, sizeof(float) * per * cap), "ba keyframe copies");
      if (RC->used) HIP_TRY(hipMemcpy(nc, RC->copies, sizeof(float) * per * RC->used, hipMemcpyDeviceToDevice),
                            "ba keyframe copies");
      if (RC->copies) (void)hipFree(RC->copies);
      RC->copies = nc;
      RC->cap = cap;
    }
    if (Kp > RC->tcap) {
      HIP_TRY(hipStreamSynchronize(s), "ba sync");
      if (RC->table) (void)hipFree(RC->table);
      if (RC->dirty) (void)hipFree(RC->dirty);
      if (RC->table_h) (void)hipHostFree(RC->table_h);
      if (RC->dirty_h) (void)hipHostFree(RC->dirty_h);
      RC->table = nullptr;
      RC->dirty = nullptr;
      RC->table_h = nullptr;
      RC->dirty_h = nullptr;
      RC->tcap = 0;
      const int tc = std::max(Kp, 64);
      HIP_TRY(hipMalloc((void**)&RC->table, sizeof(BaKfCopy) * tc), "ba reuse table");
      HIP_TRY(hipMalloc((void**)&RC->dirty, tc), "ba reuse flags");
      HIP_TRY(hipHostMalloc((void**)&RC->table_h, sizeof(BaKfCopy) * tc, hipHostMallocDefault), "ba reuse table");
      HIP_TRY(hipHostMalloc((void**)&RC->dirty_h, tc, hipHostMallocDefault), "ba reuse flags");
      RC->tcap = tc;
    }
    for (int k = 0; k < Kp; k++) {
      auto it = RC->copy_of.find(kf_uid[k]);
      if (it == RC->copy_of.end()) {
        ci[k] = RC->used++;
        RC->copy_of.emplace(kf_uid[k], ci[k]);
        RC->scale.push_back(__builtin_bit_cast(uint32_t, scale_h[k]));
        RC->primed.push_back(0);
      } else {
        ci[k] = it->second;
        for (int q = 0; q < k; q++)
          if (ci[q] == ci[k]) return fail(M3S_EINVAL, "ba reuse: duplicate keyframe uid");
      }
    }
    rc_ci.swap(ci);
  }
  // rank remap (gn_kernels.cu:161-170): unique(cat(ii,jj)) sorted; searchsorted; pin = 1 for rows
  std::vector<int64_t> hii(E), hjj(E);
  if (E > 0) {
    HIP_TRY(hipMemcpyAsync(hii.data(), ii, sizeof(int64_t) * E, hipMemcpyDeviceToHost, s), "ba ii readback");
    HIP_TRY(hipMemcpyAsync(hjj.data(), jj, sizeof(int64_t) * E, hipMemcpyDeviceToHost, s), "ba jj readback");
  }
  if (E > 0) HIP_TRY(hipStreamSynchronize(s), "ba sync");
  std::vector<int64_t> u(hii);
  u.insert(u.end(), hjj.begin(), hjj.end());
  std::sort(u.begin(), u.end());
  u.erase(std::unique(u.begin(), u.end()), u.end());
  if ((int)u.size() > Kp) return fail(M3S_EINVAL, "ba: more unique keyframe ids in ii/jj than poses in Twc");
  std::vector<int> ri(E), rj(E);
  for (int e = 0; e < E; e++) {
    ri[e] = (int)(std::lower_bound(u.begin(), u.end(), hii[e]) - u.begin());
    rj[e] = (int)(std::lower_bound(u.begin(), u.end(), hjj[e]) - u.begin());
  }
  if (RC) {
    // the keyframes of this shard's edges: only their records can be reused here, so only they are compared (a
    // sharded solve compares ~1/world of the keyframes per rank). A keyframe's scale and copy change only when it
    // is compared; one compared for the first time is dirty whatever its copy holds.
    std::vector<char> usedk(Kp, 0);
    for (int e = e0; e < e1; e++) usedk[ri[e]] = usedk[rj[e]] = 1;
    for (int k = 0; k < Kp; k++) {
      const int c = rc_ci[k];
      if (!usedk[k]) {
        kdirty[k] = 0;
        RC->table_h[k] = BaKfCopy{nullptr, nullptr, nullptr};
        continue;
      }
      const uint32_t sb = __builtin_bit_cast(uint32_t, scale_h[k]);
      kdirty[k] = !RC->primed[c] || RC->scale[c] != sb;  // the average-confidence scale 1/N changed: its records did too
      RC->scale[c] = sb;
      RC->primed[c] = 1;
      RC->table_h[k] = BaKfCopy{Xh[k], Ch[k], RC->copies + (size_t)4 * N * c};
    }
    HIP_TRY(hipMemcpyAsync(RC->table, RC->table_h, sizeof(BaKfCopy) * Kp, hipMemcpyHostToDevice, s), "ba reuse table");
    HIP_TRY(hipMemsetAsync(RC->dirty, 0, Kp, s), "ba reuse flags");
    HIP_TRY(m3s_launch_ba_kf_compare(RC->table, Kp, N, RC->dirty, s), "ba keyframe compare launch");
    HIP_TRY(hipMemcpyAsync(RC->dirty_h, RC->dirty, Kp, hipMemcpyDeviceToHost, s), "ba reuse flags readback");
    HIP_TRY(hipStreamSynchronize(s), "ba sync");
    for (int k = 0; k < Kp; k++) kdirty[k] |= RC->dirty_h[k];
  }
  // linearisation block table: this shard's edges grouped by target keyframe j, chunk-major within a
  // group, so consecutive blocks (dealt to one XCD by xcd_remap) read the same X_j slab
  std::vector<int> lin_tab;
  {
    std::vector<int> order(e1 - e0);
    for (int e = 0; e < e1 - e0; e++) order[e] = e;
    std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return rj[e0 + x] < rj[e0 + y]; });
    lin_tab.reserve((size_t)(e1 - e0) * chunks);
    for (size_t g0 = 0; g0 < order.size();) {
      size_t g1 = g0;
      while (g1 < order.size() && rj[e0 + order[g1]] == rj[e0 + order[g0]]) g1++;
      for (int c = 0; c < chunks; c++)
        for (size_t t = g0; t < g1; t++) lin_tab.push_back(order[t] * chunks + c);
      g0 = g1;
    }
  }
  {
    std::vector<char> seen(Kp, 0);
    for (int e = e0; e < e1; e++) P.n_targets += seen[rj[e]] ? 0 : (seen[rj[e]] = 1);
  }
  // record slots: an edge keeps the slot of its uid when that slot is still inside this shard's record range and
  // repacks there only if one of its keyframes changed; new edges take free slots and pack
  const int EL = e1 - e0;
  std::vector<int> slot, pack;
  if (RC) {
    slot.assign(EL, -1);
    std::vector<char> taken(EL, 0), need(EL, 0);
    for (int t = 0; t < EL; t++) {
      auto it = RC->slot_of.find(edge_uid[e0 + t]);
      if (it != RC->slot_of.end() && it->second < EL && !taken[it->second]) {
        slot[t] = it->second;
        taken[slot[t]] = 1;
        need[t] = kdirty[ri[e0 + t]] || kdirty[rj[e0 + t]];
      }
    }
    for (int t = 0, f = 0; t < EL; t++) {
      if (slot[t] >= 0) continue;
      while (taken[f]) f++;
      slot[t] = f;
      taken[f] = 1;
      need[t] = 1;
    }
    RC->slot_of.clear();
    for (int t = 0; t < EL; t++) RC->slot_of[edge_uid[e0 + t]] = slot[t];
    for (int t = 0; t < EL; t++)
      if (need[t]) pack.push_back(t);
  } else {
    for (int t = 0; t < EL; t++) pack.push_back(t);
  }
  // the pack order: grouped by source keyframe (ba_pack_kernel splits it into eighths, one per XCD, so an XCD's L2
  // holds the points and confidences of its own source keyframes; the records land in their slots whatever the order)
  std::stable_sort(pack.begin(), pack.end(), [&](int x, int y) { return ri[e0 + x] < ri[e0 + y]; });
  // the tables the pack and the linearisation read, in ONE upload ahead of the pack; the symbolic tables follow
  // in the same blob (their own upload, at the first solve)
  struct Sec {
    const void* src;
    size_t bytes;
    const void** dst;
  };
  const Sec secs[] = {
      {ri.data() + e0, sizeof(int) * (e1 - e0), (const void**)&P.a.ii_rank},
      {rj.data() + e0, sizeof(int) * (e1 - e0), (const void**)&P.a.jj_rank},
      {Xh, sizeof(const float*) * Kp, (const void**)&P.a.Xkf},
      {Ch, sizeof(const float*) * Kp, (const void**)&P.a.Ckf},
      {scale_h, sizeof(float) * Kp, (const void**)&P.a.Cscale},
      {lin_tab.data(), sizeof(int) * lin_tab.size(), (const void**)&P.a.lin_tab},
      {slot.data(), sizeof(int) * slot.size(), (const void**)&P.a.rec_slot},
      {pack.data(), sizeof(int) * pack.size(), (const void**)&P.a.pack_list},
  };
  static_assert(sizeof(secs) / sizeof(secs[0]) + BA_SYM_SECTIONS == BA_BLOB_SECTIONS, "blob sections");
  size_t total = 0;
  for (const Sec& x : secs) total += (x.bytes + 15) & ~(size_t)15;
  const size_t capacity = ba_blob_capacity(Kp, E, chunks);
  if (total > capacity) return fail(M3S_EINVAL, "ba: plan tables exceed the workspace blob");
  {
    PlanStage& st = plan_stage();
    std::lock_guard<std::mutex> lock(st.mu);
    if (st.pending) HIP_TRY(hipEventSynchronize(st.landed), "ba stage wait");
    st.pending = false;
    if (!st.landed) HIP_TRY(hipEventCreateWithFlags(&st.landed, hipEventDisableTiming), "ba stage event");
    if (st.cap < total) {
      if (st.buf) (void)hipHostFree(st.buf);
      st.buf = nullptr;
      st.cap = 0;
      const size_t want = std::max(total, (size_t)1 << 20);
      HIP_TRY(hipHostMalloc((void**)&st.buf, want, hipHostMallocDefault), "ba stage alloc");
      st.cap = want;
    }
    size_t off = 0;
    for (const Sec& x : secs) {
      if (x.bytes) memcpy(st.buf + off, x.src, x.bytes);
      *x.dst = static_cast<char*>(blob) + off;
      off += (x.bytes + 15) & ~(size_t)15;
    }
    if (total) HIP_TRY(hipMemcpyAsync(blob, st.buf, total, hipMemcpyHostToDevice, s), "ba upload");
    HIP_TRY(hipEventRecord(st.landed, s), "ba stage record");
    st.pending = true;
  }
  if (!RC) P.a.rec_slot = nullptr;  // every edge packs into its own slot (the pack list is the source-keyframe order)
  Y->dst = static_cast<char*>(blob) + total;
  HIP_TRY(hipMemsetAsync(P.a.info, 0, 8 * sizeof(int), s), "ba memset");
  HIP_TRY(hipMemsetAsync(P.a.edge_sums, 0, P.edge_sums_bytes > 0 ? P.edge_sums_bytes : 8, s), "ba memset");
  P.a.bad = P.a.info + 3;
  P.a.stalled = P.a.info + 4;
  {
    const char* e = getenv("M3S_BA_FORCE_STALL");
    P.a.force_stall = e != nullptr && atoi(e) != 0;
  }
  P.a.Twc = Twc;
  P.a.idx = idx;
  P.a.valid = valid;
  P.a.Q = Q;
  P.p.mode = cfg->mode;
  P.p.N = N;
  P.p.chunks = chunks;
  P.p.edge_offset = e0;
  // gn_kernels.cu:546, 905-906, 1341-1342: const float sigma_inv = 1.0/sigma (double division)
  P.p.inv_a = (float)(1.0 / (double)cfg->sigma_a);
  P.p.inv_b = cfg->mode == 0 ? 0.0f : (float)(1.0 / (double)cfg->sigma_b);
  P.p.C_thresh = cfg->C_thresh;
  P.p.Q_thresh = cfg->Q_thresh;
  P.p.fx = cfg->fx;
  P.p.fy = cfg->fy;
  P.p.cx = cfg->cx;
  P.p.cy = cfg->cy;
  P.p.H = cfg->height;
  P.p.W = cfg->width;
  P.p.pixel_border = cfg->pixel_border;
  P.p.z_eps = cfg->z_eps;
  P.Kp = Kp;
  P.N = N;
  P.E = E;
  P.e0 = e0;
  P.e1 = e1;
  P.delta_thresh = delta_thresh;
  P.ws = workspace;
  P.a.dx = dx_out ? dx_out : P.a.dx;
  // per-call point records of this shard's edges: the matched point, its pixel and the folded validity
  // weight do not change across GN iterations (only the poses do)
  P.n_packed = RC ? (int)pack.size() : EL;
  P.n_dirty = 0;
  for (int k = 0; k < Kp; k++) P.n_dirty += kdirty[k];
  // M3S_BA_FUSED_PACK=1 (opt-in): when every shard edge packs, the pack's gathers run inside the first
  // linearisation (ba_lin_kernel<PACK>) instead of their own launch. Measured slower at C5 (pack 4.3 ms + lin 1.9 ms
  // -> one 8.3 ms launch: the gathers' latency at the linearisation's 3 waves per SIMD), so off by default
  const char* fpe = getenv("M3S_BA_FUSED_PACK");
  const bool defer = P.n_packed == EL && EL > 0 && fpe && !strcmp(fpe, "1");
  if (defer) {
    std::lock_guard<std::mutex> lock(g_sym_mu);
    Y->pack_deferred = true;
  } else {
    Span sp("ba_pack", s);
    HIP_TRY(m3s_launch_ba_pack(&P.a, &P.p, P.n_packed, s), "ba pack launch");
  }
  if (RC) RC->valid = true;
  // the symbolic analysis of ALL E edges (every rank builds the identical system) runs on a host worker while
  // the device packs and linearises
  Y->fut = std::async(std::launch::async, build_symbolic, Y, std::move(ri), std::move(rj), E, Kp, P.a.H != nullptr,
                      capacity - total);
  memcpy(plan->opaque, &P, sizeof(P));
  return M3S_OK;
}
}  // namespace

extern "C" int m3s_ba_make_plan_reuse(const m3s_ba_config* cfg, float* Twc, const float* Xs, const float* Cs, int Kp,
                                      int N, const int64_t* ii, const int64_t* jj, int E, int e0, int e1,
                                      const int64_t* idx, const uint8_t* valid, const float* Q, float delta_thresh,
                                      float* dx_out, const m3s_ba_reuse* reuse, void* workspace,
                                      size_t workspace_bytes, m3s_ba_plan* plan, void* stream) {
  M3S_CHECK(!reuse || (reuse->edge_uid && reuse->kf_uid), "ba reuse: null uid array");
  M3S_CHECK(Xs && Cs && Kp >= 1 && N >= 1, "ba: null Xs/Cs or bad sizes");
  std::vector<const float*> xh(Kp), ch(Kp);
  std::vector<float> sh(Kp, 1.0f);  // stacked Cs is already the average confidence
  for (int k = 0; k < Kp; k++) {
    xh[k] = Xs + (size_t)k * N * 3;
    ch[k] = Cs + (size_t)k * N;
  }
  return ba_make_plan_impl(cfg, Twc, xh.data(), ch.data(), sh.data(), Kp, N, ii, jj, E, e0, e1, idx, valid, Q,
                           delta_thresh, dx_out, reuse ? reuse->edge_uid : nullptr, reuse ? reuse->kf_uid : nullptr,
                           workspace, workspace_bytes, plan, stream);
}

extern "C" int m3s_ba_make_plan_kf_reuse(const m3s_ba_config* cfg, float* Twc, const m3s_ba_keyframes* kf, int Kp,
                                         int N, const int64_t* ii, const int64_t* jj, int E, int e0, int e1,
                                         const int64_t* idx, const uint8_t* valid, const float* Q, float delta_thresh,
                                         float* dx_out, const m3s_ba_reuse* reuse, void* workspace,
                                         size_t workspace_bytes, m3s_ba_plan* plan, void* stream) {
  M3S_CHECK(!reuse || (reuse->edge_uid && reuse->kf_uid), "ba reuse: null uid array");
  M3S_CHECK(kf && kf->X && kf->C && kf->N_avg && Kp >= 1 && N >= 1, "ba: null keyframe table or bad sizes");
  std::vector<float> sh(Kp);
  for (int k = 0; k < Kp; k++) {
    M3S_CHECK(kf->X[k] && kf->C[k], "ba: null keyframe buffer");
    M3S_CHECK(kf->N_avg[k] > 0.0f, "ba: keyframe fusion count N must be positive");
    sh[k] = 1.0f / kf->N_avg[k];  // torch's C / N on a device tensor: C * float32(1/N)
  }
  return ba_make_plan_impl(cfg, Twc, kf->X, kf->C, sh.data(), Kp, N, ii, jj, E, e0, e1, idx, valid, Q, delta_thresh,
                           dx_out, reuse ? reuse->edge_uid : nullptr, reuse ? reuse->kf_uid : nullptr, workspace,
                           workspace_bytes, plan, stream);
}

extern "C" int m3s_ba_make_plan(const m3s_ba_config* cfg, float* Twc, const float* Xs, const float* Cs, int Kp, int N,
                                const int64_t* ii, const int64_t* jj, int E, int e0, int e1, const int64_t* idx,
                                const uint8_t* valid, const float* Q, float delta_thresh, float* dx_out,
                                void* workspace, size_t workspace_bytes, m3s_ba_plan* plan, void* stream) {
  return m3s_ba_make_plan_reuse(cfg, Twc, Xs, Cs, Kp, N, ii, jj, E, e0, e1, idx, valid, Q, delta_thresh, dx_out,
                                nullptr, workspace, workspace_bytes, plan, stream);
}

extern "C" int m3s_ba_make_plan_kf(const m3s_ba_config* cfg, float* Twc, const m3s_ba_keyframes* kf, int Kp, int N,
                                   const int64_t* ii, const int64_t* jj, int E, int e0, int e1, const int64_t* idx,
                                   const uint8_t* valid, const float* Q, float delta_thresh, float* dx_out,
                                   void* workspace, size_t workspace_bytes, m3s_ba_plan* plan, void* stream) {
  return m3s_ba_make_plan_kf_reuse(cfg, Twc, kf, Kp, N, ii, jj, E, e0, e1, idx, valid, Q, delta_thresh, dx_out,
                                   nullptr, workspace, workspace_bytes, plan, stream);
}

extern "C" int m3s_ba_reuse_info(const m3s_ba_plan* plan, int* packed_edges, int* changed_keyframes) {
  M3S_CHECK(plan && packed_edges && changed_keyframes, "ba: null argument");
  const BaPlanImpl* P = reinterpret_cast<const BaPlanImpl*>(plan->opaque);
  *packed_edges = P->n_packed;
  *changed_keyframes = P->n_dirty;
  return M3S_OK;
}

extern "C" int m3s_ba_plan_release(const void* workspace) {
  std::unique_ptr<PlanSym> Y;
  {
    std::lock_guard<std::mutex> lock(g_sym_mu);
    auto it = g_sym.find(workspace);
    if (it == g_sym.end()) return M3S_OK;
    Y = std::move(it->second);
    g_sym.erase(it);
  }
  if (Y && !Y->joined && Y->fut.valid()) Y->fut.wait();  // the worker writes into Y: done before it is freed
  return M3S_OK;
}

extern "C" int m3s_ba_plan_count(void) {
  std::lock_guard<std::mutex> lock(g_sym_mu);
  return (int)g_sym.size();
}

extern "C" int m3s_ba_reuse_release(const void* workspace) {
  m3s_ba_plan_release(workspace);
  std::lock_guard<std::mutex> lock(g_rec_mu);
  auto it = g_rec.find(workspace);
  if (it == g_rec.end()) return M3S_OK;
  it->second.free_all();
  g_rec.erase(it);
  return M3S_OK;
}

extern "C" int m3s_ba_edge_sums(const m3s_ba_plan* plan, size_t* byte_offset, size_t* byte_count) {
  M3S_CHECK(plan && byte_offset && byte_count, "ba: null argument");
  const BaPlanImpl* P = reinterpret_cast<const BaPlanImpl*>(plan->opaque);
  *byte_offset = P->edge_sums_off;
  *byte_count = P->edge_sums_bytes;
  return M3S_OK;
}

extern "C" int m3s_ba_plan_info(const m3s_ba_plan* plan, int* info) {
  M3S_CHECK(plan && info, "ba: null argument");
  const BaPlanImpl* P = reinterpret_cast<const BaPlanImpl*>(plan->opaque);
  int rc;
  const PlanSym* Y = plan_symbolic(P, nullptr, false, &rc);  // joins the symbolic analysis
  if (Y == nullptr) return rc;
  info[0] = P->p.chunks;
  info[1] = Y->nL;
  info[2] = Y->nlev;
  info[3] = Y->wide_steps;
  info[4] = Y->dense;
  info[5] = P->n_targets;
  info[6] = P->e1 - P->e0;
  info[7] = P->Kp;
  info[8] = info[9] = info[10] = info[11] = info[12] = 0;  // round 5's opt-in solver phases (removed in round 6)
  return M3S_OK;
}

extern "C" int m3s_ba_linearize(const m3s_ba_plan* plan, void* stream) {
  M3S_CHECK(plan, "ba: null plan");
  const BaPlanImpl* P = reinterpret_cast<const BaPlanImpl*>(plan->opaque);
  hipStream_t s = (hipStream_t)stream;
  // a shard writes only its own rows: clear the rest so the caller's all-reduce sums fresh rows
  if ((P->e0 > 0 || P->e1 < P->E) && P->edge_sums_bytes > 0)
    HIP_TRY(hipMemsetAsync(P->a.edge_sums, 0, P->edge_sums_bytes, s), "ba memset");
  int pack = 0;  // this plan's first linearisation also packs (see ba_make_plan_impl)
  {
    std::lock_guard<std::mutex> lock(g_sym_mu);
    auto it = g_sym.find(P->ws);
    if (it != g_sym.end() && it->second->gen == P->sym_gen && it->second->pack_deferred) {
      pack = 1;
      it->second->pack_deferred = false;
    }
  }
  Span sp(pack ? "ba_lin_pack" : "ba_linearize", s);
  HIP_TRY(m3s_launch_ba_lin(&P->a, &P->p, P->e1 - P->e0, pack, s), "ba linearize launch");
  return M3S_OK;
}

extern "C" int m3s_ba_solve(const m3s_ba_plan* plan, void* stream) {
  M3S_CHECK(plan, "ba: null plan");
  const BaPlanImpl* P = reinterpret_cast<const BaPlanImpl*>(plan->opaque);
  hipStream_t s = (hipStream_t)stream;
  int rc;
  const PlanSym* Y = plan_symbolic(P, s, true, &rc);  // the first solve joins the host worker and uploads its tables
  if (Y == nullptr) return rc;
  const BaArgs a = with_symbolic(P, Y);
  Span sp("ba_solve", s);
  HIP_TRY(Y->dense ? m3s_launch_ba_solve_dense(&a, P->Kp, Y->nL, P->delta_thresh, s)
                   : m3s_launch_ba_solve(&a, P->Kp, Y->nL, P->delta_thresh, Y->step_tasks, Y->step_base,
                                         Y->step_na, s),
          "ba solve launch");
  return M3S_OK;
}

extern "C" int m3s_ba_iterations(const m3s_ba_plan* plan, int* iters_out, void* stream) {
  M3S_CHECK(plan && iters_out, "ba: null argument");
  const BaPlanImpl* P = reinterpret_cast<const BaPlanImpl*>(plan->opaque);
  hipStream_t s = (hipStream_t)stream;
  int st[3];  // iters, bad, stalled (info + 2 .. + 4)
  HIP_TRY(hipMemcpyAsync(st, P->a.iters, sizeof(st), hipMemcpyDeviceToHost, s), "ba readback");
  HIP_TRY(hipStreamSynchronize(s), "ba sync");
  *iters_out = st[0];
  if (st[2] != 0)
    return fail(M3S_ESTALL, "ba: a factor-schedule hand-off stalled (bounded wait timed out); poses were not updated "
                            "by the stalled iteration and the loop stopped");
  return M3S_OK;
}

extern "C" int m3s_gauss_newton(const m3s_ba_config* cfg, float* Twc, const float* Xs, const float* Cs, int Kp, int N,
                                const int64_t* ii, const int64_t* jj, int E, const int64_t* idx,
                                const uint8_t* valid, const float* Q, int max_iter, float delta_thresh, float* dx_out,
                                int* iters_out, void* workspace, size_t workspace_bytes, void* stream) {
  M3S_CHECK(max_iter >= 0, "ba: max_iter must be >= 0");
  m3s_ba_plan plan;
  int rc = m3s_ba_make_plan(cfg, Twc, Xs, Cs, Kp, N, ii, jj, E, 0, E, idx, valid, Q, delta_thresh, dx_out, workspace,
                            workspace_bytes, &plan, stream);
  if (rc != M3S_OK) return rc;
  if (dx_out && Kp > 1)
    HIP_TRY(hipMemsetAsync(dx_out, 0, sizeof(float) * (size_t)(Kp - 1) * 7, (hipStream_t)stream), "ba memset");
  for (int it = 0; it < max_iter; it++) {
    if ((rc = m3s_ba_linearize(&plan, stream)) != M3S_OK) return rc;
    if ((rc = m3s_ba_solve(&plan, stream)) != M3S_OK) return rc;
  }
  // one readback per call (the reference's host loop syncs every iteration): the iteration count and the
  // schedule-stall check (M3S_ESTALL), so a stalled solve is an error, never silently unoptimised poses
  int iters_local = 0;
  return m3s_ba_iterations(&plan, iters_out ? iters_out : &iters_local, stream);
}

// ------------------------------------------------------------------------------------------
// measured peak (bench roofline context only)
// ------------------------------------------------------------------------------------------
extern "C" int m3s_peak_fma_f32(float* out_dev, int blocks, int iters, void* stream) {
  M3S_CHECK(out_dev && blocks > 0 && iters > 0, "peak: bad argument");
  HIP_TRY(m3s_launch_peak_fma_f32(out_dev, blocks, iters, (hipStream_t)stream), "peak launch");
  return M3S_OK;
}

// ------------------------------------------------------------------------------------------
// retrieval codebook quantization (retrieval_database.py:96-105; kernels in retrieval.hip)
// ------------------------------------------------------------------------------------------
namespace {
constexpr int RQ_ROWS = 256, RQ_QG = 304, RQ_NQT = 19;  // retrieval.hip: rows per block, queries per group
inline int rq_steps(int D) { return (D + 31) / 32; }
inline int rq_rows_padded(int C) { return (C + RQ_ROWS - 1) / RQ_ROWS * RQ_ROWS; }
inline int rq_groups(int M) { return (M + RQ_QG - 1) / RQ_QG; }

size_t codebook_carve(Carver& c, int C, int D, uint4** frag, float** cn) {
  const size_t Cp = (size_t)rq_rows_padded(C);
  *frag = c.take<uint4>(Cp / 16 * rq_steps(D) * 128);  // (Cp/16 tiles) x S x {hi, lo} x 64 lanes (rq_prep_kernel)
  *cn = c.take<float>(Cp);
  return c.off;
}

size_t quantize_carve(Carver& c, int C, int D, int M, int k, uint4** qfrag, float** qn, unsigned long long** cand) {
  const int G = rq_groups(M);
  *qfrag = c.take<uint4>((size_t)G * rq_steps(D) * RQ_NQT * 128);
  *qn = c.take<float>((size_t)G * RQ_QG);
  *cand = c.take<unsigned long long>((size_t)G * (rq_rows_padded(C) / RQ_ROWS) * RQ_QG * k);
  return c.off;
}
}  // namespace

extern "C" size_t m3s_codebook_size(int C, int D) {
  if (C <= 0 || D <= 0) return 0;
  Carver c(nullptr);
  uint4* f;
  float* n;
  return codebook_carve(c, C, D, &f, &n);
}

extern "C" int m3s_codebook_prepare(const float* centroids, int C, int D, void* codebook, size_t codebook_bytes,
                                    void* stream) {
  M3S_CHECK(centroids && codebook, "codebook: null argument");
  M3S_CHECK(C > 0 && D > 0, "codebook: C and D must be positive");
  M3S_CHECK((long long)rq_rows_padded(C) * rq_steps(D) * 32 < (1ll << 31), "codebook: too large");
  if (codebook_bytes < m3s_codebook_size(C, D)) return fail(M3S_ESPACE, "codebook: buffer too small");
  Carver c(codebook);
  uint4* frag;
  float* cn;
  codebook_carve(c, C, D, &frag, &cn);
  hipStream_t s = (hipStream_t)stream;
  const int Cp = rq_rows_padded(C);
  HIP_TRY(m3s_launch_rq_prep(centroids, C, D, rq_steps(D), Cp / 16, RQ_ROWS / 16, frag, Cp, __builtin_inff(), cn, s),
          "codebook prep launch");
  return M3S_OK;
}

extern "C" size_t m3s_quantize_workspace_size(int C, int D, int M, int k) {
  if (C <= 0 || D <= 0 || M <= 0 || k <= 0) return 0;
  Carver c(nullptr);
  uint4* q;
  float* n;
  unsigned long long* cand;
  return quantize_carve(c, C, D, M, k, &q, &n, &cand);
}

extern "C" int m3s_quantize(const void* codebook, int C, int D, const float* qvecs, int M, int k, int64_t* topk_out,
                            void* workspace, size_t workspace_bytes, void* stream) {
  M3S_CHECK(codebook && qvecs && topk_out && workspace, "quantize: null argument");
  M3S_CHECK(C > 0 && D > 0 && M > 0, "quantize: C, D and M must be positive");
  M3S_CHECK(k >= 1 && k <= 8, "quantize: k (multiple_assignment) must be in 1..8");
  M3S_CHECK(k <= C, "quantize: k larger than the codebook (torch.topk: selected index k out of range)");
  M3S_CHECK(rq_groups(M) < 65536, "quantize: too many query rows");
  if (workspace_bytes < m3s_quantize_workspace_size(C, D, M, k)) return fail(M3S_ESPACE, "quantize: workspace too small");
  Carver cb(const_cast<void*>(codebook));
  uint4* cfrag;
  float* cn;
  codebook_carve(cb, C, D, &cfrag, &cn);
  Carver c(workspace);
  uint4* qfrag;
  float* qn;
  unsigned long long* cand;
  quantize_carve(c, C, D, M, k, &qfrag, &qn, &cand);
  hipStream_t s = (hipStream_t)stream;
  const int G = rq_groups(M), S = rq_steps(D);
  HIP_TRY(m3s_launch_rq_prep(qvecs, M, D, S, G * RQ_NQT, RQ_NQT, qfrag, G * RQ_QG, 0.0f, qn, s),
          "quantize prep launch");
  {
    Span sp("quantize_topk", s);
    HIP_TRY(m3s_launch_rq_topk(cfrag, cn, qfrag, qn, S, rq_rows_padded(C) / RQ_ROWS, G, M, k, cand, topk_out, s),
            "quantize topk launch");
  }
  return M3S_OK;
}
