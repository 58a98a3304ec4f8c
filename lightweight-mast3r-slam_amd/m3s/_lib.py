"""ctypes binding of libm3s.so (the C ABI declared in include/m3s.h).

The product path has no fallback: if the HIP library or a GPU is missing, every operator raises
RuntimeError. Tensors are passed as raw device pointers together with torch's current HIP stream,
so the kernels are ordered with the caller's other torch work exactly like the reference's
extension ops (which, unlike these, always used the legacy default stream).
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# M3S_LIB: alternative build of the same library (kernel experiments); still the HIP library, no fallback
LIB_PATH = os.environ.get("M3S_LIB") or os.path.join(os.path.dirname(_HERE), "lib", "libm3s.so")

ABI_VERSION = 5  # include/m3s.h M3S_ABI_VERSION

c_int, c_float, c_double, c_size_t, c_void_p = ctypes.c_int, ctypes.c_float, ctypes.c_double, ctypes.c_size_t, ctypes.c_void_p


class BaConfig(ctypes.Structure):
    _fields_ = [("mode", c_int), ("sigma_a", c_float), ("sigma_b", c_float), ("C_thresh", c_float),
                ("Q_thresh", c_float), ("fx", c_float), ("fy", c_float), ("cx", c_float), ("cy", c_float),
                ("height", c_int), ("width", c_int), ("pixel_border", c_int), ("z_eps", c_float)]


class BaKeyframes(ctypes.Structure):
    _fields_ = [("X", ctypes.POINTER(c_void_p)), ("C", ctypes.POINTER(c_void_p)), ("N_avg", ctypes.POINTER(c_float))]


class BaReuse(ctypes.Structure):
    _fields_ = [("edge_uid", c_void_p), ("kf_uid", c_void_p)]


class BaPlan(ctypes.Structure):
    _fields_ = [("opaque", ctypes.c_ubyte * 768)]


class TrackConfig(ctypes.Structure):
    _fields_ = [("mode", c_int), ("max_iters", c_int), ("C_conf", c_float), ("Q_conf", c_float),
                ("min_match_frac", c_float), ("sigma_a", c_float), ("sigma_b", c_float), ("huber_k", c_float),
                ("rel_error", c_float), ("delta_norm", c_float), ("pixel_border", c_float),
                ("depth_eps", c_float), ("K", c_float * 9), ("H", c_int), ("W", c_int)]


class TrackInputs(ctypes.Structure):
    _fields_ = [("idx_f2k", c_void_p), ("valid_match", c_void_p), ("Xf", c_void_p), ("Cf", c_void_p),
                ("Nf", c_float), ("Qff", c_void_p), ("Xk", c_void_p), ("Ck", c_void_p), ("Nk", c_float),
                ("Qkf", c_void_p), ("T_WCf", c_void_p), ("T_WCk", c_void_p), ("direct", c_int),
                ("meas_k", c_void_p), ("valid_meas_k", c_void_p)]


class TrackFuse(ctypes.Structure):
    _fields_ = [("Xk_canon", c_void_p), ("Ck_sum", c_void_p), ("Xkf", c_void_p), ("Ckf", c_void_p),
                ("Xk_out", c_void_p), ("Ck_out", c_void_p), ("Cf", c_void_p), ("Ck_avg_out", c_void_p),
                ("Cf_avg_out", c_void_p), ("Nk_new", c_float), ("Nf", c_float), ("slot_N", c_void_p),
                ("slot_N_updates", c_void_p), ("slot_dirty", c_void_p), ("N_new", c_int), ("N_updates_new", c_int)]


class TrackResult(ctypes.Structure):
    _fields_ = [("T_WCf", c_float * 8), ("T_CkCf", c_float * 8), ("cost", c_double), ("iters", c_int),
                ("status", c_int), ("n_valid_opt", c_int), ("n_valid_kf", c_int), ("n_unique", c_int),
                ("N", c_int)]


TRACK_OK, TRACK_MAX_ITERS, TRACK_CHOLESKY_FAILED, TRACK_SKIPPED = 1, 2, 3, 4

# exported entry points and their argtypes (restype int unless noted)
_SIGS = {
    "m3s_abi_version": ([], c_int),
    "m3s_last_error": ([], ctypes.c_char_p),
    "m3s_timing_enable": ([c_int], None),
    "m3s_timing_reset": ([], None),
    "m3s_timing_query": ([ctypes.c_char_p, ctypes.POINTER(c_double), ctypes.POINTER(c_int)], c_int),
    "m3s_iter_proj": ([c_void_p] * 5 + [c_int] * 6 + [c_float, c_float, c_void_p], c_int),
    "m3s_refine_matches": ([c_int] + [c_void_p] * 4 + [c_int] * 7 + [c_void_p], c_int),
    "m3s_ba_workspace_size": ([c_int, c_int, c_int], c_size_t),
    "m3s_gauss_newton": ([ctypes.POINTER(BaConfig), c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p,
                          c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, c_float, c_void_p,
                          ctypes.POINTER(c_int), c_void_p, c_size_t, c_void_p], c_int),
    "m3s_ba_make_plan": ([ctypes.POINTER(BaConfig), c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p,
                          c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_float, c_void_p,
                          c_void_p, c_size_t, ctypes.POINTER(BaPlan), c_void_p], c_int),
    "m3s_ba_make_plan_kf": ([ctypes.POINTER(BaConfig), c_void_p, ctypes.POINTER(BaKeyframes), c_int, c_int, c_void_p,
                             c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_float, c_void_p,
                             c_void_p, c_size_t, ctypes.POINTER(BaPlan), c_void_p], c_int),
    "m3s_ba_make_plan_reuse": ([ctypes.POINTER(BaConfig), c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p,
                                c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_float, c_void_p,
                                ctypes.POINTER(BaReuse), c_void_p, c_size_t, ctypes.POINTER(BaPlan), c_void_p], c_int),
    "m3s_ba_make_plan_kf_reuse": ([ctypes.POINTER(BaConfig), c_void_p, ctypes.POINTER(BaKeyframes), c_int, c_int,
                                   c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_float,
                                   c_void_p, ctypes.POINTER(BaReuse), c_void_p, c_size_t, ctypes.POINTER(BaPlan),
                                   c_void_p], c_int),
    "m3s_ba_reuse_info": ([ctypes.POINTER(BaPlan), ctypes.POINTER(c_int), ctypes.POINTER(c_int)], c_int),
    "m3s_ba_reuse_release": ([c_void_p], c_int),
    "m3s_ba_plan_release": ([c_void_p], c_int),
    "m3s_ba_plan_count": ([], c_int),
    "m3s_ba_edge_sums": ([ctypes.POINTER(BaPlan), ctypes.POINTER(c_size_t), ctypes.POINTER(c_size_t)], c_int),
    "m3s_ba_linearize": ([ctypes.POINTER(BaPlan), c_void_p], c_int),
    "m3s_ba_solve": ([ctypes.POINTER(BaPlan), c_void_p], c_int),
    "m3s_ba_iterations": ([ctypes.POINTER(BaPlan), ctypes.POINTER(c_int), c_void_p], c_int),
    "m3s_ba_plan_info": ([ctypes.POINTER(BaPlan), ctypes.POINTER(c_int)], c_int),
    "m3s_ba_pattern_stats": ([c_void_p, c_void_p, c_int, c_int, ctypes.POINTER(c_int)], c_int),
    "m3s_peak_fma_f32": ([c_void_p, c_int, c_int, c_void_p], c_int),
    "m3s_match_workspace_size": ([c_int] * 4, c_size_t),
    "m3s_match": ([c_void_p] * 7 + [c_int] * 5 + [c_float] * 3 + [c_int, c_int, c_void_p, c_size_t, c_void_p], c_int),
    "m3s_track_workspace_size": ([c_int], c_size_t),
    "m3s_track_release": ([c_void_p], c_int),
    "m3s_codebook_size": ([c_int, c_int], c_size_t),
    "m3s_codebook_prepare": ([c_void_p, c_int, c_int, c_void_p, c_size_t, c_void_p], c_int),
    "m3s_quantize_workspace_size": ([c_int] * 4, c_size_t),
    "m3s_quantize": ([c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_void_p, c_void_p, c_size_t, c_void_p], c_int),
    "m3s_track": ([ctypes.POINTER(TrackInputs), ctypes.POINTER(TrackConfig), ctypes.POINTER(TrackFuse), c_int,
                   c_void_p, ctypes.POINTER(TrackResult), c_void_p, c_size_t, c_void_p], c_int),
}

EXPORTED = sorted(_SIGS)

_LIB = None
_GPU_OK = False  # a HIP device was verified once: later calls skip the query


def load(require_gpu=True):
    """Load libm3s.so. With require_gpu, raise unless a HIP device is visible to torch."""
    global _LIB, _GPU_OK
    if _LIB is not None and _GPU_OK:  # hot path: every operator call after the first (no device query)
        return _LIB
    if require_gpu and not torch.cuda.is_available():
        raise RuntimeError("m3s: no HIP device visible; the MI355X kernels have no CPU fallback")
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"m3s: {LIB_PATH} not built (run __graft_entry__.build() or make -C csrc)")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (args, res) in _SIGS.items():
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = res
        if lib.m3s_abi_version() != ABI_VERSION:
            raise RuntimeError(f"m3s: ABI version mismatch (library {lib.m3s_abi_version()}, bindings {ABI_VERSION})")
        _LIB = lib
    _GPU_OK = _GPU_OK or require_gpu
    return _LIB


def ba_pattern_stats(ii, jj, Kp):
    """Host-only: (factor blocks, elimination-tree levels, update groups, update sources, source-map
    entries, factor-task groups) of the
    symbolic factorisation a BA plan builds for the directed edges ii, jj (int64 host arrays)."""
    import numpy as np

    lib = load(require_gpu=False)
    ii = np.ascontiguousarray(ii, dtype=np.int64)
    jj = np.ascontiguousarray(jj, dtype=np.int64)
    out = (c_int * 6)()
    check(lib.m3s_ba_pattern_stats(c_void_p(ii.ctypes.data), c_void_p(jj.ctypes.data), len(ii), int(Kp), out))
    return tuple(out)


def check(rc):
    if rc != 0:
        msg = _LIB.m3s_last_error().decode() if _LIB is not None else ""
        raise RuntimeError(f"m3s error {rc}: {msg}")


_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_ptr(device=None):
    """torch's current HIP stream on `device` (raw handle; no Stream object on the hot path)."""
    if _RAW_STREAM is not None:
        idx = device.index if isinstance(device, torch.device) and device.index is not None else (
            device if isinstance(device, int) else torch.cuda.current_device())
        return c_void_p(_RAW_STREAM(idx))
    return c_void_p(torch.cuda.current_stream(device).cuda_stream)


def ptr(t):
    return c_void_p(t.data_ptr()) if t is not None else c_void_p(0)


_WS = {}


# key -> the ABI call that forgets a dropped buffer's per-workspace library state: the tracker's clean-scratch record,
# and the BA plan state of the workspace mast3r_slam_backends' gauss_newton_* cache under "ba" (it grows with E, so a
# growing SLAM run replaces it at nearly every backend solve; without the release every dropped buffer's PlanSym
# would stay in the library's table). HipShard / RecordCache own and release their own workspaces.
_WS_RELEASE = {"track": "m3s_track_release", "ba": "m3s_ba_plan_release"}


def workspace(key, nbytes, device, stream):
    """A cached uint8 device buffer per (key, device, stream), grown on demand (torch caching allocator).

    Contract: a buffer is only ever used by launches on the one stream it is keyed by, so consecutive
    calls reuse it in stream order; calls on another stream get their own buffer."""
    k = (key, device, stream.value)
    buf = _WS.get(k)
    if buf is None or buf.numel() < nbytes:
        if buf is not None and key in _WS_RELEASE and _LIB is not None:
            # the library's per-workspace state of the buffer being dropped (m3s_track_release: its "clean
            # scratch" record; the allocator may hand the same address to another buffer later)
            getattr(_LIB, _WS_RELEASE[key])(buf.data_ptr())
        buf = torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=device)
        _WS[k] = buf
    return buf


def require_cuda(name, *tensors):
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise RuntimeError(f"{name}: tensors must be on the HIP device (got {t.device})")
