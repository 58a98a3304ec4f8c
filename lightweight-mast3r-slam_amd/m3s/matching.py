"""Dense matching: the reference's ``mast3r_slam/matching.py`` surface over fused HIP kernels.

``match`` / ``match_iterative_proj`` keep the reference signatures and return values
(``matching.py:8-90``): ``idx_1_to_2`` (B, H*W) int64 and ``valid_match2`` (B, H*W, 1) bool. The
whole function is one C-ABI call (``m3s_match``): ray-image prep + iterative projection + occlusion
test + half-precision descriptor refine + linear index, three kernels, no host sync.
"""
import torch

from m3s import _lib
from m3s.config import config


def pixel_to_lin(p1, w):
    return p1[..., 0] + (w * p1[..., 1])  # matching.py:13-15


def lin_to_pixel(idx_1_to_2, w):
    u = idx_1_to_2 % w  # matching.py:18-22
    v = idx_1_to_2 // w
    return torch.stack((u, v), dim=-1)


def match(X11, X21, D11, D21, idx_1_to_2_init=None):
    return match_iterative_proj(X11, X21, D11, D21, idx_1_to_2_init)


def _f32(t):
    return t if (t.dtype == torch.float32 and t.is_contiguous()) else t.float().contiguous()


def match_iterative_proj(X11, X21, D11, D21, idx_1_to_2_init=None):
    _lib.require_cuda("match", X11, X21, D11, D21, idx_1_to_2_init)
    b, h, w = X21.shape[:3]
    F = D11.shape[-1]
    X11, X21, D11 = _f32(X11), _f32(X21), _f32(D11)
    D21 = _f32(D21).reshape(b, h, w, F)
    if tuple(X11.shape) != (b, h, w, 3) or tuple(D11.shape) != (b, h, w, F):
        raise RuntimeError("match: X11/X21 (B,H,W,3) and D11/D21 (B,H,W,F) must agree")
    return _match(X11.data_ptr(), X21.data_ptr(), D11.data_ptr(), D21.data_ptr(), b, h, w, F, X11.device,
                  idx_1_to_2_init)


def match_halves(X, D, idx_1_to_2_init=None):
    """``match(X[:b], X[b:], D[:b], D[b:], init)`` for stacked decoder outputs X (2b,H,W,3), D (2b,H,W,F)
    (mast3r_utils.py:238-240), with the halves passed as pointer offsets instead of four slice tensors."""
    _lib.require_cuda("match", X, D, idx_1_to_2_init)
    b2, h, w = X.shape[:3]
    F = D.shape[-1]
    X, D = _f32(X), _f32(D)
    if b2 % 2 or tuple(X.shape) != (b2, h, w, 3) or tuple(D.shape) != (b2, h, w, F):
        raise RuntimeError("match: X (2B,H,W,3) and D (2B,H,W,F) must agree")
    b = b2 // 2
    xp, dp = X.data_ptr(), D.data_ptr()
    return _match(xp, xp + b * h * w * 3 * 4, dp, dp + b * h * w * F * 4, b, h, w, F, X.device, idx_1_to_2_init)


# Output tensors for the NEXT call of a shape, allocated right after this call's launch (while the matcher runs
# on the device) instead of on the host's critical path between a frame's result and the next frame's first
# launch. Each pair is a fresh allocation handed out once: the same tensors torch.empty would give at call time.
_SPARE = {}
_WS_BYTES = {}


def _outputs(dev, b, n, st):
    pair = _SPARE.pop((dev, b, n, st.value), None)
    if pair is None:
        pair = (torch.empty((b, n), dtype=torch.int64, device=dev), torch.empty((b, n, 1), dtype=torch.bool, device=dev))
    return pair


def _match(x11, x21, d11, d21, b, h, w, F, dev, idx_1_to_2_init):
    cfg = config["matching"]
    lib = _lib.load()
    init = 0
    if idx_1_to_2_init is not None:
        init_t = idx_1_to_2_init
        if init_t.dtype != torch.int64 or not init_t.is_contiguous():
            init_t = init_t.to(torch.int64).contiguous()
        if init_t.numel() != b * h * w:
            raise RuntimeError("match: idx_1_to_2_init must hold B*H*W indices")
        init = init_t.data_ptr()
    st = _lib.stream_ptr(dev)
    idx, valid = _outputs(dev, b, h * w, st)
    key = (b, h, w, F)
    nbytes = _WS_BYTES.get(key)
    if nbytes is None:
        nbytes = _WS_BYTES[key] = lib.m3s_match_workspace_size(b, h, w, F)
    ws = _lib.workspace("match", nbytes, dev, st)
    _lib.check(lib.m3s_match(x11, x21, d11, d21, init, idx.data_ptr(), valid.data_ptr(), b, h, w, F,
                             int(cfg["max_iter"]), float(cfg["lambda_init"]), float(cfg["convergence_thresh"]),
                             float(cfg["dist_thresh"]), int(cfg["radius"]), int(cfg["dilation_max"]), ws.data_ptr(),
                             ws.numel(), st))
    _SPARE[(dev, b, h * w, st.value)] = (torch.empty((b, h * w), dtype=torch.int64, device=dev),
                               torch.empty((b, h * w, 1), dtype=torch.bool, device=dev))
    return idx, valid
