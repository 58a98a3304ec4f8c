"""ORACLE — test infrastructure only (never imported by the product package).

Python side of the CPU oracle:

* ctypes bindings of ``liboracle_m3s.so`` (``m3s_oracle.c``: the plain-C restatement of the
  reference's CUDA kernels and BA host loop);
* numpy restatements of the reference's Python glue on the hot path:
  - ``prep_for_iter_proj``  <- ``mast3r_slam/matching.py:25-49`` + ``image.py:5-38``
  - ``match``               <- ``mast3r_slam/matching.py:8-90``
  - ``track_rays`` / ``track_calib`` <- ``mast3r_slam/tracker.py:156-266`` with
    ``geometry.py:17-123`` and ``nonlinear_optimizer.py:5-33`` (fp64 "truth" arithmetic)
  - ``Sim3`` math in fp64 (lietorch semantics, see ``lietorch_shim.py``)

Who may import this: ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

_f32p = ctypes.POINTER(ctypes.c_float)
_f64p = ctypes.POINTER(ctypes.c_double)
_u8p = ctypes.POINTER(ctypes.c_uint8)
_u16p = ctypes.POINTER(ctypes.c_uint16)
_i64p = ctypes.POINTER(ctypes.c_int64)


_LIB64 = None


def lib64():
    """The fp64 truth build of the same restatement (oracle/Makefile F64): BA only."""
    global _LIB64
    if _LIB64 is None:
        path = os.path.join(_HERE, "liboracle_m3s_f64.so")
        if not os.path.exists(path):
            import subprocess

            subprocess.check_call(["make", "-C", _HERE, "-s", "liboracle_m3s_f64.so"])
        L = ctypes.CDLL(path)
        L.m3o_gauss_newton.argtypes = (
            [ctypes.c_int, _f64p, _f64p, _f64p] + [ctypes.c_int] * 3 + [_i64p, _i64p, _i64p, _u8p, _f64p, _f64p]
            + [ctypes.c_int, ctypes.c_double, _f64p]
        )
        L.m3o_gauss_newton.restype = ctypes.c_int
        _LIB64 = L
    return _LIB64


def lib():
    """Load (building on demand) the oracle C library."""
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle_m3s.so")
        if not os.path.exists(path):
            import subprocess

            subprocess.check_call(["make", "-C", _HERE, "-s"])
        L = ctypes.CDLL(path)
        L.m3o_iter_proj.argtypes = [_f32p, _f32p, _f32p, _f32p, _u8p] + [ctypes.c_int] * 5 + [ctypes.c_float] * 2
        L.m3o_iter_proj_diag.argtypes = ([_f32p, _f32p, _f32p, _f32p, _u8p] + [ctypes.c_int] * 5 + [ctypes.c_float] * 2
                                         + [_f32p])
        L.m3o_refine_matches_f16.argtypes = [_u16p, _u16p, _i64p, _i64p] + [ctypes.c_int] * 7
        L.m3o_refine_matches_f32.argtypes = [_f32p, _f32p, _i64p, _i64p] + [ctypes.c_int] * 7
        L.m3o_f32_to_f16.argtypes = [_f32p, _u16p, ctypes.c_int64]
        L.m3o_gauss_newton.argtypes = (
            [ctypes.c_int, _f32p, _f32p, _f32p] + [ctypes.c_int] * 3 + [_i64p, _i64p, _i64p, _u8p, _f32p, _f32p]
            + [ctypes.c_int, ctypes.c_float, _f32p]
        )
        L.m3o_gauss_newton.restype = ctypes.c_int
        L.m3o_ba_linearize.argtypes = [ctypes.c_int, _f32p, _f32p, _f32p, ctypes.c_int, ctypes.c_int,
                                       _i64p, _i64p, _i64p, _u8p, _f32p, _f32p, _f64p, _f64p]
        L.m3o_pose_retr.argtypes = [_f32p, _f32p, ctypes.c_int, ctypes.c_int]
        L.m3o_exp_sim3.argtypes = [_f32p, _f32p]
        L.m3o_norm3.argtypes = [_f32p, _f32p, ctypes.c_int64]
        L.m3o_normalize3.argtypes = [_f32p, _f32p, ctypes.c_int64]
        L.m3o_img_gradient.argtypes = [_f32p, _f32p, _f32p, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.m3o_set_threads.argtypes = [ctypes.c_int]
        L.m3o_set_ref_order.argtypes = [ctypes.c_int]
        L.m3o_act_sim3.argtypes = [_f32p, _f32p, _f32p]
        L.m3o_rel_sim3.argtypes = [_f32p, _f32p, _f32p]
        _LIB = L
    return _LIB


def _p(a, t):
    return a.ctypes.data_as(t)


def _c(a, dtype):
    return np.ascontiguousarray(a, dtype=dtype)


# --------------------------------------------------------------------------------------------
# kernels (C restatement)
# --------------------------------------------------------------------------------------------
def iter_proj(rays, pts, p_init, max_iter, lambda_init, cost_thresh):
    """matching_kernels.cu:119-316 — rays (B,H,W,9), pts (B,N,3), p_init (B,N,2) -> p_new, converged."""
    rays, pts, p_init = _c(rays, np.float32), _c(pts, np.float32), _c(p_init, np.float32)
    B, H, W, C = rays.shape
    assert C == 9
    N = pts.shape[1]
    p_new = np.zeros((B, N, 2), np.float32)
    conv = np.zeros((B, N), np.uint8)
    lib().m3o_iter_proj(_p(rays, _f32p), _p(pts, _f32p), _p(p_init, _f32p), _p(p_new, _f32p), _p(conv, _u8p),
                        B, H, W, N, int(max_iter), float(lambda_init), float(cost_thresh))
    return p_new, conv.astype(bool)


def iter_proj_diag(rays, pts, p_init, max_iter, lambda_init, cost_thresh):
    """iter_proj + per-pixel rounding margins (m3s_oracle.c iter_proj_impl): (p_new, converged, diag (B,N,2)) with
    diag[..., 0] the smallest LM accept margin and diag[..., 1] the convergence-threshold margin."""
    rays, pts, p_init = _c(rays, np.float32), _c(pts, np.float32), _c(p_init, np.float32)
    B, H, W, C = rays.shape
    assert C == 9
    N = pts.shape[1]
    p_new = np.zeros((B, N, 2), np.float32)
    conv = np.zeros((B, N), np.uint8)
    diag = np.zeros((B, N, 2), np.float32)
    lib().m3o_iter_proj_diag(_p(rays, _f32p), _p(pts, _f32p), _p(p_init, _f32p), _p(p_new, _f32p), _p(conv, _u8p),
                             B, H, W, N, int(max_iter), float(lambda_init), float(cost_thresh), _p(diag, _f32p))
    return p_new, conv.astype(bool), diag


def to_half_bits(x):
    x = _c(x, np.float32)
    out = np.empty(x.shape, np.uint16)
    lib().m3o_f32_to_f16(_p(x, _f32p), _p(out, _u16p), x.size)
    return out


def refine_matches(D11, D21, p1, radius, dilation_max, half=True):
    """matching_kernels.cu:25-116. D11 (B,H,W,F), D21 (B,N,F) float arrays; half=True emulates the
    caller's ``.half()`` (matching.py:80-81) and c10::Half step rounding."""
    p1 = _c(p1, np.int64)
    B, H, W, F = D11.shape
    N = p1.shape[1]
    out = np.zeros((B, N, 2), np.int64)
    if half:
        a = D11 if D11.dtype == np.uint16 else to_half_bits(D11)
        b = D21 if D21.dtype == np.uint16 else to_half_bits(D21)
        a, b = _c(a, np.uint16), _c(b, np.uint16)
        lib().m3o_refine_matches_f16(_p(a, _u16p), _p(b, _u16p), _p(p1, _i64p), _p(out, _i64p),
                                     B, H, W, F, N, int(radius), int(dilation_max))
    else:
        a, b = _c(D11, np.float32), _c(D21, np.float32)
        lib().m3o_refine_matches_f32(_p(a, _f32p), _p(b, _f32p), _p(p1, _i64p), _p(out, _i64p),
                                     B, H, W, F, N, int(radius), int(dilation_max))
    return out


_MODES = {"points": 0, "rays": 1, "calib": 2}


def ba_params(mode, sigma_a, sigma_b=0.0, C_thresh=0.0, Q_thresh=1.5, K=None, height=0, width=0,
              pixel_border=0, z_eps=0.0):
    fx = fy = cx = cy = 0.0
    if K is not None:
        K = np.asarray(K, np.float32)
        fx, fy, cx, cy = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
    return np.array([sigma_a, sigma_b, C_thresh, Q_thresh, fx, fy, cx, cy, height, width, pixel_border, z_eps],
                    np.float32)


def set_ref_order(on):
    """BA sums in the reference's own fp32 order (256 per-thread float accumulators + the float blockReduce tree,
    gn_kernels.cu:36-55) instead of per-point fp32 products summed in fp64 (the default)."""
    lib().m3o_set_ref_order(1 if on else 0)


def set_threads(n):
    """OpenMP threads of the C restatement's parallel loops."""
    lib().m3o_set_threads(int(n))


def gauss_newton(mode, Twc, Xs, Cs, ii, jj, idx, valid, Q, params, max_iter, delta_thresh):
    """gn_kernels.cu gauss_newton_*_cuda. Returns (Twc_new, dx, iters). Twc is not modified."""
    Twc = np.array(Twc, np.float32, copy=True, order="C")
    Xs, Cs = _c(Xs, np.float32), _c(Cs, np.float32)
    K, N = Xs.shape[:2]
    ii, jj = _c(ii, np.int64), _c(jj, np.int64)
    E = ii.shape[0]
    idx = _c(idx, np.int64).reshape(E, N)
    valid = _c(valid, np.uint8).reshape(E, N)
    Q = _c(Q, np.float32).reshape(E, N)
    dx = np.zeros((max(K - 1, 0), 7), np.float32)
    its = lib().m3o_gauss_newton(_MODES[mode], _p(Twc, _f32p), _p(Xs, _f32p), _p(Cs, _f32p), K, N, E,
                                 _p(ii, _i64p), _p(jj, _i64p), _p(idx, _i64p), _p(valid, _u8p), _p(Q, _f32p),
                                 _p(_c(params, np.float32), _f32p), int(max_iter), float(delta_thresh),
                                 _p(dx, _f32p))
    if its < 0:
        raise RuntimeError("oracle gauss_newton: more unique keyframe ids than poses")
    return Twc, dx, its


def gauss_newton_f64(mode, Twc, Xs, Cs, ii, jj, idx, valid, Q, params, max_iter, delta_thresh):
    """fp64 truth of gauss_newton (every float of the restatement computed in double)."""
    Twc = np.array(Twc, np.float64, copy=True, order="C")
    Xs, Cs = _c(Xs, np.float64), _c(Cs, np.float64)
    K, N = Xs.shape[:2]
    ii, jj = _c(ii, np.int64), _c(jj, np.int64)
    E = ii.shape[0]
    idx = _c(idx, np.int64).reshape(E, N)
    valid = _c(valid, np.uint8).reshape(E, N)
    Q = _c(Q, np.float64).reshape(E, N)
    dx = np.zeros((max(K - 1, 0), 7), np.float64)
    its = lib64().m3o_gauss_newton(_MODES[mode], _p(Twc, _f64p), _p(Xs, _f64p), _p(Cs, _f64p), K, N, E,
                                   _p(ii, _i64p), _p(jj, _i64p), _p(idx, _i64p), _p(valid, _u8p), _p(Q, _f64p),
                                   _p(_c(params, np.float64), _f64p), int(max_iter), float(delta_thresh),
                                   _p(dx, _f64p))
    if its < 0:
        raise RuntimeError("oracle gauss_newton_f64: more unique keyframe ids than poses")
    return Twc, dx, its


def ba_linearize(mode, Twc, Xs, Cs, ii_rank, jj_rank, idx, valid, Q, params):
    """Per-edge Hs (4,E,7,7) / gs (2,E,7) in fp64 for dense-rank edges."""
    Twc, Xs, Cs = _c(Twc, np.float32), _c(Xs, np.float32), _c(Cs, np.float32)
    K, N = Xs.shape[:2]
    ii_rank, jj_rank = _c(ii_rank, np.int64), _c(jj_rank, np.int64)
    E = ii_rank.shape[0]
    Hs = np.zeros((4, E, 7, 7), np.float64)
    gs = np.zeros((2, E, 7), np.float64)
    lib().m3o_ba_linearize(_MODES[mode], _p(Twc, _f32p), _p(Xs, _f32p), _p(Cs, _f32p), N, E,
                           _p(ii_rank, _i64p), _p(jj_rank, _i64p), _p(_c(idx, np.int64), _i64p),
                           _p(_c(valid, np.uint8), _u8p), _p(_c(Q, np.float32), _f32p),
                           _p(_c(params, np.float32), _f32p), _p(Hs, _f64p), _p(gs, _f64p))
    return Hs, gs


def pose_retr(Twc, dx, num_fix=1):
    Twc = np.array(Twc, np.float32, copy=True, order="C")
    dx = _c(dx, np.float32)
    lib().m3o_pose_retr(_p(Twc, _f32p), _p(dx, _f32p), Twc.shape[0], num_fix)
    return Twc


def exp_sim3_f32(xi):
    xi = _c(xi, np.float32)
    out = np.zeros(8, np.float32)
    lib().m3o_exp_sim3(_p(xi, _f32p), _p(out, _f32p))
    return out


# --------------------------------------------------------------------------------------------
# glue (numpy restatement)
# --------------------------------------------------------------------------------------------
def norm3(x):
    """torch.linalg.vector_norm(x, dim=-1) of fp32 3-vectors on torch's CPU: sqrt(fma(z, z, fma(y, y, x * x))) in fp32
    (m3s_oracle.c m3o_norm3; bit-exact against the reference run's golden vectors)."""
    x = _c(x, np.float32)
    out = np.empty(x.shape[:-1], np.float32)
    lib().m3o_norm3(_p(x, _f32p), _p(out, _f32p), out.size)
    return out


def normalize(x, eps=1e-12):
    """torch.nn.functional.normalize(x, dim=-1) of fp32 3-vectors: x / max(norm3(x), eps) in fp32."""
    assert eps == 1e-12
    x = _c(x, np.float32)
    out = np.empty_like(x)
    lib().m3o_normalize3(_p(x, _f32p), _p(out, _f32p), x.size // 3)
    return out


def img_gradient(img):
    """image.py:5-38 on (B,H,W,3): Scharr-like 3x3 / 32, reflect pad 1, depthwise, in the reference's fp32 order
    (m3s_oracle.c m3o_img_gradient: row-major FMA chain over the 9 taps)."""
    img = _c(img, np.float32)
    B, H, W, C = img.shape
    assert C == 3
    gx, gy = np.empty_like(img), np.empty_like(img)
    lib().m3o_img_gradient(_p(img, _f32p), _p(gx, _f32p), _p(gy, _f32p), B, H, W)
    return gx, gy


def lin_to_pixel(idx, w):
    return np.stack((idx % w, idx // w), axis=-1)


def pixel_to_lin(p, w):
    return p[..., 0] + w * p[..., 1]


def prep_for_iter_proj(X11, X21, idx_init=None):
    """matching.py:25-49."""
    b, h, w, _ = X11.shape
    rays = normalize(X11.astype(np.float32))
    gx, gy = img_gradient(rays)
    rays_with_grad = np.concatenate((rays, gx, gy), axis=-1)
    pts = normalize(X21.reshape(b, -1, 3).astype(np.float32))
    if idx_init is None:
        idx_init = np.tile(np.arange(h * w)[None], (b, 1))
    p_init = lin_to_pixel(np.asarray(idx_init), w).astype(np.float32)
    return rays_with_grad, pts, p_init


def match(X11, X21, D11, D21, idx_init=None, max_iter=10, lambda_init=1e-8, convergence_thresh=1e-6,
          dist_thresh=0.1, radius=3, dilation_max=5):
    """matching.py:52-90 (config/base.yaml:8-14 defaults). Returns idx (B,N) int64, valid (B,N,1)."""
    b, h, w = X21.shape[:3]
    rays, pts, p_init = prep_for_iter_proj(X11, X21, idx_init)
    p_new, conv = iter_proj(rays, pts, p_init, max_iter, lambda_init, convergence_thresh)
    p1 = p_new.astype(np.int64)  # .long() truncation
    Xg = X11[np.arange(b)[:, None], p1[..., 1], p1[..., 0], :].reshape(b, h, w, 3)
    d = norm3(Xg.astype(np.float32) - X21.astype(np.float32))  # torch.linalg.norm(..., dim=-1) in fp32
    valid = conv & (d < np.float32(dist_thresh)).reshape(b, -1)
    if radius > 0:
        p1 = refine_matches(D11, D21.reshape(b, h * w, -1), p1, radius, dilation_max)
    return pixel_to_lin(p1, w), valid[..., None]


def match_diag(X11, X21, D11, D21, idx_init=None, max_iter=10, lambda_init=1e-8, convergence_thresh=1e-6,
               dist_thresh=0.1, radius=3, dilation_max=5):
    """``match`` with its intermediates, for the fused match's mismatch census (tests/test_gpu_configs.py): a dict
    of idx, valid (the outputs of ``match``), p_new (B,N,2) float, p1 (B,N) linear truncated index before the refine,
    conv, the occlusion distance d (B,N) and the LM margins of ``iter_proj_diag``."""
    b, h, w = X21.shape[:3]
    rays, pts, p_init = prep_for_iter_proj(X11, X21, idx_init)
    p_new, conv, diag = iter_proj_diag(rays, pts, p_init, max_iter, lambda_init, convergence_thresh)
    p1 = p_new.astype(np.int64)
    Xg = X11[np.arange(b)[:, None], p1[..., 1], p1[..., 0], :].reshape(b, h, w, 3)
    d = norm3(Xg.astype(np.float32) - X21.astype(np.float32)).reshape(b, -1)
    valid = conv & (d < np.float32(dist_thresh))
    p1r = refine_matches(D11, D21.reshape(b, h * w, -1), p1, radius, dilation_max) if radius > 0 else p1
    return {"idx": pixel_to_lin(p1r, w), "valid": valid[..., None], "p_new": p_new, "p1": pixel_to_lin(p1, w),
            "conv": conv, "d": d, "accept_margin": diag[..., 0], "conv_margin": diag[..., 1]}


# ---- Sim3 fp64 (lietorch semantics) ----
def _qmul(a, b):
    ax, ay, az, aw = a
    bx, by, bz, bw = b
    return np.array([aw * bx + ax * bw + ay * bz - az * by, aw * by - ax * bz + ay * bw + az * bx,
                     aw * bz + ax * by - ay * bx + az * bw, aw * bw - ax * bx - ay * by - az * bz])


def _qrot(q, p):
    qv, w = q[:3], q[3]
    uv = 2.0 * np.cross(np.broadcast_to(qv, p.shape), p)
    return p + w * uv + np.cross(np.broadcast_to(qv, p.shape), uv)


def sim3_mul(a, b):
    q = _qmul(a[3:7], b[3:7])
    q = q / np.linalg.norm(q)
    t = a[:3] + a[7] * _qrot(a[3:7], b[:3])
    return np.concatenate((t, q, [a[7] * b[7]]))


def sim3_inv(a):
    qi = a[3:7] * np.array([-1, -1, -1, 1.0])
    si = 1.0 / a[7]
    return np.concatenate((-si * _qrot(qi, a[:3]), qi, [si]))


def sim3_act(a, p):
    return a[7] * _qrot(a[3:7], p) + a[:3]


def sim3_exp(xi):
    tau, phi, sigma = np.asarray(xi[:3], np.float64), np.asarray(xi[3:6], np.float64), float(xi[6])
    th2 = float(phi @ phi)
    th = np.sqrt(th2)
    if th2 < 1e-6:
        imag = 0.5 - th2 / 48.0 + th2 * th2 / 3840.0
        real = 1.0 - th2 / 8.0 + th2 * th2 / 384.0
    else:
        imag, real = np.sin(0.5 * th) / th, np.cos(0.5 * th)
    q = np.concatenate((imag * phi, [real]))
    S = np.exp(sigma)
    if abs(sigma) < 1e-6:
        C = 1.0
        if th < 1e-6:
            A, B = 0.5, 1.0 / 6.0
        else:
            A, B = (1 - np.cos(th)) / th2, (th - np.sin(th)) / (th2 * th)
    else:
        C = (S - 1.0) / sigma
        if th < 1e-6:
            s2 = sigma * sigma
            A = ((sigma - 1) * S + 1) / s2
            B = (S * 0.5 * s2 + S - 1 - sigma * S) / (s2 * sigma)
        else:
            a, b = S * np.sin(th), S * np.cos(th)
            c = th2 + sigma * sigma
            A = (a * sigma + (1 - b) * th) / (th * c)
            B = (C - ((b - 1) * sigma + a * th) / c) / th2
    pxt = np.cross(phi, tau)
    t = C * tau + A * pxt + B * np.cross(phi, pxt)
    return np.concatenate((t, q, [S]))


def sim3_retr(a, xi):
    return sim3_mul(sim3_exp(xi), a)


def _huber_w(r, k):
    ra = np.abs(r)
    return np.where(ra < k, 1.0, k / np.maximum(ra, 1e-300))


def _solve(sqrt_info, r, J, k):
    """tracker.py:156-171 in fp64."""
    robust = sqrt_info * np.sqrt(_huber_w(sqrt_info * r, k))
    A = (robust[..., None] * J).reshape(-1, 7)
    b = (robust * r).reshape(-1, 1)
    H = A.T @ A
    g = -A.T @ b
    cost = 0.5 * float((b.T @ b)[0, 0])
    L = np.linalg.cholesky(H)
    tau = np.linalg.solve(L.T, np.linalg.solve(L, g)).reshape(-1)
    return tau, cost


def _act_jac(T, X):
    Y = sim3_act(T, X)
    n = X.shape[0]
    J = np.zeros((n, 3, 7))
    J[:, 0, 0] = J[:, 1, 1] = J[:, 2, 2] = 1.0
    x, y, z = Y[:, 0], Y[:, 1], Y[:, 2]
    # -skew(Y) columns 3..5
    J[:, 0, 4], J[:, 0, 5] = z, -y
    J[:, 1, 3], J[:, 1, 5] = -z, x
    J[:, 2, 3], J[:, 2, 4] = y, -x
    J[:, :, 6] = Y
    return Y, J


def track_rays(Xf, Xk, T_WCf, T_WCk, Qk, valid, sigma_ray=0.003, sigma_dist=10.0, huber_k=1.345,
               max_iters=50, rel_error=1e-3, delta_norm=1e-3, fixed_iters=None):
    """tracker.py:173-214 (opt_pose_ray_dist_sim3) in fp64. Returns (T_WCf, T_CkCf, iters)."""
    Xf, Xk = Xf.astype(np.float64), Xk.astype(np.float64)
    v = valid.reshape(-1, 1).astype(np.float64)
    sq = np.sqrt(Qk.reshape(-1, 1).astype(np.float64))
    sqrt_info = np.concatenate((np.repeat(v * sq / sigma_ray, 3, 1), v * sq / sigma_dist), 1)
    T = sim3_mul(sim3_inv(np.asarray(T_WCk, np.float64)), np.asarray(T_WCf, np.float64))
    dk = np.linalg.norm(Xk, axis=-1, keepdims=True)
    rd_k = np.concatenate((Xk / dk, dk), -1)
    old = np.inf
    iters = max_iters if fixed_iters is None else fixed_iters
    it = 0
    for step in range(iters):
        Y, dY = _act_jac(T, Xf)
        d = np.linalg.norm(Y, axis=-1, keepdims=True)
        r_ = Y / d
        rd = np.concatenate((r_, d), -1)
        I = np.eye(3)[None]
        dr = (1.0 / d)[..., None] * (I - (1.0 / d ** 2)[..., None] * (Y[:, :, None] * Y[:, None, :]))
        drd = np.concatenate((dr, r_[:, None, :]), 1)
        r = rd_k - rd
        J = -drd @ dY
        tau, cost = _solve(sqrt_info, r, J, huber_k)
        T = sim3_retr(T, tau)
        it = step + 1
        if fixed_iters is None:
            rel = abs((old - cost) / old) if np.isfinite(old) else np.nan
            if rel < rel_error or np.linalg.norm(tau) < delta_norm:
                break
        old = cost
    return sim3_mul(np.asarray(T_WCk, np.float64), T), T, it


def track_calib(Xf, Xk, T_WCf, T_WCk, Qk, valid, meas_k, valid_meas_k, K, img_size, sigma_pixel=1.0,
                sigma_depth=10.0, huber_k=1.345, pixel_border=-10, depth_eps=1e-6, max_iters=50,
                rel_error=1e-3, delta_norm=1e-3, fixed_iters=None):
    """tracker.py:216-266 (opt_pose_calib_sim3) + geometry.project_calib in fp64."""
    Xf = Xf.astype(np.float64)
    v = valid.reshape(-1, 1).astype(np.float64)
    sq = np.sqrt(Qk.reshape(-1, 1).astype(np.float64))
    sqrt_info = np.concatenate((np.repeat(v * sq / sigma_pixel, 2, 1), v * sq / sigma_depth), 1)
    K = np.asarray(K, np.float64)
    fx, fy, cx, cy = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
    h, w = img_size
    T = sim3_mul(sim3_inv(np.asarray(T_WCk, np.float64)), np.asarray(T_WCf, np.float64))
    meas_k = meas_k.astype(np.float64)
    vm = valid_meas_k.reshape(-1, 1)
    old = np.inf
    iters = max_iters if fixed_iters is None else fixed_iters
    it = 0
    for step in range(iters):
        Y, dY = _act_jac(T, Xf)
        x, y, z = Y[:, 0:1], Y[:, 1:2], Y[:, 2:3]
        with np.errstate(divide="ignore", invalid="ignore"):
            u = fx * x / z + cx
            vv = fy * y / z + cy
            valid_z = z > depth_eps
            logz = np.where(valid_z, np.log(np.where(valid_z, z, 1.0)), 0.0)
            zi = 1.0 / z[:, 0]
        valid_p = (u > pixel_border) & (u < w - 1 - pixel_border) & (vv > pixel_border) & (vv < h - 1 - pixel_border) & valid_z
        pz = np.concatenate((u, vv, logz), -1)
        dpz = np.zeros((Y.shape[0], 3, 3))
        dpz[:, 0, 0] = fx * zi
        dpz[:, 1, 1] = fy * zi
        dpz[:, 0, 2] = -fx * x[:, 0] * zi * zi
        dpz[:, 1, 2] = -fy * y[:, 0] * zi * zi
        dpz[:, 2, 2] = zi
        si2 = (valid_p & vm) * sqrt_info
        r = meas_k - pz
        J = -dpz @ dY
        tau, cost = _solve(si2, r, J, huber_k)
        T = sim3_retr(T, tau)
        it = step + 1
        if fixed_iters is None:
            rel = abs((old - cost) / old) if np.isfinite(old) else np.nan
            if rel < rel_error or np.linalg.norm(tau) < delta_norm:
                break
        old = cost
    return sim3_mul(np.asarray(T_WCk, np.float64), T), T, it


def backproject_constrain(X, K, img_size):
    """geometry.constrain_points_to_ray: X (..., H*W, 3) -> points on pixel rays with X's depth."""
    h, w = img_size
    K = np.asarray(K, np.float32)
    u, v = np.meshgrid(np.arange(w, dtype=np.float32), np.arange(h, dtype=np.float32), indexing="xy")
    t1 = ((u.reshape(-1) - K[0, 2]) / K[0, 0]).astype(np.float32)
    t2 = ((v.reshape(-1) - K[1, 2]) / K[1, 1]).astype(np.float32)
    z = X[..., 2]
    return np.stack((z * t1, z * t2, z * 1.0), -1).astype(np.float32)


# ---------------------------------------------------------------- retrieval quantization
def quantize_custom(centroids, qvecs, k, dtype=np.float64):
    """``RetrievalDatabase.quantize_custom`` (``mast3r_slam/retrieval_database.py:96-105``) in numpy:
    l2 = (|q|^2 + |c|^2) - 2 q c^T in ``dtype`` (fp64 = the truth the tests measure against), the k
    smallest per row in ascending order (ties -> lower index). Returns (indices int64 (M, k), l2)."""
    c = np.asarray(centroids, dtype=dtype)
    q = np.asarray(qvecs, dtype=dtype)
    l2 = (np.sum(q * q, axis=1)[:, None] + np.sum(c * c, axis=1)[None, :]) - 2.0 * (q @ c.T)
    part = np.argpartition(l2, k - 1, axis=1)[:, :k] if k < l2.shape[1] else np.tile(np.arange(l2.shape[1]), (len(l2), 1))
    rows = np.arange(len(l2))[:, None]
    order = np.lexsort((part, l2[rows, part]), axis=1)
    return part[rows, order].astype(np.int64), l2


def topk_equivalent(got, ref, l2, tol):
    """True where ``got`` and ``ref`` pick the same index at each rank, or indices whose fp64 distances
    differ by at most ``tol`` (a near-tie that any fp32-rounded GEMM may order either way)."""
    rows = np.arange(len(l2))[:, None]
    return (got == ref) | (np.abs(l2[rows, got] - l2[rows, ref]) <= tol)
