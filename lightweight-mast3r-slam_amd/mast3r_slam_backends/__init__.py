"""Drop-in replacement for the reference's native extension ``mast3r_slam_backends``.

Same module name, same five functions, same argument order, dtypes, return lists, in-place
``Twc`` semantics and contiguity errors as
``/root/reference/mast3r_slam/backend/src/gn.cpp:116-123`` (declarations ``backend/include/gn.h``).
Behind each function is the C ABI of ``libm3s.so`` (``include/m3s.h``) running hand-written HIP
kernels for gfx950. There is no CPU path: non-HIP tensors raise ``RuntimeError``.

Differences that a caller can observe (all stricter, none looser):
  * dtype / shape errors raise ``RuntimeError`` (the reference has only contiguity checks, gn.h:5);
  * kernels run on torch's *current* stream instead of the legacy default stream;
  * ``iter_proj`` / ``refine_matches`` guard ``n < N`` (the reference reads out of bounds when N is
    not a multiple of 16, matching_kernels.cu:36,131).
"""
import ctypes

import torch

from m3s import _lib

__all__ = ["iter_proj", "refine_matches", "gauss_newton_points", "gauss_newton_rays", "gauss_newton_calib"]


def _contig(name, **tensors):
    for k, t in tensors.items():
        if not t.is_contiguous():
            raise RuntimeError(f"{k} must be contiguous")  # gn.h:5 CHECK_CONTIGUOUS message


def _dtype(name, t, dt, what):
    if t.dtype != dt:
        raise RuntimeError(f"{name}: {what} must be {dt}, got {t.dtype}")


def iter_proj(rays_img_with_grad, pts_3d_norm, p_init, max_iter, lambda_init, cost_thresh):
    """gn.cpp:84-99 -> [p_new (B,N,2) f32, converged (B,N) bool]."""
    _contig("iter_proj", rays_img_with_grad=rays_img_with_grad, pts_3d_norm=pts_3d_norm, p_init=p_init)
    lib = _lib.load()
    _lib.require_cuda("iter_proj", rays_img_with_grad, pts_3d_norm, p_init)
    for t, w in ((rays_img_with_grad, "rays_img_with_grad"), (pts_3d_norm, "pts_3d_norm"), (p_init, "p_init")):
        _dtype("iter_proj", t, torch.float32, w)
    if rays_img_with_grad.dim() != 4 or pts_3d_norm.dim() != 3 or p_init.dim() != 3:
        raise RuntimeError("iter_proj: expected rays (B,H,W,9), pts (B,N,3), p_init (B,N,2)")
    B, H, W, C = rays_img_with_grad.shape
    Bp, N, two = p_init.shape
    if Bp != B or two != 2 or pts_3d_norm.shape[0] != B or pts_3d_norm.shape[1] != N or pts_3d_norm.shape[2] != 3:
        raise RuntimeError("iter_proj: inconsistent batch / point dimensions")
    p_new = torch.zeros((B, N, 2), dtype=torch.float32, device=p_init.device)
    conv = torch.zeros((B, N), dtype=torch.bool, device=p_init.device)
    _lib.check(lib.m3s_iter_proj(_lib.ptr(rays_img_with_grad), _lib.ptr(pts_3d_norm), _lib.ptr(p_init),
                                 _lib.ptr(p_new), _lib.ptr(conv), B, H, W, C, N, int(max_iter),
                                 float(lambda_init), float(cost_thresh), _lib.stream_ptr(p_init.device)))
    return [p_new, conv]


def refine_matches(D11, D21, p1, radius, dilation_max):
    """gn.cpp:101-114 -> [p1_new (B,N,2) i64]. f16 inputs use c10::Half step rounding."""
    _contig("refine_matches", D11=D11, D21=D21, p1=p1)
    lib = _lib.load()
    _lib.require_cuda("refine_matches", D11, D21, p1)
    if D11.dtype != D21.dtype or D11.dtype not in (torch.float16, torch.float32):
        raise RuntimeError("refine_matches: D11/D21 must both be float16 or float32")
    _dtype("refine_matches", p1, torch.int64, "p1")
    if D11.dim() != 4 or D21.dim() != 3 or p1.dim() != 3:
        raise RuntimeError("refine_matches: expected D11 (B,H,W,F), D21 (B,N,F), p1 (B,N,2)")
    B, H, W, F = D11.shape
    N = p1.shape[1]
    if D21.shape[0] != B or D21.shape[1] != N or D21.shape[2] != F or p1.shape[0] != B or p1.shape[2] != 2:
        raise RuntimeError("refine_matches: inconsistent shapes")
    out = torch.zeros((B, N, 2), dtype=torch.int64, device=p1.device)
    dt = 0 if D11.dtype == torch.float16 else 1
    _lib.check(lib.m3s_refine_matches(dt, _lib.ptr(D11), _lib.ptr(D21), _lib.ptr(p1), _lib.ptr(out), B, H, W, F, N,
                                      int(radius), int(dilation_max), _lib.stream_ptr(p1.device)))
    return [out]


def _gauss_newton(mode, Twc, Xs, Cs, ii, jj, idx_ii2jj, valid_match, Q, cfg, max_iter, delta_thresh, K=None):
    tensors = dict(Twc=Twc, Xs=Xs, Cs=Cs, ii=ii, jj=jj, idx_ii2jj=idx_ii2jj, valid_match=valid_match, Q=Q)
    if K is not None:
        tensors["K"] = K
    _contig("gauss_newton", **tensors)
    lib = _lib.load()
    _lib.require_cuda("gauss_newton", *tensors.values())
    for name, dt in (("Twc", torch.float32), ("Xs", torch.float32), ("Cs", torch.float32), ("ii", torch.int64),
                     ("jj", torch.int64), ("idx_ii2jj", torch.int64), ("Q", torch.float32)):
        _dtype("gauss_newton", tensors[name], dt, name)
    if valid_match.dtype not in (torch.bool, torch.uint8):
        raise RuntimeError("gauss_newton: valid_match must be bool")
    if Twc.dim() != 2 or Twc.shape[1] != 8:
        raise RuntimeError("gauss_newton: Twc must be (K,8)")
    Kp, N = Xs.shape[0], Xs.shape[1]
    E = ii.shape[0]
    if Xs.shape[2] != 3 or Cs.numel() != Kp * N or Twc.shape[0] != Kp:
        raise RuntimeError("gauss_newton: Xs (K,N,3), Cs (K,N,1), Twc (K,8) disagree")
    if jj.shape[0] != E or idx_ii2jj.numel() != E * N or valid_match.numel() != E * N or Q.numel() != E * N:
        raise RuntimeError("gauss_newton: edge tensors disagree with ii (E,) x N")
    dev = Twc.device
    dx = torch.zeros((max(Kp - 1, 0), 7), dtype=torch.float32, device=dev)
    nbytes = lib.m3s_ba_workspace_size(Kp, N, E)
    st = _lib.stream_ptr(dev)
    ws = _lib.workspace("ba", nbytes, dev, st)
    _lib.check(lib.m3s_gauss_newton(ctypes.byref(cfg), _lib.ptr(Twc), _lib.ptr(Xs), _lib.ptr(Cs), Kp, N,
                                    _lib.ptr(ii), _lib.ptr(jj), E, _lib.ptr(idx_ii2jj), _lib.ptr(valid_match),
                                    _lib.ptr(Q), int(max_iter), float(delta_thresh), _lib.ptr(dx), None,
                                    _lib.ptr(ws), ws.numel(), st))
    return [dx]


def gauss_newton_points(Twc, Xs, Cs, ii, jj, idx_ii2jj, valid_match, Q, sigma_point, C_thresh, Q_thresh, max_iter,
                        delta_thresh):
    """gn.cpp:3-26 (point_align_kernel). Mutates Twc in place; returns [dx]."""
    cfg = _lib.BaConfig(mode=0, sigma_a=sigma_point, sigma_b=0.0, C_thresh=C_thresh, Q_thresh=Q_thresh)
    return _gauss_newton(0, Twc, Xs, Cs, ii, jj, idx_ii2jj, valid_match, Q, cfg, max_iter, delta_thresh)


def gauss_newton_rays(Twc, Xs, Cs, ii, jj, idx_ii2jj, valid_match, Q, sigma_ray, sigma_dist, C_thresh, Q_thresh,
                      max_iter, delta_thresh):
    """gn.cpp:28-52 (ray_align_kernel). Mutates Twc in place; returns [dx]."""
    cfg = _lib.BaConfig(mode=1, sigma_a=sigma_ray, sigma_b=sigma_dist, C_thresh=C_thresh, Q_thresh=Q_thresh)
    return _gauss_newton(1, Twc, Xs, Cs, ii, jj, idx_ii2jj, valid_match, Q, cfg, max_iter, delta_thresh)


def gauss_newton_calib(Twc, Xs, Cs, K, ii, jj, idx_ii2jj, valid_match, Q, height, width, pixel_border, z_eps,
                       sigma_pixel, sigma_depth, C_thresh, Q_thresh, max_iter, delta_thresh):
    """gn.cpp:54-82 (calib_proj_kernel). Mutates Twc in place; returns [dx]."""
    Kh = K.detach().float().cpu()
    cfg = _lib.BaConfig(mode=2, sigma_a=sigma_pixel, sigma_b=sigma_depth, C_thresh=C_thresh, Q_thresh=Q_thresh,
                        fx=float(Kh[0, 0]), fy=float(Kh[1, 1]), cx=float(Kh[0, 2]), cy=float(Kh[1, 2]),
                        height=int(height), width=int(width), pixel_border=int(pixel_border), z_eps=float(z_eps))
    return _gauss_newton(2, Twc, Xs, Cs, ii, jj, idx_ii2jj, valid_match, Q, cfg, max_iter, delta_thresh, K=K)
