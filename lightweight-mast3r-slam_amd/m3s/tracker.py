"""``FrameTracker`` with the reference surface (``/root/reference/mast3r_slam/tracker.py:15-266``).

``track(frame) -> (new_kf, match_info, try_reloc)`` keeps the reference's return triple and failure
behaviour (low match fraction or Cholesky failure -> ``(False, [], True)``). The post-matching work
— confidence / validity setup, the Sim(3) Gauss-Newton loop to convergence, the keyframe pointmap
fusion and the keyframe-selection statistics — is ONE C-ABI call (``m3s_track``): 2 + 2*iters HIP
kernels and a single host readback per frame, instead of ~30 torch launches and a ``.item()`` sync
per GN iteration.

``opt_pose_ray_dist_sim3`` / ``opt_pose_calib_sim3`` keep their reference signatures and run the
same HIP GN kernels in "direct" mode; ``solve`` is the generic whitened normal-equation step of
``tracker.py:156-171`` (torch ops on the device, not on the fused path).
"""
import ctypes

import torch

from m3s import _lib
from m3s.config import config
from m3s.frame import Frame, slot_frame, slot_rows
from m3s.matching import match, match_halves
from m3s.sim3 import Sim3


def huber(r, k=1.345):
    """nonlinear_optimizer.py:28-33."""
    unit = torch.ones((1), dtype=r.dtype, device=r.device)
    r_abs = torch.abs(r)
    return torch.where(r_abs < k, unit, k / r_abs)


def asymmetric_inference(model, frame_i, frame_j):
    """X, C, D, Q (2b,H,W,·) of the pair. Models with ``asymmetric_inference`` (synthetic / replayed
    pointmaps) answer directly; the real AsymmetricMASt3R goes through the reference's own ViT helper
    (``mast3r_utils.py:190-217``, stock PyTorch-ROCm, outside this package's scope)."""
    fn = getattr(model, "asymmetric_inference", None)
    if fn is not None:
        return fn(frame_i, frame_j)
    from mast3r_slam.mast3r_utils import mast3r_asymmetric_inference

    return mast3r_asymmetric_inference(model, frame_i, frame_j)


def mast3r_match_asymmetric(model, frame_i, frame_j, idx_i2j_init=None):
    """mast3r_utils.py:220-242 with the ViT call behind ``model.asymmetric_inference`` (stock
    PyTorch-ROCm, out of scope); returns idx_i2j, valid_match_j, Xii, Cii, Qii, Xji, Cji, Qji."""
    X, C, D, Q = asymmetric_inference(model, frame_i, frame_j)
    b = X.shape[0] // 2
    h, w = X.shape[1:3]
    idx_i2j, valid_match_j = match_halves(X, D, idx_1_to_2_init=idx_i2j_init)  # match(X[:b], X[b:], D[:b], D[b:])
    Xr = X.reshape(2 * b, h * w, 3)
    Cr = C.reshape(2 * b, h * w, 1)
    Qr = Q.reshape(2 * b, h * w, 1)
    return idx_i2j, valid_match_j, Xr[0], Cr[0], Qr[0], Xr[1], Cr[1], Qr[1]


_K_CACHE = {}


def _host_K(K):
    """Host copy of the intrinsics, cached per live tensor and version: a device->host read every frame would
    serialise the host against the matcher kernels still in flight. The entry holds a weak reference to the
    tensor it was read from, so a new tensor that reuses a freed one's address (or Python id) never hits."""
    import weakref

    e = _K_CACHE.get(id(K))
    if e is not None and e[0]() is K and e[1] == K._version and e[2] == K.data_ptr():
        return e[3]
    Kh = K.detach().float().cpu().reshape(-1).tolist()
    if len(_K_CACHE) > 64:
        _K_CACHE.clear()
    _K_CACHE[id(K)] = (weakref.ref(K), K._version, K.data_ptr(), Kh)
    return Kh


def _as(t, dt=torch.float32):
    """t as a contiguous dt tensor, without a dispatcher round trip when it already is one."""
    if t is None or (t.dtype == dt and t.is_contiguous()):
        return t
    return t.to(dt).contiguous()


def _dp(t):
    return 0 if t is None else t.data_ptr()


def frame_img_size(frame):
    """(H, W): ``frame.img.shape[-2:]`` for a reference Frame (tracker.py:47), ``img_size`` for m3s.frame."""
    size = getattr(frame, "img_size", None)
    if size is None:
        size = frame.img.shape[-2:]
    return tuple(int(x) for x in size)


def _track_config(cfg, use_calib, img_size, K):
    tc = _lib.TrackConfig()
    tc.mode = 1 if use_calib else 0
    tc.max_iters = int(cfg["max_iters"])
    tc.C_conf, tc.Q_conf, tc.min_match_frac = float(cfg["C_conf"]), float(cfg["Q_conf"]), float(cfg["min_match_frac"])
    if use_calib:
        tc.sigma_a, tc.sigma_b = float(cfg["sigma_pixel"]), float(cfg["sigma_depth"])
        Kh = _host_K(K)
        for i in range(9):
            tc.K[i] = Kh[i]
    else:
        tc.sigma_a, tc.sigma_b = float(cfg["sigma_ray"]), float(cfg["sigma_dist"])
    tc.huber_k, tc.rel_error, tc.delta_norm = float(cfg["huber"]), float(cfg["rel_error"]), float(cfg["delta_norm"])
    tc.pixel_border, tc.depth_eps = float(cfg["pixel_border"]), float(cfg["depth_eps"])
    tc.H, tc.W = int(img_size[0]), int(img_size[1])
    return tc


class FrameTracker:
    def __init__(self, model, frames, device):
        self.cfg = config["tracking"]
        self.model = model
        self.keyframes = frames
        self.device = device
        self.first_chunk = 8  # GN iterations enqueued before the first host readback
        self.last_result = None
        # fuse straight into a buffer-backed store's slot (SharedKeyframes) instead of tracker.py:101's full-record
        # copy; False: the reference's copy (A/B tests and the bench's comparison leg)
        self.slot_writeback = True
        self.reset_idx_f2k()

    def reset_idx_f2k(self):
        self.idx_f2k = None

    def _config(self, use_calib, img_size, K, max_iters):
        """m3s_track_config, rebuilt only when the inputs that shape it change."""
        cfg = self.cfg
        kkey = None if (K is None or not use_calib) else tuple(_host_K(K))  # the values (a freed K's address can recur)
        key = (use_calib, tuple(img_size), kkey, max_iters, tuple(cfg.items()))
        if getattr(self, "_cfg_key", None) != key:
            c = dict(cfg)
            if max_iters is not None:
                c["max_iters"] = max_iters
            self._cfg_struct = _track_config(c, use_calib, img_size, K)
            self._cfg_key = key
        return self._cfg_struct

    # ------------------------------------------------------------------ fused track
    def track(self, frame):
        """tracker.py:28-127."""
        keyframe, kf_slot = self._last_keyframe()
        idx_f2k, valid_match_k, Xff, Cff, Qff, Xkf, Ckf, Qkf = mast3r_match_asymmetric(
            self.model, frame, keyframe, idx_i2j_init=self.idx_f2k)
        # tracker.py:45 clones; the fused matcher returns a fresh tensor that nothing writes to, so the
        # warm-start reference keeps it without a copy
        self.idx_f2k = idx_f2k
        idx_f2k = idx_f2k[0]
        valid_match_k = valid_match_k[0]
        if isinstance(frame, Frame):
            frame.update_pointmap(Xff, Cff, own=True)  # fresh model outputs: no clone (frame.py:41-45 clones)
        else:  # the reference's Frame (m3s/hook.py): its own update_pointmap
            frame.update_pointmap(Xff, Cff)

        use_calib = config["use_calib"]
        img_size = frame_img_size(frame)
        K = keyframe.K if use_calib else None
        cfg = self.cfg
        # weighted_pointmap on an initialised keyframe is fused on the device (frame.py:74-77); every
        # other filtering mode / an empty keyframe goes through keyframe.update_pointmap
        fuse_fused = cfg["filtering_mode"] == "weighted_pointmap" and keyframe.N > 0
        # SharedKeyframes (frame.py:220-289): the fusion kernel writes X / C and the slot's N, N_updates, is_dirty
        # into the slot itself; the rest of the record (img, uimg, feat, pos, T_WC) is what the slot already holds
        slot = None
        if fuse_fused and self.slot_writeback:
            slot = slot_rows(self.keyframes, keyframe, kf_slot)

        res, T_f, T_r = self._run_track(
            idx=idx_f2k, valid=valid_match_k, Xf=frame.X_canon, Cf=frame.C, Nf=frame.N, Qff=Qff,
            Xk=keyframe.X_canon, Ck=keyframe.C, Nk=keyframe.N, Qkf=Qkf, T_WCf=frame.T_WC, T_WCk=keyframe.T_WC,
            use_calib=use_calib, img_size=img_size, K=K,
            fuse=(keyframe, Xkf, Ckf, slot) if fuse_fused else None)

        if res.status == _lib.TRACK_SKIPPED:
            print(f"Skipped frame {frame.frame_id}")
            return False, [], True
        if res.status == _lib.TRACK_CHOLESKY_FAILED:
            print(f"Cholesky failed {frame.frame_id}")
            return False, [], True

        # fresh (1, 8) views of this call's output, made before the launch: no copy, no op after the wait
        frame.T_WC = Sim3(T_f)
        T_CkCf = Sim3(T_r)
        if fuse_fused:  # X/C fused on the device by m3s_track (frame.py:74-77): new tensors, or the slot in place
            keyframe.X_canon, keyframe.C = self._fused
            keyframe.N += 1
            keyframe.N_updates += 1
        else:
            keyframe.update_pointmap(T_CkCf.act(Xkf), Ckf)
        if slot is None:  # write back the filtered pointmap (tracker.py:101)
            self.keyframes[kf_slot] = keyframe

        n = res.N
        match_frac_k = res.n_valid_kf / n
        unique_frac_f = res.n_unique / n
        new_kf = min(match_frac_k, unique_frac_f) < cfg["match_frac_thresh"]
        if new_kf:
            self.reset_idx_f2k()
        if fuse_fused:  # C / N of both frames, written by the fuse kernel (frame.py:83-84)
            Ck_avg, Cf_avg = self._avg
        else:
            Ck_avg, Cf_avg = keyframe.get_average_conf(), frame.get_average_conf()
        return (new_kf, [keyframe.X_canon, Ck_avg, frame.X_canon, Cf_avg, Qkf, Qff], False)

    def _last_keyframe(self):
        """(keyframes.last_keyframe(), its slot index) with one store round trip: tracker.py:29 reads the last
        keyframe and tracker.py:101 writes it back at len(keyframes) - 1. Only the frontend appends keyframes
        (main.py), so the index read with the keyframe is the one len() would return at the write-back. A
        lock-guarded store (the reference's SharedKeyframes, frame.py:220-327: every Manager lock and Value access
        is an IPC) is read under one lock hold: n_size once, then the slot, instead of last_keyframe()'s two n_size
        reads plus a separate len(); a buffer-backed slot is read inside that hold (slot_frame: no nested lock, one
        D2H copy for its three scalars instead of three)."""
        kfs = self.keyframes
        lock, n_size = getattr(kfs, "lock", None), getattr(kfs, "n_size", None)
        if lock is not None and n_size is not None and hasattr(n_size, "value"):
            with lock:
                n = n_size.value
                if n <= 0:
                    return None, -1
                kf = slot_frame(kfs, n - 1)
                return (kfs[n - 1] if kf is None else kf), n - 1
        n = len(kfs)
        return (kfs[n - 1], n - 1) if n > 0 else (None, -1)

    def _run_track(self, idx, valid, Xf, Cf, Nf, Qff, Xk, Ck, Nk, Qkf, T_WCf, T_WCk, use_calib, img_size, K,
                   fuse=None, direct=False, meas_k=None, valid_meas_k=None, max_iters=None):
        lib = _lib.load()
        dev = Xf.device
        _lib.require_cuda("track", Xf, Xk, Qff, valid)
        tc = self._config(use_calib, img_size, K, max_iters)
        N = tc.H * tc.W
        c = _as
        Xf, Xk, Qff, Qkf, Cf, Ck = c(Xf), c(Xk), c(Qff), c(Qkf), c(Cf), c(Ck)
        idx = c(idx, torch.int64)
        valid = c(valid.reshape(-1), torch.bool)
        meas_k = c(meas_k)
        valid_meas_k = None if valid_meas_k is None else c(valid_meas_k.reshape(-1), torch.bool)
        TWf = c(T_WCf.data.reshape(8))
        TWk = c(T_WCk.data.reshape(8))
        for t in (Xf, Xk):
            if t is not None and t.numel() != 3 * N:
                raise RuntimeError("track: pointmaps must have H*W points")
        dp = _dp
        ins = _lib.TrackInputs(
            idx_f2k=dp(idx), valid_match=dp(valid), Xf=dp(Xf), Cf=dp(Cf), Nf=float(Nf or 1), Qff=dp(Qff),
            Xk=dp(Xk), Ck=dp(Ck), Nk=float(Nk or 1), Qkf=dp(Qkf), T_WCf=dp(TWf), T_WCk=dp(TWk),
            direct=1 if direct else 0, meas_k=dp(meas_k), valid_meas_k=dp(valid_meas_k))
        fz = _lib.TrackFuse()
        keep = []
        self._fused = self._avg = None
        if fuse is not None:  # out of place like frame.py:75-76 (earlier holders keep the old tensors), or in the slot
            kf, Xkf, Ckf, slot = fuse
            Xin, Cin = c(kf.X_canon), c(kf.C)
            Xkf_c, Ckf_c = c(Xkf), c(Ckf)
            if slot is not None:
                Xo, Co = slot[0], slot[1]
            else:
                Xo, Co = torch.empty_like(Xin), torch.empty_like(Cin)
            Cka, Cfa = torch.empty_like(Cin), torch.empty_like(Cf)
            keep += [Xin, Cin, Xkf_c, Ckf_c]
            self._fused = (Xo, Co)
            self._avg = (Cka, Cfa)
            fz = _lib.TrackFuse(Xk_canon=dp(Xin), Ck_sum=dp(Cin), Xkf=dp(Xkf_c), Ckf=dp(Ckf_c), Xk_out=dp(Xo),
                                Ck_out=dp(Co), Cf=dp(Cf), Ck_avg_out=dp(Cka), Cf_avg_out=dp(Cfa),
                                Nk_new=float(kf.N + 1), Nf=float(Nf or 1))
            if slot is not None:
                fz.slot_N, fz.slot_N_updates, fz.slot_dirty = dp(slot[2]), dp(slot[3]), dp(slot[4])
                fz.N_new, fz.N_updates_new = int(kf.N) + 1, int(kf.N_updates) + 1
        T_out = torch.empty((2, 1, 8), dtype=torch.float32, device=dev)  # T_WCf | T_CkCf
        T_f, T_r = T_out.unbind(0)
        res = _lib.TrackResult()
        st = _lib.stream_ptr(dev)
        ws = _lib.workspace("track", lib.m3s_track_workspace_size(N), dev, st)
        _lib.check(lib.m3s_track(ctypes.byref(ins), ctypes.byref(tc), ctypes.byref(fz), int(self.first_chunk),
                                 T_out.data_ptr(), ctypes.byref(res), ws.data_ptr(), ws.numel(), st))
        self.last_result = res
        if not direct:  # next frame: enqueue as many GN launches as this one needed (+1) before reading back
            self.first_chunk = max(2, min(int(tc.max_iters), res.iters + 1))
        return res, T_f, T_r

    # ------------------------------------------------------------------ reference method surface
    def get_points_poses(self, frame, keyframe, idx_f2k, img_size, use_calib, K=None):
        """tracker.py:129-154 (torch glue; the fused path does this inside track_setup)."""
        from m3s.geometry import constrain_points_to_ray, get_pixel_coords

        Xf, Xk = frame.X_canon, keyframe.X_canon
        Cf, Ck = frame.get_average_conf(), keyframe.get_average_conf()
        meas_k = valid_meas_k = None
        if use_calib:
            Xf = constrain_points_to_ray(img_size, Xf[None], K).squeeze(0)
            Xk = constrain_points_to_ray(img_size, Xk[None], K).squeeze(0)
            uv_k = get_pixel_coords(1, img_size, device=Xf.device, dtype=Xf.dtype).view(-1, 2)
            meas_k = torch.cat((uv_k, torch.log(Xk[..., 2:3])), dim=-1)
            valid_meas_k = Xk[..., 2:3] > self.cfg["depth_eps"]
            meas_k[~valid_meas_k.repeat(1, 3)] = 0.0
        return Xf[idx_f2k], Xk, frame.T_WC, keyframe.T_WC, Cf[idx_f2k], Ck, meas_k, valid_meas_k

    def solve(self, sqrt_info, r, J):
        """tracker.py:156-171 (generic step; raises on Cholesky failure like torch.linalg.cholesky)."""
        whitened_r = sqrt_info * r
        robust_sqrt_info = sqrt_info * torch.sqrt(huber(whitened_r, k=self.cfg["huber"]))
        mdim = J.shape[-1]
        A = (robust_sqrt_info[..., None] * J).view(-1, mdim)
        b = (robust_sqrt_info * r).view(-1, 1)
        H = A.T @ A
        g = -A.T @ b
        cost = 0.5 * (b.T @ b).item()
        L = torch.linalg.cholesky(H, upper=False)
        tau_j = torch.cholesky_solve(g, L, upper=False).view(1, -1)
        return tau_j, cost

    def _direct(self, Xf, Xk, T_WCf, T_WCk, Qk, valid, use_calib, img_size, K, meas_k=None, valid_meas_k=None):
        n = Xf.shape[0]
        if img_size is None:
            img_size = (1, n)
        res, T_f, T_r = self._run_track(idx=None, valid=valid, Xf=Xf, Cf=None, Nf=1, Qff=Qk.reshape(-1), Xk=Xk, Ck=None,
                                     Nk=1, Qkf=None, T_WCf=T_WCf, T_WCk=T_WCk, use_calib=use_calib,
                                     img_size=img_size, K=K, direct=True, meas_k=meas_k, valid_meas_k=valid_meas_k)
        if res.status == _lib.TRACK_CHOLESKY_FAILED:
            raise RuntimeError("linalg.cholesky: The factorization could not be completed")
        return Sim3(T_f), Sim3(T_r)

    def opt_pose_ray_dist_sim3(self, Xf, Xk, T_WCf, T_WCk, Qk, valid):
        """tracker.py:173-214 -> (T_WCf, T_CkCf)."""
        return self._direct(Xf, Xk, T_WCf, T_WCk, Qk, valid, False, None, None)

    def opt_pose_calib_sim3(self, Xf, Xk, T_WCf, T_WCk, Qk, valid, meas_k, valid_meas_k, K, img_size):
        """tracker.py:216-266 -> (T_WCf, T_CkCf)."""
        return self._direct(Xf, Xk, T_WCf, T_WCk, Qk, valid, True, img_size, K, meas_k, valid_meas_k)
