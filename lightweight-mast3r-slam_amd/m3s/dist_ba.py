"""Edge-sharded global BA across GPUs (one process per GPU, RCCL over xGMI).

No reference counterpart: the reference runs BA in one process with a CPU Eigen solve
(``gn_kernels.cu:1181-1225``). Here:

* the E directed edges are split into contiguous, equal shards (every edge carries the same N
  points, so equal edge counts are equal work);
* each rank linearises only its shard into its rows of the (E, 36) fp64 edge-sum table
  (``M = A L A^T`` upper 28 + ``g = A v`` 7 per edge) — ~0.56 MB at E = 2000;
* ONE all-reduce(sum) of that table per GN iteration is the only exchange;
* every rank then assembles the identical block-sparse system in a fixed order, factorises it and
  retracts the poses, so poses stay bit-identical across ranks without a broadcast.

The backend is pluggable so the protocol itself can be exercised on CPU with ``gloo`` (tests use
an oracle backend); the product backend is ``HipShard`` over ``libm3s.so``.
"""
import ctypes
from ctypes import c_void_p

import numpy as np
import torch
import torch.distributed as dist

from m3s import _lib

BA_MODES = {"points": 0, "rays": 1, "calib": 2}
M3S_ESTALL = -4  # include/m3s.h


def shard_range(E, rank, world):
    """Contiguous balanced split of E edges: the first E % world ranks get one extra edge."""
    q, r = divmod(E, world)
    e0 = rank * q + min(rank, r)
    return e0, e0 + q + (1 if rank < r else 0)


def ba_config(mode, cfg, K=None, height=0, width=0):
    m = BA_MODES[mode]
    c = _lib.BaConfig(mode=m, C_thresh=float(cfg["C_conf"]), Q_thresh=float(cfg["Q_conf"]))
    if m == 0:
        c.sigma_a = float(cfg["sigma_point"])
    elif m == 1:
        c.sigma_a, c.sigma_b = float(cfg["sigma_ray"]), float(cfg["sigma_dist"])
    else:
        Kh = K.detach().float().cpu()
        c.sigma_a, c.sigma_b = float(cfg["sigma_pixel"]), float(cfg["sigma_depth"])
        c.fx, c.fy, c.cx, c.cy = float(Kh[0, 0]), float(Kh[1, 1]), float(Kh[0, 2]), float(Kh[1, 2])
        c.height, c.width = int(height), int(width)
        c.pixel_border, c.z_eps = int(cfg["pixel_border"]), float(cfg["depth_eps"])
    return c


class RecordCache:
    """A BA workspace kept across solves so the point records of unchanged edges carry over
    (``m3s_ba_make_plan*_reuse``): the backend solves once per new keyframe (main.py:150-155) while its edge set
    only grows. Grown with 2x headroom as the graph grows (a doubling of the edge count); a regrown workspace starts
    a fresh cache (one full pack, what every solve costs without reuse)."""

    def __init__(self):
        self.ws = None

    def workspace(self, nbytes, device):
        if self.ws is None or self.ws.device != device or self.ws.numel() < nbytes:
            self.release()
            self.ws = torch.empty(int(nbytes) * 2 + 256, dtype=torch.uint8, device=device)
        return self.ws

    def release(self):
        if self.ws is not None:
            _lib.check(_lib.load().m3s_ba_reuse_release(_lib.ptr(self.ws)))
            self.ws = None

    def __del__(self):
        try:
            self.release()
        except Exception:  # interpreter shutdown
            pass


class HipShard:
    """One rank's view of a sharded BA problem on its GPU (libm3s split API).

    The keyframe points come either stacked (``Xs`` (K,N,3), ``Cs`` (K,N) average confidences, as
    ``get_poses_points`` builds them) or, with ``Xs=None``, zero-copy from the keyframes' own buffers:
    ``keyframes = (X_list, C_list, N_list)`` with each X (N,3), C (N or N,1) the confidence sum and N the
    fusion count (``m3s_ba_make_plan_kf``)."""

    def __init__(self, cfg_struct, Twc, Xs, Cs, ii, jj, idx, valid, Q, delta_thresh, e0, e1, keyframes=None,
                 reuse=None, cache=None):
        """reuse = (edge_uid, kf_uid) int64 host arrays + cache (a RecordCache): pack only the edges whose records
        are not already in the cache's workspace (bit-identical results)."""
        lib = _lib.load()
        self.lib = lib
        self.dev = Twc.device
        if Xs is None:
            X_list, C_list, N_list = keyframes
            Kp, N = len(X_list), X_list[0].shape[-2]
            for x, cc in zip(X_list, C_list):
                if x.dtype != torch.float32 or cc.dtype != torch.float32 or not x.is_contiguous() or \
                        not cc.is_contiguous() or x.numel() != 3 * N or cc.numel() != N:
                    raise RuntimeError("ba: keyframe X (N,3) / C (N) must be contiguous float32")
        else:
            Kp, N = Xs.shape[0], Xs.shape[1]
        E = ii.shape[0]
        self.Kp, self.E = Kp, E
        self.dx = torch.zeros((max(Kp - 1, 0), 7), dtype=torch.float32, device=self.dev)
        nbytes = lib.m3s_ba_workspace_size(Kp, N, E)
        if reuse is not None and cache is not None:
            self.ws = cache.workspace(nbytes, self.dev)
            edge_uid = np.ascontiguousarray(reuse[0], dtype=np.int64)
            kf_uid = np.ascontiguousarray(reuse[1], dtype=np.int64)
            if edge_uid.shape != (E,) or kf_uid.shape != (Kp,):
                raise RuntimeError(f"ba reuse: need {E} edge uids and {Kp} keyframe uids")
            self._uids = (edge_uid, kf_uid)
            ru = ctypes.byref(_lib.BaReuse(edge_uid.ctypes.data, kf_uid.ctypes.data))
        else:
            self.ws = torch.empty(nbytes, dtype=torch.uint8, device=self.dev)
            self._own_ws = True
            ru = None
        self.keep = (Twc, Xs, Cs, ii, jj, idx, valid, Q, keyframes)
        self.plan = _lib.BaPlan()
        self.cfg = cfg_struct
        head = (_lib.ptr(ii), _lib.ptr(jj), E, int(e0), int(e1), _lib.ptr(idx), _lib.ptr(valid), _lib.ptr(Q),
                float(delta_thresh), _lib.ptr(self.dx))
        tail = (_lib.ptr(self.ws), self.ws.numel(), ctypes.byref(self.plan), _lib.stream_ptr(self.dev))
        if Xs is None:
            kt = _lib.BaKeyframes((c_void_p * Kp)(*[x.data_ptr() for x in X_list]),
                                  (c_void_p * Kp)(*[cc.data_ptr() for cc in C_list]),
                                  (ctypes.c_float * Kp)(*[float(n) for n in N_list]))
            _lib.check(lib.m3s_ba_make_plan_kf_reuse(ctypes.byref(cfg_struct), _lib.ptr(Twc), ctypes.byref(kt), Kp, N,
                                                     *head, ru, *tail))
        else:
            _lib.check(lib.m3s_ba_make_plan_reuse(ctypes.byref(cfg_struct), _lib.ptr(Twc), _lib.ptr(Xs), _lib.ptr(Cs),
                                                  Kp, N, *head, ru, *tail))
        off, cnt = ctypes.c_size_t(), ctypes.c_size_t()
        _lib.check(lib.m3s_ba_edge_sums(ctypes.byref(self.plan), ctypes.byref(off), ctypes.byref(cnt)))
        self.edge_sums = self.ws[off.value: off.value + cnt.value].view(torch.float64)

    def __del__(self):
        # a workspace of its own (not the RecordCache's): the library's plan state for it goes with it
        try:
            if getattr(self, "_own_ws", False) and _lib._LIB is not None:
                _lib._LIB.m3s_ba_plan_release(_lib.ptr(self.ws))
        except Exception:  # interpreter shutdown
            pass

    def reuse_info(self):
        """(shard edges the pack wrote, keyframes found changed)."""
        packed, changed = ctypes.c_int(), ctypes.c_int()
        _lib.check(self.lib.m3s_ba_reuse_info(ctypes.byref(self.plan), ctypes.byref(packed), ctypes.byref(changed)))
        return packed.value, changed.value

    def linearize(self):
        _lib.check(self.lib.m3s_ba_linearize(ctypes.byref(self.plan), _lib.stream_ptr(self.dev)))

    def solve(self):
        _lib.check(self.lib.m3s_ba_solve(ctypes.byref(self.plan), _lib.stream_ptr(self.dev)))

    def iterations(self):
        it = ctypes.c_int()
        _lib.check(self.lib.m3s_ba_iterations(ctypes.byref(self.plan), ctypes.byref(it), _lib.stream_ptr(self.dev)))
        return it.value

    def status(self):
        """This rank's loop status code, without raising: 0, M3S_ESTALL (its factor schedule stalled and its GN
        loop stopped) or another m3s error code. One readback (syncs the stream)."""
        it = ctypes.c_int()
        return int(self.lib.m3s_ba_iterations(ctypes.byref(self.plan), ctypes.byref(it), _lib.stream_ptr(self.dev)))

    def stalled(self):
        """True when this rank's factor schedule stalled; any other error raises."""
        rc = self.status()
        if rc == M3S_ESTALL:
            return True
        _lib.check(rc)
        return False


def _shard_status(shard):
    if hasattr(shard, "status"):
        return int(shard.status())
    if hasattr(shard, "stalled"):
        return M3S_ESTALL if shard.stalled() else 0
    return 0


def run_sharded(shard, max_iter, group=None):
    """GN loop of one rank: linearise shard -> all-reduce edge sums -> identical solve/retract.

    The all-reduce runs whenever a process group exists (also at world size 1, where it is the identity:
    the RCCL path is then exercised on one GPU); without one the loop is the plain single-GPU solve."""
    reduce = dist.is_available() and dist.is_initialized()
    for _ in range(int(max_iter)):
        shard.linearize()
        if reduce:
            dist.all_reduce(shard.edge_sums, op=dist.ReduceOp.SUM, group=group)
        shard.solve()
    # The outcome is decided globally: a rank whose bounded factor-schedule wait timed out stops its own loop (its
    # edge-sum rows stay zero), so its peers solved without that shard, and a rank whose status readback failed
    # otherwise must not raise alone either (its peers would wait for it at their next collective). Every rank reads
    # its status code without raising, one MAX all-reduce of {stalled, failed, |code|} follows, and then every rank
    # raises the same error together.
    rc = _shard_status(shard)
    stalled, failed, code = float(rc == M3S_ESTALL), float(rc != 0 and rc != M3S_ESTALL), float(abs(rc))
    if reduce:
        flag = torch.tensor([stalled, failed, code if failed else 0.0], dtype=torch.float64,
                            device=shard.edge_sums.device)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=group)
        stalled, failed, code = (float(v) for v in flag.tolist())
    if failed > 0.0:
        raise RuntimeError(f"m3s error {-int(code)}: ba: the GN loop failed on a rank; the poses are not valid")
    if stalled > 0.0:
        raise RuntimeError(f"m3s error {M3S_ESTALL}: ba: a factor-schedule hand-off stalled on a rank (bounded wait "
                           "timed out); the GN loop stopped and the poses are not valid")
    return shard


def gauss_newton_sharded(mode, Twc, Xs, Cs, ii, jj, idx, valid, Q, cfg, max_iter, delta_thresh, K=None, height=0,
                         width=0, group=None, keyframes=None, reuse=None, cache=None, info=None):
    """Multi-GPU drop-in for mast3r_slam_backends.gauss_newton_*: same inputs (every rank holds the
    full problem, replicated), Twc updated in place identically on every rank; returns [dx]. With
    ``Xs=None`` the keyframe points come zero-copy from ``keyframes`` (see ``HipShard``); with ``reuse`` and
    ``cache`` the records of unchanged edges carry over from the previous solve (``info``, a dict, receives
    ``packed_edges`` / ``changed_keyframes``)."""
    rank = dist.get_rank(group) if dist.is_available() and dist.is_initialized() else 0
    world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
    e0, e1 = shard_range(ii.shape[0], rank, world)
    c = lambda t: t.contiguous()
    if Xs is not None:
        Xs, Cs = c(Xs), c(Cs.reshape(Xs.shape[0], -1))
    shard = HipShard(ba_config(mode, cfg, K, height, width), c(Twc), Xs, Cs, c(ii), c(jj), c(idx),
                     c(valid.reshape(idx.shape)), c(Q.reshape(idx.shape)), delta_thresh, e0, e1, keyframes=keyframes,
                     reuse=reuse, cache=cache)
    if info is not None:
        info["packed_edges"], info["changed_keyframes"] = shard.reuse_info()
    run_sharded(shard, max_iter, group)  # raises RuntimeError (M3S_ESTALL) on every rank if any rank stalled
    return [shard.dx]
