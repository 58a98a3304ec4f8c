"""``FactorGraph`` with the reference surface (``/root/reference/mast3r_slam/global_opt.py:14-226``).

Edge insertion (``add_factors``) batches the symmetric matches of all new edges through the fused
HIP matcher; ``solve_GN_rays`` / ``solve_GN_calib`` run the split BA API of ``m3s.dist_ba`` with record reuse
across solves (only new edges and edges of changed keyframes are re-packed; bit-identical to a fresh solve) and,
when ``torch.distributed`` is initialised with more than one rank, edge-sharded over RCCL (identical result on
every rank). With ``reuse_records = False`` a single-GPU solve calls the drop-in ``mast3r_slam_backends``
operators.
"""
import numpy as np
import torch
import torch.distributed as dist

import mast3r_slam_backends
from m3s.config import config
from m3s.geometry import constrain_points_to_ray
from m3s.matching import match
from m3s.sim3 import Sim3
from m3s.tracker import frame_img_size


def mast3r_match_symmetric(model, kfs_i, kfs_j):
    """mast3r_utils.py:149-187 with the ViT decode behind ``model.symmetric_inference`` returning
    X (4,b,H,W,3), C (4,b,H,W), D (4,b,H,W,F), Q (4,b,H,W) ordered ii, ji, jj, ij."""
    fn = getattr(model, "symmetric_inference", None)
    if fn is not None:
        X, C, D, Q = fn(kfs_i, kfs_j)
    else:  # the real ViT: the reference's own batched decode (mast3r_utils.py:117-146), stock PyTorch-ROCm
        from mast3r_slam.mast3r_utils import mast3r_decode_symmetric_batch

        X, C, D, Q = mast3r_decode_symmetric_batch(
            model, torch.cat([k.feat for k in kfs_i]), torch.cat([k.pos for k in kfs_i]),
            torch.cat([k.feat for k in kfs_j]), torch.cat([k.pos for k in kfs_j]),
            [k.img_true_shape for k in kfs_i], [k.img_true_shape for k in kfs_j])
    b = X.shape[1]
    X11 = torch.cat((X[0], X[2]), dim=0)
    X21 = torch.cat((X[1], X[3]), dim=0)
    D11 = torch.cat((D[0], D[2]), dim=0)
    D21 = torch.cat((D[1], D[3]), dim=0)
    idx_1_to_2, valid_match_2 = match(X11, X21, D11, D21)
    return (idx_1_to_2[:b], idx_1_to_2[b:], valid_match_2[:b], valid_match_2[b:],
            Q[0].reshape(b, -1, 1), Q[2].reshape(b, -1, 1), Q[1].reshape(b, -1, 1), Q[3].reshape(b, -1, 1))


class FactorGraph:
    def __init__(self, model, frames, K=None, device="cuda"):
        self.model = model
        self.frames = frames
        self.device = device
        self.cfg = config["local_opt"]
        e = lambda dt: torch.as_tensor([], dtype=dt, device=device)
        self.ii, self.jj = e(torch.long), e(torch.long)
        self.idx_ii2jj, self.idx_jj2ii = e(torch.long), e(torch.long)
        self.valid_match_j, self.valid_match_i = e(torch.bool), e(torch.bool)
        self.Q_ii2jj, self.Q_jj2ii = e(torch.float32), e(torch.float32)
        self.window_size = self.cfg["window_size"]
        self.K = K
        self.group = None  # torch.distributed group for the sharded solve (None = WORLD)
        # record reuse across solves (m3s.dist_ba.RecordCache): edges are append-only here, so directed edge
        # 2u + d (undirected edge u, direction d) names the same match data in every later solve
        self.reuse_records = True
        self._records = None
        self.ba_info = {}

    def add_factors(self, ii, jj, min_match_frac, is_reloc=False):
        """global_opt.py:32-101."""
        kf_ii = [self.frames[i] for i in ii]
        kf_jj = [self.frames[j] for j in jj]
        idx_i2j, idx_j2i, valid_match_j, valid_match_i, Qii, Qjj, Qji, Qij = mast3r_match_symmetric(
            self.model, kf_ii, kf_jj)
        bi = torch.arange(idx_i2j.shape[0], device=idx_i2j.device)[:, None].repeat(1, idx_i2j.shape[1])
        Qj = torch.sqrt(Qii[bi, idx_i2j] * Qji)
        Qi = torch.sqrt(Qjj[bi, idx_j2i] * Qij)
        valid_j = valid_match_j & (Qj > self.cfg["Q_conf"])
        valid_i = valid_match_i & (Qi > self.cfg["Q_conf"])
        match_frac_j = valid_j.sum(dim=(1, 2)) / (valid_j.shape[1] * valid_j.shape[2])
        match_frac_i = valid_i.sum(dim=(1, 2)) / (valid_i.shape[1] * valid_i.shape[2])
        ii_t = torch.as_tensor(ii, device=self.device)
        jj_t = torch.as_tensor(jj, device=self.device)
        invalid = torch.minimum(match_frac_j, match_frac_i) < min_match_frac
        invalid = (~(ii_t == (jj_t - 1))) & invalid  # consecutive edges are always kept
        if invalid.any() and is_reloc:
            return False
        keep = ~invalid
        self.ii = torch.cat([self.ii, ii_t[keep]])
        self.jj = torch.cat([self.jj, jj_t[keep]])
        self.idx_ii2jj = torch.cat([self.idx_ii2jj, idx_i2j[keep]])
        self.idx_jj2ii = torch.cat([self.idx_jj2ii, idx_j2i[keep]])
        self.valid_match_j = torch.cat([self.valid_match_j, valid_match_j[keep]])
        self.valid_match_i = torch.cat([self.valid_match_i, valid_match_i[keep]])
        self.Q_ii2jj = torch.cat([self.Q_ii2jj, Qj[keep]])
        self.Q_jj2ii = torch.cat([self.Q_jj2ii, Qi[keep]])
        return keep.sum() > 0

    def get_unique_kf_idx(self):
        return torch.unique(torch.cat([self.ii, self.jj]), sorted=True)

    def prep_two_way_edges(self):
        ii = torch.cat((self.ii, self.jj), dim=0)
        jj = torch.cat((self.jj, self.ii), dim=0)
        idx_ii2jj = torch.cat((self.idx_ii2jj, self.idx_jj2ii), dim=0)
        valid_match = torch.cat((self.valid_match_j, self.valid_match_i), dim=0)
        Q_ii2jj = torch.cat((self.Q_ii2jj, self.Q_jj2ii), dim=0)
        return ii, jj, idx_ii2jj, valid_match, Q_ii2jj

    def get_poses_points(self, unique_kf_idx):
        kfs = [self.frames[int(i)] for i in unique_kf_idx]
        Xs = torch.stack([kf.X_canon for kf in kfs])
        T_WCs = Sim3(torch.stack([kf.T_WC.data.reshape(1, 8) for kf in kfs]))
        Cs = torch.stack([kf.get_average_conf() for kf in kfs])
        return Xs, T_WCs, Cs

    def get_poses_keyframes(self, unique_kf_idx):
        """Zero-copy counterpart of get_poses_points: the poses are stacked (K x 8
        floats) but the points stay in the keyframes' own X_canon / C buffers, which the BA plan reads
        through a pointer table (``m3s_ba_make_plan_kf``); the average confidence C / N is applied in the
        pack kernel. Returns None when a keyframe's buffers do not qualify (then the stacked path runs)."""
        kfs = [self.frames[int(i)] for i in unique_kf_idx]
        X = [kf.X_canon for kf in kfs]
        C = [kf.C for kf in kfs]
        ok = all(x.is_cuda and x.dtype == torch.float32 and x.is_contiguous() and c.dtype == torch.float32 and
                 c.is_contiguous() and x.numel() == X[0].numel() and c.numel() * 3 == x.numel() for x, c in zip(X, C))
        if not ok:
            return None
        T_WCs = Sim3(torch.stack([kf.T_WC.data.reshape(1, 8) for kf in kfs]))
        return T_WCs, (X, C, [float(kf.N) for kf in kfs])

    @staticmethod
    def _pin(cfg):
        """cfg.pin: the C++ solvers fix exactly one pose (num_fix = 1, gn_kernels.cu:741,1157,1566) while the
        Python slices the write-back by cfg.pin (global_opt.py:125,161). pin = 1 is the configured value
        (config/base.yaml:36). pin = 0 is accepted as the reference runs it: pose 0 stays fixed in the solve, so writing
        T_WCs[0:] back writes it unchanged, and a graph with one keyframe has nothing to solve (the early return uses
        max(pin, 1)). pin > 1 would drop solved poses from the write-back: rejected (SURVEY.md §8 a-note 8)."""
        pin = int(cfg["pin"])
        if pin not in (0, 1):
            raise ValueError(f"local_opt.pin = {pin}: only pin = 0 or 1 is supported (the solver fixes one pose)")
        return pin

    def _sharded(self):
        return dist.is_available() and dist.is_initialized() and dist.get_world_size(self.group) > 1

    def _reuse_kw(self, unique_kf_idx):
        """gauss_newton_sharded keywords for record reuse ({} when disabled)."""
        if not self.reuse_records:
            return {}
        from m3s.dist_ba import RecordCache

        if self._records is None:
            self._records = RecordCache()
        u = np.arange(self.ii.numel(), dtype=np.int64)
        edge_uid = np.concatenate([2 * u, 2 * u + 1])
        kf_uid = unique_kf_idx.cpu().numpy().astype(np.int64)
        self.ba_info = {}
        return {"reuse": (edge_uid, kf_uid), "cache": self._records, "info": self.ba_info}

    def solve_GN_rays(self):
        """global_opt.py:123-161, with the keyframe points read in place (no torch.stack of K x N x 16 B)."""
        cfg = self.cfg
        pin = self._pin(cfg)
        unique_kf_idx = self.get_unique_kf_idx()
        if unique_kf_idx.numel() <= max(pin, 1):
            return
        ii, jj, idx_ii2jj, valid_match, Q_ii2jj = self.prep_two_way_edges()
        rk = self._reuse_kw(unique_kf_idx)
        zc = self.get_poses_keyframes(unique_kf_idx)
        if zc is not None:
            from m3s.dist_ba import gauss_newton_sharded

            T_WCs, keyframes = zc
            gauss_newton_sharded("rays", T_WCs.data[:, 0, :], None, None, ii, jj, idx_ii2jj, valid_match, Q_ii2jj,
                                 cfg, cfg["max_iters"], cfg["delta_norm"],
                                 group=self.group, keyframes=keyframes, **rk)
            self.frames.update_T_WCs(T_WCs[pin:], unique_kf_idx[pin:])
            return
        Xs, T_WCs, Cs = self.get_poses_points(unique_kf_idx)
        pose_data = T_WCs.data[:, 0, :]
        if self._sharded() or rk:
            from m3s.dist_ba import gauss_newton_sharded

            gauss_newton_sharded("rays", pose_data, Xs, Cs, ii, jj, idx_ii2jj, valid_match, Q_ii2jj, cfg,
                                 cfg["max_iters"], cfg["delta_norm"], group=self.group, **rk)
        else:
            mast3r_slam_backends.gauss_newton_rays(pose_data, Xs, Cs, ii, jj, idx_ii2jj, valid_match, Q_ii2jj,
                                                   cfg["sigma_ray"], cfg["sigma_dist"], cfg["C_conf"], cfg["Q_conf"],
                                                   cfg["max_iters"], cfg["delta_norm"])
        self.frames.update_T_WCs(T_WCs[pin:], unique_kf_idx[pin:])

    def solve_GN_calib(self):
        """global_opt.py:163-226."""
        cfg = self.cfg
        K = self.K
        pin = self._pin(cfg)
        unique_kf_idx = self.get_unique_kf_idx()
        if unique_kf_idx.numel() <= max(pin, 1):
            return
        Xs, T_WCs, Cs = self.get_poses_points(unique_kf_idx)
        img_size = frame_img_size(self.frames[0])
        Xs = constrain_points_to_ray(img_size, Xs, K)
        ii, jj, idx_ii2jj, valid_match, Q_ii2jj = self.prep_two_way_edges()
        pose_data = T_WCs.data[:, 0, :]
        height, width = img_size
        rk = self._reuse_kw(unique_kf_idx)
        if self._sharded() or rk:
            from m3s.dist_ba import gauss_newton_sharded

            gauss_newton_sharded("calib", pose_data, Xs, Cs, ii, jj, idx_ii2jj, valid_match, Q_ii2jj, cfg,
                                 cfg["max_iters"], cfg["delta_norm"], K=K, height=height, width=width,
                                 group=self.group, **rk)
        else:
            mast3r_slam_backends.gauss_newton_calib(pose_data, Xs, Cs, K, ii, jj, idx_ii2jj, valid_match, Q_ii2jj,
                                                    height, width, cfg["pixel_border"], cfg["depth_eps"],
                                                    cfg["sigma_pixel"], cfg["sigma_depth"], cfg["C_conf"],
                                                    cfg["Q_conf"], cfg["max_iters"], cfg["delta_norm"])
        self.frames.update_T_WCs(T_WCs[pin:], unique_kf_idx[pin:])
