"""Conditioning of the BA pose system on the K=256 chess graph, and how many steps of fp64 iterative
refinement an fp32 Cholesky needs to reach the fp64 solve (feasibility of a mixed-precision factor).
usage: python scripts/ba_cond.py [H] [W]"""
import os
import sys

import numpy as np
import scipy.linalg as sl
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "lightweight-mast3r-slam_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
from m3s.config import config  # noqa: E402
from m3s.dist_ba import HipShard, ba_config  # noqa: E402
from m3s.geometry import constrain_points_to_ray  # noqa: E402
from m3s.synthetic import chess_poses, make_traj_graph, make_graph, two_way  # noqa: E402

H = int(sys.argv[1]) if len(sys.argv) > 1 else 48
W = int(sys.argv[2]) if len(sys.argv) > 2 else 64
dev = torch.device("cuda")


def system(es, ii, jj):
    u = np.unique(np.concatenate((ii, jj)))
    ri, rj = np.searchsorted(u, ii) - 1, np.searchsorted(u, jj) - 1
    n = (len(u) - 1) * 7
    Hs, g = np.zeros((n, n)), np.zeros(n)
    iu = np.triu_indices(7)
    for e in range(es.shape[0]):
        M = np.zeros((7, 7))
        M[iu] = es[e, :28]
        M = M + np.triu(M, 1).T
        gv = es[e, 28:35]
        a, b = ri[e], rj[e]
        if a >= 0:
            Hs[7 * a:7 * a + 7, 7 * a:7 * a + 7] += M
            g[7 * a:7 * a + 7] -= gv
        if b >= 0:
            Hs[7 * b:7 * b + 7, 7 * b:7 * b + 7] += M
            g[7 * b:7 * b + 7] += gv
        if a >= 0 and b >= 0:
            Hs[7 * a:7 * a + 7, 7 * b:7 * b + 7] -= M
            Hs[7 * b:7 * b + 7, 7 * a:7 * a + 7] -= M
    return Hs, g


for graph in ("chess", "circle"):
    for mode in ("rays", "calib"):
        if graph == "chess":
            G = make_traj_graph(chess_poses(256), H, W, seed=1, device=dev)
            ii, jj, idx = G["ii"], G["jj"], G["idx"].contiguous()
            valid, Q = G["valid"][..., 0].contiguous(), G["Q"][..., 0].contiguous()
        else:
            G = make_graph(n_kf=256, H=H, W=W, seed=1)
            ii, jj, idx, valid, Q = two_way(G)
            ii, jj, idx = ii.to(dev), jj.to(dev), idx.to(dev).contiguous()
            valid, Q = valid[..., 0].to(dev).contiguous(), Q[..., 0].to(dev).contiguous()
        Xs, Cs = G["Xs"].to(dev).contiguous(), G["Cs"][..., 0].to(dev).contiguous()
        if mode == "calib":
            Xs = constrain_points_to_ray((H, W), Xs, G["K"].to(dev)).contiguous()
        cfg = ba_config(mode, config["local_opt"], K=G["K"], height=H, width=W)
        sh = HipShard(cfg, G["Twc0"].to(dev).contiguous(), Xs, Cs, ii, jj, idx, valid, Q, 0.0, 0, ii.shape[0])
        sh.linearize()
        es = sh.edge_sums.view(-1, 36).cpu().numpy().copy()
        A, b = system(es, ii.cpu().numpy(), jj.cpu().numpy())
        x64 = np.linalg.solve(A, b)
        ev = np.linalg.eigvalsh(A)
        # fp32 Cholesky, fp64 residuals
        L32 = np.linalg.cholesky(A.astype(np.float32))
        x = np.zeros_like(b)
        errs = []
        for it in range(6):
            r = b - A @ x
            d = sl.cho_solve((L32, True), r.astype(np.float32)).astype(np.float64)
            x = x + d
            errs.append(np.abs(x - x64).max() / np.abs(x64).max())
        # Jacobi-scaled variant
        s = 1.0 / np.sqrt(np.diag(A))
        As = A * s[:, None] * s[None, :]
        evs = np.linalg.eigvalsh(As)
        print(f"{graph:6s} {mode:5s} n={A.shape[0]} cond {ev[-1] / ev[0]:.3e} (Jacobi-scaled {evs[-1] / evs[0]:.3e}); "
              f"fp32 chol + refinement rel err per step: " + " ".join(f"{e:.1e}" for e in errs), flush=True)
