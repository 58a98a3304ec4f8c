"""BA accuracy census of one libm3s build (M3S_LIB): max |pose - fp64 truth| on every BA parity fixture.

usage: M3S_LIB=... python scripts/ba_acc.py [--quick]
Fixtures: the ill-conditioned 6-KF golden graph (24x32, rays / calib), the 24-KF medium graph (48x64), the
full-chunk 6-KF graph (128x192, 48 point rounds per lane), the K=256 chess (rays / calib) and EuRoC (rays) graphs
at 48x64. The truth is the oracle's fp64 build (oracle/liboracle_m3s_f64.so) on the same inputs."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "lightweight-mast3r-slam_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle.oracle as O  # noqa: E402
from test_gpu_ba import SIG, _call, _graph_inputs  # noqa: E402


def err(mode, Twc0, Xs, Cs, ii, jj, idx, valid, Q, K, H, W):
    sa, sb = SIG[mode]
    p = O.ba_params(mode, sa, sb, 0.0, 1.5, K=K, height=H, width=W, pixel_border=-10, z_eps=1e-6)
    T_ref, _, _ = O.gauss_newton_f64(mode, Twc0.astype(np.float64), Xs.astype(np.float64),
                                     Cs[..., 0].astype(np.float64), ii, jj, idx, valid[..., 0],
                                     Q[..., 0].astype(np.float64), p, 10, 1e-8)
    T, _ = _call(mode, Twc0, Xs, Cs, ii, jj, idx, valid, Q, K, H, W)
    return float(np.abs(T - T_ref).max())


def main():
    from m3s.synthetic import chess_poses, euroc_poses, make_graph, make_traj_graph, two_way

    out = {}
    g = dict(np.load(os.path.join(REPO, "tests", "golden", "ba_6kf_24x32.npz")))
    for mode in ("rays", "calib"):
        Xs, ii, jj = _graph_inputs(g, mode, 24, 32)
        out[f"6kf_{mode}"] = err(mode, g["Twc0"], Xs, g["Cs"], ii, jj, g["idx2"], g["valid2"], g["Q2"], g["K"], 24, 32)
    for name, (nkf, H, W, seed) in {"medium": (24, 48, 64, 5), "fullchunk": (6, 128, 192, 11)}.items():
        if name == "fullchunk":
            os.environ["M3S_BA_CHUNK_POINTS"] = "24576"
        G = make_graph(n_kf=nkf, H=H, W=W, seed=seed)
        ii, jj, idx, valid, Q = (t.numpy() for t in two_way(G))
        K = G["K"].numpy()
        for mode in ("rays", "calib"):
            Xs = G["Xs"].numpy() if mode == "rays" else O.backproject_constrain(G["Xs"].numpy(), K, (H, W))
            out[f"{name}_{mode}"] = err(mode, G["Twc0"].numpy(), Xs, G["Cs"].numpy(), ii, jj, idx, valid, Q, K, H, W)
        os.environ.pop("M3S_BA_CHUNK_POINTS", None)
    if "--quick" not in sys.argv:
        for traj, modes in (("chess", ("rays", "calib")), ("euroc", ("rays",))):
            G = make_traj_graph((chess_poses if traj == "chess" else euroc_poses)(256), 48, 64, seed=1)
            G = {k: (v.numpy() if torch.is_tensor(v) else v) for k, v in G.items()}
            for mode in modes:
                Xs = G["Xs"] if mode == "rays" else O.backproject_constrain(G["Xs"], G["K"], (48, 64))
                out[f"k256_{traj}_{mode}"] = err(mode, G["Twc0"], Xs, G["Cs"], G["ii"], G["jj"], G["idx"],
                                                 G["valid"], G["Q"], G["K"], 48, 64)
    out["max"] = max(out.values())
    print(json.dumps({k: float(f"{v:.3e}") for k, v in out.items()}), flush=True)


if __name__ == "__main__":
    main()
