"""Writes the 256-keyframe trajectories of the C4/C5 BA graphs as data fixtures, so the
graphs of bench.py and tests/ can be rebuilt on the GPU box, where /root/reference does not exist:

* m3s/data/chess_kf256.txt: 7-Scenes chess ground truth (groundtruths/7-scenes/chess.txt, 1000 poses
  `i tx ty tz qx qy qz qw`) at rows round(linspace(0, 999, 256)) — every ~3.9th pose, the "every 4th pose"
  of §8(d) stretched to exactly K=256;
* m3s/data/euroc_mh02_kf256.txt: EuRoC MH_02_easy ground truth (groundtruths/euroc/MH_02_easy.txt, 29993
  poses `t tx ty tz qx qy qz qw`; MH_01, C4's sequence, is not among the reference's ground-truth files)
  at rows round(linspace(0, n-1, 256)).

Rows are Sim(3) [t(3), q(xyzw), s=1].

    python scripts/make_traj_poses.py
"""
import os

import numpy as np

REF = "/root/reference/groundtruths"
DATA = os.path.join(os.path.dirname(__file__), "..", "lightweight-mast3r-slam_amd", "m3s", "data")
SETS = {
    "chess_kf256.txt": (os.path.join(REF, "7-scenes", "chess.txt"), "7-Scenes chess GT (groundtruths/7-scenes/chess.txt)"),
    "euroc_mh02_kf256.txt": (os.path.join(REF, "euroc", "MH_02_easy.txt"), "EuRoC MH_02_easy GT (groundtruths/euroc/MH_02_easy.txt)"),
}


def main():
    for dst, (src, what) in SETS.items():
        a = np.loadtxt(src)
        assert a.ndim == 2 and a.shape[1] == 8, a.shape
        sel = np.round(np.linspace(0, len(a) - 1, 256)).astype(int)
        P = np.concatenate((a[sel, 1:4], a[sel, 4:8], np.ones((256, 1))), axis=1)
        P[:, 3:7] /= np.linalg.norm(P[:, 3:7], axis=1, keepdims=True)
        hdr = f"{what}, rows round(linspace(0,{len(a) - 1},256)); tx ty tz qx qy qz qw s"
        out = os.path.join(DATA, dst)
        np.savetxt(out, P, fmt="%.9f", header=hdr)
        print("wrote", os.path.normpath(out), P.shape)


if __name__ == "__main__":
    main()
