"""Writes m3s/data/chess_kf256.txt: 256 keyframe poses of the 7-Scenes chess ground truth
(/root/reference/groundtruths/7-scenes/chess.txt, 1000 poses `i tx ty tz qx qy qz qw`), sampled at
round(linspace(0, 999, 256)) — every ~3.9th pose, the "every 4th pose" of SURVEY.md §8(d) stretched to
exactly K=256 — as Sim(3) rows [t(3), q(xyzw), s=1]. The file is data (a fixture), so the C4/C5 BA graphs
of bench.py and tests/ can be rebuilt on the GPU box, where /root/reference does not exist.

    python scripts/make_chess_poses.py
"""
import os

import numpy as np

SRC = "/root/reference/groundtruths/7-scenes/chess.txt"
DST = os.path.join(os.path.dirname(__file__), "..", "lightweight-mast3r-slam_amd", "m3s", "data", "chess_kf256.txt")


def main():
    a = np.loadtxt(SRC)
    assert a.shape == (1000, 8), a.shape
    sel = np.round(np.linspace(0, len(a) - 1, 256)).astype(int)
    P = np.concatenate((a[sel, 1:4], a[sel, 4:8], np.ones((256, 1))), axis=1)
    P[:, 3:7] /= np.linalg.norm(P[:, 3:7], axis=1, keepdims=True)
    hdr = "7-Scenes chess GT (groundtruths/7-scenes/chess.txt), rows round(linspace(0,999,256)); tx ty tz qx qy qz qw s"
    np.savetxt(DST, P, fmt="%.9f", header=hdr)
    print("wrote", os.path.normpath(DST), P.shape)


if __name__ == "__main__":
    main()
