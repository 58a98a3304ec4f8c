"""Dump the fused tracker's outputs over a few frames (poses, fused keyframe X / C, match_info tensors, per-frame
iteration counts) into one .npz (argv[1]), calib and rays modes at 512x512, so two builds of libm3s (M3S_LIB) can be
compared bit for bit."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lightweight-mast3r-slam_amd"))
from m3s.config import config  # noqa: E402
from m3s.frame import Frame, Keyframes  # noqa: E402
from m3s.sim3 import Sim3  # noqa: E402
from m3s.synthetic import SyntheticModel, make_pair  # noqa: E402
from m3s.tracker import FrameTracker  # noqa: E402

out = {}
H = W = 512
config["tracking"]["filtering_mode"] = "weighted_pointmap"
for mode in ("calib", "rays"):
    config["use_calib"] = mode == "calib"
    pairs = [make_pair(H, W, seed=600 + r) for r in range(3)]
    model = SyntheticModel(pairs, "cuda")
    kf = Frame(0, (H, W), T_WC=Sim3.Identity(1, device="cuda"))
    kf.K = pairs[0]["K"].cuda()
    kf.update_pointmap(pairs[0]["Xk"].cuda(), pairs[0]["Ck"].cuda())
    kfs = Keyframes()
    kfs.append(kf)
    tr = FrameTracker(model, kfs, "cuda")
    for f in range(6):
        frame = Frame(1 + f, (H, W), T_WC=Sim3.Identity(1, device="cuda"))
        new_kf, info, reloc = tr.track(frame)
        out[f"{mode}_{f}_T"] = frame.T_WC.data.cpu().numpy()
        out[f"{mode}_{f}_iters"] = np.array([tr.last_result.iters, int(new_kf), int(reloc)])
        for k, t in enumerate(info):
            out[f"{mode}_{f}_info{k}"] = t.cpu().numpy()
    out[f"{mode}_kfX"] = kfs[0].X_canon.cpu().numpy()
    out[f"{mode}_kfC"] = kfs[0].C.cpu().numpy()
config["use_calib"] = False
np.savez(sys.argv[1], **out)
print("dumped", len(out), "arrays to", sys.argv[1])
