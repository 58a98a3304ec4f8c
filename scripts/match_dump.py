"""Dump the fused match's idx / valid on a set of cases into one .npz
(argv[1]), so two builds of libm3s (M3S_LIB) can be compared bit for bit: 512x512 cold and warm starts, a ragged
batch of 2, scattered and negative / out-of-range warm starts, max_iter 0 and 1."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lightweight-mast3r-slam_amd"))
from m3s.config import config  # noqa: E402
from m3s.matching import match  # noqa: E402
from m3s.synthetic import make_pair  # noqa: E402


def dev(a):
    return torch.as_tensor(np.ascontiguousarray(a)).cuda()


out = {}
rng = np.random.default_rng(9)
for name, (B, H, W), warm, iters in [("full_cold", (1, 512, 512), "none", 10), ("full_warm", (1, 512, 512), "flow", 10),
                                     ("ragged", (2, 50, 70), "none", 10), ("scatter", (1, 33, 47), "scatter", 10),
                                     ("negative", (1, 8, 9), "negative", 10), ("iter0", (1, 96, 128), "flow", 0),
                                     ("iter1", (1, 96, 128), "flow", 1)]:
    Ps = [make_pair(H, W, seed=70 + b) for b in range(B)]
    X11 = dev(np.stack([p["X"][0].numpy() for p in Ps]))
    X21 = dev(np.stack([p["X"][1].numpy() for p in Ps]))
    D11 = dev(np.stack([p["D"][0].numpy() for p in Ps]))
    D21 = dev(np.stack([p["D"][1].numpy() for p in Ps]))
    init = None
    if warm == "flow":
        init, _ = match(X11, X21, D11, D21)
    elif warm == "scatter":
        init = dev(rng.integers(0, H * W, size=(B, H * W)).astype(np.int64))
    elif warm == "negative":
        init = dev(rng.integers(-3 * H * W, 3 * H * W, size=(B, H * W)).astype(np.int64))
    config["matching"]["max_iter"] = iters
    idx, valid = match(X11, X21, D11, D21, init)
    config["matching"]["max_iter"] = 10
    out[name + "_idx"] = idx.cpu().numpy()
    out[name + "_valid"] = valid.cpu().numpy()
np.savez(sys.argv[1], **out)
print("dumped", len(out), "arrays to", sys.argv[1])
