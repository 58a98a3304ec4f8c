"""proj_occlusion time vs the LM iteration count (HIP-event spans of m3s_match's launches), windowed (M3S_PROJ_WIN=1)
and global-gather (0) kernels, 512x512 synthetic pair, warm-started like the bench. Where the kernel's time goes:
the per-iteration slope against the fixed part (loads, setup, occlusion gather, stores)."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lightweight-mast3r-slam_amd"))
from m3s import _lib  # noqa: E402
from m3s.config import config  # noqa: E402
from m3s.matching import match  # noqa: E402
from m3s.synthetic import make_pair  # noqa: E402

lib = _lib.load()
P, Q = make_pair(512, 512, seed=500), make_pair(512, 512, seed=501)
X, D = P["X"].cuda(), P["D"].cuda()
X2, D2 = Q["X"].cuda(), Q["D"].cuda()
init, _ = match(X2[:1], X2[1:], D2[:1], D2[1:])
for win in ("1",):
    os.environ["M3S_PROJ_WIN"] = win
    for it in (0, 1, 2, 5, 10):
        config["matching"]["max_iter"] = it
        for _ in range(5):
            match(X[:1], X[1:], D[:1], D[1:], init)
        torch.cuda.synchronize()
        lib.m3s_timing_reset()
        lib.m3s_timing_enable(1)
        for _ in range(50):
            match(X[:1], X[1:], D[:1], D[1:], init)
        torch.cuda.synchronize()
        lib.m3s_timing_enable(0)
        ms, cnt = ctypes.c_double(), ctypes.c_int()
        _lib.check(lib.m3s_timing_query(b"proj_occlusion", ctypes.byref(ms), ctypes.byref(cnt)))
        print(f"win={win} max_iter={it:2d} proj_occlusion {1e3 * ms.value / max(cnt.value, 1):7.2f} us", flush=True)
config["matching"]["max_iter"] = 10
