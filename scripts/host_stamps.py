"""Host-side time stamps of the tracking bench's per-frame path (run on the GPU box).

Wraps the functions a tracked frame passes through with perf_counter_ns stamps at entry / exit and
prints the median time between consecutive stamps over the timed frames, to locate host time between
one frame's sync and the next frame's first launch."""
import os
import sys
import time
from collections import defaultdict

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lightweight-mast3r-slam_amd"))

from m3s import _lib, matching, tracker  # noqa: E402
from m3s.config import config  # noqa: E402
from m3s.frame import Frame, Keyframes  # noqa: E402
from m3s.sim3 import Sim3  # noqa: E402
from m3s.synthetic import SyntheticModel, make_pair  # noqa: E402

ST = []


def stamp(tag):
    ST.append((tag, time.perf_counter_ns()))


def wrap(mod, name, tag):
    f = getattr(mod, name)

    def w(*a, **k):
        stamp(tag + ">")
        r = f(*a, **k)
        stamp(tag + "<")
        return r

    setattr(mod, name, w)


lib = _lib.load()
orig_track = lib.m3s_track
orig_match = lib.m3s_match


class LibProxy:
    def __getattr__(self, n):
        return getattr(lib, n)

    def m3s_track(self, *a):
        stamp("c_track>")
        r = orig_track(*a)
        stamp("c_track<")
        return r

    def m3s_match(self, *a):
        stamp("c_match>")
        r = orig_match(*a)
        stamp("c_match<")
        return r


proxy = LibProxy()
_lib.load = lambda: proxy
wrap(matching, "match_iterative_proj", "match")
wrap(tracker, "match_halves", "tmatch")
wrap(tracker.FrameTracker, "_run_track", "run_track")
wrap(tracker.FrameTracker, "track", "track")
wrap(SyntheticModel, "asymmetric_inference", "model")

dev = torch.device("cuda:0")
H = W = 512
config["use_calib"] = True
pairs = [make_pair(H, W, seed=r) for r in range(6)]
model = SyntheticModel(pairs, dev)
kf = Frame(0, (H, W), T_WC=Sim3.Identity(1, device=dev))
kf.K = pairs[0]["K"].to(dev)
kf.update_pointmap(pairs[0]["Xk"].to(dev), pairs[0]["Ck"].to(dev))
kfs = Keyframes()
kfs.append(kf)
tr = tracker.FrameTracker(model, kfs, dev)
prev = kf.T_WC
for i in range(400):
    stamp("frame>")
    fr = Frame(i, (H, W), T_WC=kf.T_WC)
    stamp("frame_made")
    tr.track(fr)
    stamp("frame<")
    if i == 99:
        ST.clear()
torch.cuda.synchronize()
d = defaultdict(list)
for (t0, a), (t1, b) in zip(ST[:-1], ST[1:]):
    d[f"{t0} -> {t1}"].append((b - a) / 1e3)
fr = [b - a for (t, a), (u, b) in zip(ST, ST[1:]) if False]
tot = 0.0
for k, v in d.items():
    m = float(np.median(v))
    tot += m * len(v) / 300
    print(f"{k:32s} n={len(v):4d} median {m:8.2f} us  p90 {np.percentile(v, 90):8.2f}")
print(f"sum of medians per frame {tot:.1f} us")
