"""Refine-kernel experiment: kernel time (HIP events inside libm3s) vs dilation_max and grid size."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "lightweight-mast3r-slam_amd"))
import torch  # noqa: E402

from m3s import _lib  # noqa: E402
from m3s.config import config  # noqa: E402
from m3s.matching import match  # noqa: E402
from m3s.synthetic import make_pair  # noqa: E402

lib = _lib.load()


def timed(X, D, reps=20):
    for _ in range(3):
        match(X[:1], X[1:], D[:1], D[1:])
    lib.m3s_timing_reset()
    lib.m3s_timing_enable(1)
    for _ in range(reps):
        match(X[:1], X[1:], D[:1], D[1:])
    torch.cuda.synchronize()
    lib.m3s_timing_enable(0)
    out = {}
    for name in ("prep_rays", "proj_occlusion", "refine_lin"):
        ms, cnt = ctypes.c_double(), ctypes.c_int()
        _lib.check(lib.m3s_timing_query(name.encode(), ms, cnt))
        out[name] = 1000 * ms.value / max(cnt.value, 1)
    return out


QUICK = os.environ.get("REFINE_EXP_QUICK") == "1"  # profiling: only 512x512 at dilation_max 5
for (h, w) in ((512, 512),) if QUICK else ((512, 512), (8, 512)):
    P = make_pair(h, w, seed=0)
    X, D = P["X"].cuda(), P["D"].cuda()
    row = []
    for dm in (5,) if QUICK else (1, 2, 3, 4, 5):
        config["matching"]["dilation_max"] = dm
        row.append(timed(X, D)["refine_lin"])
    config["matching"]["dilation_max"] = 5
    print(f"{h}x{w} blocks={h * w // 256}: refine us by dmax 1..5: " + " ".join(f"{t:7.1f}" for t in row), flush=True)

P = make_pair(512, 512, seed=0)
X, D = P["X"].cuda(), P["D"].cuda()
idx, valid = match(X[:1], X[1:], D[:1], D[1:])
print("idx checksum", int(idx.sum().item()), "lib", _lib.LIB_PATH)
if hasattr(lib, "m3s_debug_refine_stats"):
    buf = (ctypes.c_ulonglong * 64)()
    lib.m3s_debug_refine_stats(buf, 1)
    idx, valid = match(X[:1], X[1:], D[:1], D[1:])
    lib.m3s_debug_refine_stats(buf, 0)
    for d in range(5, 0, -1):
        print(f"d={d}: outlier lanes {buf[2 * d]}  waves with outliers {buf[2 * d + 1]} / {512 * 512 // 64}; "
              f"screen survivors per pixel {buf[32 + 2 * d] / (512 * 512):.3f}, per-wave max (mean) "
              f"{buf[33 + 2 * d] / (512 * 512 // 64):.3f}")
