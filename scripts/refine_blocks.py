"""Refine-kernel block balance (M3S_REFINE_BSTAMPS build): per-block durations of refine_tile_kernel at 512x512."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "lightweight-mast3r-slam_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from m3s import _lib  # noqa: E402
from m3s.matching import match  # noqa: E402
from m3s.synthetic import make_pair  # noqa: E402

lib = _lib.load()
P = make_pair(512, 512, seed=0)
X, D = P["X"].cuda(), P["D"].cuda()
for _ in range(5):
    match(X[:1], X[1:], D[:1], D[1:])
torch.cuda.synchronize()
nb = 512 * 512 // 256
buf = (ctypes.c_ulonglong * (8192 * 4))()
lib.m3s_debug_refine_bstamps(buf)
a = np.frombuffer(buf, dtype=np.uint64).reshape(8192, 4)[:nb].astype(np.float64)
t0 = a[:, 0].min()
start, end = (a[:, 0] - t0) / 100.0, (a[:, 1] - t0) / 100.0  # us (100 MHz)
dur = end - start
hw = a[:, 2].astype(np.int64)
cu = (hw >> 8) & 0xF
sh = (hw >> 12) & 1
se = (hw >> 13) & 0x7
act = a[:, 3]
print(f"blocks {nb}: kernel span {end.max():.1f} us, block start {start.min():.1f}..{start.max():.1f} us")
print("block duration us: min %.1f p10 %.1f median %.1f p90 %.1f max %.1f mean %.1f" % (
    dur.min(), *np.percentile(dur, [10, 50, 90]), dur.max(), dur.mean()))
print("active lanes per block (of 256): min %d median %d max %d" % (act.min(), np.median(act), act.max()))
slow = np.argsort(dur)[-8:]
print("slowest blocks (block, dur us, start us, active, se, cu):",
      [(int(b), round(dur[b], 1), round(start[b], 1), int(act[b]), int(se[b]), int(cu[b])) for b in slow])
print("corr(duration, active lanes) %.3f" % np.corrcoef(dur, act)[0, 1])
# tile of each block (refine.hip: lb = xcd_remap(block), 32x8 tiles, 16 per row at 512 wide)
q8, r8 = nb // 8, nb % 8
xb = np.arange(nb) % 8
lb = np.where(xb < r8, xb * (q8 + 1), r8 * (q8 + 1) + (xb - r8) * q8) + np.arange(nb) // 8
tx, ty = lb % 16, lb // 16
grid = np.zeros((64, 16))
grid[ty, tx] = dur
print("mean block duration by tile row band (8 tile rows = 64 px each):",
      " ".join(f"{grid[r:r + 8].mean():.0f}" for r in range(0, 64, 8)))
print("mean block duration by tile column (32 px each):", " ".join(f"{grid[:, c].mean():.0f}" for c in range(16)))
print("XCD (block % 8) mean durations:", " ".join(f"{dur[xb == x].mean():.0f}" for x in range(8)))
