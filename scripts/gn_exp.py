"""GN-iteration experiment: in-kernel s_memrealtime stamps (M3S_GN_STAMPS build) of one tracked frame."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "lightweight-mast3r-slam_amd"))
import torch  # noqa: E402

from m3s import _lib  # noqa: E402
from m3s.config import config  # noqa: E402
from m3s.frame import Frame, Keyframes  # noqa: E402
from m3s.sim3 import Sim3  # noqa: E402
from m3s.synthetic import SyntheticModel, make_pair  # noqa: E402
from m3s.tracker import FrameTracker  # noqa: E402

H = W = 512
dev = torch.device("cuda")
config["use_calib"] = os.environ.get("MODE", "calib") == "calib"
pairs = [make_pair(H, W, seed=r) for r in range(2)]
model = SyntheticModel(pairs, dev)
kf = Frame(0, (H, W), T_WC=Sim3.Identity(1, device=dev))
kf.K = pairs[0]["K"].to(dev)
kf.update_pointmap(pairs[0]["Xk"].to(dev), pairs[0]["Ck"].to(dev))
kfs = Keyframes()
kfs.append(kf)
tracker = FrameTracker(model, kfs, dev)
lib = _lib.load()
for i in range(6):
    tracker.track(Frame(i, (H, W), T_WC=Sim3(kf.T_WC.data.clone())))
torch.cuda.synchronize()
import numpy as np  # noqa: E402

NB = 8 * 256 * 8
buf = (ctypes.c_ulonglong * NB)()
lib.m3s_debug_gn_stamps(buf)  # read + clear the warm-up frames' stamps
tracker.track(Frame(6, (H, W), T_WC=Sim3(kf.T_WC.data.clone())))
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * NB)()
lib.m3s_debug_gn_stamps(buf)
st = np.frombuffer(buf, dtype=np.uint64).reshape(8, 256, 8).astype(np.float64)
iters = tracker.last_result.iters
print("iters", iters, "- per-block s_memrealtime stamps (100 MHz), us from the iteration's earliest block start:")
names = ["start", "points done", "partial stored", "shard-last start", "shard sum published", "shard sums polled",
         "solved"]
for it in range(iters):
    t0 = st[it, :, 0][st[it, :, 0] > 0].min()
    parts = []
    for k, n in enumerate(names):
        v = st[it, :, k]
        v = v[v > 0]
        if v.size:
            parts.append(f"{n} {(v.min() - t0) / 100:.2f}..{(v.max() - t0) / 100:.2f}")
    print(f"iter {it}: " + " | ".join(parts))
