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
buf = (ctypes.c_ulonglong * 128)()
lib.m3s_debug_gn_stamps(buf)
print("iters", tracker.last_result.iters, "(stamps in us from block-0 start; 100 MHz clock)")
names = ["b0 start", "b0 points done", "b0 partial stored", "shard-last start", "shard sum published",
         "b0 shard sums polled", "b0 solved"]
for it in range(tracker.last_result.iters):
    t0 = buf[it * 16]
    nxt = f"  next b0 start={(buf[(it + 1) * 16] - t0) / 100:.2f}" if it + 1 < tracker.last_result.iters else ""
    print(f"iter {it}: " + "  ".join(f"{n}={(buf[it * 16 + k] - t0) / 100:.2f}" for k, n in enumerate(names)) + nxt)
