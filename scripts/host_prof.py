"""Host-side profile of the tracking step (cProfile over FrameTracker.track on synthetic pairs)."""
import cProfile
import os
import pstats
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "lightweight-mast3r-slam_amd"))
import torch  # noqa: E402

from m3s.config import config  # noqa: E402
from m3s.frame import Frame, Keyframes  # noqa: E402
from m3s.sim3 import Sim3  # noqa: E402
from m3s.synthetic import SyntheticModel, make_pair  # noqa: E402
from m3s.tracker import FrameTracker  # noqa: E402

H = W = 512
dev = torch.device("cuda")
config["use_calib"] = True
pairs = [make_pair(H, W, seed=r) for r in range(3)]
model = SyntheticModel(pairs, dev)
kf = Frame(0, (H, W), T_WC=Sim3.Identity(1, device=dev))
kf.K = pairs[0]["K"].to(dev)
kf.update_pointmap(pairs[0]["Xk"].to(dev), pairs[0]["Ck"].to(dev))
kfs = Keyframes()
kfs.append(kf)
tracker = FrameTracker(model, kfs, dev)


def step(i):
    return tracker.track(Frame(i, (H, W), T_WC=Sim3(kf.T_WC.data.clone())))


for i in range(20):
    step(i)
torch.cuda.synchronize()
n = 300
t0 = time.perf_counter()
pr = cProfile.Profile()
pr.enable()
for i in range(n):
    step(i)
pr.disable()
torch.cuda.synchronize()
print(f"{(time.perf_counter() - t0) / n * 1e6:.1f} us/frame under cProfile")
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
