"""Profiling driver: the fused matcher alone on a 512x512 synthetic pair (for rocprofv3)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "lightweight-mast3r-slam_amd"))
import torch  # noqa: E402

from m3s.matching import match  # noqa: E402
from m3s.synthetic import make_pair  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
P = make_pair(512, 512, seed=0)
X, D = P["X"].cuda(), P["D"].cuda()
for _ in range(reps):
    idx, valid = match(X[:1], X[1:], D[:1], D[1:])
torch.cuda.synchronize()
print("valid frac", valid.float().mean().item())
