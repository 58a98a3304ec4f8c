"""Determinism probe (GPU): the fused match twice on the same 512x512 pair (idx / valid bit-equal?), then the tracker's
unique-match count for the separate and the folded setup (M3S_TRACK_FOLD_SETUP), each run three times, with the
byte map's population counted independently on the host (unique(idx[valid])) for reference."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "lightweight-mast3r-slam_amd"))
import torch  # noqa: E402

from m3s.config import config, reset_config  # noqa: E402
from m3s.frame import Frame, Keyframes  # noqa: E402
from m3s.matching import match  # noqa: E402
from m3s.sim3 import Sim3  # noqa: E402
from m3s.synthetic import SyntheticModel, make_pair  # noqa: E402
import m3s.tracker as T  # noqa: E402
from m3s.tracker import FrameTracker  # noqa: E402

_cap = {}
_orig = T.mast3r_match_asymmetric


def _capture(*a, **k):
    out = _orig(*a, **k)
    _cap["idx"], _cap["valid"] = out[0], out[1]
    return out


T.mast3r_match_asymmetric = _capture

H = W = 512
P = make_pair(H, W, seed=2)
X, D = P["X"].cuda(), P["D"].cuda()
res = [match(X[:1], X[1:], D[:1], D[1:]) for _ in range(3)]
for r in res[1:]:
    print("match repeat: idx equal", torch.equal(r[0], res[0][0]), "valid equal", torch.equal(r[1], res[0][1]),
          "idx diffs", int((r[0] != res[0][0]).sum()), flush=True)

for fold in ("0", "1", "0", "1"):
    os.environ["M3S_TRACK_FOLD_SETUP"] = fold
    for rep in range(2):
        reset_config()
        model = SyntheticModel([P], "cuda")
        kf = Frame(0, (H, W))
        kf.T_WC = Sim3.Identity(1, device="cuda")
        kf.update_pointmap(P["Xk"].cuda(), P["Ck"].cuda())
        kfs = Keyframes()
        kfs.append(kf)
        tr = FrameTracker(model, kfs, "cuda")
        frame = Frame(1, (H, W), T_WC=Sim3.Identity(1, device="cuda"))
        tr.track(frame)
        r = tr.last_result
        idx = _cap["idx"].reshape(-1)
        v = _cap["valid"].reshape(-1).bool()
        host_unique = int(torch.unique(idx[v]).numel())
        print(f"fold={fold} rep={rep}: cost {r.cost:.6f} iters {r.iters} status {r.status} n_valid {r.n_valid_opt} "
              f"{r.n_valid_kf} n_unique {r.n_unique} host unique {host_unique} idx sum {int(idx.sum())}", flush=True)
