"""Child process of tests/test_gpu_ba.py::test_rccl_all_reduce_path_equals_unsharded (not collected by pytest).

Initialises torch.distributed with the "nccl" backend (RCCL on ROCm) at world size 1 BEFORE any other GPU call,
runs the edge-sharded BA (m3s.dist_ba.gauss_newton_sharded: linearise -> dist.all_reduce of the fp64 edge-sum
table -> solve, per iteration) on a 12-keyframe graph and compares it with the unsharded
mast3r_slam_backends.gauss_newton_rays bit for bit. Prints RCCL_BA_OK on success."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "lightweight-mast3r-slam_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

dev = torch.device("cuda", 0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
assert dist.get_backend() == "nccl"

import mast3r_slam_backends as B  # noqa: E402
from m3s.config import config  # noqa: E402
from m3s.dist_ba import gauss_newton_sharded  # noqa: E402
from m3s.synthetic import make_graph, two_way  # noqa: E402

calls = {"n": 0, "bytes": 0}
_all_reduce = dist.all_reduce


def counting_all_reduce(t, *a, **k):
    assert t.is_cuda and t.dtype == torch.float64
    calls["n"] += 1
    if t.numel() > 1:
        calls["bytes"] = t.numel() * 8
    return _all_reduce(t, *a, **k)


dist.all_reduce = counting_all_reduce

G = make_graph(n_kf=12, H=48, W=64, seed=5)
ii, jj, idx, valid, Q = (t.to(dev) for t in two_way(G))
Xs, Cs = G["Xs"].to(dev).contiguous(), G["Cs"][..., 0].to(dev).contiguous()
c = config["local_opt"]
iters = 10
T_sh = G["Twc0"].to(dev).clone()
dx_sh = gauss_newton_sharded("rays", T_sh, Xs, Cs, ii, jj, idx, valid, Q, c, iters, 0.0)[0]
torch.cuda.synchronize()
# one all-reduce of the edge-sum table per iteration + the run's one-element stall decision (run_sharded)
assert calls["n"] == iters + 1, f"expected {iters + 1} all-reduces, saw {calls['n']}"

T_un = G["Twc0"].to(dev).clone()
dx_un = B.gauss_newton_rays(T_un, Xs, G["Cs"].to(dev).contiguous(), ii, jj, idx.contiguous(), valid.contiguous(),
                            Q.contiguous(),
                            c["sigma_ray"], c["sigma_dist"], c["C_conf"], c["Q_conf"], iters, 0.0)[0]
torch.cuda.synchronize()
assert torch.isfinite(T_sh).all()
assert torch.equal(T_sh, T_un), (T_sh - T_un).abs().max().item()
assert torch.equal(dx_sh, dx_un), (dx_sh - dx_un).abs().max().item()
print(f"RCCL_BA_OK all_reduces={calls['n']} bytes_each={calls['bytes']} max|dT|="
      f"{(T_sh - G['Twc0'].to(dev)).abs().max().item():.3e}", flush=True)
dist.destroy_process_group()
