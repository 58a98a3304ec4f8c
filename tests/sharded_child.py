"""Child process of tests/test_gpu_ba.py::test_sharded_hip_path_world2 (not collected by pytest).

One rank of a world-size-2 gloo process group, both ranks on cuda:0 (the one-GPU box). Runs the product's sharded
BA (m3s.dist_ba.gauss_newton_sharded -> HipShard over libm3s.so + run_sharded: linearise the rank's edge range ->
all-reduce the fp64 edge-sum table -> replicated solve) on a 48-keyframe graph in rays and calib mode, fresh and with
record reuse (a RecordCache: the first call packs every shard edge, the second none), and the unsharded
mast3r_slam_backends.gauss_newton_* on the same inputs. Saves everything to OUT_DIR/rank<r>.npz; the parent
compares ranks with each other and with the unsharded solve (the reference call site: global_opt.py:123-226)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "lightweight-mast3r-slam_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo", rank=rank, world_size=world)

import mast3r_slam_backends as B  # noqa: E402
from m3s.config import config  # noqa: E402
from m3s.dist_ba import RecordCache, gauss_newton_sharded  # noqa: E402
from m3s.synthetic import make_graph, two_way  # noqa: E402

dev = torch.device("cuda", 0)
H, W = 24, 32
G = make_graph(n_kf=48, H=H, W=W, seed=11)
ii, jj, idx, valid, Q = (t.to(dev).contiguous() for t in two_way(G))
valid, Q = valid.reshape(idx.shape).contiguous(), Q.reshape(idx.shape).contiguous()
Cs3 = G["Cs"].to(dev).contiguous()
Cs = Cs3[..., 0].contiguous()
K = G["K"].to(dev)
c = config["local_opt"]
iters = 6
out = {}
for mode in ("rays", "calib"):
    Xs = G["Xs"].to(dev).contiguous()
    if mode == "calib":
        from m3s.geometry import constrain_points_to_ray

        Xs = constrain_points_to_ray((H, W), Xs, K).contiguous()
    kw = dict(K=K, height=H, width=W) if mode == "calib" else {}
    E, Kp = ii.shape[0], Xs.shape[0]
    T = G["Twc0"].to(dev).clone()
    dx = gauss_newton_sharded(mode, T, Xs, Cs, ii, jj, idx, valid, Q, c, iters, 0.0, **kw)[0]
    out[f"{mode}_T"], out[f"{mode}_dx"] = T.cpu().numpy(), dx.cpu().numpy()
    cache = RecordCache()
    uids = (np.arange(E, dtype=np.int64), np.arange(Kp, dtype=np.int64))
    for n in range(2):
        info = {}
        T = G["Twc0"].to(dev).clone()
        dx = gauss_newton_sharded(mode, T, Xs, Cs, ii, jj, idx, valid, Q, c, iters, 0.0, reuse=uids, cache=cache,
                                  info=info, **kw)[0]
        out[f"{mode}_reuse{n}_T"], out[f"{mode}_reuse{n}_dx"] = T.cpu().numpy(), dx.cpu().numpy()
        out[f"{mode}_reuse{n}_packed"] = np.array(info["packed_edges"])
    cache.release()
    T = G["Twc0"].to(dev).clone()
    if mode == "rays":
        dx = B.gauss_newton_rays(T, Xs, Cs3, ii, jj, idx, valid, Q, c["sigma_ray"], c["sigma_dist"], c["C_conf"],
                                 c["Q_conf"], iters, 0.0)[0]
    else:
        dx = B.gauss_newton_calib(T, Xs, Cs3, K, ii, jj, idx, valid, Q, H, W, c["pixel_border"], c["depth_eps"],
                                  c["sigma_pixel"], c["sigma_depth"], c["C_conf"], c["Q_conf"], iters, 0.0)[0]
    out[f"{mode}_un_T"], out[f"{mode}_un_dx"] = T.cpu().numpy(), dx.cpu().numpy()
    out["E"] = np.array(E)
out["Twc0"] = G["Twc0"].numpy()
torch.cuda.synchronize()
np.savez(os.path.join(os.environ["OUT_DIR"], f"rank{rank}.npz"), **out)
dist.barrier()
dist.destroy_process_group()
print(f"SHARDED_OK rank {rank}", flush=True)
