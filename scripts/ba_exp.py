"""BA experiment: per-iteration linearize / solve time (HIP-event spans in libm3s) on a synthetic graph.
usage: python scripts/ba_exp.py [K] [H] [W] [iters] [graph: circle|chess|euroc] [mode: rays|calib]"""
import ctypes
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "lightweight-mast3r-slam_amd"))
import torch  # noqa: E402

from m3s import _lib  # noqa: E402
from m3s.config import config  # noqa: E402
from m3s.dist_ba import HipShard, ba_config, run_sharded  # noqa: E402
from m3s.synthetic import chess_poses, euroc_poses, make_graph, make_traj_graph  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 64
H = int(sys.argv[2]) if len(sys.argv) > 2 else 384
W = int(sys.argv[3]) if len(sys.argv) > 3 else 512
iters = int(sys.argv[4]) if len(sys.argv) > 4 else 10
graph = sys.argv[5] if len(sys.argv) > 5 else "circle"
mode = sys.argv[6] if len(sys.argv) > 6 else "rays"
dev = torch.device("cuda")
t0 = time.time()
if graph in ("chess", "euroc"):  # SURVEY §8(d) C5 / C4 trajectories, built on the GPU
    G = make_traj_graph((chess_poses if graph == "chess" else euroc_poses)(K), H, W, seed=1, device=dev)
    ii, jj, idx = G["ii"], G["jj"], G["idx"].contiguous()
    valid, Q = G["valid"][..., 0].contiguous(), G["Q"][..., 0].contiguous()
else:
    G = make_graph(n_kf=K, H=H, W=W, seed=1, device="cpu")
    ii = torch.cat((G["ii"], G["jj"])).to(dev)
    jj = torch.cat((G["jj"], G["ii"])).to(dev)
    idx = torch.cat((G["idx"], G["idx"].flip(1))).to(dev).contiguous()
    valid = torch.cat((G["valid"], G["valid"].flip(1)))[..., 0].to(dev).contiguous()
    Q = torch.cat((G["Q"], G["Q"].flip(1)))[..., 0].to(dev).contiguous()
print(f"graph {graph} K={K} {H}x{W} built in {time.time() - t0:.1f}s", flush=True)
Xs, Cs = G["Xs"].to(dev).contiguous(), G["Cs"][..., 0].to(dev).contiguous()
if mode == "calib":  # global_opt.py:163-201: the calib solve sees the points constrained to their rays
    from m3s.geometry import constrain_points_to_ray

    Xs = constrain_points_to_ray((H, W), Xs, G["K"].to(dev)).contiguous()
E = ii.shape[0]
cfg = ba_config(mode, config["local_opt"], K=G["K"], height=H, width=W)
lib = _lib.load()
for rep in range(2):
    Twc = G["Twc0"].to(dev).clone()  # gauss_newton mutates Twc in place: never the graph's own initial poses
    shard = HipShard(cfg, Twc, Xs, Cs, ii, jj, idx, valid, Q, 0.0, 0, E)
    torch.cuda.synchronize()
    lib.m3s_timing_reset()
    lib.m3s_timing_enable(1)
    t0 = time.perf_counter()
    run_sharded(shard, iters)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    lib.m3s_timing_enable(0)
    out = {}
    for name in ("ba_linearize", "ba_solve"):
        ms, cnt = ctypes.c_double(), ctypes.c_int()
        _lib.check(lib.m3s_timing_query(name.encode(), ms, cnt))
        out[name] = ms.value / max(cnt.value, 1)
    import hashlib
    twc_hash = hashlib.sha1(Twc.cpu().numpy().tobytes()).hexdigest()[:12]
    info = (ctypes.c_int * 13)()
    _lib.check(lib.m3s_ba_plan_info(ctypes.byref(shard.plan), info))
    # the linearisation's compulsory bytes per launch (bench.py ba roofline): 16 B record per point and
    # edge + 12 B X_j per point and target keyframe + 17 partial / edge-sum rows of 288 B per edge
    gb = (16 * H * W * E + 12 * H * W * info[5] + 17 * 288 * E) / 1e6  # MB -> MB/ms = GB/s
    print(f"rep {rep}: Twc sha1 {twc_hash} E={E} {el / iters * 1e3:.3f} ms/iter  lin {out['ba_linearize']:.3f} ms ({gb / out['ba_linearize']:.0f} GB/s "
          f"compulsory)  solve {out['ba_solve']:.3f} ms  edges/s {E * iters / el:.0f}  wide steps {info[3]} "
          f"of {info[2]} levels", flush=True)


if hasattr(lib, "m3s_debug_sp_stamps"):  # M3S_SP_STAMPS build: phases of the last factor launch
    buf = (ctypes.c_ulonglong * 4096)()
    lib.m3s_debug_sp_stamps(buf)
    st = _lib.ba_pattern_stats(ii.cpu().numpy(), jj.cpu().numpy(), Xs.shape[0])
    nlev = st[1]
    t = [(buf[k] - buf[0]) / 100.0 for k in range(5 + 2 * nlev)]  # us (100 MHz)
    steps = [t[2 + l] - t[1 + l] for l in range(nlev + 1)]
    print(f"factor stamps: nlev {nlev} blocks {st[0]} groups {st[2]} sources {st[3]} sidx {st[4]} "
          f"pull groups {st[5]}: prologue {t[1]:.1f} us, factor {t[2 + nlev] - t[1]:.1f} us, "
          f"back {t[3 + 2 * nlev] - t[2 + nlev]:.1f} us, tail {t[4 + 2 * nlev] - t[3 + 2 * nlev]:.1f} us, "
          f"total {t[4 + 2 * nlev]:.1f}")
    if all(buf[2 + l] != 0 for l in range(nlev)):  # level stamps exist only in the level-synchronous build
        print("steps:", " ".join(f"{x:.2f}" for x in steps))
    # back substitution: stamps only after barriers (runs of single-column levels share one), root level first
    bs = [(buf[3 + nlev + (nlev - 1 - l)] - buf[0]) / 100.0 for l in range(nlev - 1, -1, -1)]
    prev, segs = t[2 + nlev], []
    for l, x in zip(range(nlev - 1, -1, -1), bs):
        if buf[3 + nlev + (nlev - 1 - l)] != 0 and x >= prev:
            segs.append(f"L{l}:{x - prev:.2f}")
            prev = x
    print("back (level: us since the previous barrier):", " ".join(segs))
    # dataflow build (flow schedule): per-task wait-done / end stamps of the factor lists, per-column end stamps of
    # the back substitution; per wave the time spent waiting vs working, and the wave-0 timeline
    info = (ctypes.c_int * 13)()
    _lib.check(lib.m3s_ba_plan_info(ctypes.byref(shard.plan), info))
    if os.environ.get("M3S_BA_FLOW", "1") != "0" and buf[1000] != 0:
        ts = [(buf[1000 + k] - buf[0]) / 100.0 for k in range(2000)]
        n = max(k for k in range(1000) if buf[1001 + 2 * k] != 0) + 1
        f0 = t[1]
        print(f"flow: {n} factor tasks; factor phase ends {t[2 + nlev]:.1f} us, back ends {t[3 + 2 * nlev]:.1f} us")
        bt = [(buf[3000 + k] - buf[0]) / 100.0 for k in range(1000) if buf[3000 + k] != 0]
        print("back columns stamped:", len(bt), "last", f"{max(bt):.1f}" if bt else "-")
        prev = f0
        line = []
        for k in range(n):
            if ts[2 * k] < prev - 0.05:  # next wave's list starts (stamps restart earlier)
                break
            line.append(f"{ts[2 * k] - prev:.2f}/{ts[2 * k + 1] - ts[2 * k]:.2f}")
            prev = ts[2 * k + 1]
        print("wave 0 tasks (wait/work us):", " ".join(line))
