"""BA experiment: per-iteration linearize / solve time (HIP-event spans in libm3s) on a synthetic graph.
usage: python scripts/ba_exp.py [K] [H] [W] [iters]"""
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
from m3s.synthetic import make_graph  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 64
H = int(sys.argv[2]) if len(sys.argv) > 2 else 384
W = int(sys.argv[3]) if len(sys.argv) > 3 else 512
iters = int(sys.argv[4]) if len(sys.argv) > 4 else 10
dev = torch.device("cuda")
t0 = time.time()
G = make_graph(n_kf=K, H=H, W=W, seed=1, device="cpu")
print(f"graph K={K} {H}x{W} built in {time.time() - t0:.1f}s", flush=True)
ii = torch.cat((G["ii"], G["jj"])).to(dev)
jj = torch.cat((G["jj"], G["ii"])).to(dev)
idx = torch.cat((G["idx"], G["idx"].flip(1))).to(dev).contiguous()
valid = torch.cat((G["valid"], G["valid"].flip(1)))[..., 0].to(dev).contiguous()
Q = torch.cat((G["Q"], G["Q"].flip(1)))[..., 0].to(dev).contiguous()
Xs, Cs = G["Xs"].to(dev).contiguous(), G["Cs"][..., 0].to(dev).contiguous()
E = ii.shape[0]
cfg = ba_config("rays", config["local_opt"])
lib = _lib.load()
for rep in range(2):
    Twc = G["Twc0"].to(dev).contiguous()
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
    gb = E * H * W * 45 / 1e6  # MB -> MB/ms = GB/s
    print(f"rep {rep}: E={E} {el / iters * 1e3:.3f} ms/iter  lin {out['ba_linearize']:.3f} ms ({gb / out['ba_linearize']:.0f} GB/s "
          f"alg)  solve {out['ba_solve']:.3f} ms  edges/s {E * iters / el:.0f}", flush=True)

if hasattr(lib, "m3s_debug_chol_stamps"):
    buf = (ctypes.c_ulonglong * 1024)()
    lib.m3s_debug_chol_stamps(buf)
    n = (K - 1) * 7
    npan = min(64, (n + 63) // 64)
    names = {1: "loaded", 2: "diag look-ahead", 3: "L0", 4: "L1", 5: "L2", 6: "L3", 7: "chain end", 8: "X look-ahead",
             9: "T0", 10: "T1", 11: "T2", 12: "T3", 13: "synced", 14: "stored"}
    for sel in (range(1, 2), range(npan // 2, npan // 2 + 1), range(npan - 1, npan)):
        for p in sel:
            t0 = buf[p * 16]
            print(f"panel {p}: " + "  ".join(f"{nm}={(buf[p * 16 + k] - t0) / 100.0:.2f}" for k, nm in names.items()))
    gaps = [(buf[(p + 1) * 16] - buf[p * 16 + 14]) / 100.0 for p in range(npan - 1)]
    print(f"gap from panel-block-0 end to next launch's block-0 start: mean {sum(gaps) / len(gaps):.2f} us")
