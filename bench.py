"""Benchmark: tracked frames/s (match + GN, 512x512 pointmaps) and BA edges/s.

  python bench.py --gpus N --steps K --warmup W
  (N > 1: launched by torch.distributed.run, one rank per GPU, RCCL)

A "step" is one FrameTracker.track() of one frame against its keyframe on synthetic MASt3R-shaped
outputs resident in HBM: fused matching (prep, iterative projection, occlusion, fp16 refine) +
confidence setup + Sim(3) GN to convergence + keyframe pointmap fusion + selection statistics.
Workload = BASELINE.json configs[1] (TUM fr1_room, config/calib.yaml: calibrated mode, tracking
only) at the metric's 512x512 pointmap size. Tracking does not shard (frames are sequential):
at N > 1 every rank tracks its own sequence ("replicas only", weak scaling). The BA leg shards one
synthetic factor graph's edges over the ranks (strong scaling, one RCCL all-reduce per iteration).

Prints ONE JSON line on rank 0.
"""
import argparse
import ctypes
import platform
import glob
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "lightweight-mast3r-slam_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
MFMA_BF16_PEAK_TFLOPS = 2500.0  # MI355X dense bf16 matrix-core peak (no sparsity)
VALU_F32_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: FP32 vector spec


OUT = sys.stdout  # the JSON line's stream (main() points it at the original stdout)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--height", type=int, default=512)
    ap.add_argument("--width", type=int, default=512)
    ap.add_argument("--mode", choices=["calib", "rays"], default="calib")
    ap.add_argument("--ring", type=int, default=6, help="distinct synthetic pairs cycled (ring > L3)")
    ap.add_argument("--ba-kf", type=int, default=256)  # C4/C5: 256-keyframe factor graphs (BA_LEGS)
    ap.add_argument("--ba-iters", type=int, default=10)
    ap.add_argument("--no-ba", action="store_true")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-retrieval", action="store_true")
    ap.add_argument("--no-store", action="store_true", help="skip the SharedKeyframes write-back leg")
    ap.add_argument("--no-peaks", action="store_true", help="skip the measured HBM-copy / FMA peak probes")
    ap.add_argument("--no-kernel-timing", action="store_true",
                    help="diagnostic: no HIP-event spans inside the timed loop (no roofline)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--launch-probe", action="store_true",
                    help="test the N-rank launcher only (gloo, no GPU): rank 0 prints world size and a rank sum")
    return ap.parse_args()


def sync_all(world):
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()


def max_over_ranks(x, world):
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def bench_tracking(args, rank, world, dev):
    from m3s import _lib
    from m3s.config import config
    from m3s.frame import Frame, Keyframes
    from m3s.sim3 import Sim3
    from m3s.synthetic import SyntheticModel, make_pair
    from m3s.tracker import FrameTracker

    H, W = args.height, args.width
    config["use_calib"] = args.mode == "calib"
    t0 = time.time()
    pairs = [make_pair(H, W, seed=1000 * rank + r) for r in range(args.ring)]
    log(f"[rank {rank}] generated {args.ring} synthetic {H}x{W} pairs in {time.time() - t0:.1f}s")
    model = SyntheticModel(pairs, dev)
    kf = Frame(0, (H, W), T_WC=Sim3.Identity(1, device=dev))
    kf.K = pairs[0]["K"].to(dev)
    kf.update_pointmap(pairs[0]["Xk"].to(dev), pairs[0]["Ck"].to(dev))
    kfs = Keyframes()
    kfs.append(kf)
    tracker = FrameTracker(model, kfs, dev)
    lib = _lib.load()

    def step(i):
        # initial pose: the keyframe's (main.py:314-319 hands create_frame the last pose object; track()
        # replaces frame.T_WC rather than writing it, so sharing needs no clone)
        fr = Frame(i, (H, W), T_WC=kf.T_WC)
        return tracker.track(fr)

    for i in range(args.warmup):
        step(i)
    iters = []
    step_s = []
    sync_all(world)
    t0 = time.perf_counter()
    tp = t0
    for i in range(args.steps):
        new_kf, _, reloc = step(args.warmup + i)
        # track() returns once the frame's result is published to the host, so host stamps bracket each
        # frame's device work (the last fusion blocks overlap the next frame's host work)
        tn = time.perf_counter()
        step_s.append(tn - tp)
        tp = tn
        iters.append(tracker.last_result.iters)
        assert not reloc, "synthetic tracking failed"
    sync_all(world)
    elapsed = time.perf_counter() - t0
    # Kernel durations: the same K steps again with HIP-event spans around every launch (libm3s,
    # on the launch stream). The event records cost host time in this sync-bound loop (~15%), so
    # they stay out of the pass that produces `value`.
    kern = {}
    if not args.no_kernel_timing:
        lib.m3s_timing_reset()
        lib.m3s_timing_enable(1)
        for i in range(args.steps):
            step(args.warmup + args.steps + i)
        sync_all(world)
        lib.m3s_timing_enable(0)
        for name in ("prep_rays", "proj_occlusion", "refine_lin", "track_setup", "gn_iters"):
            ms, cnt = _lib.c_double(), _lib.c_int()
            _lib.check(lib.m3s_timing_query(name.encode(), ms, cnt))
            kern[name] = (ms.value, cnt.value)
        lib.m3s_timing_reset()
    elapsed = max_over_ranks(elapsed, world)
    return elapsed, kern, float(np.mean(iters)), H * W, step_s


def bench_configs(args, dev, frames=60, warmup=10):
    """Per-config tracking throughput at each config's own shape, beside the headline C2-shaped
    512x512 line: C1 = one 512x512 synthetic pair, rays (base config), exactly 5 GN iterations (convergence tests
    off); C2 = TUM fr1_room, 512x384 calib, GN to convergence. Host-stamped per-frame wall, median and frames/s."""
    from m3s.config import config
    from m3s.frame import Frame, Keyframes
    from m3s.sim3 import Sim3
    from m3s.synthetic import SyntheticModel, make_pair
    from m3s.tracker import FrameTracker

    out = {}
    for name, H, W, calib, fixed in (("C1", 512, 512, False, 5), ("C2", 384, 512, True, None)):
        config["use_calib"] = calib
        saved = dict(config["tracking"])
        if fixed:
            config["tracking"].update(max_iters=fixed, rel_error=0.0, delta_norm=0.0)
        try:
            pairs = [make_pair(H, W, seed=700 + r) for r in range(args.ring)]
            model = SyntheticModel(pairs, dev)
            kf = Frame(0, (H, W), T_WC=Sim3.Identity(1, device=dev))
            kf.K = pairs[0]["K"].to(dev)
            kf.update_pointmap(pairs[0]["Xk"].to(dev), pairs[0]["Ck"].to(dev))
            kfs = Keyframes()
            kfs.append(kf)
            tr = FrameTracker(model, kfs, dev)
            st, its = [], []
            for i in range(warmup + frames):
                t0 = time.perf_counter()
                _, _, reloc = tr.track(Frame(i + 1, (H, W), T_WC=kf.T_WC))
                st.append(time.perf_counter() - t0)
                its.append(tr.last_result.iters)
                assert not reloc, "synthetic tracking failed"
            torch.cuda.synchronize()
            med = float(np.median(st[warmup:]))
            out[name] = {"frames_per_s": 1.0 / med, "median_ms": med * 1e3, "shape": [H, W],
                         "mode": "calib" if calib else "rays", "gn_iters_mean": float(np.mean(its[warmup:]))}
        finally:
            config["tracking"].clear()
            config["tracking"].update(saved)
    config["use_calib"] = args.mode == "calib"
    return out


def bench_store(args, dev, frames=60, warmup=10):
    """tracking through the reference's multi-process keyframe store (m3s.frame.SharedKeyframes =
    frame.py:220-327: share_memory_ buffers behind a Manager RLock, 512x512, the reference's 1024-dim feat / pos
    record). Per-frame wall (median, host stamps as the headline) with the fused in-slot write-back (the fusion
    kernel writes X / C / N / N_updates / is_dirty into the slot) and with tracker.py:101's full-record __setitem__
    copy (img, uimg on the host, X, C, feat, pos, T_WC, counters) for comparison; and the single-process store."""
    import multiprocessing as mp

    from m3s.config import config
    from m3s.frame import Frame, Keyframes, SharedKeyframes
    from m3s.sim3 import Sim3
    from m3s.synthetic import SyntheticModel, make_pair
    from m3s.tracker import FrameTracker

    H, W = args.height, args.width
    config["use_calib"] = args.mode == "calib"
    pairs = [make_pair(H, W, seed=500 + r) for r in range(args.ring)]
    manager = mp.get_context("spawn").Manager()
    out = {}
    try:
        for label in ("slot_writeback", "full_copy", "single_process"):
            model = SyntheticModel(pairs, dev)
            kf = Frame(0, (H, W), T_WC=Sim3.Identity(1, device=dev))
            kf.K = pairs[0]["K"].to(dev)
            kf.update_pointmap(pairs[0]["Xk"].to(dev), pairs[0]["Ck"].to(dev))
            if label == "single_process":
                kfs = Keyframes()
            else:
                kfs = SharedKeyframes(manager, H, W, buffer=8, device=dev)
                kf.img = torch.zeros(3, H, W, device=dev)
                kf.uimg = torch.zeros(H, W, 3)
                kf.img_shape = torch.tensor([[H, W]], dtype=torch.int, device=dev)
                kf.img_true_shape = kf.img_shape.clone()
                kf.feat = torch.zeros(1, kfs.num_patches, kfs.feat_dim, device=dev)
                kf.pos = torch.zeros(1, kfs.num_patches, 2, dtype=torch.long, device=dev)
                if config["use_calib"]:
                    kfs.set_intrinsics(kf.K)
            kfs.append(kf)
            tr = FrameTracker(model, kfs, dev)
            tr.slot_writeback = label != "full_copy"
            T0 = kfs[0].T_WC if label != "single_process" else kf.T_WC
            st = []
            for i in range(warmup + frames):
                t0 = time.perf_counter()
                _, _, reloc = tr.track(Frame(i + 1, (H, W), T_WC=T0))
                st.append(time.perf_counter() - t0)
                assert not reloc, "synthetic tracking failed"
            torch.cuda.synchronize()
            out[label] = float(np.median(st[warmup:])) * 1e3
    finally:
        manager.shutdown()
    return {"median_ms": out, "saved_ms_per_frame": out["full_copy"] - out["slot_writeback"],
            "frames": frames, "shape": [H, W],
            "note": "track() per frame through SharedKeyframes (Manager RLock, share_memory_ slots): fused in-slot "
                    "write-back vs the reference's full-record copy (tracker.py:101, frame.py:271-289); "
                    "single_process = the Keyframes list store of the headline"}


def roofline(kern, N, gn_iters_mean):
    """Algorithmic bytes / flops per launch / measured HIP-event duration."""
    per_px_bytes = {
        # X11 in, rays9 out; + the D11 f32 -> f16 descriptor conversion, which runs in prep_rays (csrc/matching.hip
        # prep_rays_kernel; DESIGN.md §4: 192 B/px)
        "prep_rays": 12 + 36 + 96 + 48,
        "proj_occlusion": 12 + 8 + 36 + 12 + 8 + 1,  # X21, idx_init, rays9, X11 gather, p1, valid (77 B/px)
        "refine_lin": 48 + 96 + 8 + 8,  # D11 f16 centre rows, D21 f32, p1, idx
        "track_setup": 8 + 1 + 12 + 4 + 4 + 12 + 4 + 4 + 32,  # idx, valid, Xf, Cf, Qff, Xk, Ck, Qkf -> rec
        "gn_iters": 32 * gn_iters_mean,  # 32 B record per point per iteration
    }
    out = {}
    for k, (ms, cnt) in kern.items():
        if cnt == 0:
            continue
        avg_s = ms / cnt / 1e3
        out[k] = {"avg_us": avg_s * 1e6, "GBps": per_px_bytes[k] * N / avg_s / 1e9}
    refine_flops = 245 * 24 * 2 * N  # half products + half adds
    if "refine_lin" in out:
        out["refine_lin"]["TFLOPs"] = refine_flops / (out["refine_lin"]["avg_us"] * 1e-6) / 1e12
    return out


def kernel_table(rl, N, gn_iters_mean):
    """Per kernel: HIP-event duration, algorithmic bytes and their rate, and beside them the HBM traffic per launch of
    the newest committed PMC summary (profiles/r??_pmc.json, FETCH_SIZE x2 + WRITE_SIZE) over the same duration, so
    the two rates can be compared kernel by kernel (gn_iters: per frame, all iterations in one launch)."""
    alg = {"prep_rays": 192, "proj_occlusion": 77, "refine_lin": 160, "track_setup": 80, "gn_iters": 32 * gn_iters_mean}
    out = {}
    for k, v in rl.items():
        e = pmc_entry(k)
        t = e["traffic_bytes"] if e else None
        out[k] = {"avg_us": round(v["avg_us"], 2), "alg_MB": round(alg[k] * N / 1e6, 2), "alg_GBps": round(v["GBps"], 1),
                  "pmc_MB": round(t / 1e6, 2) if t else None,
                  "pmc_GBps": round(t / (v["avg_us"] * 1e-6) / 1e9, 1) if t else None,
                  "pmc_source": e["file"] if e else None}
    return out


KERNEL_SYMBOL = {"prep_rays": "prep_rays_kernel", "proj_occlusion": "proj_occlusion_kernel",
                 "refine_lin": "refine_tile_kernel", "track_setup": "track_setup_kernel", "gn_iters": "gn_loop_kernel"}


def pmc_entry(name, pattern="r[0-9][0-9]_pmc.json"):
    """The newest committed rocprofv3 PMC summary entry of kernel `name` (profiles/<round>_*pmc.json,
    FETCH_SIZE x2 + WRITE_SIZE per launch, scripts/profile_summary.py) with its file name; None if absent."""
    files = sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", pattern)))
    if not files:
        return None
    for k, v in json.load(open(files[-1])).items():
        if KERNEL_SYMBOL.get(name, name) in k:
            return dict(v, file=os.path.basename(files[-1]))
    return None


def pmc_traffic(name, pattern="r[0-9][0-9]_pmc.json"):
    e = pmc_entry(name, pattern)
    return e["traffic_bytes"] if e else None


# SURVEY.md §8(d) BA legs: C5 = 256-keyframe chess graph, calib, 512x384 (7-Scenes shape); C4 = EuRoC-shaped
# graph (MH_02_easy trajectory), rays (eval_no_calib), 512x320
# C5 = 7-Scenes chess (384x512 calib) + ETH3D (512x304 calib; its ground truth is not in the reference, so the chess
# trajectory carries the ETH3D image shape); C4 = EuRoC MH_02 (320x512 rays)
BA_LEGS = {"C5": dict(traj="chess", mode="calib", H=384, W=512), "C4": dict(traj="euroc", mode="rays", H=320, W=512),
           "C5e": dict(traj="chess", mode="calib", H=304, W=512)}
BA_PMC_TAG = {"C5": "_ba", "C4": "_ba_c4", "C5e": "_ba_eth3d"}
# Compulsory HBM bytes of the build's BA loop. Once per call the pack streams, per point and edge,
# valid 1 + idx 8 + Q 4 in and the record out, and gathers from the keyframes' X (12 B) and C (4 B), compulsory once
# per keyframe point. Every GN iteration then streams only the record of each point of each edge and the 12-B X_j of
# each point of each distinct target keyframe (the edges of one target share that slab in L2), plus per edge its
# chunk partials (36 doubles written by ba_lin, read back by ba_edge) and its edge-sum row. Records (ba.hip
# pack_record): calib 12 B {u | v << 16, log z_i, sw}, points 16 B {X_i, sw}, rays 16 B {X_i / |X_i|, sw} + 4 B |X_i|.
BA_PACK_IN_BYTES = 13
BA_PACK_KF_BYTES = 16
BA_REC_BYTES = {"calib": 12, "points": 16, "rays": 20}
BA_XJ_BYTES = 12
BA_SUM_BYTES = 36 * 8


def ba_plan_info(lib, plan):
    from m3s import _lib

    info = (ctypes.c_int * 13)()
    _lib.check(lib.m3s_ba_plan_info(ctypes.byref(plan), info))
    keys = ("chunks", "factor_blocks", "levels", "wide_steps", "dense", "targets", "edges", "poses")
    return dict(zip(keys, list(info)[:len(keys)]))


def bench_ba(args, rank, world, dev, leg):
    from m3s import _lib
    from m3s.config import config
    from m3s.dist_ba import HipShard, ba_config, run_sharded, shard_range
    from m3s.geometry import constrain_points_to_ray
    from m3s.synthetic import chess_poses, euroc_poses, make_traj_graph

    L = BA_LEGS[leg]
    H, W, mode = L["H"], L["W"], L["mode"]
    poses = (chess_poses if L["traj"] == "chess" else euroc_poses)(args.ba_kf)
    G = make_traj_graph(poses, H, W, seed=1, device=dev)  # same seed on every rank: identical graphs
    ii, jj, idx = G["ii"], G["jj"], G["idx"].contiguous()
    valid, Q = G["valid"][..., 0].contiguous(), G["Q"][..., 0].contiguous()
    Xs, Cs = G["Xs"].contiguous(), G["Cs"][..., 0].contiguous()
    if mode == "calib":  # global_opt.py:163-201: the calib solve sees the points constrained to their rays
        Xs = constrain_points_to_ray((H, W), Xs, G["K"]).contiguous()
    Twc0 = G["Twc0"].clone()  # the stated initial poses; every call starts from a fresh copy
    E = ii.shape[0]
    N = H * W
    e0, e1 = shard_range(E, rank, world)
    cfg = ba_config(mode, config["local_opt"], K=G["K"], height=H, width=W)
    lib = _lib.load()
    # ba_lin_pack: the first linearisation of a call that packs every edge builds the records itself (the separate
    # ba_pack launch only runs for partial packs: record reuse)
    names = ("ba_pack", "ba_lin_pack", "ba_linearize", "ba_solve")

    def run(iters, timed_kernels=False):
        # the whole gauss_newton call is timed: plan (rank remap, symbolic factorisation, per-call
        # point records of this rank's edges) + iters x (linearise, all-reduce, solve, retract)
        Twc = Twc0.clone()  # gauss_newton mutates Twc in place (gn.cpp): never the graph's own initial poses
        sync_all(world)
        if timed_kernels:
            lib.m3s_timing_reset()
            lib.m3s_timing_enable(1)
        t0 = time.perf_counter()
        shard = HipShard(cfg, Twc, Xs, Cs, ii, jj, idx, valid, Q, 0.0, e0, e1)  # delta 0: no early exit
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        run_sharded(shard, iters)
        sync_all(world)
        el = time.perf_counter() - t0
        spans = {}
        if timed_kernels:
            lib.m3s_timing_enable(0)
            for name in names:
                ms, cnt = ctypes.c_double(), ctypes.c_int()
                _lib.check(lib.m3s_timing_query(name.encode(), ms, cnt))
                spans[name] = ms.value / max(cnt.value, 1)
                spans[name + "#"] = cnt.value
        return el, t1 - t0, spans, shard, Twc

    run(1)  # warmup
    el, setup, _, shard, Twc = run(args.ba_iters)
    el = max_over_ranks(el, world)
    setup = max_over_ranks(setup, world)
    _, _, spans, _, Twc2 = run(args.ba_iters, timed_kernels=True)  # HIP-event spans, a second pass
    assert torch.equal(Twc, Twc2), "BA: two calls from the same initial poses differ"
    info = ba_plan_info(lib, shard.plan)
    # roofline of the dominant kernel (the linearisation) at the build's compulsory bytes per iteration
    lin_s = spans["ba_linearize"] * 1e-3
    n_e = e1 - e0
    rec_bytes = BA_REC_BYTES[mode]
    alg = n_e * N * rec_bytes + info["targets"] * N * BA_XJ_BYTES + n_e * (2 * info["chunks"] + 1) * BA_SUM_BYTES
    pmc = pmc_entry(f"ba_lin_kernel<{1 if mode == 'rays' else 2}, false>", pattern=f"r[0-9][0-9]{BA_PMC_TAG[leg]}_pmc.json")
    traffic = pmc["traffic_bytes"] if pmc else None
    roof = {"kernel": "ba_lin_kernel + ba_edge_kernel", "bound": "hbm", "achieved": alg / lin_s / 1e9,
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": alg / lin_s / 1e9 / HBM_PEAK_GBS,
            "traffic": traffic, "traffic_over_alg": (traffic / alg) if traffic else None,
            "traffic_source": pmc["file"] if pmc else None, "avg_us": spans["ba_linearize"] * 1e3,
            "alg_bytes": f"{rec_bytes} B record x {N} points x {n_e} edges + {BA_XJ_BYTES} B X_j x {N} points x "
                         f"{info['targets']} target keyframes + {2 * info['chunks'] + 1} x {BA_SUM_BYTES} B partial/"
                         f"edge-sum rows x {n_e} edges per launch (compulsory traffic, DESIGN.md §4)"}
    # the backend's next solve (main.py:150-155) on the same graph after tracking re-fused the newest keyframe, with
    # record reuse (m3s_ba_make_plan_reuse via RecordCache): only that keyframe's edges repack; the calls alternate
    # two versions of its points, so every timed call sees it changed
    from m3s.dist_ba import RecordCache

    cache = RecordCache()
    uids = (np.arange(E, dtype=np.int64), np.arange(args.ba_kf, dtype=np.int64))
    Xs_b = Xs.clone()
    Xs_b[-1] *= 1.0001

    def run_reuse(X_in, iters):
        Twc = Twc0.clone()
        sync_all(world)
        t0 = time.perf_counter()
        sh = HipShard(cfg, Twc, X_in, Cs, ii, jj, idx, valid, Q, 0.0, e0, e1, reuse=uids, cache=cache)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        run_sharded(sh, iters)
        sync_all(world)
        return time.perf_counter() - t0, t1 - t0, sh.reuse_info(), Twc

    run_reuse(Xs, args.ba_iters)  # fills the cache (every edge packs)
    run_reuse(Xs_b, args.ba_iters)
    r_el, r_setup, r_info = [], [], None
    for X_in in (Xs, Xs_b):
        a_el, a_setup, r_info, Twc_r = run_reuse(X_in, args.ba_iters)
        r_el.append(max_over_ranks(a_el, world))
        r_setup.append(max_over_ranks(a_setup, world))
    Twc_fresh = Twc0.clone()
    fresh = HipShard(cfg, Twc_fresh, Xs_b, Cs, ii, jj, idx, valid, Q, 0.0, e0, e1)
    run_sharded(fresh, args.ba_iters)
    torch.cuda.synchronize()
    assert torch.equal(Twc_r, Twc_fresh), "BA: record reuse differs from a fresh solve"
    reuse = {"ms_per_call": 1e3 * sum(r_el) / len(r_el), "ms_setup": 1e3 * sum(r_setup) / len(r_setup),
             "packed_edges": r_info[0], "changed_keyframes": r_info[1], "shard_edges": e1 - e0,
             "note": "the next backend solve after the newest keyframe was re-fused (its X changed), record reuse "
                     "(m3s_ba_make_plan_reuse): only its edges repack; poses bit-identical to a fresh solve"}
    cache.release()
    del fresh, Xs_b
    fused = spans["ba_lin_pack#"] > 0
    # the pack's cost: its own launch, or what it adds to the first linearisation when fused into it
    ms_pack = spans["ba_lin_pack"] - spans["ba_linearize"] if fused else spans["ba_pack"]
    pack_s = (spans["ba_lin_pack"] if fused else spans["ba_pack"]) * 1e-3
    pack_bytes = n_e * N * (BA_PACK_IN_BYTES + rec_bytes) + args.ba_kf * N * BA_PACK_KF_BYTES
    pack_pmc = pmc_entry(f"ba_pack_kernel<{1 if mode == 'rays' else 2}>",
                         pattern=f"r[0-9][0-9]{BA_PMC_TAG[leg]}_pmc.json")
    out = {"edges_per_s": E * args.ba_iters / el, "n_gpus": world, "keyframes": args.ba_kf, "edges_dir": E,
           "points_per_kf": N, "shape": [H, W], "mode": mode, "trajectory": L["traj"], "iters": args.ba_iters,
           "ms_per_call": el * 1e3, "ms_setup": setup * 1e3, "ms_per_iter": (el - setup) / args.ba_iters * 1e3,
           "ms_pack": ms_pack, "ms_plan_host": max(setup * 1e3 - (0.0 if fused else spans["ba_pack"]), 0.0),
           "ms_first_lin_with_pack": spans["ba_lin_pack"] if fused else None,
           "ms_lin_per_iter": spans["ba_linearize"], "ms_solve_per_iter": spans["ba_solve"],
           "factor": {"blocks": info["factor_blocks"], "levels": info["levels"], "wide_steps": info["wide_steps"],
                      "dense": bool(info["dense"]), "dense_blocks": (args.ba_kf - 1) * args.ba_kf // 2},
           "scaling": "strong", "roofline": roof,
           "pack": {"GBps": (pack_bytes + (alg if fused else 0)) / pack_s / 1e9,
                    "frac": (pack_bytes + (alg if fused else 0)) / pack_s / 1e9 / HBM_PEAK_GBS,
                    "bytes": pack_bytes, "fused_into_first_linearisation": fused,
                    "traffic": None if fused else (pack_pmc["traffic_bytes"] if pack_pmc else None),
                    "note": f"once per call: {BA_PACK_IN_BYTES + rec_bytes} B per point and edge + {BA_PACK_KF_BYTES} B per "
                            f"keyframe point (compulsory)" + ("; fused into the first linearisation (ba_lin_kernel"
                            "<PACK>): GBps counts the pack's and that iteration's compulsory bytes over its time, "
                            "ms_pack what the pack adds to it" if fused else "")},
           "reuse": reuse}
    del G, idx, valid, Q, Xs, Cs, shard
    torch.cuda.empty_cache()
    return out


def ba_cpu_baseline(args, leg="C5", n_kf=8, iters=2):
    """The oracle's gauss_newton (C restatement of gn_kernels.cu, OpenMP over points) on a bounded sample of
    the same workload: the first n_kf keyframes of the leg's trajectory at its full shape."""
    import oracle.oracle as O
    from m3s.config import config
    from m3s.synthetic import chess_poses, euroc_poses, make_traj_graph

    L = BA_LEGS[leg]
    H, W, mode = L["H"], L["W"], L["mode"]
    G = make_traj_graph((chess_poses if L["traj"] == "chess" else euroc_poses)(n_kf), H, W, seed=1, device="cpu")
    Xs = G["Xs"].numpy()
    K = G["K"].numpy()
    if mode == "calib":
        Xs = O.backproject_constrain(Xs, K, (H, W))
    c = config["local_opt"]
    sa, sb = (c["sigma_pixel"], c["sigma_depth"]) if mode == "calib" else (c["sigma_ray"], c["sigma_dist"])
    p = O.ba_params(mode, sa, sb, c["C_conf"], c["Q_conf"], K=K, height=H, width=W, pixel_border=c["pixel_border"],
                    z_eps=c["depth_eps"])
    E = G["ii"].shape[0]
    out = {}
    avail = len(os.sched_getaffinity(0))
    # thread sweep (16 = the box's share, 64, every affinity core) + one thread; value = the best thread count
    legs = [(f"t{t}", t, iters) for t in sorted({t for t in (16, 64, avail) if t <= avail})] + [("one_thread", 1, 1)]
    for label, threads, its in legs:
        O.set_threads(threads)
        t0 = time.perf_counter()
        O.gauss_newton(mode, G["Twc0"].numpy(), Xs, G["Cs"].numpy()[..., 0], G["ii"].numpy(), G["jj"].numpy(),
                       G["idx"].numpy(), G["valid"].numpy()[..., 0], G["Q"].numpy()[..., 0], p, its, 0.0)
        el = time.perf_counter() - t0
        out[label] = {"value": E * its / el, "cores": threads, "seconds": el}
    O.set_threads(min(16, avail))
    best = max((k for k in out if k != "one_thread"), key=lambda k: out[k]["value"])
    share = out.get("t16")
    return {"value": out[best]["value"], "unit": "edges/s", "cores": out[best]["cores"], "kind": "port",
            "threads_sweep": {str(v["cores"]): v["value"] for k, v in out.items() if k != "one_thread"},
            "one_thread": out["one_thread"]["value"], "affinity_cores": avail,
            "box_share_16": share["value"] if share else None,
            "sample": f"{leg} shape ({H}x{W}, {mode}), first {n_kf} keyframes ({E} directed edges) through the oracle's "
                      f"gauss_newton (C, OpenMP): {iters} iterations at "
                      + ", ".join(f"{v['cores']} threads in {v['seconds']:.1f}s" for k, v in out.items() if k != "one_thread")
                      + f", 1 on one thread in {out['one_thread']['seconds']:.1f}s; value = the best thread count "
                      f"({out[best]['cores']})"}


def bench_retrieval(dev):
    """RetrievalDatabase.quantize_custom (retrieval_database.py:96-105) at the reference's
    shapes (64k x 1024 asmk codebook, 300 local features, multiple_assignment 5). Roofline of the fused
    GEMM + block top-k (+ merge) launch pair: matrix-core flops actually issued (3 bf16 products per fp32
    product, 304 padded query rows) against the dense bf16 peak, and the codebook stream against HBM."""
    import torch.nn.functional as F

    from m3s import _lib
    from m3s.retrieval import Codebook

    C, D, M, k = 65536, 1024, 300, 5
    g = torch.Generator(device=dev).manual_seed(0)
    c = F.normalize(torch.randn(C, D, device=dev, generator=g), dim=1)
    q = F.normalize(torch.randn(M, D, device=dev, generator=g), dim=1)
    cb = Codebook(c)
    for _ in range(3):
        cb.quantize(q, k)
    torch.cuda.synchronize()
    reps = 50
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        cb.quantize(q, k)
    e1.record()
    e1.synchronize()
    ms = e0.elapsed_time(e1) / reps
    lib = _lib.load()
    lib.m3s_timing_enable(1)
    lib.m3s_timing_reset()
    for _ in range(reps):
        cb.quantize(q, k)
    torch.cuda.synchronize()
    tot, cnt = _lib.c_double(), _lib.c_int()
    lib.m3s_timing_query(b"quantize_topk", tot, cnt)
    lib.m3s_timing_enable(0)
    kms = tot.value / max(cnt.value, 1)
    mfma_flops = 3 * 2 * ((M + 303) // 304 * 304) * C * D
    def torch_ref():  # the reference's formulation on the same GPU (fp32 GEMM + topk), for context
        l2 = torch.sum(q ** 2, dim=1)[:, None] + torch.sum(c ** 2, dim=1)[None, :] - 2 * (q @ c.mT)
        return torch.topk(l2, k, dim=1, largest=False).indices

    for _ in range(3):
        torch_ref()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(10):
        torch_ref()
    e1.record()
    e1.synchronize()
    achieved = mfma_flops / (kms * 1e-3) / 1e12
    return {"calls_per_s": 1e3 / ms, "ms_per_call": ms, "kernel_ms": kms,
            "shape": {"codebook": [C, D], "queries": M, "k": k},
            "dtype": "bf16 hi/lo split (3 MFMA per fp32 product), fp32 accumulate",
            "roofline": {"kernel": "rq_gemm_topk + rq_merge", "bound": "mfma", "achieved": achieved,
                         "peak": MFMA_BF16_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": achieved / MFMA_BF16_PEAK_TFLOPS,
                         "alg_TFLOPs": 2.0 * M * C * D / (kms * 1e-3) / 1e12,
                         "codebook_GBps": C * D * 4 / (kms * 1e-3) / 1e9},
            "torch_fp32_topk_ms": e0.elapsed_time(e1) / 10}


def measured_peaks(dev):
    """re-measure the peaks on the box — a STREAM-like device copy (torch, 2 x 2 GiB) and a
    v_fma_f32 loop (libm3s peak probe, 4 waves per SIMD on every CU)."""
    from m3s import _lib

    lib = _lib.load()
    n = 1 << 29  # 2 GiB of fp32
    a = torch.empty(n, dtype=torch.float32, device=dev).fill_(1.0)
    b = torch.empty_like(a)
    b.copy_(a)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 10
    e0.record()
    for _ in range(reps):
        b.copy_(a)
    e1.record()
    e1.synchronize()
    hbm = 2 * 4 * n * reps / (e0.elapsed_time(e1) * 1e-3) / 1e9
    del a, b
    out = torch.empty(256, dtype=torch.float32, device=dev)
    blocks, it = 256 * 16, 4096
    stream = _lib.stream_ptr(dev)
    _lib.check(lib.m3s_peak_fma_f32(out.data_ptr(), blocks, it, stream))
    e0.record()
    _lib.check(lib.m3s_peak_fma_f32(out.data_ptr(), blocks, it, stream))
    e1.record()
    e1.synchronize()
    fma = blocks * 256 * it * 8 * 2 / (e0.elapsed_time(e1) * 1e-3) / 1e12
    return {"hbm_copy_GBps": hbm, "fp32_fma_TFLOPs": fma,
            "how": "torch device copy of 2 GiB (read + write bytes) x10; libm3s v_fma_f32 loop, 4096 blocks x 256"}


def frame_roofline(step_s, N, gn_iters_mean, mode):
    """BASELINE.md §3 per tracked frame: bytes = N (233 + 16 + 29 it), flops = N (11760 + 1700 + c it) with
    c = 510 (rays) / 380 (calib); fraction = max(bytes / 8 TB/s, flops / 157.3 TFLOP/s) / t_frame (median)."""
    med = float(np.median(step_s))
    it = gn_iters_mean
    byts = N * (233 + 16 + 29 * it)
    flops = N * (11760 + 1700 + (380 if mode == "calib" else 510) * it)
    t_b, t_f = byts / (HBM_PEAK_GBS * 1e9), flops / (VALU_F32_PEAK_TFLOPS * 1e12)
    return {"median_ms": med * 1e3, "p90_ms": float(np.percentile(step_s, 90)) * 1e3,
            "mean_ms": float(np.mean(step_s)) * 1e3, "max_ms": float(np.max(step_s)) * 1e3,
            "first_ms": [round(float(x) * 1e3, 4) for x in step_s[:3]], "bytes": byts,
            "flops": flops, "bound": "hbm" if t_b > t_f else "valu", "frac": max(t_b, t_f) / med,
            "note": "host-stamped per-frame wall (track() returns once its result is published), ViT excluded"}


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def cpu_baseline(args):
    """Oracle (C restatement + numpy glue) on the host cores, bounded sample of the same workload: frames on
    16, 64 and every affinity core for ~cpu_seconds in all (value = the best), then one frame on one thread."""
    import oracle.oracle as O
    from m3s.synthetic import make_pair

    avail = len(os.sched_getaffinity(0))
    H, W = args.height, args.width
    P = make_pair(H, W, seed=0)
    X, C, D, Q = (P[k].numpy() for k in ("X", "C", "D", "Q"))
    Xk, K = P["Xk"].numpy(), P["K"].numpy()
    I = np.array([0, 0, 0, 0, 0, 0, 1, 1.0])

    def frame():
        idx, valid = O.match(X[:1], X[1:], D[:1], D[1:])
        i = idx[0]
        Qk = np.sqrt(Q[0].reshape(-1)[i] * Q[1].reshape(-1))
        v = valid[0, :, 0] & (Qk > 1.5)
        if args.mode == "calib":
            Xf = O.backproject_constrain(X[0].reshape(1, -1, 3), K, (H, W))[0][i]
            u, vv = np.meshgrid(np.arange(W, dtype=np.float32), np.arange(H, dtype=np.float32), indexing="xy")
            z = Xk[:, 2]
            vm = z > 1e-6
            meas = np.stack((u.reshape(-1), vv.reshape(-1), np.log(np.where(vm, z, 1.0))), -1) * vm[:, None]
            O.track_calib(Xf, Xk, I, I, Qk, v, meas, vm, K, (H, W))
        else:
            O.track_rays(X[0].reshape(-1, 3)[i], Xk, I, I, Qk, v)

    def timed(threads, seconds):
        O.set_threads(threads)
        t0 = time.perf_counter()
        frames = 0
        while True:
            frame()
            frames += 1
            if time.perf_counter() - t0 > seconds or frames >= 50:
                break
        return frames, time.perf_counter() - t0

    # thread sweep: the box's 16-core share, 64, and every core of the affinity mask; `value` is the best of them
    # with its thread count (the OpenMP loops and the numpy glue stop scaling past a few dozen threads)
    counts = sorted({t for t in (16, 64, avail) if t <= avail})
    sweep = {}
    for t in counts:
        frames, el = timed(t, args.cpu_seconds / len(counts))
        sweep[t] = (frames, el)
    best = max(sweep, key=lambda t: sweep[t][0] / sweep[t][1])
    O.set_threads(1)
    t1 = time.perf_counter()
    frame()
    el1 = time.perf_counter() - t1
    O.set_threads(min(16, avail))
    share = sweep.get(16)
    return {"value": sweep[best][0] / sweep[best][1], "unit": "tracked frames/s", "cores": best, "kind": "port",
            "threads_sweep": {str(t): f / e for t, (f, e) in sweep.items()},
            "one_thread": 1.0 / el1, "affinity_cores": avail, "cpu_model": cpu_model(),
            "box_share_16": share[0] / share[1] if share else None,
            "sample": f"tracked frames ({H}x{W}, {args.mode}) through oracle/ (C kernels, OpenMP, + numpy fp64 glue) at "
                      + ", ".join(f"{t} threads: {f} frames in {e:.1f}s" for t, (f, e) in sweep.items())
                      + f"; one frame on one thread in {el1:.1f}s; value = the best thread count ({best})"}


def free_port():
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args):
    """`python bench.py --gpus N` with no launcher around it (WORLD_SIZE unset): start N rank processes of this
    script, one per GPU (LOCAL_RANK = device), rendezvous on 127.0.0.1, and return the worst exit code. The parent
    touches no GPU (torch.cuda.device_count() does not initialise HIP on this image); rank 0 prints the JSON line
    to the inherited stdout. With M3S_BENCH_DEVICE set (the rehearsal of the N-rank path on one GPU, usually with
    M3S_DIST_BACKEND=gloo) every rank runs on that device, so no device count is required."""
    import signal
    import subprocess

    n = args.gpus
    rehearsal = os.environ.get("M3S_BENCH_DEVICE") is not None or args.launch_probe
    if not rehearsal:
        have = torch.cuda.device_count()
        if have < n:
            log(f"bench.py: --gpus {n} needs {n} visible GPUs, this node has {have}; "
                f"set M3S_BENCH_DEVICE=<dev> M3S_DIST_BACKEND=gloo to rehearse {n} ranks on one device")
            return 2
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), M3S_BENCH_LAUNCHER="bench.py")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    log(f"bench.py: launched {n} ranks (pids {[p.pid for p in procs]}) on 127.0.0.1:{port}")
    codes = [None] * n
    try:
        while any(c is None for c in codes):
            for i, p in enumerate(procs):
                if codes[i] is None:
                    codes[i] = p.poll()
            bad = [c for c in codes if c not in (None, 0)]
            if bad:  # one rank failed: its peers would wait for it at their next collective
                for i, p in enumerate(procs):
                    if codes[i] is None:
                        p.send_signal(signal.SIGTERM)
                for i, p in enumerate(procs):
                    if codes[i] is None:
                        try:
                            codes[i] = p.wait(timeout=30)
                        except subprocess.TimeoutExpired:
                            p.kill()
                            codes[i] = p.wait()
                break
            time.sleep(0.2)
    except BaseException:
        for p in procs:
            if p.poll() is None:
                p.kill()
        raise
    worst = max((abs(c) for c in codes), default=0)
    if worst:
        log(f"bench.py: rank exit codes {codes}")
    return worst


def launch_probe(world, rank, args):
    """--launch-probe: the launcher contract without a GPU (CPU test): every rank joins a gloo group, checks
    world == --gpus, all-reduces its rank, and rank 0 prints one JSON line."""
    dist.init_process_group("gloo")
    t = torch.tensor([float(rank + 1)])
    dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({"probe": True, "n_gpus": world, "gpus_arg": args.gpus, "rank_sum": float(t.item()),
                          "launcher": os.environ.get("M3S_BENCH_LAUNCHER", "external")}), file=OUT, flush=True)
    dist.barrier()
    dist.destroy_process_group()


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"bench.py: rank {rank} sees WORLD_SIZE={world} but --gpus {args.gpus}; launch one rank per GPU "
            f"(torch.distributed.run --nproc-per-node {args.gpus}, or plain `python bench.py --gpus {args.gpus}`)")
        sys.exit(2)
    # stdout carries exactly one line, the JSON record: anything else a library prints there (gloo's "[Gloo] Rank ...
    # is connected" lines, RCCL banners) goes to stderr
    global OUT
    OUT = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    if args.launch_probe:
        launch_probe(world, rank, args)
        return
    # M3S_BENCH_DEVICE / M3S_DIST_BACKEND: rehearsal of the N-rank path on a 1-GPU box (all ranks on
    # one device over gloo); the driver's multi-GPU runs use one GPU per rank over RCCL ("nccl").
    ndev = os.environ.get("M3S_BENCH_DEVICE")
    local_dev = int(ndev) if ndev is not None else local
    torch.cuda.set_device(local_dev)
    dev = torch.device("cuda", local_dev)
    if world > 1:
        backend = os.environ.get("M3S_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    import __graft_entry__  # noqa: F401  (sys.path)

    elapsed, kern, gn_iters, N, step_s = bench_tracking(args, rank, world, dev)
    total_frames = args.steps * world
    value = total_frames / elapsed
    rl = roofline(kern, N, gn_iters)
    log(f"[rank {rank}] kernels: {json.dumps(rl)}")
    roof = None
    if rl:
        name, d = max(rl.items(), key=lambda kv: kv[1]["avg_us"] * kern[kv[0]][1])
        if name == "refine_lin":
            roof = {"kernel": name, "bound": "valu", "achieved": d["TFLOPs"], "peak": VALU_F32_PEAK_TFLOPS,
                    "unit": "TFLOP/s", "frac": d["TFLOPs"] / VALU_F32_PEAK_TFLOPS}
        else:
            roof = {"kernel": name, "bound": "hbm", "achieved": d["GBps"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": d["GBps"] / HBM_PEAK_GBS}
        roof["traffic"] = pmc_traffic(name)
        roof["avg_us"] = d["avg_us"]
        roof["timing"] = "HIP events on the launch stream, second pass of the same K steps"
    frame = frame_roofline(step_s, N, gn_iters, args.mode)
    peaks = measured_peaks(dev) if (rank == 0 and not args.no_peaks) else None
    ba = None
    if not args.no_ba:
        ba = bench_ba(args, rank, world, dev, "C5")
        ba["c4"] = bench_ba(args, rank, world, dev, "C4")
        ba["eth3d"] = bench_ba(args, rank, world, dev, "C5e")
    retrieval = bench_retrieval(dev) if (rank == 0 and not args.no_retrieval) else None
    store = bench_store(args, dev) if (rank == 0 and not args.no_store) else None
    configs = bench_configs(args, dev) if (rank == 0 and not args.no_store) else None
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(args)
        if ba is not None:
            ba["cpu_baseline"] = ba_cpu_baseline(args)
    if rank == 0:
        rec = {
            "metric": "tracked frames/s (match+GN, 512x512 pointmaps) @1 GPU; BA edges/s @1/2/4/8",
            "value": value, "unit": "tracked frames/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32 (refine f16, GN accum f64)",
            "data": "synthetic MASt3R-shaped pointmaps/descriptors/confidences (no checkpoint, no dataset)",
            "config": {"workload": f"TUM fr1_room tracking-only, config/calib.yaml "
                                   f"({'calib' if args.mode == 'calib' else 'rays'} mode), {args.height}x"
                                   f"{args.width} pointmap pairs, GN to convergence",
                       "parallelism": f"replicas x{world} (tracking does not shard)",
                       "launch": {"world_size": world, "gpus_arg": args.gpus,
                                  "launcher": os.environ.get("M3S_BENCH_LAUNCHER", "torch.distributed.run"
                                                             if "TORCHELASTIC_RUN_ID" in os.environ else
                                                             ("external" if world > 1 else "none")),
                                  "backend": dist.get_backend() if world > 1 else None},
                       "gn_iters_mean": gn_iters, "ring_pairs": args.ring},
            "kernels_us": {k: round(v["avg_us"], 2) for k, v in rl.items()},
            "kernels": kernel_table(rl, N, gn_iters),
            "roofline": roof, "frame": frame, "peaks_measured": peaks, "cpu_baseline": cpu, "ba": ba,
            "retrieval": retrieval, "store": store, "configs": configs,
        }
        print(json.dumps(rec), file=OUT, flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
