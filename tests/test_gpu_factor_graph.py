"""FactorGraph edge insertion and the C3 backend chain.

* ``add_factors`` (``/root/reference/mast3r_slam/global_opt.py:32-101``, symmetric matching
  ``mast3r_utils.py:149-187``) against the golden ``add_factors_32x48.npz``: the reference's own
  ``FactorGraph.add_factors`` run by ``tests/golden/make_golden.py`` over four calls on synthetic symmetric
  decoder outputs (the Q filter, the both-directions min-match-fraction rule, the consecutive-edge
  exemption, the ``is_reloc`` early return, the append order). The inputs are regenerated here from their
  seeds with ``m3s.synthetic`` and pinned by the golden's checksums (host test, no GPU).
* the C3 chain of the backend loop (``main.py:116-165``): track a frame, quantize its features against the
  retrieval codebook, insert the factor-graph edges, ``solve_GN_calib`` — each stage checked against the
  oracle / golden.
"""
import numpy as np
import pytest
import torch

import oracle.oracle as O


def _sym_outputs(seed, H, W, kind):
    """tests/golden/make_golden.py _sym_outputs: decoder outputs (ii, ji, jj, ij) of one keyframe pair."""
    from m3s import synthetic

    A = synthetic.make_pair(H, W, seed=seed)
    B = synthetic.make_pair(H, W, seed=seed + 1000)
    X = torch.stack((A["X"][0], A["X"][1], B["X"][0], B["X"][1]))
    C = torch.stack((A["C"][0], A["C"][1], B["C"][0], B["C"][1]))
    D = torch.stack((A["D"][0], A["D"][1], B["D"][0], B["D"][1]))
    Q = torch.stack((A["Q"][0], A["Q"][1], B["Q"][0], B["Q"][1]))
    if kind == "poor":
        Q = torch.ones_like(Q)
    elif kind == "one_sided":
        Q[2:] = 1.0
    return X, C, D, Q


def _call_inputs(g, c, H=32, W=48):
    outs = [_sym_outputs(int(s), H, W, str(k)) for s, k in zip(g[f"c{c}_seeds"], g[f"c{c}_kinds"])]
    return tuple(torch.stack([o[t] for o in outs], dim=1) for t in range(4))  # (4, b, H, W, ...)


def test_add_factors_inputs_regenerate(golden):
    """The synthetic decoder outputs behind the golden regenerate bit for bit (checksums)."""
    g = golden("add_factors_32x48.npz")
    for c in range(int(g["ncalls"])):
        X, C, D, Q = _call_inputs(g, c)
        got = np.array([float(t.double().sum()) for t in (X, C, D, Q)])
        np.testing.assert_array_equal(got, g[f"c{c}_csum"])


class _SymModel:
    """Stands in for MASt3R's symmetric decoder: returns queued (X, C, D, Q) of shape (4, b, H, W, ...)."""

    def __init__(self):
        self.queue = []

    def symmetric_inference(self, kfs_i, kfs_j):
        X, C, D, Q = self.queue.pop(0)
        assert X.shape[1] == len(kfs_i) == len(kfs_j)
        return X, C, D, Q


@pytest.mark.gpu
def test_add_factors_matches_reference(golden):
    from m3s.global_opt import FactorGraph

    g = golden("add_factors_32x48.npz")
    dev = torch.device("cuda")
    model = _SymModel()
    fg = FactorGraph(model, [object() for _ in range(5)], device=dev)
    for c in range(int(g["ncalls"])):
        model.queue.append(tuple(t.to(dev) for t in _call_inputs(g, c)))
        ret = fg.add_factors(g[f"c{c}_ii"].tolist(), g[f"c{c}_jj"].tolist(), float(g[f"c{c}_mmf"]),
                             is_reloc=bool(g[f"c{c}_reloc"]))
        assert bool(ret) == bool(g[f"c{c}_ret"]), c
        np.testing.assert_array_equal(fg.ii.cpu().numpy(), g[f"c{c}_ii_out"])
        np.testing.assert_array_equal(fg.jj.cpu().numpy(), g[f"c{c}_jj_out"])
        np.testing.assert_array_equal(fg.idx_ii2jj.cpu().numpy(), g[f"c{c}_idx_ii2jj"])
        np.testing.assert_array_equal(fg.idx_jj2ii.cpu().numpy(), g[f"c{c}_idx_jj2ii"])
        np.testing.assert_array_equal(fg.valid_match_j.cpu().numpy(), g[f"c{c}_valid_j"])
        np.testing.assert_array_equal(fg.valid_match_i.cpu().numpy(), g[f"c{c}_valid_i"])
        # sqrt(Qii[idx] * Qji): torch's device sqrt on ROCm is the hardware v_sqrt_f32 (within 1 ulp, not
        # always correctly rounded like the CPU's)
        np.testing.assert_allclose(fg.Q_ii2jj.cpu().numpy(), g[f"c{c}_Q_ii2jj"], rtol=2.5e-7, atol=0)
        np.testing.assert_allclose(fg.Q_jj2ii.cpu().numpy(), g[f"c{c}_Q_jj2ii"], rtol=2.5e-7, atol=0)


@pytest.mark.gpu
def test_c3_backend_chain(monkeypatch):
    """C3 (TUM fr1_room full pipeline) on synthetic model outputs: FrameTracker.track -> Codebook.quantize ->
    FactorGraph.add_factors -> solve_GN_calib, the way main.py's backend loop chains them (main.py:116-165)."""
    from m3s.config import config
    from m3s.frame import Frame, Keyframes
    from m3s.global_opt import FactorGraph
    from m3s.retrieval import Codebook
    from m3s.sim3 import Sim3
    from m3s.synthetic import SyntheticModel, make_pair, retrieval_inputs, tum_fr1_intrinsics
    from m3s.tracker import FrameTracker

    monkeypatch.setitem(config, "use_calib", True)
    dev = torch.device("cuda")
    H, W = 48, 64
    K = tum_fr1_intrinsics(H, W)
    # 1. track frame 1 against keyframe 0 (calib mode, as config/calib.yaml)
    P = make_pair(H, W, seed=4, K=K)
    kfs = Keyframes()
    kf0 = Frame(0, (H, W), T_WC=Sim3.Identity(1, device=dev))
    kf0.K = K.to(dev)
    kf0.update_pointmap(P["Xk"].to(dev), P["Ck"].to(dev))
    kfs.append(kf0)
    tr = FrameTracker(SyntheticModel([P], dev), kfs, dev)
    f1 = Frame(1, (H, W), T_WC=Sim3.Identity(1, device=dev))
    f1.K = K.to(dev)
    new_kf, info, reloc = tr.track(f1)
    assert not reloc
    # pose against the oracle's tracker GN on the same inputs (tracker.py:28-114 restated)
    X, C, D, Q = (P[k].numpy() for k in ("X", "C", "D", "Q"))
    Xk, Ck, Kn = P["Xk"].numpy(), P["Ck"].numpy()[:, 0], K.numpy()
    ref_idx, ref_valid = O.match(X[:1], X[1:], D[:1], D[1:])
    i = ref_idx[0]
    Qk = np.sqrt(Q[0].reshape(-1)[i] * Q[1].reshape(-1))
    v = ref_valid[0, :, 0] & (C[0].reshape(-1)[i] > 0.0) & (Ck > 0.0) & (Qk > 1.5)
    Xf = O.backproject_constrain(X[0].reshape(1, -1, 3), Kn, (H, W))[0][i]
    z = O.backproject_constrain(Xk[None], Kn, (H, W))[0][:, 2]
    u, vv = np.meshgrid(np.arange(W, dtype=np.float32), np.arange(H, dtype=np.float32), indexing="xy")
    vmk = z > 1e-6
    meas = np.stack((u.reshape(-1), vv.reshape(-1), np.log(np.where(vmk, z, 1.0))), -1) * vmk[:, None]
    I8 = np.array([0, 0, 0, 0, 0, 0, 1, 1.0])
    T_ref, _, _ = O.track_calib(Xf, Xk, I8, I8, Qk, v, meas, vmk, Kn, (H, W))
    np.testing.assert_allclose(f1.T_WC.data.cpu().numpy()[0], T_ref, atol=1e-5)
    # 2. retrieval: the new keyframe's local features against the codebook (retrieval_database.py:119)
    cent, qv = retrieval_inputs(7, 4096, 128, 120)
    cb = Codebook(torch.from_numpy(cent).to(dev))
    ids = cb.quantize(torch.from_numpy(qv).to(dev), 5).cpu().numpy()
    ref_ids, l2 = O.quantize_custom(cent, qv, 5)
    assert O.topk_equivalent(ids, ref_ids, l2, 1e-4).all()
    # 3. edge insertion: consecutive edge (0, 1) from the symmetric decode of the same pair
    model = _SymModel()
    kfs.append(f1)
    fg = FactorGraph(model, kfs, K=K.to(dev), device=dev)
    Xs = torch.stack((P["X"][0], P["X"][1], P["X"][1], P["X"][0]))[:, None]
    Ds = torch.stack((P["D"][0], P["D"][1], P["D"][1], P["D"][0]))[:, None]
    Qs = torch.stack((P["Q"][0], P["Q"][1], P["Q"][1], P["Q"][0]))[:, None]
    Cs = torch.stack((P["C"][0], P["C"][1], P["C"][1], P["C"][0]))[:, None]
    model.queue.append((Xs.to(dev), Cs.to(dev), Ds.to(dev), Qs.to(dev)))
    assert fg.add_factors([0], [1], config["local_opt"]["min_match_frac"])
    assert fg.ii.tolist() == [0] and fg.jj.tolist() == [1]
    # 4. global BA over the graph (calib): against the fp64 oracle on the graph's own tensors
    f1.update_pointmap(P["X"][1].reshape(-1, 3).to(dev), P["C"][1].reshape(-1, 1).to(dev))
    uniq = fg.get_unique_kf_idx()
    Xg, T_WCs, Cg = fg.get_poses_points(uniq)
    from m3s.geometry import constrain_points_to_ray

    Xg = constrain_points_to_ray((H, W), Xg, K.to(dev))
    ii, jj, idx, valid, Qe = fg.prep_two_way_edges()
    c = config["local_opt"]
    p = O.ba_params("calib", c["sigma_pixel"], c["sigma_depth"], c["C_conf"], c["Q_conf"], K=Kn, height=H, width=W,
                    pixel_border=c["pixel_border"], z_eps=c["depth_eps"])
    T_ref, _, _ = O.gauss_newton_f64("calib", T_WCs.data[:, 0, :].cpu().numpy().astype(np.float64),
                                     Xg.cpu().numpy().astype(np.float64), Cg.cpu().numpy()[..., 0].astype(np.float64),
                                     ii.cpu().numpy(), jj.cpu().numpy(), idx.cpu().numpy(),
                                     valid.cpu().numpy()[..., 0], Qe.cpu().numpy()[..., 0].astype(np.float64), p,
                                     c["max_iters"], c["delta_norm"])
    fg.solve_GN_calib()
    got = np.stack([kfs[k].T_WC.data.cpu().numpy()[0] for k in range(2)])
    assert np.isfinite(got).all()
    np.testing.assert_allclose(got, T_ref, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("mode,traj", [("calib", "chess"), ("rays", "euroc")])
def test_backend_replay_growing_graph_vs_fp64_truth(mode, traj, monkeypatch):
    """The backend loop of main.py:116-155 replayed over 20 keyframes (C3: 7-Scenes chess trajectory, calib mode,
    TUM fr1 K at 120x160; C4: EuRoC MH_02 trajectory, rays mode): for every new keyframe its retrieval features
    are quantized on the matrix cores (checked against the reference's quantize_custom restated), earlier keyframes
    are retrieved by shared visual words (ASMK scoring is out of scope), the consecutive + retrieved loop edges go
    through FactorGraph.add_factors (fused symmetric matching on SceneReplay's decoder outputs) and
    solve_GN_calib / solve_GN_rays runs on the grown graph. After EVERY call the poses must sit within 1e-5 of the
    oracle's fp64 truth run on the same graph tensors (SURVEY §8c a-note 6)."""
    from m3s.config import config
    from m3s.frame import Frame, Keyframes
    from m3s.geometry import constrain_points_to_ray
    from m3s.global_opt import FactorGraph
    from m3s.retrieval import Codebook
    from m3s.sim3 import Sim3
    from m3s.synthetic import SceneReplay, chess_poses, euroc_poses, intrinsics, retrieve, tum_fr1_intrinsics

    calib = mode == "calib"
    monkeypatch.setitem(config, "use_calib", calib)
    dev = torch.device("cuda")
    n_kf, H, W = 20, 120, 160
    K = tum_fr1_intrinsics(H, W) if calib else intrinsics(H, W)
    S = SceneReplay((chess_poses if traj == "chess" else euroc_poses)(n_kf), H, W, K=K, device=dev)
    kfs = Keyframes()
    Kd = K.to(dev)
    fg = FactorGraph(S, kfs, K=Kd, device=dev)
    rng = np.random.default_rng(11)
    cent = rng.standard_normal((2048, 128)).astype(np.float32)
    cent /= np.linalg.norm(cent, axis=1, keepdims=True)
    cb = Codebook(torch.from_numpy(cent).to(dev))
    c = config["local_opt"]
    sa, sb = (c["sigma_pixel"], c["sigma_depth"]) if calib else (c["sigma_ray"], c["sigma_dist"])
    p = O.ba_params(mode, sa, sb, c["C_conf"], c["Q_conf"], K=K.numpy(), height=H, width=W,
                    pixel_border=c["pixel_border"], z_eps=c["depth_eps"])
    words, loops, errs = {}, 0, []
    for idx in range(n_kf):
        X, C = S.keyframe(idx)
        f = Frame(idx, (H, W), T_WC=Sim3(S.Twc0[idx].view(1, 8).clone()))
        f.K = Kd
        f.update_pointmap(X, C)
        kfs.append(f)
        q = S.features(idx)
        ids = cb.quantize(q, 5).cpu().numpy()
        ref_ids, l2 = O.quantize_custom(cent, q.cpu().numpy(), 5)
        assert O.topk_equivalent(ids, ref_ids, l2, 1e-4).all()
        words[idx] = ids
        if idx == 0:
            continue
        retrieved = retrieve(words, idx, config["retrieval"]["k"], config["retrieval"]["min_thresh"])
        kf_idx = sorted(set([idx - 1] + retrieved) - {idx})  # main.py:117-141
        loops += len(set(retrieved) - {idx - 1})
        fg.add_factors(kf_idx, [idx] * len(kf_idx), c["min_match_frac"])
        # the fp64 truth on the graph's own tensors, from the poses the solve starts at
        uniq = fg.get_unique_kf_idx()
        Xg, T_WCs, Cg = fg.get_poses_points(uniq)
        if calib:
            Xg = constrain_points_to_ray((H, W), Xg, Kd)
        ii, jj, idx2, valid, Qe = fg.prep_two_way_edges()
        T_ref, _, _ = O.gauss_newton_f64(mode, T_WCs.data[:, 0, :].cpu().numpy().astype(np.float64),
                                         Xg.cpu().numpy().astype(np.float64),
                                         Cg.cpu().numpy()[..., 0].astype(np.float64), ii.cpu().numpy(),
                                         jj.cpu().numpy(), idx2.cpu().numpy(), valid.cpu().numpy()[..., 0],
                                         Qe.cpu().numpy()[..., 0].astype(np.float64), p, c["max_iters"],
                                         c["delta_norm"])
        (fg.solve_GN_calib if calib else fg.solve_GN_rays)()
        got = np.stack([kfs[int(k)].T_WC.data.cpu().numpy()[0] for k in uniq.tolist()])
        assert np.isfinite(got).all()
        errs.append(float(np.abs(got - T_ref).max()))
        np.testing.assert_allclose(got, T_ref, atol=1e-5, err_msg=f"after keyframe {idx}")
    print(f"replay {traj} {mode}: {fg.ii.numel()} edges ({loops} retrieved loop edges), max pose error vs fp64 "
          f"truth per call: max {max(errs):.2e}")
    assert loops > 0
    # the optimised trajectory is closer to the ground truth than the initial one
    T_fin = np.stack([kfs[k].T_WC.data.cpu().numpy()[0] for k in range(n_kf)])
    gt, t0 = S.Twc_gt.cpu().numpy(), S.Twc0.cpu().numpy()
    assert np.abs(T_fin[:, :3] - gt[:, :3]).mean() < np.abs(t0[:, :3] - gt[:, :3]).mean()


@pytest.mark.gpu
@pytest.mark.parametrize("mode,traj", [("calib", "chess"), ("rays", "euroc")])
def test_backend_replay_record_reuse_bit_identical(mode, traj, monkeypatch):
    """Record reuse across solves (m3s_ba_make_plan*_reuse): the replayed backend loop (main.py:116-155) with
    FactorGraph's default reuse must give poses bit-identical to a fresh solve of the same graph from the same
    start after EVERY call, while packing only the new edges and the edges of keyframes that changed. Every third
    keyframe, the previous keyframe is re-fused first (tracking's update_pointmap), so changed keyframes are
    exercised too; the workspace regrows several times as the graph grows (a fresh cache each time)."""
    import mast3r_slam_backends as B
    from m3s.config import config
    from m3s.frame import Frame, Keyframes
    from m3s.geometry import constrain_points_to_ray
    from m3s.global_opt import FactorGraph
    from m3s.sim3 import Sim3
    from m3s.synthetic import SceneReplay, chess_poses, euroc_poses, intrinsics, tum_fr1_intrinsics

    calib = mode == "calib"
    monkeypatch.setitem(config, "use_calib", calib)
    dev = torch.device("cuda")
    n_kf, H, W = 14, 120, 160
    K = tum_fr1_intrinsics(H, W) if calib else intrinsics(H, W)
    S = SceneReplay((chess_poses if traj == "chess" else euroc_poses)(n_kf), H, W, K=K, device=dev)
    kfs = Keyframes()
    Kd = K.to(dev)
    fg = FactorGraph(S, kfs, K=Kd, device=dev)
    assert fg.reuse_records
    c = config["local_opt"]
    packed_total, edges_total, changed_seen = 0, 0, 0
    for idx in range(n_kf):
        X, C = S.keyframe(idx)
        f = Frame(idx, (H, W), T_WC=Sim3(S.Twc0[idx].view(1, 8).clone()))
        f.K = Kd
        f.update_pointmap(X, C)
        kfs.append(f)
        if idx == 0:
            continue
        refused = idx >= 3 and idx % 3 == 0
        if refused:  # tracking fused a frame into the previous keyframe: its points, confidences and N change
            Xp, Cp = S.keyframe(idx - 1)
            kfs[idx - 1].update_pointmap(Xp * 1.001, Cp * 0.5)
        loop = [idx - 3] if idx >= 3 else []
        fg.add_factors(sorted(set([idx - 1] + loop)), [idx] * len(set([idx - 1] + loop)), c["min_match_frac"])
        uniq = fg.get_unique_kf_idx()
        Xg, T_WCs, Cg = fg.get_poses_points(uniq)
        if calib:
            Xg = constrain_points_to_ray((H, W), Xg, Kd)
        ii, jj, idx2, valid, Qe = fg.prep_two_way_edges()
        T_fresh = T_WCs.data[:, 0, :].clone().contiguous()
        if calib:
            B.gauss_newton_calib(T_fresh, Xg, Cg, Kd, ii, jj, idx2, valid, Qe, H, W, c["pixel_border"], c["depth_eps"],
                                 c["sigma_pixel"], c["sigma_depth"], c["C_conf"], c["Q_conf"], c["max_iters"],
                                 c["delta_norm"])
            fg.solve_GN_calib()
        else:
            B.gauss_newton_rays(T_fresh, Xg, Cg, ii, jj, idx2, valid, Qe, c["sigma_ray"], c["sigma_dist"], c["C_conf"],
                                c["Q_conf"], c["max_iters"], c["delta_norm"])
            fg.solve_GN_rays()
        got = np.stack([kfs[int(k)].T_WC.data.cpu().numpy()[0] for k in uniq.tolist()])
        want = T_fresh.cpu().numpy()
        pin = c["pin"]
        assert np.array_equal(got[pin:], want[pin:]), f"after keyframe {idx}: reuse differs from a fresh solve"
        E = ii.numel()
        packed, changed = fg.ba_info["packed_edges"], fg.ba_info["changed_keyframes"]
        assert packed <= E
        packed_total += packed
        edges_total += E
        changed_seen += changed if refused else 0
    print(f"record reuse {traj} {mode}: packed {packed_total} of {edges_total} edge records over {n_kf - 1} solves")
    assert packed_total < 0.6 * edges_total
    assert changed_seen > 0


@pytest.mark.gpu
def test_record_reuse_cache_invalidation():
    """The reuse cache of a workspace: a second reuse plan packs nothing; a plain plan on the same workspace drops
    the cache (the next reuse plan packs every edge again); changed keyframe data repacks exactly that keyframe's
    edges; a duplicate keyframe uid is rejected; poses always equal a fresh solve's."""
    import ctypes

    from m3s import _lib
    from m3s.config import config
    from m3s.dist_ba import HipShard, RecordCache, ba_config, run_sharded
    from m3s.synthetic import make_graph, two_way

    H, W = 24, 32
    G = make_graph(n_kf=6, H=H, W=W, seed=5)
    ii, jj, idx, valid, Q = (t.cuda().contiguous() for t in two_way(G))
    valid, Q = valid.reshape(idx.shape).contiguous(), Q.reshape(idx.shape).contiguous()
    Xs, Cs = G["Xs"].cuda().contiguous(), G["Cs"][..., 0].cuda().contiguous()
    E, K = ii.shape[0], Xs.shape[0]
    cfg = ba_config("rays", config["local_opt"])
    cache = RecordCache()
    uids = (np.arange(E, dtype=np.int64), np.arange(K, dtype=np.int64))

    def solve(X, reuse=True):
        T = G["Twc0"].cuda().clone()
        sh = HipShard(cfg, T, X, Cs, ii, jj, idx, valid, Q, 0.0, 0, E, reuse=uids if reuse else None,
                      cache=cache if reuse else None)
        run_sharded(sh, 5)
        return T.cpu().numpy(), (sh.reuse_info() if reuse else None)

    T_fresh, _ = solve(Xs, reuse=False)
    T1, info1 = solve(Xs)
    assert info1 == (E, K) and np.array_equal(T1, T_fresh)
    T2, info2 = solve(Xs)
    assert info2 == (0, 0) and np.array_equal(T2, T_fresh)
    # a plain plan on the cache's own workspace drops the cache
    lib = _lib.load()
    plan = _lib.BaPlan()
    dx = torch.zeros((K - 1, 7), dtype=torch.float32, device="cuda")
    Tp = G["Twc0"].cuda().clone()
    _lib.check(lib.m3s_ba_make_plan(ctypes.byref(cfg), _lib.ptr(Tp), _lib.ptr(Xs), _lib.ptr(Cs), K, H * W,
                                    _lib.ptr(ii), _lib.ptr(jj), E, 0, E, _lib.ptr(idx), _lib.ptr(valid), _lib.ptr(Q),
                                    0.0, _lib.ptr(dx), _lib.ptr(cache.ws), cache.ws.numel(), ctypes.byref(plan),
                                    _lib.stream_ptr(torch.device("cuda"))))
    torch.cuda.synchronize()
    T3, info3 = solve(Xs)
    assert info3[0] == E and np.array_equal(T3, T_fresh)
    # keyframe 2 changed: exactly its edges repack, and the result is the fresh solve of the changed data
    X2 = Xs.clone()
    X2[2] *= 1.001
    T_fresh2, _ = solve(X2, reuse=False)
    T4, info4 = solve(X2)
    n2 = int(((ii == 2) | (jj == 2)).sum())
    assert info4 == (n2, 1) and np.array_equal(T4, T_fresh2)
    # duplicate keyframe uids are rejected
    bad = (uids[0], np.zeros(K, dtype=np.int64))
    with pytest.raises(RuntimeError):
        HipShard(cfg, G["Twc0"].cuda().clone(), Xs, Cs, ii, jj, idx, valid, Q, 0.0, 0, E, reuse=bad, cache=cache)
    cache.release()
