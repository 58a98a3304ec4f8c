"""GPU parity: tracking GN (FrameTracker.track, opt_pose_*) vs the reference glue's golden vectors.

Contract (BASELINE.json north_star): pose/points to 1e-5 for identical inputs. The golden vectors
come from the reference's own tracker.py run on the same synthetic inputs (make_golden.py).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _setup(g, use_calib, N, H, W):
    from m3s.config import config
    from m3s.frame import Frame, Keyframes
    from m3s.sim3 import Sim3

    config["use_calib"] = use_calib
    dev = "cuda"
    kf = Frame(0, (H, W), T_WC=Sim3(torch.from_numpy(g["T_WCk"]).view(1, 8).to(dev)))
    kf.K = torch.from_numpy(g["K"]).to(dev)
    kf.update_pointmap(torch.from_numpy(g["Xk"]).to(dev), torch.from_numpy(g["Ck"]).to(dev))
    frame = Frame(1, (H, W), T_WC=Sim3(kf.T_WC.data.clone()))
    kfs = Keyframes()
    kfs.append(kf)

    class Model:
        def asymmetric_inference(self, fi, fj):
            return (torch.from_numpy(g["X"]).to(dev), torch.from_numpy(g["C"]).to(dev),
                    torch.from_numpy(g["D"]).to(dev), torch.from_numpy(g["Q"]).to(dev))

    return kf, frame, kfs, Model()


@pytest.mark.parametrize("mode", ["rays", "calib"])
def test_track_matches_reference(golden, mode):
    from m3s.tracker import FrameTracker

    g = golden("tracking_48x64.npz")
    H, W = 48, 64
    kf, frame, kfs, model = _setup(g, mode == "calib", H * W, H, W)
    tr = FrameTracker(model, kfs, "cuda")
    new_kf, info, reloc = tr.track(frame)
    assert bool(new_kf) == bool(g[f"{mode}_new_kf"]) and bool(reloc) == bool(g[f"{mode}_reloc"])
    assert tr.last_result.iters == int(g[f"{mode}_iters"])
    np.testing.assert_allclose(frame.T_WC.data.cpu().numpy(), g[f"{mode}_T_WCf"], atol=1e-5)
    # fused points carry the pose error times |X| (metres): 1e-5 absolute + 1e-5 relative
    np.testing.assert_allclose(kf.X_canon.cpu().numpy(), g[f"{mode}_kf_X"], atol=1e-5, rtol=1e-5)
    np.testing.assert_allclose(kf.C.cpu().numpy(), g[f"{mode}_kf_C"], atol=1e-5)
    assert kf.N == 2
    assert len(info) == 6
    # match_info average confidences (fuse kernel outputs) == C / N (frame.py:83-84), exactly
    assert torch.equal(info[1], kf.C / kf.N) and torch.equal(info[3], frame.C / frame.N)


@pytest.mark.parametrize("mode", ["rays", "calib"])
def test_opt_pose_matches_reference(golden, mode):
    from m3s.sim3 import Sim3
    from m3s.tracker import FrameTracker

    g = golden("optpose_32x48.npz")
    d = lambda k: torch.from_numpy(g[k]).cuda()
    tr = FrameTracker(None, None, "cuda")
    if mode == "rays":
        Tf, Tr = tr.opt_pose_ray_dist_sim3(d("Xf"), d("Xk"), Sim3(d("T_WCf")), Sim3(d("T_WCk")), d("Qk"), d("valid"))
    else:
        Tf, Tr = tr.opt_pose_calib_sim3(d("Xf_c"), d("Xk"), Sim3(d("T_WCf")), Sim3(d("T_WCk")), d("Qk"), d("valid"),
                                        d("meas"), d("vmeas"), d("K"), (32, 48))
    np.testing.assert_allclose(Tf.data.cpu().numpy(), g[f"{mode}_T_WCf"], atol=1e-5)
    np.testing.assert_allclose(Tr.data.cpu().numpy(), g[f"{mode}_T_CkCf"], atol=1e-5)


def test_track_skips_low_match_fraction(golden):
    """tracker.py:67-70: match_frac < min_match_frac -> (False, [], True), keyframe untouched."""
    from m3s.config import config
    from m3s.tracker import FrameTracker

    g = golden("tracking_48x64.npz")
    kf, frame, kfs, model = _setup(g, False, 48 * 64, 48, 64)
    config["tracking"]["Q_conf"] = 1e9  # nothing passes the Q test
    X0 = kf.X_canon.clone()
    tr = FrameTracker(model, kfs, "cuda")
    assert tr.track(frame) == (False, [], True)
    assert torch.equal(kf.X_canon, X0) and kf.N == 1


def test_track_full_size_converges_to_ground_truth():
    """512x512 synthetic pair: the tracked relative pose recovers the generating T_CkCf."""
    from m3s.frame import Frame, Keyframes
    from m3s.sim3 import Sim3
    from m3s.synthetic import SyntheticModel, make_pair
    from m3s.tracker import FrameTracker

    P = make_pair(512, 512, seed=2)
    model = SyntheticModel([P], "cuda")
    kf = Frame(0, (512, 512))
    kf.T_WC = Sim3.Identity(1, device="cuda")
    kf.update_pointmap(P["Xk"].cuda(), P["Ck"].cuda())
    kfs = Keyframes()
    kfs.append(kf)
    tr = FrameTracker(model, kfs, "cuda")
    frame = Frame(1, (512, 512), T_WC=Sim3.Identity(1, device="cuda"))
    new_kf, info, reloc = tr.track(frame)
    assert not reloc
    T = frame.T_WC.data.cpu().numpy()[0]
    T_gt = P["T_gt"].numpy()
    assert np.abs(T[:3] - T_gt[:3]).max() < 2e-3
    assert abs(T[7] - T_gt[7]) < 2e-3
    assert abs(abs(float(np.dot(T[3:7], T_gt[3:7]))) - 1.0) < 1e-5


def _mode_cfg(key, value):
    from m3s.config import config

    config["tracking"][key] = value


def test_track_cholesky_failure_returns_reloc(golden):
    """tracker.py:84-89: a failed factorisation (here: no valid residual, H = 0) -> (False, [], True)."""
    from m3s.tracker import FrameTracker

    g = golden("tracking_48x64.npz")
    kf, frame, kfs, model = _setup(g, False, 48 * 64, 48, 64)
    _mode_cfg("min_match_frac", 0.0)
    _mode_cfg("Q_conf", 1e9)
    X0 = kf.X_canon.clone()
    tr = FrameTracker(model, kfs, "cuda")
    assert tr.track(frame) == (False, [], True)
    assert torch.equal(kf.X_canon, X0) and kf.N == 1


def test_opt_pose_raises_on_cholesky_failure(golden):
    """torch.linalg.cholesky raises on a singular H (tracker.py:168): so does the direct surface."""
    from m3s.sim3 import Sim3
    from m3s.tracker import FrameTracker

    g = golden("optpose_32x48.npz")
    d = lambda k: torch.from_numpy(g[k]).cuda()
    tr = FrameTracker(None, None, "cuda")
    with pytest.raises(RuntimeError, match="cholesky"):
        tr.opt_pose_ray_dist_sim3(d("Xf"), d("Xk"), Sim3(d("T_WCf")), Sim3(d("T_WCk")), d("Qk"),
                                  torch.zeros_like(d("valid")))


def test_track_max_iters_still_updates(golden):
    """max_iters reached without convergence: the pose and the fusion are still applied (tracker.py:76-101)."""
    from m3s import _lib
    from m3s.tracker import FrameTracker

    g = golden("tracking_48x64.npz")
    kf, frame, kfs, model = _setup(g, False, 48 * 64, 48, 64)
    _mode_cfg("max_iters", 1)
    tr = FrameTracker(model, kfs, "cuda")
    new_kf, info, reloc = tr.track(frame)
    assert not reloc and tr.last_result.iters == 1 and tr.last_result.status == _lib.TRACK_MAX_ITERS
    assert kf.N == 2 and len(info) == 6


def test_track_recent_filtering_replaces_keyframe(golden):
    """filtering_mode 'recent' (frame.py:59-62) takes the update_pointmap path: X = T_CkCf.act(Xkf), N = 1."""
    from m3s.sim3 import Sim3
    from m3s.tracker import FrameTracker

    g = golden("tracking_48x64.npz")
    kf, frame, kfs, model = _setup(g, False, 48 * 64, 48, 64)
    _mode_cfg("filtering_mode", "recent")
    tr = FrameTracker(model, kfs, "cuda")
    new_kf, info, reloc = tr.track(frame)
    assert not reloc
    T_CkCf = Sim3(kf.T_WC.data).inv() * frame.T_WC
    Xkf = torch.from_numpy(g["X"][1].reshape(-1, 3)).cuda()
    np.testing.assert_allclose(kf.X_canon.cpu().numpy(), T_CkCf.act(Xkf).cpu().numpy(), atol=2e-5, rtol=1e-5)
    assert kf.N == 1 and kf.N_updates == 2


def test_track_while_ba_runs_on_another_stream():
    """The reference runs the backend's global BA concurrently with tracking on the same GPU (main.py:268-269).
    A 512x512 frame tracked while a K=64 chess-trajectory gauss_newton (30 iterations, enqueued first) occupies
    the CUs from a second stream: the persistent GN launch's blocks become resident as the BA blocks drain and
    the frame's pose, fused keyframe points and iteration count equal the solo run bit for bit; the BA result
    equals its own solo run too."""
    import mast3r_slam_backends as B
    from m3s.config import config
    from m3s.frame import Frame, Keyframes
    from m3s.sim3 import Sim3
    from m3s.synthetic import SyntheticModel, chess_poses, make_pair, make_traj_graph
    from m3s.tracker import FrameTracker

    config["use_calib"] = True
    P = make_pair(512, 512, seed=4)
    model = SyntheticModel([P], "cuda")

    def track_once():
        kf = Frame(0, (512, 512), T_WC=Sim3.Identity(1, device="cuda"))
        kf.K = P["K"].cuda()
        kf.update_pointmap(P["Xk"].cuda(), P["Ck"].cuda())
        kfs = Keyframes()
        kfs.append(kf)
        tr = FrameTracker(model, kfs, "cuda")
        frame = Frame(1, (512, 512), T_WC=Sim3.Identity(1, device="cuda"))
        new_kf, info, reloc = tr.track(frame)
        assert not reloc
        return frame.T_WC.data.clone(), kf.X_canon.clone(), kf.C.clone(), tr.last_result.iters

    G = make_traj_graph(chess_poses(64), 384, 512, seed=1, device="cuda")
    c = config["local_opt"]
    ba_args = (G["Xs"].contiguous(), G["Cs"].contiguous(), G["ii"], G["jj"], G["idx"].contiguous(),
               G["valid"].contiguous(), G["Q"].contiguous(), c["sigma_ray"], c["sigma_dist"], c["C_conf"],
               c["Q_conf"], 30, 0.0)

    def ba(stream):
        T = G["Twc0"].clone()
        with torch.cuda.stream(stream):
            dx = B.gauss_newton_rays(T, *ba_args)[0]
        return T, dx

    solo = track_once()
    s2 = torch.cuda.Stream()
    T_ba_solo, dx_ba_solo = ba(s2)
    torch.cuda.synchronize()
    T_ba, dx_ba = ba(s2)  # enqueued: ~30 linearisation launches of ~500 edge blocks each on stream 2
    both = track_once()   # meanwhile on the default stream
    torch.cuda.synchronize()
    for a, b in zip(solo, both):
        assert (a == b) if isinstance(a, int) else torch.equal(a, b)
    assert torch.equal(T_ba, T_ba_solo) and torch.equal(dx_ba, dx_ba_solo)


def _shared_store(P, H, W, manager):
    """A SharedKeyframes (the reference's multi-process store, frame.py:220-327) holding one keyframe record."""
    from m3s.frame import Frame, SharedKeyframes
    from m3s.sim3 import Sim3

    kfs = SharedKeyframes(manager, H, W, buffer=4, device="cuda", feat_dim=64)
    kf = Frame(0, (H, W), T_WC=Sim3.Identity(1, device="cuda"))
    kf.K = P["K"].cuda()
    kf.update_pointmap(P["Xk"].cuda(), P["Ck"].cuda())
    g = torch.Generator().manual_seed(3)
    kf.img = torch.rand(3, H, W, generator=g).cuda()
    kf.uimg = torch.rand(H, W, 3, generator=g)
    kf.img_shape = torch.tensor([[H, W]], dtype=torch.int).cuda()
    kf.img_true_shape = kf.img_shape.clone()
    kf.feat = torch.rand(1, H * W // 256, 64, generator=g).cuda()
    kf.pos = torch.randint(0, 100, (1, H * W // 256, 2), generator=g).cuda()
    kfs.append(kf)
    kfs.set_intrinsics(P["K"].cuda())
    kfs.get_dirty_idx()  # clean
    return kfs


def test_track_writes_fused_keyframe_into_shared_slot():
    """SURVEY §8f row 2 (keyframe-buffer write-back): with a SharedKeyframes store the fused tracker writes the fused
    X / C and the slot's N, N_updates, is_dirty straight into the slot (fusion kernel, in place) instead of
    tracker.py:101's full-record __setitem__ copy (frame.py:271-289). Over several tracked frames every buffer of the
    store is bit-identical to the reference's full-copy path (slot_writeback = False), and so are the poses and
    the returned match_info."""
    import multiprocessing as mp

    from m3s.config import config
    from m3s.frame import Frame
    from m3s.sim3 import Sim3
    from m3s.synthetic import SyntheticModel, make_pair
    from m3s.tracker import FrameTracker

    config["use_calib"] = True
    config["tracking"]["filtering_mode"] = "weighted_pointmap"
    H, W = 64, 96
    pairs = [make_pair(H, W, seed=s) for s in (11, 12, 13)]
    manager = mp.get_context("spawn").Manager()
    try:
        out = {}
        for direct in (True, False):
            kfs = _shared_store(pairs[0], H, W, manager)
            tr = FrameTracker(SyntheticModel(pairs, "cuda"), kfs, "cuda")
            tr.slot_writeback = direct
            poses, infos = [], []
            for f in range(5):
                frame = Frame(1 + f, (H, W), T_WC=Sim3.Identity(1, device="cuda"))
                new_kf, info, reloc = tr.track(frame)
                assert not reloc
                poses.append(frame.T_WC.data.cpu().clone())
                infos.append([t.cpu().clone() for t in info])
            torch.cuda.synchronize()
            bufs = {k: getattr(kfs, k).cpu().clone() for k in ("dataset_idx", "img", "uimg", "img_shape",
                                                                   "img_true_shape", "T_WC", "X", "C", "N",
                                                                   "N_updates", "feat", "pos", "is_dirty")}
            out[direct] = (bufs, poses, infos, len(kfs))
        a, b = out[True], out[False]
        assert a[3] == b[3] == 1
        for k in a[0]:
            assert torch.equal(a[0][k], b[0][k]), f"slot buffer {k} differs"
        assert int(a[0]["N"][0]) == 6 and int(a[0]["N_updates"][0]) == 6 and bool(a[0]["is_dirty"][0])
        for pa, pb in zip(a[1], b[1]):
            assert torch.equal(pa, pb)
        for ia, ib in zip(a[2], b[2]):
            assert all(torch.equal(x, y) for x, y in zip(ia, ib))
    finally:
        manager.shutdown()
        config["use_calib"] = False


def _track_once(g, mode, H, W, cfg):
    from m3s.tracker import FrameTracker

    kf, frame, kfs, model = _setup(g, mode == "calib", H * W, H, W)
    for k, v in cfg.items():
        _mode_cfg(k, v)
    tr = FrameTracker(model, kfs, "cuda")
    out = tr.track(frame)
    r = tr.last_result
    res = None if r is None else (list(r.T_WCf), list(r.T_CkCf), r.cost, r.iters, r.status, r.n_valid_opt,
                                  r.n_valid_kf, r.n_unique)
    return (bool(out[0]), bool(out[2]), res, frame.T_WC.data.cpu().clone(), kf.X_canon.cpu().clone(),
            kf.C.cpu().clone(), kf.N)


@pytest.mark.parametrize("case", ["rays", "calib", "skip", "cholesky", "max_iters"])
def test_track_folded_setup_bit_identical(golden, monkeypatch, case):
    """M3S_TRACK_FOLD_SETUP=1 (setup inside the GN launch's first iteration, the skip test after its hand-off) gives
    the separate-setup path's result bit for bit: decisions, iterations, status, counts, pose, cost, fused points and
    confidences. track.hip is built without FMA contraction (csrc/Makefile FLAGS_track), so the shared setup_point /
    track_state_init code rounds the same in both instantiations."""
    from m3s.config import reset_config

    g = golden("tracking_48x64.npz")
    mode = "calib" if case == "calib" else "rays"
    cfg = {"skip": {"Q_conf": 1e9}, "cholesky": {"min_match_frac": 0.0, "Q_conf": 1e9},
           "max_iters": {"max_iters": 1}}.get(case, {})
    outs = []
    for fold in ("0", "1"):
        monkeypatch.setenv("M3S_TRACK_FOLD_SETUP", fold)
        reset_config()
        outs.append(_track_once(g, mode, 48, 64, cfg))
    a, b = outs
    assert a[:2] == b[:2]
    if a[2] is None or b[2] is None:
        assert a[2] is None and b[2] is None
    else:
        assert a[2] == b[2]
    assert torch.equal(a[3], b[3])
    assert torch.equal(a[4], b[4])
    assert torch.equal(a[5], b[5]) and a[6] == b[6]


def test_track_folded_setup_full_size(monkeypatch):
    """512x512 (every point in the GN launch's registers) and 640x480 (points past the first round: records built in
    iteration 0 into the record buffer, read back later), folded vs separate setup, both modes (tolerances as
    above: bit for bit)."""
    from m3s.config import config, reset_config
    from m3s.frame import Frame, Keyframes
    from m3s.sim3 import Sim3
    from m3s.synthetic import SyntheticModel, make_pair
    from m3s.tracker import FrameTracker

    for (H, W) in ((512, 512), (480, 640)):
        P = make_pair(H, W, seed=2)
        for calib in (False, True):
            outs = []
            for fold in ("0", "1"):
                monkeypatch.setenv("M3S_TRACK_FOLD_SETUP", fold)
                reset_config()
                config["use_calib"] = calib
                model = SyntheticModel([P], "cuda")
                kf = Frame(0, (H, W))
                kf.T_WC = Sim3.Identity(1, device="cuda")
                kf.K = P["K"].cuda()
                kf.update_pointmap(P["Xk"].cuda(), P["Ck"].cuda())
                kfs = Keyframes()
                kfs.append(kf)
                tr = FrameTracker(model, kfs, "cuda")
                frame = Frame(1, (H, W), T_WC=Sim3.Identity(1, device="cuda"))
                frame.K = P["K"].cuda()
                tr.track(frame)
                r = tr.last_result
                outs.append(((r.iters, r.status, r.n_valid_opt, r.n_valid_kf, r.n_unique), r.cost,
                             frame.T_WC.data.cpu(), kf.X_canon.cpu(), kf.C.cpu()))
            a, b = outs
            assert a[0] == b[0], (H, W, calib)
            assert a[1] == b[1], (H, W, calib)
            assert torch.equal(a[2], b[2]) and torch.equal(a[3], b[3]) and torch.equal(a[4], b[4]), (H, W, calib)


def test_track_unique_count_after_frame_of_another_size(golden):
    """The frame scratch (byte map, records, partials) is laid out per image size, so a workspace whose last frame had
    another size gets its scratch re-initialised: a 48x64 frame then a 512x512 frame on the same workspace, and the
    512x512 frame's unique-match count equals |unique(idx[valid])| computed on the host (the 48x64 frame's records
    once left 5540 stale byte-map entries under it)."""
    import m3s.tracker as T
    from m3s.config import config
    from m3s.frame import Frame, Keyframes
    from m3s.sim3 import Sim3
    from m3s.synthetic import SyntheticModel, make_pair
    from m3s.tracker import FrameTracker

    cap = {}
    orig = T.mast3r_match_asymmetric

    def capture(*a, **k):
        out = orig(*a, **k)
        cap["idx"], cap["valid"] = out[0], out[1]
        return out

    T.mast3r_match_asymmetric = capture
    P = make_pair(512, 512, seed=2)

    def big():
        config["use_calib"] = False
        kf = Frame(0, (512, 512), T_WC=Sim3.Identity(1, device="cuda"))
        kf.update_pointmap(P["Xk"].cuda(), P["Ck"].cuda())
        kfs = Keyframes()
        kfs.append(kf)
        tr = FrameTracker(SyntheticModel([P], "cuda"), kfs, "cuda")
        tr.track(Frame(1, (512, 512), T_WC=Sim3.Identity(1, device="cuda")))
        idx, v = cap["idx"].reshape(-1), cap["valid"].reshape(-1).bool()
        assert tr.last_result.n_unique == int(torch.unique(idx[v]).numel())

    try:
        big()  # the workspace grows to the 512x512 layout
        g = golden("tracking_48x64.npz")
        kf, frame, kfs, model = _setup(g, False, 48 * 64, 48, 64)
        FrameTracker(model, kfs, "cuda").track(frame)  # same buffer, the 48x64 layout
        big()
    finally:
        T.mast3r_match_asymmetric = orig
