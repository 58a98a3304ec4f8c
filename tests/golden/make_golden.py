"""Generate the golden fixtures under tests/golden/ by running the REFERENCE's own Python glue.

Runs only in the build container, where /root/reference exists (read-only). The reference never
travels: only the resulting .npz vectors are committed. What runs from the reference:

  mast3r_slam/matching.py     prep_for_iter_proj, match_iterative_proj (the glue around the kernels)
  mast3r_slam/image.py        img_gradient
  mast3r_slam/geometry.py     point_to_ray_dist, act_Sim3, project_calib, constrain_points_to_ray, ...
  mast3r_slam/tracker.py      FrameTracker.track / opt_pose_ray_dist_sim3 / opt_pose_calib_sim3 / solve
  mast3r_slam/global_opt.py   FactorGraph.solve_GN_rays / solve_GN_calib (prep_two_way_edges, pin, write-back),
                              FactorGraph.add_factors (Q filter, min-match fraction, consecutive rule, reloc)
  mast3r_slam/frame.py        Frame.update_pointmap (weighted_pointmap fusion)
  mast3r_slam/retrieval_database.py  RetrievalDatabase.quantize_custom (distance GEMM + top-k), called
                              unbound on a stand-in `self` holding the centroids

Stand-ins (the reference's native / third-party pieces cannot run here — no nvcc, no lietorch,
no ViT checkpoint):
  lietorch               -> oracle/lietorch_shim.py (restated published algorithm; parity unpinned)
  mast3r_slam_backends   -> oracle/m3s_oracle.c via oracle/oracle.py (restated CUDA kernels)
  mast3r_slam.mast3r_utils -> stub; the synthetic "model outputs" are fed to the glue directly.
  mast3r.retrieval.*, asmk -> stubs (only quantize_custom runs, which needs neither).

Usage:  python tests/golden/make_golden.py
"""
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.dont_write_bytecode = True
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "lightweight-mast3r-slam_amd"))

import oracle.oracle as O  # noqa: E402
import oracle.lietorch_shim as shim  # noqa: E402

# ---------------------------------------------------------------- stand-ins for absent modules
sys.modules["lietorch"] = shim


def _np(t):
    return t.detach().cpu().numpy()


class _OracleBackends(types.ModuleType):
    """mast3r_slam_backends over the C oracle, torch-tensor in / torch-tensor out."""

    def iter_proj(self, rays, pts, p_init, max_iter, lambda_init, cost_thresh):
        p, c = O.iter_proj(_np(rays), _np(pts), _np(p_init), max_iter, lambda_init, cost_thresh)
        return [torch.from_numpy(p), torch.from_numpy(c)]

    def refine_matches(self, D11, D21, p1, radius, dilation_max):
        if D11.dtype == torch.float16:
            out = O.refine_matches(_np(D11.view(torch.int16)).view(np.uint16), _np(D21.view(torch.int16)).view(np.uint16),
                                   _np(p1), radius, dilation_max, half=True)
        else:
            out = O.refine_matches(_np(D11), _np(D21), _np(p1), radius, dilation_max, half=False)
        return [torch.from_numpy(out)]

    def _gn(self, mode, Twc, Xs, Cs, ii, jj, idx, valid, Q, params, max_iter, delta):
        T, dx, _ = O.gauss_newton(mode, _np(Twc), _np(Xs), _np(Cs).reshape(Xs.shape[0], -1), _np(ii), _np(jj),
                                  _np(idx), _np(valid), _np(Q), params, max_iter, delta)
        Twc.copy_(torch.from_numpy(T))
        return [torch.from_numpy(dx)]

    def gauss_newton_rays(self, Twc, Xs, Cs, ii, jj, idx, valid, Q, s_ray, s_dist, C_t, Q_t, max_iter, delta):
        return self._gn("rays", Twc, Xs, Cs, ii, jj, idx, valid, Q, O.ba_params("rays", s_ray, s_dist, C_t, Q_t),
                        max_iter, delta)

    def gauss_newton_calib(self, Twc, Xs, Cs, K, ii, jj, idx, valid, Q, h, w, border, z_eps, s_pix, s_depth, C_t,
                           Q_t, max_iter, delta):
        p = O.ba_params("calib", s_pix, s_depth, C_t, Q_t, K=_np(K), height=h, width=w, pixel_border=border,
                        z_eps=z_eps)
        return self._gn("calib", Twc, Xs, Cs, ii, jj, idx, valid, Q, p, max_iter, delta)

    def gauss_newton_points(self, Twc, Xs, Cs, ii, jj, idx, valid, Q, s_pt, C_t, Q_t, max_iter, delta):
        return self._gn("points", Twc, Xs, Cs, ii, jj, idx, valid, Q, O.ba_params("points", s_pt, 0.0, C_t, Q_t),
                        max_iter, delta)


sys.modules["mast3r_slam_backends"] = _OracleBackends("mast3r_slam_backends")
_mu = types.ModuleType("mast3r_slam.mast3r_utils")
_mu.mast3r_match_asymmetric = None
_mu.mast3r_match_symmetric = None
_mu.resize_img = None
sys.modules["mast3r_slam.mast3r_utils"] = _mu
sys.path.insert(0, REF)

from mast3r_slam import config as ref_config  # noqa: E402

ref_config.load_config(os.path.join(REF, "config", "base.yaml"))
import mast3r_slam.frame as ref_frame  # noqa: E402
import mast3r_slam.geometry as ref_geom  # noqa: E402
import mast3r_slam.global_opt as ref_go  # noqa: E402
import mast3r_slam.matching as ref_matching  # noqa: E402
import mast3r_slam.tracker as ref_tracker  # noqa: E402
from m3s import synthetic  # noqa: E402  (synthetic inputs only; no product compute)

torch.set_num_threads(8)
torch.cuda.synchronize = lambda *a, **k: None  # reference profiler.timer syncs CUDA; CPU-only here


def save(name, **arrays):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **{k: np.asarray(v) for k, v in arrays.items()})
    print("wrote", name, {k: np.asarray(v).shape for k, v in arrays.items()})


# ---------------------------------------------------------------- matching
def gen_matching(H=48, W=64, seed=0):
    P = synthetic.make_pair(H, W, seed=seed)
    X, D = P["X"], P["D"]
    X11, X21, D11, D21 = X[:1], X[1:], D[:1], D[1:]
    rays, pts, p_init = ref_matching.prep_for_iter_proj(X11, X21, None)
    cfg = ref_config.config["matching"]
    p_new, conv = sys.modules["mast3r_slam_backends"].iter_proj(rays, pts, p_init, cfg["max_iter"],
                                                               cfg["lambda_init"], cfg["convergence_thresh"])
    idx, valid = ref_matching.match(X11, X21, D11, D21, None)
    # warm start from a shifted previous solution (tracker re-uses idx_f2k)
    idx_init = torch.clamp(idx + 1, max=H * W - 1)
    idx_w, valid_w = ref_matching.match(X11, X21, D11, D21, idx_init)
    D11h = D11.half().view(torch.int16)
    save(f"matching_{H}x{W}.npz", X11=_np(X11), X21=_np(X21), D11=_np(D11), D21=_np(D21), rays=_np(rays),
         pts=_np(pts), p_init=_np(p_init), p_new=_np(p_new), converged=_np(conv), idx=_np(idx), valid=_np(valid),
         idx_init=_np(idx_init), idx_warm=_np(idx_w), valid_warm=_np(valid_w), D11h=_np(D11h).view(np.uint16))


# ---------------------------------------------------------------- matching at the config sizes, as digests
def _digest(a):
    import hashlib

    a = np.ascontiguousarray(_np(a) if torch.is_tensor(a) else a)
    return hashlib.sha256(a.tobytes()).hexdigest()


def gen_match_digest():
    """The reference's prep_for_iter_proj and match (its torch glue + the oracle's kernels) at the BASELINE config
    sizes, stored as sha256 digests of the exact bytes (the arrays themselves would be ~10 MB each): C1 512x512
    (make_pair seed 11, the GPU config tests' pair) and C2 384x512 with the TUM fr1 intrinsics (seed 11)."""
    out = {}
    for name, H, W, K in (("C1", 512, 512, None), ("C2", 384, 512, synthetic.tum_fr1_intrinsics(384, 512))):
        P = synthetic.make_pair(H, W, seed=11, K=K)
        X, D = P["X"], P["D"]
        X11, X21, D11, D21 = X[:1], X[1:], D[:1], D[1:]
        rays, pts, p_init = ref_matching.prep_for_iter_proj(X11, X21, None)
        idx, valid = ref_matching.match(X11, X21, D11, D21, None)
        out[f"{name}_shape"] = np.array([H, W])
        for k, v in (("rays", rays), ("pts", pts), ("idx", idx), ("valid", valid)):
            out[f"{name}_{k}_sha256"] = np.array(_digest(v))
        out[f"{name}_rays_row0"] = _np(rays[0, 0])  # a readable slice beside the digest
        print(name, "valid fraction", float(valid.float().mean()))
    # C3w: a batch of two TUM-shaped 384x512 pairs (seeds 21, 22) matched from a warm start (synthetic.make_warm_batch:
    # a shifted identity with out-of-range entries), the batched call global_opt's loop-closure matching makes
    H, W = 384, 512
    X11, X21, D11, D21, init = synthetic.make_warm_batch(H, W, (21, 22), K=synthetic.tum_fr1_intrinsics(H, W))
    rays, pts, p_init = ref_matching.prep_for_iter_proj(X11, X21, init)
    idx, valid = ref_matching.match(X11, X21, D11, D21, init)
    out["C3w_shape"] = np.array([H, W])
    for k, v in (("rays", rays), ("pts", pts), ("p_init", p_init), ("idx", idx), ("valid", valid)):
        out[f"C3w_{k}_sha256"] = np.array(_digest(v))
    out["C3w_rays_row0"] = _np(rays[0, 0])
    print("C3w valid fraction", float(valid.float().mean()))
    save("match_digest.npz", **out)


# ---------------------------------------------------------------- tracking (opt_pose_* and track())
class _KFs:
    def __init__(self, kf):
        self.kfs = [kf]

    def last_keyframe(self):
        return self.kfs[-1]

    def __len__(self):
        return len(self.kfs)

    def __getitem__(self, i):
        return self.kfs[i]

    def __setitem__(self, i, v):
        self.kfs[i] = v


def _mk_frame(fid, H, W, T=None):
    img = torch.zeros(1, 3, H, W)
    f = ref_frame.Frame(fid, img, torch.tensor([[H, W]]), torch.tensor([[H, W]]), torch.zeros(H, W, 3))
    f.T_WC = T if T is not None else shim.Sim3.Identity(1)
    return f


def gen_tracking(H=48, W=64, seed=3):
    P = synthetic.make_pair(H, W, seed=seed)
    X, C, D, Q = P["X"], P["C"], P["D"], P["Q"]
    N = H * W
    K = P["K"]
    out = {}
    for use_calib in (False, True):
        ref_config.config["use_calib"] = use_calib
        kf = _mk_frame(0, H, W, shim.Sim3(torch.tensor([[0.1, -0.2, 0.05, 0.0, 0.0, 0.0, 1.0, 1.0]])))
        kf.K = K
        kf.update_pointmap(P["Xk"], P["Ck"])
        frame = _mk_frame(1, H, W, kf.T_WC)
        tr = ref_tracker.FrameTracker(None, _KFs(kf), "cpu")

        def fake_match(model, frame_i, frame_j, idx_i2j_init=None):
            idx, valid = ref_matching.match(X[:1], X[1:], D[:1], D[1:], idx_i2j_init)
            return (idx, valid, X[0].reshape(N, 3), C[0].reshape(N, 1), Q[0].reshape(N, 1), X[1].reshape(N, 3),
                    C[1].reshape(N, 1), Q[1].reshape(N, 1))

        ref_tracker.mast3r_match_asymmetric = fake_match
        steps = []
        orig = ref_tracker.check_convergence

        def counting(*a, **k):
            steps.append(1)
            return orig(*a, **k)

        ref_tracker.check_convergence = counting
        new_kf, info, reloc = tr.track(frame)
        ref_tracker.check_convergence = orig
        tag = "calib" if use_calib else "rays"
        out[tag] = dict(new_kf=np.array(new_kf), reloc=np.array(reloc), T_WCf=_np(frame.T_WC.data),
                        kf_X=_np(kf.X_canon), kf_C=_np(kf.C), idx=_np(tr.idx_f2k) if tr.idx_f2k is not None else
                        np.zeros(0), iters=np.array(len(steps)))
    ref_config.config["use_calib"] = False
    save(f"tracking_{H}x{W}.npz", X=_np(X), C=_np(C), D=_np(D), Q=_np(Q), Xk=_np(P["Xk"]), Ck=_np(P["Ck"]), K=_np(K),
         T_WCk=np.array([0.1, -0.2, 0.05, 0.0, 0.0, 0.0, 1.0, 1.0], np.float32),
         **{f"{t}_{k}": v for t, d in out.items() for k, v in d.items()})


def gen_track_config():
    """The reference's FrameTracker.track (its torch glue, fp32 GN, weighted_pointmap fusion) at the BASELINE config
    sizes on the GPU config tests' pairs and set-up (tests/test_gpu_configs.py: seed 11, keyframe at the identity,
    frame starting at the identity): C1 512x512 rays and calib, C2 384x512 calib with the TUM fr1 intrinsics. Stores
    the frame pose, the GN step count, new_kf and every 997th fused keyframe point (the full pointmap is 3 MB)."""
    out = {}
    for name, H, W, calib, K in (("C1_rays", 512, 512, False, None), ("C1_calib", 512, 512, True, None),
                                 ("C2_calib", 384, 512, True, synthetic.tum_fr1_intrinsics(384, 512))):
        P = synthetic.make_pair(H, W, seed=11, K=K)
        X, C, D, Q = P["X"], P["C"], P["D"], P["Q"]
        N = H * W
        ref_config.config["use_calib"] = calib
        kf = _mk_frame(0, H, W)
        kf.K = P["K"]
        kf.update_pointmap(P["Xk"], P["Ck"])
        frame = _mk_frame(1, H, W)
        tr = ref_tracker.FrameTracker(None, _KFs(kf), "cpu")

        def fake_match(model, frame_i, frame_j, idx_i2j_init=None):
            idx, valid = ref_matching.match(X[:1], X[1:], D[:1], D[1:], idx_i2j_init)
            return (idx, valid, X[0].reshape(N, 3), C[0].reshape(N, 1), Q[0].reshape(N, 1), X[1].reshape(N, 3),
                    C[1].reshape(N, 1), Q[1].reshape(N, 1))

        ref_tracker.mast3r_match_asymmetric = fake_match
        steps = []
        orig = ref_tracker.check_convergence

        def counting(*a, **k):
            steps.append(1)
            return orig(*a, **k)

        ref_tracker.check_convergence = counting
        new_kf, info, reloc = tr.track(frame)
        ref_tracker.check_convergence = orig
        sub = np.arange(0, N, 997)
        out.update({f"{name}_T_WCf": _np(frame.T_WC.data), f"{name}_iters": np.array(len(steps)),
                    f"{name}_new_kf": np.array(new_kf), f"{name}_reloc": np.array(reloc), f"{name}_sub": sub,
                    f"{name}_kf_X_sub": _np(kf.X_canon)[sub], f"{name}_shape": np.array([H, W])})
        print(name, "iters", len(steps), "new_kf", new_kf, "T", _np(frame.T_WC.data))
    ref_config.config["use_calib"] = False
    save("track_config.npz", **out)


def gen_track_seq():
    """Three frames tracked in sequence by the reference's own FrameTracker.track against one keyframe, the bench's
    workload (bench.py bench_tracking): 512x512, the bench's synthetic pairs (seeds 0, 1, 2), the keyframe at the
    identity from pair 0, each frame starting at the previous frame's pose, the tracker's own idx_f2k warm start
    from frame to frame and weighted_pointmap fusion accumulating in the keyframe (N = 1 -> 4). S1 calib (the
    headline mode), S2 rays. Stores every frame's pose, GN step count and new_kf, and the final keyframe's N,
    points and confidences (every 997th)."""
    H, W = 512, 512
    pairs = [synthetic.make_pair(H, W, seed=s) for s in (0, 1, 2)]
    N = H * W
    cur = {"P": None}

    def fake_match(model, frame_i, frame_j, idx_i2j_init=None):
        X, C, D, Q = (cur["P"][k] for k in ("X", "C", "D", "Q"))
        idx, valid = ref_matching.match(X[:1], X[1:], D[:1], D[1:], idx_i2j_init)
        return (idx, valid, X[0].reshape(N, 3), C[0].reshape(N, 1), Q[0].reshape(N, 1), X[1].reshape(N, 3),
                C[1].reshape(N, 1), Q[1].reshape(N, 1))

    ref_tracker.mast3r_match_asymmetric = fake_match
    orig = ref_tracker.check_convergence
    out = {}
    for case, calib in (("S1", True), ("S2", False)):
        ref_config.config["use_calib"] = calib
        kf = _mk_frame(0, H, W)
        kf.K = pairs[0]["K"]
        kf.update_pointmap(pairs[0]["Xk"], pairs[0]["Ck"])
        tr = ref_tracker.FrameTracker(None, _KFs(kf), "cpu")
        out.update({f"{case}_shape": np.array([H, W]), f"{case}_seeds": np.array([0, 1, 2]),
                    f"{case}_calib": np.array(calib)})
        T = kf.T_WC
        for k, P in enumerate(pairs):
            cur["P"] = P
            steps = []

            def counting(*a, **kw):
                steps.append(1)
                return orig(*a, **kw)

            ref_tracker.check_convergence = counting
            frame = _mk_frame(k + 1, H, W, T)
            new_kf, info, reloc = tr.track(frame)
            ref_tracker.check_convergence = orig
            assert not reloc, "sequence frame lost"
            T = frame.T_WC
            out[f"{case}_f{k}_T_WCf"] = _np(T.data)
            out[f"{case}_f{k}_iters"] = np.array(len(steps))
            out[f"{case}_f{k}_new_kf"] = np.array(new_kf)
            print(case, "frame", k, "iters", len(steps), "new_kf", new_kf, "T", _np(T.data))
        sub = np.arange(0, N, 997)
        out.update({f"{case}_sub": sub, f"{case}_kf_X_sub": _np(kf.X_canon)[sub],
                    f"{case}_kf_C_sub": _np(kf.C)[sub], f"{case}_kf_N": np.array(kf.N)})
    ref_config.config["use_calib"] = False
    save("track_seq.npz", **out)


def gen_opt_pose(H=32, W=48, seed=5):
    """opt_pose_* on pre-gathered inputs, fixed seeds (tracker.py:173-266)."""
    P = synthetic.make_pair(H, W, seed=seed)
    N = H * W
    g = torch.Generator().manual_seed(seed)
    Xf = P["X"][1].reshape(N, 3)  # frame points at the matched pixels
    Xk = P["Xk"]
    Qk = P["Q"][0].reshape(N, 1)
    valid = (torch.rand(N, 1, generator=g) < 0.9)
    T_WCk = shim.Sim3(torch.tensor([[0.3, 0.1, -0.2, 0.0, 0.0, 0.0, 1.0, 1.0]]))
    T_WCf = shim.Sim3(torch.tensor([[0.3, 0.1, -0.2, 0.0, 0.0, 0.0, 1.0, 1.0]]))
    tr = ref_tracker.FrameTracker(None, None, "cpu")
    T1, Tr1 = tr.opt_pose_ray_dist_sim3(Xf, Xk, T_WCf, T_WCk, Qk, valid)
    K = P["K"]
    Xf_c = ref_geom.constrain_points_to_ray((H, W), Xf[None], K).squeeze(0)
    Xk_c = ref_geom.constrain_points_to_ray((H, W), Xk[None], K).squeeze(0)
    uv = ref_geom.get_pixel_coords(1, (H, W), device="cpu", dtype=torch.float32).view(-1, 2)
    meas = torch.cat((uv, torch.log(Xk_c[..., 2:3])), dim=-1)
    vmeas = Xk_c[..., 2:3] > 1e-6
    meas[~vmeas.repeat(1, 3)] = 0.0
    T2, Tr2 = tr.opt_pose_calib_sim3(Xf_c, Xk, T_WCf, T_WCk, Qk, valid, meas, vmeas, K, (H, W))
    save(f"optpose_{H}x{W}.npz", Xf=_np(Xf), Xk=_np(Xk), Qk=_np(Qk), valid=_np(valid), T_WCk=_np(T_WCk.data),
         T_WCf=_np(T_WCf.data), K=_np(K), Xf_c=_np(Xf_c), meas=_np(meas), vmeas=_np(vmeas),
         rays_T_WCf=_np(T1.data), rays_T_CkCf=_np(Tr1.data), calib_T_WCf=_np(T2.data), calib_T_CkCf=_np(Tr2.data))


# ---------------------------------------------------------------- BA through FactorGraph
class _BAFrames:
    def __init__(self, Xs, Cs, Twc, img):
        self.fr = []
        for k in range(Xs.shape[0]):
            f = _mk_frame(k, *img, shim.Sim3(Twc[k].view(1, 8).clone()))
            f.X_canon, f.C, f.N = Xs[k].clone(), Cs[k].clone(), 1
            self.fr.append(f)

    def __getitem__(self, i):
        return self.fr[int(i)]

    def update_T_WCs(self, T, idx):
        for k, i in enumerate(idx.tolist()):
            self.fr[int(i)].T_WC = shim.Sim3(T.data[k].reshape(1, 8).clone())


def gen_ba(n_kf=6, H=24, W=32, seed=1):
    G = synthetic.make_graph(n_kf=n_kf, H=H, W=W, seed=seed)
    res = {}
    for mode in ("rays", "calib"):
        frames = _BAFrames(G["Xs"], G["Cs"], G["Twc0"], (H, W))
        fg = ref_go.FactorGraph(None, frames, K=G["K"], device="cpu")
        ii2, jj2, idx2, valid2, Q2 = synthetic.two_way(G)
        E = G["ii"].shape[0]
        fg.ii, fg.jj = G["ii"].clone(), G["jj"].clone()
        fg.idx_ii2jj, fg.idx_jj2ii = idx2[:E].clone(), idx2[E:].clone()
        fg.valid_match_j, fg.valid_match_i = valid2[:E].clone(), valid2[E:].clone()
        fg.Q_ii2jj, fg.Q_jj2ii = Q2[:E].clone(), Q2[E:].clone()
        (fg.solve_GN_rays if mode == "rays" else fg.solve_GN_calib)()
        res[mode] = np.stack([_np(frames[k].T_WC.data[0]) for k in range(n_kf)])
    ii2, jj2, idx2, valid2, Q2 = synthetic.two_way(G)
    save(f"ba_{n_kf}kf_{H}x{W}.npz", Xs=_np(G["Xs"]), Cs=_np(G["Cs"]), Twc0=_np(G["Twc0"]), Twc_gt=_np(G["Twc_gt"]),
         ii=_np(G["ii"]), jj=_np(G["jj"]), idx2=_np(idx2), valid2=_np(valid2), Q2=_np(Q2), K=_np(G["K"]),
         rays_Twc=res["rays"], calib_Twc=res["calib"])


# ---------------------------------------------------------------- FactorGraph.add_factors
def _sym_outputs(seed, H, W, kind):  # restated in tests/test_gpu_factor_graph.py (the inputs are regenerated)
    """Synthetic symmetric-decoder outputs of one keyframe pair, ordered (ii, ji, jj, ij) like
    mast3r_decode_symmetric_batch: the i->j pair from one synthetic pair, the j->i pair from another.
    kind 'good': natural confidences; 'poor': every Q = 1 (no match passes Q_conf); 'one_sided': Qjj = Qij
    = 1 (the j->i direction fails, i->j passes)."""
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


def gen_add_factors(H=32, W=48):
    """The reference's FactorGraph.add_factors (global_opt.py:32-101) over four calls on synthetic symmetric
    decoder outputs, the matcher being the reference's matching.match over the C oracle. Covers the Q filter,
    the both-directions min-match-fraction rule, the consecutive-edge exemption, the is_reloc early return
    (state untouched) and the append order."""
    calls = [  # (ii, jj, kinds, min_match_frac, is_reloc)
        ([0, 1, 0], [1, 2, 2], ["good", "poor", "one_sided"], ref_config.config["local_opt"]["min_match_frac"], False),
        ([2, 0], [3, 3], ["good", "good"], ref_config.config["local_opt"]["min_match_frac"], False),
        ([1, 2], [4, 4], ["poor", "good"], ref_config.config["reloc"]["min_match_frac"], True),
        ([3], [4], ["poor"], ref_config.config["reloc"]["min_match_frac"], True),
    ]
    queue = []

    def match_symmetric(model, feat_i, pos_i, feat_j, pos_j, shape_i, shape_j):
        # mast3r_utils.py:149-187 on the queued decoder outputs
        X, C, D, Q = queue.pop(0)
        b = X.shape[1]
        X11 = torch.cat((X[0], X[2]), dim=0)
        X21 = torch.cat((X[1], X[3]), dim=0)
        D11 = torch.cat((D[0], D[2]), dim=0)
        D21 = torch.cat((D[1], D[3]), dim=0)
        idx_1_to_2, valid_match_2 = ref_matching.match(X11, X21, D11, D21)
        return (idx_1_to_2[:b], idx_1_to_2[b:], valid_match_2[:b], valid_match_2[b:], Q[0].view(b, -1, 1),
                Q[2].view(b, -1, 1), Q[1].view(b, -1, 1), Q[3].view(b, -1, 1))

    ref_go.mast3r_match_symmetric = match_symmetric

    class _KF:
        feat = torch.zeros(1, 1)
        pos = torch.zeros(1, 1, 2)
        img_true_shape = torch.tensor([[H, W]])

    fg = ref_go.FactorGraph(None, [_KF() for _ in range(5)], device="cpu")
    out = {}
    for c, (ii, jj, kinds, mmf, reloc) in enumerate(calls):
        outs = [_sym_outputs(100 * c + 10 * e, H, W, k) for e, k in enumerate(kinds)]
        X, C, D, Q = (torch.stack([o[t] for o in outs], dim=1) for t in range(4))  # (4, b, H, W, ...)
        queue.append((X, C, D, Q))
        ret = fg.add_factors(ii, jj, mmf, is_reloc=reloc)
        # the inputs are regenerated by the test from (seed, kind) with m3s.synthetic; a checksum pins them
        csum = np.array([float(t.double().sum()) for t in (X, C, D, Q)])
        out.update({f"c{c}_seeds": np.array([100 * c + 10 * e for e in range(len(kinds))]),
                    f"c{c}_kinds": np.array(kinds), f"c{c}_csum": csum, f"c{c}_ii": np.array(ii), f"c{c}_jj": np.array(jj), f"c{c}_mmf": np.float32(mmf),
                    f"c{c}_reloc": np.bool_(reloc), f"c{c}_ret": np.bool_(bool(ret)),
                    f"c{c}_ii_out": _np(fg.ii), f"c{c}_jj_out": _np(fg.jj), f"c{c}_idx_ii2jj": _np(fg.idx_ii2jj),
                    f"c{c}_idx_jj2ii": _np(fg.idx_jj2ii), f"c{c}_valid_j": _np(fg.valid_match_j),
                    f"c{c}_valid_i": _np(fg.valid_match_i), f"c{c}_Q_ii2jj": _np(fg.Q_ii2jj),
                    f"c{c}_Q_jj2ii": _np(fg.Q_jj2ii)})
    out["ncalls"] = np.int32(len(calls))
    save(f"add_factors_{H}x{W}.npz", **out)


# ---------------------------------------------------------------- oracle BA rows vs reference geometry
def gen_ba_rows(N=512, seed=11):
    """With T_i = identity the adjoint is I, so the oracle's H_jj / g_j for one edge must equal the
    whitened normal equations built from the reference's own geometry.py Jacobians."""
    g = torch.Generator().manual_seed(seed)
    H, W = 16, 32
    N = H * W
    K = synthetic.intrinsics(H, W)
    Xj = torch.randn(N, 3, generator=g) * 0.3 + torch.tensor([0.0, 0.0, 2.0])
    Tj = torch.tensor([0.02, -0.01, 0.03, 0.01, -0.02, 0.015, 1.0, 1.02])
    Tj[3:7] = Tj[3:7] / Tj[3:7].norm()
    Tij = shim.Sim3(Tj.view(1, 8))
    Xp = Tij.act(Xj)
    idx = torch.randperm(N, generator=g)  # point k of j matches pixel idx[k] of i
    Xs_i_full = torch.zeros(N, 3)
    Xs_i_full[idx] = Xp + 0.01 * torch.randn(N, 3, generator=g)
    Xi = Xs_i_full[idx]
    q = 1.0 + torch.empty(N).exponential_(0.25, generator=g)
    valid_in = torch.rand(N, generator=g) < 0.85
    valid = valid_in & (q > 1.5)  # the kernels' Q_thresh test (gn_kernels.cu:953-957), C = 2 > C_thresh
    out = {}
    pW, dX = ref_geom.act_Sim3(Tij, Xj, jacobian=True)
    for mode in ("points", "rays", "calib"):
        sig = {"points": (0.05, 0.0), "rays": (0.003, 10.0), "calib": (1.0, 10.0)}[mode]
        if mode == "points":
            e = pW - Xi
            J = dX
            sw = torch.where(valid, (1.0 / sig[0]) * q.sqrt(), torch.zeros(()))[:, None].repeat(1, 3)
        elif mode == "rays":
            rd, drd = ref_geom.point_to_ray_dist(pW, jacobian=True)
            rdi = ref_geom.point_to_ray_dist(Xi)
            e = rd - rdi
            J = drd @ dX
            s = torch.where(valid, q.sqrt(), torch.zeros(()))[:, None]
            sw = torch.cat(((1.0 / sig[0]) * s.repeat(1, 3), (1.0 / sig[1]) * s), dim=1)
        else:
            pz, dpz, vproj = ref_geom.project_calib(pW, K, (H, W), jacobian=True, border=-10, z_eps=1e-6)
            tgt = torch.stack(((idx % W).float(), (idx // W).float(), torch.log(Xi[:, 2])), dim=-1)
            e = pz - tgt
            J = dpz @ dX
            ok = valid & vproj[:, 0] & (Xi[:, 2] > 1e-6)
            s = torch.where(ok, q.sqrt(), torch.zeros(()))[:, None]
            sw = torch.cat(((1.0 / sig[0]) * s.repeat(1, 2), (1.0 / sig[1]) * s), dim=1)
        wr = sw * e
        hub = torch.where(wr.abs() < 1.345, torch.ones(()), 1.345 / wr.abs())
        w = hub * sw * sw
        Hm = torch.einsum("nr,nra,nrb->ab", w.double(), J.double(), J.double())
        gv = torch.einsum("nr,nr,nra->a", w.double(), e.double(), J.double())
        out[mode] = (Hm.numpy(), gv.numpy())
    Xs = torch.stack((Xs_i_full, Xj))
    save("ba_rows.npz", Xs=_np(Xs), idx=_np(idx), valid=_np(valid_in), q=_np(q), Tj=_np(Tj), K=_np(K), H=H, W=W,
         **{f"{m}_H": v[0] for m, v in out.items()}, **{f"{m}_g": v[1] for m, v in out.items()})


# ---------------------------------------------------------------- retrieval quantization
def gen_retrieval():
    for name in ("mast3r", "mast3r.retrieval", "mast3r.retrieval.processor", "mast3r.retrieval.model", "asmk",
                 "asmk.io_helpers"):
        sys.modules.setdefault(name, types.ModuleType(name))
    sys.modules["mast3r.retrieval.processor"].Retriever = object
    sys.modules["mast3r.retrieval.model"].how_select_local = None
    sys.modules["asmk"].io_helpers = sys.modules["asmk.io_helpers"]
    import mast3r_slam.retrieval_database as ref_rd

    out = {}
    # (seed, C, D, M, k): ragged codebook / feature sizes, one and two query groups, query and build k
    cases = [(21, 1000, 200, 37, 5), (22, 2048, 64, 310, 1), (23, 777, 96, 64, 8)]
    for i, (seed, C, D, M, k) in enumerate(cases):
        c, q = synthetic.retrieval_inputs(seed, C, D, M)
        fake = types.SimpleNamespace(centroids=torch.from_numpy(c))
        idx = ref_rd.RetrievalDatabase.quantize_custom(fake, torch.from_numpy(q), {"quantize": {"multiple_assignment": k}})
        out[f"case{i}"] = np.array([seed, C, D, M, k])
        out[f"case{i}_topk"] = _np(idx)
        out[f"case{i}_checksum"] = np.array([c.astype(np.float64).sum(), q.astype(np.float64).sum()])
    save("retrieval_quantize.npz", **out)


if __name__ == "__main__":
    if len(sys.argv) > 1:
        for name in sys.argv[1:]:
            globals()["gen_" + name]()
        sys.exit(0)
    gen_matching()
    gen_match_digest()
    gen_tracking()
    gen_track_config()
    gen_track_seq()
    gen_opt_pose()
    gen_ba()
    gen_ba_rows()
    gen_retrieval()
    gen_add_factors()
