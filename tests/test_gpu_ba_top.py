"""GPU parity: the dense top phase of the BA factorisation (M3S_BA_TOP=t: ba_top_plan in ba_pattern.cpp,
ba_dense_top_kernel in ba.hip; the root end of the elimination tree factored densely on the matrix cores between a
factor-only and a back-substitution-only run of the one-workgroup kernel) against the fp64 truth
(oracle/liboracle_m3s_f64.so, the checker only), the column-task solver and itself.

The factorisation replaced is SparseBlock + SimplicialLLT (/root/reference/mast3r_slam/backend/src/gn_kernels.cu:57-159),
called every GN iteration from the host loop (gn_kernels.cu:1181-1225)."""
import numpy as np
import pytest
import torch

import oracle.oracle as O

pytestmark = pytest.mark.gpu

SIG = {"points": (0.05, 0.0), "rays": (0.003, 10.0), "calib": (1.0, 10.0)}


def _traj(traj, H, W):
    from m3s.synthetic import chess_poses, euroc_poses, make_traj_graph

    G = make_traj_graph((chess_poses if traj == "chess" else euroc_poses)(256), H, W, seed=1, device="cpu")
    return {k: (v.numpy() if torch.is_tensor(v) else v) for k, v in G.items()}


def _solve(monkeypatch, G, mode, top, iters=4, delta=0.0):
    import mast3r_slam_backends as B

    monkeypatch.setenv("M3S_BA_SOLVER", "sparse")  # (the cost model may pick the dense solver for small graphs)
    if top:
        monkeypatch.setenv("M3S_BA_TOP", str(top))
    else:
        monkeypatch.delenv("M3S_BA_TOP", raising=False)
    c = lambda a, dt=None: (torch.from_numpy(np.ascontiguousarray(a)) if dt is None
                            else torch.from_numpy(np.ascontiguousarray(a)).to(dt)).cuda()
    Xs = G["Xs"]
    H, W = int(G["H"]), int(G["W"])
    if mode == "calib":
        Xs = O.backproject_constrain(Xs, G["K"], (H, W))
    args = (c(Xs), c(G["Cs"]), c(G["ii"]), c(G["jj"]), c(G["idx"]), c(G["valid"], torch.bool), c(G["Q"]))
    T = c(G["Twc0"])
    sa, sb = SIG[mode]
    if mode == "rays":
        dx = B.gauss_newton_rays(T, *args, sa, sb, 0.0, 1.5, iters, delta)[0]
    else:
        Xs_, Cs_, ii_, jj_, idx_, v_, Q_ = args
        dx = B.gauss_newton_calib(T, Xs_, Cs_, c(G["K"]), ii_, jj_, idx_, v_, Q_, H, W, -10, 1e-6, sa, sb, 0.0, 1.5,
                                  iters, delta)[0]
    return T.cpu().numpy(), dx.cpu().numpy(), Xs


def _top_poses(monkeypatch, G, mode, top):
    """m3s_ba_plan_info[12] of a plan of this graph under M3S_BA_TOP=top (HipShard: the plan API the solves use)."""
    import ctypes

    from m3s import _lib
    from m3s.config import config
    from m3s.dist_ba import HipShard, ba_config

    monkeypatch.setenv("M3S_BA_TOP", str(top))
    monkeypatch.setenv("M3S_BA_SOLVER", "sparse")
    d = lambda a, dt=None: (torch.from_numpy(np.ascontiguousarray(a)) if dt is None
                            else torch.from_numpy(np.ascontiguousarray(a)).to(dt)).cuda()
    H, W = int(G["H"]), int(G["W"])
    Xs = G["Xs"] if mode != "calib" else O.backproject_constrain(G["Xs"], G["K"], (H, W))
    cfg = ba_config(mode, config["local_opt"], K=d(G["K"]), height=H, width=W)
    E = G["ii"].shape[0]
    sh = HipShard(cfg, d(G["Twc0"]), d(Xs), d(G["Cs"][..., 0]), d(G["ii"]), d(G["jj"]), d(G["idx"]),
                  d(G["valid"][..., 0]), d(G["Q"][..., 0]), 0.0, 0, E)
    info = (ctypes.c_int * 13)()
    _lib.check(_lib.load().m3s_ba_plan_info(ctypes.byref(sh.plan), info))
    return info[12]


# the chess graph: its dataflow schedule fits the one-workgroup kernel's LDS (the top phase needs it; the 24x32 EuRoC
# graph's tables do not fit, so its plans run level-synchronously without a top phase)
@pytest.mark.parametrize("traj,mode", [("chess", "calib"), ("chess", "rays")])
@pytest.mark.parametrize("top", [8, 25])
def test_dense_top_k256_vs_fp64_truth_and_column_solver(monkeypatch, traj, mode, top):
    """The K = 256 chess trajectory graph (the C5 bench graph's trajectory at 24x32), calib and rays: with the top phase (the plan reports its poses,
    m3s_ba_plan_info[12]) the solve stays within 1e-5 of the fp64 truth and within 1e-6 of the column-task solver (fp64
    factors that differ only in summation order), and is deterministic."""
    G = _traj(traj, 24, 32)
    T_top, dx_top, Xs = _solve(monkeypatch, G, mode, top)
    T_col, dx_col, _ = _solve(monkeypatch, G, mode, 0)
    sa, sb = SIG[mode]
    p = O.ba_params(mode, sa, sb, 0.0, 1.5, K=G["K"], height=int(G["H"]), width=int(G["W"]), pixel_border=-10,
                    z_eps=1e-6)
    T64, dx64, _ = O.gauss_newton_f64(mode, G["Twc0"], Xs, G["Cs"][..., 0], G["ii"], G["jj"], G["idx"],
                                      G["valid"][..., 0], G["Q"][..., 0], p, 4, 0.0)
    print(f"{traj} {mode} top {top}: vs fp64 truth {np.abs(T_top - T64).max():.2e} (dx {np.abs(dx_top - dx64).max():.2e}),"
          f" vs column solver {np.abs(T_top - T_col).max():.2e} (dx {np.abs(dx_top - dx_col).max():.2e})")
    np.testing.assert_allclose(T_top, T64, rtol=0, atol=1e-5)
    np.testing.assert_allclose(dx_top, dx64, rtol=0, atol=1e-5)
    np.testing.assert_allclose(T_top, T_col, rtol=0, atol=1e-6)
    np.testing.assert_allclose(dx_top, dx_col, rtol=0, atol=1e-6)
    assert _top_poses(monkeypatch, G, mode, top) > 0, "the plan has no dense top phase"
    again = _solve(monkeypatch, G, mode, top)
    assert np.array_equal(again[0], T_top) and np.array_equal(again[1], dx_top)


def test_dense_top_singular_system_returns_zero_step(monkeypatch):
    """No valid matches -> a singular system -> a non-positive pivot (in the dense top phase: every column of this
    3-keyframe graph is in it) -> dx = 0, Twc unchanged (gn_kernels.cu:147-150)."""
    import mast3r_slam_backends as B

    monkeypatch.setenv("M3S_BA_TOP", "25")
    monkeypatch.setenv("M3S_BA_SOLVER", "sparse")
    N = 256
    Xs = np.random.default_rng(0).standard_normal((3, N, 3)).astype(np.float32) + np.array([0, 0, 3], np.float32)
    Twc0 = np.tile(np.array([0, 0, 0, 0, 0, 0, 1, 1], np.float32), (3, 1))
    Twc0[1, 0] = 0.1
    c = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    T = c(Twc0)
    dx = B.gauss_newton_rays(T, c(Xs), c(np.full((3, N, 1), 2.0, np.float32)), c(np.array([0, 1])),
                             c(np.array([1, 2])), c(np.tile(np.arange(N), (2, 1))), c(np.zeros((2, N, 1), bool)),
                             c(np.full((2, N, 1), 2.0, np.float32)), 0.003, 10.0, 0.0, 1.5, 10, 1e-8)[0]
    assert torch.all(dx == 0) and np.array_equal(T.cpu().numpy(), Twc0)


@pytest.mark.parametrize("mode", ["points", "rays", "calib"])
def test_dense_top_golden_6kf(golden, monkeypatch, mode):
    """The 6-keyframe golden graph (tests/golden/ba_6kf_24x32.npz, made by the reference's own global_opt glue): the
    solve with the dense top phase within 1e-5 of the fp64 truth."""
    import mast3r_slam_backends as B

    monkeypatch.setenv("M3S_BA_TOP", "25")
    monkeypatch.setenv("M3S_BA_SOLVER", "sparse")
    g = golden("ba_6kf_24x32.npz")
    H, W = 24, 32
    Xs = g["Xs"] if mode != "calib" else O.backproject_constrain(g["Xs"], g["K"], (H, W))
    ii, jj = np.concatenate((g["ii"], g["jj"])), np.concatenate((g["jj"], g["ii"]))
    sa, sb = SIG[mode]
    c = lambda a, dt=None: (torch.from_numpy(np.ascontiguousarray(a)) if dt is None
                            else torch.from_numpy(np.ascontiguousarray(a)).to(dt)).cuda()
    args = (c(Xs), c(g["Cs"]), c(ii), c(jj), c(g["idx2"]), c(g["valid2"], torch.bool), c(g["Q2"]))
    T = c(g["Twc0"])
    if mode == "rays":
        B.gauss_newton_rays(T, *args, sa, sb, 0.0, 1.5, 10, 1e-8)
    elif mode == "points":
        B.gauss_newton_points(T, *args, sa, 0.0, 1.5, 10, 1e-8)
    else:
        a_ = args
        B.gauss_newton_calib(T, a_[0], a_[1], c(g["K"]), a_[2], a_[3], a_[4], a_[5], a_[6], H, W, -10, 1e-6, sa, sb,
                             0.0, 1.5, 10, 1e-8)
    p = O.ba_params(mode, sa, sb, 0.0, 1.5, K=g["K"], height=H, width=W, pixel_border=-10, z_eps=1e-6)
    T64, _, _ = O.gauss_newton_f64(mode, g["Twc0"], Xs, g["Cs"][..., 0], ii, jj, g["idx2"], g["valid2"][..., 0],
                                   g["Q2"][..., 0], p, 10, 1e-8)
    err = np.abs(T.cpu().numpy() - T64).max()
    print(f"6-KF {mode} dense top vs fp64 truth {err:.2e}")
    assert err <= 1e-5
