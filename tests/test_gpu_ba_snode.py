"""GPU parity: the supernodal BA factorisation (M3S_BA_SOLVER=snode: ba_snode.hip + ba_snode.cpp) against the fp64
truth (oracle/liboracle_m3s_f64.so, the checker only), the column-task solver and itself.

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


def _solve(monkeypatch, G, mode, env, iters=4, delta=0.0):
    import mast3r_slam_backends as B

    for k in ("M3S_BA_SOLVER", "M3S_BA_SN_CUT"):
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
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


@pytest.mark.parametrize("traj,mode", [("chess", "calib"), ("euroc", "rays")])
def test_snode_k256_vs_fp64_truth_and_column_solver(monkeypatch, traj, mode):
    """K = 256 trajectory graphs (the C5 / C4 bench graphs at 24x32): the supernodal solve within 1e-5 of the fp64
    truth, within 1e-6 of the column-task solver (fp64 factors that differ only in summation order), deterministic,
    and bit-identical at every supernodal cut (the cut moves supernodes between launches, never their arithmetic)."""
    G = _traj(traj, 24, 32)
    T_sn, dx_sn, Xs = _solve(monkeypatch, G, mode, {"M3S_BA_SOLVER": "snode"})
    T_sp, dx_sp, _ = _solve(monkeypatch, G, mode, {"M3S_BA_SOLVER": "sparse"})
    sa, sb = SIG[mode]
    p = O.ba_params(mode, sa, sb, 0.0, 1.5, K=G["K"], height=int(G["H"]), width=int(G["W"]), pixel_border=-10,
                    z_eps=1e-6)
    T64, dx64, _ = O.gauss_newton_f64(mode, G["Twc0"], Xs, G["Cs"][..., 0], G["ii"], G["jj"], G["idx"],
                                      G["valid"][..., 0], G["Q"][..., 0], p, 4, 0.0)
    print(f"{traj} {mode}: snode vs fp64 truth {np.abs(T_sn - T64).max():.2e} (dx {np.abs(dx_sn - dx64).max():.2e}), "
          f"vs column solver {np.abs(T_sn - T_sp).max():.2e}")
    np.testing.assert_allclose(T_sn, T64, rtol=0, atol=1e-5)
    np.testing.assert_allclose(dx_sn, dx64, rtol=0, atol=1e-5)
    np.testing.assert_allclose(T_sn, T_sp, rtol=0, atol=1e-6)
    again = _solve(monkeypatch, G, mode, {"M3S_BA_SOLVER": "snode"})
    assert np.array_equal(again[0], T_sn) and np.array_equal(again[1], dx_sn)
    for cut in ("0", "1", "3", "1000"):
        T, dx, _ = _solve(monkeypatch, G, mode, {"M3S_BA_SOLVER": "snode", "M3S_BA_SN_CUT": cut})
        assert np.array_equal(T, T_sn) and np.array_equal(dx, dx_sn), f"cut {cut}"


def test_snode_singular_system_returns_zero_step(monkeypatch):
    """No valid matches -> singular system -> a non-positive pivot -> dx = 0, Twc unchanged (gn_kernels.cu:147-150)."""
    import mast3r_slam_backends as B

    monkeypatch.setenv("M3S_BA_SOLVER", "snode")
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
def test_snode_golden_6kf(golden, monkeypatch, mode):
    """The 6-keyframe golden graph (tests/golden/ba_6kf_24x32.npz, made by the reference's own global_opt glue): the
    supernodal solve within 1e-5 of the fp64 truth."""
    import mast3r_slam_backends as B

    monkeypatch.setenv("M3S_BA_SOLVER", "snode")
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
    print(f"6-KF {mode} snode vs fp64 truth {err:.2e}")
    assert err <= 1e-5
