"""CPU: host logic, the C-ABI library surface, the Sim3 stand-in and config handling."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

import oracle.oracle as O

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_abi_library_exports_every_declared_symbol():
    from m3s import _lib

    header = open(os.path.join(REPO, "include", "m3s.h")).read()
    declared = set(re.findall(r"\b(m3s_[a-z0-9_]+)\s*\(", header))
    assert declared, "no declarations parsed"
    lib = ctypes.CDLL(_lib.LIB_PATH)  # loads without a GPU
    missing = [s for s in sorted(declared) if not hasattr(lib, s)]
    assert not missing, missing
    assert declared == set(_lib.EXPORTED)  # the ctypes table binds exactly the header
    lib.m3s_abi_version.restype = ctypes.c_int
    hdr_version = int(re.search(r"#define M3S_ABI_VERSION (\d+)", header).group(1))
    assert lib.m3s_abi_version() == hdr_version == _lib.ABI_VERSION


def test_workspace_sizes_are_monotone():
    from m3s import _lib

    lib = ctypes.CDLL(_lib.LIB_PATH)
    for name, args in (("m3s_match_workspace_size", [(1, 64, 64, 24), (2, 64, 64, 24), (1, 512, 512, 24)]),
                       ("m3s_track_workspace_size", [(1024,), (4096,), (262144,)]),
                       ("m3s_ba_workspace_size", [(4, 1024, 6), (8, 1024, 20), (256, 196608, 2000)]),
                       ("m3s_codebook_size", [(100, 64), (1000, 200), (65536, 1024)]),
                       ("m3s_quantize_workspace_size", [(100, 64, 10, 1), (1000, 64, 310, 5), (65536, 1024, 300, 8)])):
        fn = getattr(lib, name)
        fn.restype = ctypes.c_size_t
        sizes = [fn(*a) for a in args]
        assert sizes == sorted(sizes) and sizes[0] > 0


def test_backends_reject_like_reference_and_never_fall_back():
    import mast3r_slam_backends as B

    rays = torch.zeros(1, 8, 8, 9).transpose(1, 2)
    with pytest.raises(RuntimeError, match="must be contiguous"):
        B.iter_proj(rays, torch.zeros(1, 64, 3), torch.zeros(1, 64, 2), 10, 1e-8, 1e-6)
    if not torch.cuda.is_available():
        with pytest.raises(RuntimeError, match="no HIP device"):
            B.iter_proj(torch.zeros(1, 8, 8, 9), torch.zeros(1, 64, 3), torch.zeros(1, 64, 2), 10, 1e-8, 1e-6)
        with pytest.raises(RuntimeError, match="no HIP device"):
            B.refine_matches(torch.zeros(1, 8, 8, 24, dtype=torch.float16), torch.zeros(1, 64, 24, dtype=torch.float16),
                             torch.zeros(1, 64, 2, dtype=torch.int64), 3, 5)


def _shim():
    import oracle.lietorch_shim as shim

    return shim


def test_sim3_matches_oracle_shim_and_fp64():
    from m3s.sim3 import Sim3

    shim = _shim()
    g = torch.Generator().manual_seed(0)
    xi = torch.randn(16, 7, generator=g) * torch.tensor([0.3, 0.3, 0.3, 0.5, 0.5, 0.5, 0.2])
    xi[0] = 0
    xi[1, 3:6] = 1e-5  # small-angle branch
    xi[2, 6] = 1e-8  # |sigma| < EPS branch
    a = Sim3.exp(xi)
    b = shim.Sim3.exp(xi)
    np.testing.assert_allclose(a.data.numpy(), b.data.numpy(), atol=2e-6)
    for k in range(16):
        # the float closed form (lietorch / gn_kernels.cu:360-372) cancels for small theta & sigma:
        # vs the fp64 truth only ~1e-4; vs the float restatement tightly
        np.testing.assert_allclose(a.data[k].numpy(), O.sim3_exp(xi[k].double().numpy()), atol=1e-4)
        np.testing.assert_allclose(a.data[k].numpy(), O.exp_sim3_f32(xi[k].numpy()), atol=2e-6)
    p = torch.randn(16, 5, 3, generator=g)
    T1, T2 = Sim3.exp(xi), Sim3.exp(xi.flip(0))
    np.testing.assert_allclose((T1 * T2).act(p).numpy(), T1.act(T2.act(p)).numpy(), atol=2e-5)
    np.testing.assert_allclose((T1.inv() * T1).data.numpy(), Sim3.Identity(16).data.numpy(), atol=2e-6)
    np.testing.assert_allclose(T1.retr(xi.flip(0)).data.numpy(), (Sim3.exp(xi.flip(0)) * T1).data.numpy(), atol=1e-6)
    M = T1.matrix()
    ph = torch.cat((p, torch.ones(16, 5, 1)), -1)
    np.testing.assert_allclose((M[:, None] @ ph[..., None])[..., :3, 0].numpy(), T1.act(p).numpy(), atol=2e-5)


def test_config_loads_reference_style_yaml(tmp_path):
    from m3s.config import config, load_config

    base = tmp_path / "base.yaml"
    base.write_text("matching:\n  radius: 2\n  lambda_init: 1e-7\ntracking:\n  sigma_ray: 5e-3\n")
    child = tmp_path / "child.yaml"
    child.write_text(f'inherit: "{base}"\nuse_calib: True\ndataset:\n  subsample: 2\n')
    load_config(str(child))
    assert config["use_calib"] is True and config["matching"]["radius"] == 2
    assert isinstance(config["matching"]["lambda_init"], float) and config["matching"]["lambda_init"] == 1e-7
    assert config["tracking"]["sigma_ray"] == 5e-3 and config["tracking"]["max_iters"] == 50  # defaults kept
    assert config["dataset"]["subsample"] == 2


def test_shard_range_partitions_edges():
    from m3s.dist_ba import shard_range

    for E in (0, 1, 7, 2000, 2001):
        for world in (1, 2, 3, 8):
            rs = [shard_range(E, r, world) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == E
            assert all(rs[r][1] == rs[r + 1][0] for r in range(world - 1))
            sizes = [b - a for a, b in rs]
            assert max(sizes) - min(sizes) <= 1


def test_frame_weighted_fusion_matches_reference_formula():
    from m3s.frame import Frame

    g = torch.Generator().manual_seed(0)
    f = Frame(0, (4, 4))
    X1, C1 = torch.randn(16, 3, generator=g), torch.rand(16, 1, generator=g) + 1
    X2, C2 = torch.randn(16, 3, generator=g), torch.rand(16, 1, generator=g) + 1
    f.update_pointmap(X1, C1)
    f.update_pointmap(X2, C2)
    assert f.N == 2 and f.N_updates == 2
    torch.testing.assert_close(f.X_canon, (C1 * X1 + C2 * X2) / (C1 + C2))
    torch.testing.assert_close(f.get_average_conf(), (C1 + C2) / 2)


def test_frame_owned_pointmap_is_copied_before_in_place_modes():
    """update_pointmap(own=True) keeps the caller's tensors (no clone); indep_conf, the one in-place
    mode (frame.py:57-61), copies them first, so the caller's buffer is never written."""
    from m3s.config import config
    from m3s.frame import Frame

    g = torch.Generator().manual_seed(1)
    X1, C1 = torch.randn(16, 3, generator=g), torch.rand(16, 1, generator=g) + 1
    X2, C2 = torch.randn(16, 3, generator=g), torch.rand(16, 1, generator=g) + 2
    X1_ref, C1_ref = X1.clone(), C1.clone()
    mode = config["tracking"]["filtering_mode"]
    try:
        config["tracking"]["filtering_mode"] = "indep_conf"
        f = Frame(0, (4, 4))
        f.update_pointmap(X1, C1, own=True)
        assert f.X_canon is X1 and f.shared
        f.update_pointmap(X2, C2)
        torch.testing.assert_close(X1, X1_ref)  # caller buffer untouched
        torch.testing.assert_close(C1, C1_ref)
        m = C2 > C1_ref
        torch.testing.assert_close(f.X_canon, torch.where(m, X2, X1_ref))
        assert not f.shared
    finally:
        config["tracking"]["filtering_mode"] = mode


@pytest.mark.parametrize("use_calib", [False, True])
def test_slot_frame_is_the_store_record(use_calib):
    """FrameTracker._last_keyframe reads a buffer-backed store's last slot inside its one lock hold (slot_frame): the
    same record SharedKeyframes.__getitem__ returns (frame.py:248-267), views of the same slot rows and the same
    scalars, without the nested lock and with one scalar copy instead of three."""
    import multiprocessing as mp

    from m3s.config import config
    from m3s.frame import Frame, SharedKeyframes, slot_frame
    from m3s.sim3 import Sim3
    from m3s.tracker import FrameTracker

    H, W = 16, 32
    g = torch.Generator().manual_seed(5)
    manager = mp.get_context("spawn").Manager()
    config["use_calib"] = use_calib
    try:
        kfs = SharedKeyframes(manager, H, W, buffer=4, device="cpu", feat_dim=8)
        for fid in (7, 9):
            kf = Frame(fid, (H, W), T_WC=Sim3(torch.randn(1, 8, generator=g)))
            kf.update_pointmap(torch.randn(H * W, 3, generator=g), torch.rand(H * W, 1, generator=g) + 1)
            kf.update_pointmap(torch.randn(H * W, 3, generator=g), torch.rand(H * W, 1, generator=g) + 1)
            kf.img, kf.uimg = torch.rand(3, H, W, generator=g), torch.rand(H, W, 3, generator=g)
            kf.img_shape = torch.tensor([[H, W]], dtype=torch.int)
            kf.img_true_shape = kf.img_shape.clone()
            kf.feat = torch.rand(1, H * W // 256, 8, generator=g)
            kf.pos = torch.randint(0, 9, (1, H * W // 256, 2), generator=g)
            kfs.append(kf)
        ref, got = kfs[1], slot_frame(kfs, 1)
        assert (got.frame_id, got.N, got.N_updates) == (ref.frame_id, ref.N, ref.N_updates) == (9, 2, 2)
        assert all(type(v) is int for v in (got.frame_id, got.N, got.N_updates))
        for a in ("img", "uimg", "img_shape", "img_true_shape", "X_canon", "C", "feat", "pos"):
            assert getattr(got, a).data_ptr() == getattr(ref, a).data_ptr(), a
        assert got.T_WC.data.data_ptr() == ref.T_WC.data.data_ptr() and got.shared
        assert (got.K is kfs.K) if use_calib else got.K is None
        kf, idx = FrameTracker(None, kfs, "cpu")._last_keyframe()
        assert idx == 1 and kf.frame_id == 9 and kf.X_canon.data_ptr() == kfs.X[1].data_ptr()
        assert slot_frame([], 0) is None  # not buffer-backed: the tracker falls back to store[idx]
    finally:
        config["use_calib"] = False
        manager.shutdown()


def test_synthetic_pair_is_consistent():
    from m3s.sim3 import Sim3
    from m3s.synthetic import make_pair

    P = make_pair(32, 48, seed=0, noise=0.0)
    X21 = P["X"][1].reshape(-1, 3)
    np.testing.assert_allclose(Sim3(P["T_gt"].view(1, 8)).act(X21).numpy(), P["Xk"].numpy(), atol=1e-5)
    D = P["D"]
    np.testing.assert_allclose(D.norm(dim=-1).numpy(), 1.0, atol=1e-5)
    assert (P["Q"] > 1.0).all() and (P["C"] > 1.0).all()


def test_se3_is_sim3_with_unit_scale_and_as_se3_pattern():
    """lietorch_utils.py:6-13 (as_SE3) against the package's lietorch: SE3 from a Sim3's t, q."""
    import lietorch
    import torch

    g = torch.Generator().manual_seed(0)
    q = torch.randn(5, 4, generator=g, dtype=torch.float64)
    q = q / q.norm(dim=-1, keepdim=True)
    t = torch.randn(5, 3, generator=g, dtype=torch.float64)
    s = torch.ones(5, 1, dtype=torch.float64)
    T = lietorch.Sim3(torch.cat((t, q, s), -1))
    t_, q_, _ = T.data.split([3, 4, 1], -1)
    E = lietorch.SE3(torch.cat([t_, q_], dim=-1))
    p = torch.randn(5, 3, generator=g, dtype=torch.float64)
    assert isinstance(E, lietorch.SE3)
    torch.testing.assert_close(E.act(p), T.act(p))
    torch.testing.assert_close((E * E.inv()).data, lietorch.SE3.Identity(5, dtype=torch.float64).data,
                               atol=1e-12, rtol=0)
    torch.testing.assert_close(E.matrix(), T.matrix())
    assert lietorch.Sim3.embedded_dim == 8 and lietorch.SE3.embedded_dim == 7


def test_retrieval_abi_validates_before_any_launch():
    """m3s_codebook_* / m3s_quantize reject bad sizes, k and buffers with an error code and a message before
    touching the device (runs without a GPU)."""
    from m3s import _lib

    lib = ctypes.CDLL(_lib.LIB_PATH)
    lib.m3s_last_error.restype = ctypes.c_char_p
    for name in ("m3s_codebook_size", "m3s_quantize_workspace_size"):
        getattr(lib, name).restype = ctypes.c_size_t
    assert lib.m3s_codebook_size(0, 64) == 0 and lib.m3s_quantize_workspace_size(10, 64, 5, 0) == 0
    buf = ctypes.create_string_buffer(16)
    p = ctypes.cast(buf, ctypes.c_void_p)
    q = ctypes.c_void_p
    rc = lib.m3s_quantize(p, 10, 64, p, 5, 9, p, p, ctypes.c_size_t(1 << 30), q(0))
    assert rc != 0 and b"multiple_assignment" in lib.m3s_last_error()
    rc = lib.m3s_quantize(p, 4, 64, p, 5, 5, p, p, ctypes.c_size_t(1 << 30), q(0))
    assert rc != 0 and b"larger than the codebook" in lib.m3s_last_error()
    rc = lib.m3s_quantize(p, 100, 64, p, 5, 5, p, p, ctypes.c_size_t(16), q(0))
    assert rc != 0 and b"workspace too small" in lib.m3s_last_error()
    rc = lib.m3s_codebook_prepare(p, 100, 64, p, ctypes.c_size_t(16), q(0))
    assert rc != 0 and b"too small" in lib.m3s_last_error()
    rc = lib.m3s_quantize(q(0), 100, 64, p, 5, 5, p, p, ctypes.c_size_t(1 << 30), q(0))
    assert rc != 0 and b"null" in lib.m3s_last_error()


def _min_degree_symbolic(ii, jj, Kp):
    """Independent restatement of the plan's symbolic analysis (ba_pattern.cpp): minimum-degree
    elimination on the pose graph (pin removed, ties to the lowest index), the factor's block count,
    its elimination-tree height, and the update groups: one per (source level, target column), the
    group of a column's children's level run by its own factor task."""
    u = np.unique(np.concatenate([ii, jj]))
    ri, rj = np.searchsorted(u, ii) - 1, np.searchsorted(u, jj) - 1
    nb = Kp - 1
    adj = [set() for _ in range(nb)]
    for a, b in zip(ri, rj):
        if a >= 0 and b >= 0 and a != b:
            adj[a].add(b)
            adj[b].add(a)
    alive, order, struct = set(range(nb)), [], {}
    while alive:
        v = min(alive, key=lambda x: (len(adj[x]), x))
        order.append(v)
        alive.remove(v)
        nv = set(adj[v])
        struct[v] = nv
        for a in nv:
            adj[a] |= nv
            adj[a] -= {a, v}
        adj[v] = set()
    pos = {v: k for k, v in enumerate(order)}
    S = [sorted(pos[a] for a in struct[order[j]]) for j in range(nb)]
    lev = [0] * nb
    for j in range(nb):
        if S[j]:
            lev[S[j][0]] = max(lev[S[j][0]], lev[j] + 1)
    nlev = max(lev) + 1 if nb else 0
    pairs_kj = [(k, j) for k in range(nb) for j in S[k]]
    groups = len({(lev[k], j) for k, j in pairs_kj})
    sidx = sum(len(S[j]) + 1 for k, j in pairs_kj)
    pulls = len({j for k, j in pairs_kj if lev[k] == lev[j] - 1})
    return nb + len(pairs_kj), nlev, groups, len(pairs_kj), sidx, pulls


@pytest.mark.parametrize("kind", ["chain", "loops", "chess"])
def test_ba_symbolic_factorisation_matches_restatement(kind):
    """The BA plan's block-sparse pattern (SparseBlock's system, gn_kernels.cu:57-159) against an
    independent Python elimination: identical fill, elimination-tree height and update lists."""
    from m3s import _lib

    if kind == "chain":  # consecutive edges only: tridiagonal, no fill
        K = 40
        und = [(k - 1, k) for k in range(1, K)]
    elif kind == "loops":
        K, g = 60, np.random.default_rng(3)
        und = [(k - 1, k) for k in range(1, K)] + [(int(c), k) for k in range(4, K)
                                                   for c in g.choice(k - 1, 3, replace=False)]
    else:  # the K=256 chess trajectory's loop-closure graph used by the BA bench and config tests
        from m3s.synthetic import chess_poses, make_traj_graph

        G = make_traj_graph(chess_poses(256), 12, 16, covis_grid=(12, 16))
        K = 256
        und = list(zip(G["ii"][: G["E_und"]].tolist(), G["jj"][: G["E_und"]].tolist()))
    ii = np.array([a for a, b in und] + [b for a, b in und], dtype=np.int64) * 3 + 7  # global ids, remapped
    jj = np.array([b for a, b in und] + [a for a, b in und], dtype=np.int64) * 3 + 7
    got = _lib.ba_pattern_stats(ii, jj, K)
    want = _min_degree_symbolic(ii, jj, K)
    assert got == want
    nb = K - 1
    assert got[0] <= nb * (nb + 1) // 2
    if kind == "chain":
        assert got[0] == 2 * nb - 1
    if kind == "chess":  # the point of the sparse solve: little fill, a short elimination tree
        assert got[0] < 0.1 * nb * (nb + 1) // 2 and got[1] < nb // 2


def test_factor_graph_rejects_pin_above_one():
    """SURVEY.md §8 a-note 8: the C++ solvers fix exactly one pose (gn_kernels.cu:741,1157,1566) while the Python
    write-back slices by cfg.pin (global_opt.py:125,161): a pin above 1 would drop solved poses and is rejected before
    a solve starts; pin = 0 is accepted (pose 0 is fixed in the solve either way)."""
    from m3s.global_opt import FactorGraph

    fg = FactorGraph(None, [], device="cpu")
    for pin in (0, 1):
        assert FactorGraph._pin(dict(fg.cfg, pin=pin)) == pin
    for pin in (2, 3):
        fg.cfg = dict(fg.cfg, pin=pin)
        for fn in (fg.solve_GN_rays, fg.solve_GN_calib):
            with pytest.raises(ValueError, match="pin"):
                fn()


def test_workspace_release_entry_points_are_safe_without_state():
    """m3s_track_release / m3s_ba_plan_release / m3s_ba_reuse_release forget the library's per-workspace host state
    (a freed workspace's address can be reused): they succeed on an address the library never saw and
    need no GPU."""
    from m3s import _lib

    lib = ctypes.CDLL(_lib.LIB_PATH)
    for name in ("m3s_track_release", "m3s_ba_plan_release", "m3s_ba_reuse_release"):
        fn = getattr(lib, name)
        fn.argtypes = [ctypes.c_void_p]
        fn.restype = ctypes.c_int
        assert fn(ctypes.c_void_p(0x1234000)) == 0
        assert fn(None) == 0


def test_isa_spill_check_flags_spilling_kernels(tmp_path):
    """scripts/isa_check_spills.py (the Makefile's no-spill gate on refine_tile_kernel and ba_lin_kernel) fails on a
    named kernel whose AMDGPU metadata reports spilled VGPRs, passes when none do, and fails when no kernel matches."""
    import subprocess
    import sys

    def meta(name, spills):
        return (f"  - .agpr_count:     0\n    .args:\n      - .offset:         0\n        .size:           8\n"
                f"    .name:           {name}\n    .sgpr_spill_count: 0\n    .vgpr_count:     128\n"
                f"    .vgpr_spill_count: {spills}\n    .wavefront_size: 64\n")

    script = os.path.join(os.path.dirname(__file__), "..", "scripts", "isa_check_spills.py")
    run = lambda text, *names: subprocess.run([sys.executable, script, str(tmp_path / "k.s"), *names],
                                              capture_output=True, text=True) if (tmp_path / "k.s").write_text(text) \
        else None
    ok = run("amdhsa.kernels:\n" + meta("_Z10refine_tile_kernelILi1EEvv", 0) + meta("_Z5otherv", 9), "refine_tile")
    assert ok.returncode == 0, ok.stdout
    bad = run("amdhsa.kernels:\n" + meta("_Z10refine_tile_kernelILi1EEvv", 3), "refine_tile")
    assert bad.returncode == 1 and "3 spilled VGPRs" in bad.stdout
    none = run("amdhsa.kernels:\n" + meta("_Z5otherv", 0), "refine_tile")
    assert none.returncode == 1
