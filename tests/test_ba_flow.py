"""Host check of the BA dataflow schedule (csrc/ba_pattern.cpp ba_flow_schedule): scripts/ba_flow_check.cpp
interprets every wave's task list with ba_sparse_factor_kernel's wait conditions and fails on a deadlock, an
update group applied out of step order, a column factored before its groups landed, or an unfinished column."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "lightweight-mast3r-slam_amd", "csrc")


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    cxx = shutil.which("g++") or shutil.which("c++")
    if cxx is None:
        pytest.skip("no host C++ compiler")
    exe = str(tmp_path_factory.mktemp("flow") / "ba_flow_check")
    subprocess.check_call([cxx, "-O2", "-std=c++17", "-I", CSRC, os.path.join(REPO, "scripts", "ba_flow_check.cpp"),
                           os.path.join(CSRC, "ba_pattern.cpp"), "-o", exe])
    return exe


# (K, loop edges per keyframe, seed, wide steps, subtree cut): trajectory-like graphs, a pure chain (one spine),
# tiny graphs, all-in-workgroup (wide 0) and mostly-launched splits; the subtree phase at forced cuts and at the
# plan's cost-model cut (-1)
CASES = [(256, 3, 1, 31, 0), (256, 3, 2, 0, 0), (256, 3, 3, 15, 0), (64, 2, 4, 5, 0), (2, 0, 1, 0, 0), (3, 0, 1, 0, 0),
         (300, 5, 9, 40, 0), (128, 0, 1, 3, 0), (97, 1, 7, 200, 0),
         (256, 3, 1, 0, -1), (256, 3, 2, 0, 12), (64, 2, 4, 0, 30), (2, 0, 1, 0, -1), (3, 0, 1, 0, 1),
         (128, 0, 1, 0, 20), (97, 1, 7, 0, 200)]


@pytest.mark.parametrize("K,loops,seed,wide,sub", CASES)
def test_flow_schedule_completes_in_order(checker, K, loops, seed, wide, sub):
    out = subprocess.run([checker, str(K), str(loops), str(seed), str(wide), str(sub)], capture_output=True, text=True)
    assert out.returncode == 0 and out.stdout.startswith("OK"), out.stdout + out.stderr


@pytest.mark.parametrize("traj", ["chess", "euroc"])
@pytest.mark.parametrize("sub", [-1, 8, 24])
def test_subtree_phase_on_trajectory_graphs(checker, tmp_path, traj, sub):
    """The C5 / C4 trajectory graphs (K = 256, 2028 directed edges; the edge set does not depend on the image size):
    the subtree phase's workgroup steps and the one-workgroup schedule together factor every column with every
    update group in step order."""
    import sys

    sys.path.insert(0, os.path.join(REPO, "lightweight-mast3r-slam_amd"))
    from m3s.synthetic import chess_poses, euroc_poses, make_traj_graph

    G = make_traj_graph((chess_poses if traj == "chess" else euroc_poses)(256), 24, 32, seed=1)
    f = tmp_path / "edges.txt"
    f.write_text("".join(f"{a} {b}\n" for a, b in zip(G["ii"].tolist(), G["jj"].tolist())))
    out = subprocess.run([checker, "-f", str(f), "0", str(sub)], capture_output=True, text=True)
    assert out.returncode == 0 and out.stdout.startswith("OK"), out.stdout + out.stderr
    assert " sub 0 " not in out.stdout, out.stdout  # these graphs do get a subtree phase


@pytest.fixture(scope="module")
def front_checker(tmp_path_factory):
    cxx = shutil.which("g++") or shutil.which("c++")
    if cxx is None:
        pytest.skip("no host C++ compiler")
    exe = str(tmp_path_factory.mktemp("front") / "ba_front_check")
    subprocess.check_call([cxx, "-O2", "-std=c++17", "-I", CSRC, os.path.join(REPO, "scripts", "ba_front_check.cpp"),
                           os.path.join(CSRC, "ba_pattern.cpp"), "-o", exe])
    return exe


# (K, loop edges per keyframe, seed, cut): random loop graphs, a pure chain, tiny graphs, cuts past the tree height
FRONT_CASES = [(256, 3, 1, 1), (256, 3, 1, 2), (64, 2, 4, 3), (128, 0, 1, 20), (3, 0, 1, 1), (2, 0, 1, 1),
               (97, 1, 7, 5), (97, 1, 7, 200), (300, 1, 9, 12)]


@pytest.mark.parametrize("K,loops,seed,cut", FRONT_CASES)
def test_front_phase_solves_like_dense_cholesky(front_checker, K, loops, seed, cut):
    """The frontal subtree phase's translated tables (ba_front_plan), interpreted with ba_front_kernel's semantics,
    then the U columns, the remaining steps without the replaced groups and the back substitution: the solution of a
    random SPD system on the plan's pattern matches a dense Cholesky solve (and the all-groups factorisation)."""
    out = subprocess.run([front_checker, str(K), str(loops), str(seed), str(cut)], capture_output=True, text=True)
    assert out.returncode == 0 and out.stdout.startswith("OK"), out.stdout + out.stderr


@pytest.mark.parametrize("traj,cut", [("chess", 8), ("chess", 18), ("euroc", 8), ("euroc", 14)])
def test_front_phase_on_trajectory_graphs(front_checker, tmp_path, traj, cut):
    """C5 / C4 trajectory graphs at cuts that fit the workgroup's LDS image."""
    import sys

    sys.path.insert(0, os.path.join(REPO, "lightweight-mast3r-slam_amd"))
    from m3s.synthetic import chess_poses, euroc_poses, make_traj_graph

    G = make_traj_graph((chess_poses if traj == "chess" else euroc_poses)(256), 24, 32, seed=1)
    f = tmp_path / "edges.txt"
    f.write_text("".join(f"{a} {b}\n" for a, b in zip(G["ii"].tolist(), G["jj"].tolist())))
    out = subprocess.run([front_checker, "-f", str(f), str(cut)], capture_output=True, text=True)
    assert out.returncode == 0 and out.stdout.startswith("OK") and " nwg 0 " not in out.stdout, out.stdout + out.stderr


@pytest.fixture(scope="module")
def snode_checker(tmp_path_factory):
    cxx = shutil.which("g++") or shutil.which("c++")
    if cxx is None:
        pytest.skip("no host C++ compiler")
    exe = str(tmp_path_factory.mktemp("snode") / "ba_snode_check")
    subprocess.check_call([cxx, "-O2", "-std=c++17", "-I", CSRC, os.path.join(REPO, "scripts", "ba_snode_check.cpp"),
                           os.path.join(CSRC, "ba_pattern.cpp"), os.path.join(CSRC, "ba_snode.cpp"), "-o", exe])
    return exe


def test_snode_plan_random_graphs(snode_checker):
    """The supernodal plan (csrc/ba_snode.cpp) interpreted with ba_snode_kernel's arithmetic and wait rules
    (scripts/ba_snode_check.cpp) on random trajectory-like graphs, smax 1..6, cost-model and forced cuts: every
    workgroup list drains (no deadlock) and factor + forward substitution equal a dense Cholesky to 1e-9."""
    out = subprocess.run([snode_checker], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.count("rel err") >= 8, out.stdout


@pytest.mark.parametrize("traj", ["chess", "euroc"])
def test_snode_plan_trajectory_graphs(snode_checker, tmp_path, traj):
    """The C5 / C4 trajectory graphs (K = 256): every cut (all top, cost model, all bottom) and smax 1, 2, 4, 6."""
    import sys

    sys.path.insert(0, os.path.join(REPO, "lightweight-mast3r-slam_amd"))
    from m3s.synthetic import chess_poses, euroc_poses, make_traj_graph

    G = make_traj_graph((chess_poses if traj == "chess" else euroc_poses)(256), 24, 32, seed=1)
    f = tmp_path / "edges.txt"
    f.write_text("".join(f"{a} {b}\n" for a, b in zip(G["ii"].tolist(), G["jj"].tolist())))
    out = subprocess.run([snode_checker, str(f)], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.count("rel err") == 8, out.stdout
