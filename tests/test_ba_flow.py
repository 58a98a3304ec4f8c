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


# (K, loop edges per keyframe, seed, wide steps): trajectory-like graphs, a pure chain (one spine), tiny graphs,
# all-in-workgroup (wide 0) and mostly-launched splits
CASES = [(256, 3, 1, 31), (256, 3, 2, 0), (256, 3, 3, 15), (64, 2, 4, 5), (2, 0, 1, 0), (3, 0, 1, 0),
         (300, 5, 9, 40), (128, 0, 1, 3), (97, 1, 7, 200), (128, 0, 1, 0), (97, 1, 7, 0)]


@pytest.mark.parametrize("K,loops,seed,wide", CASES)
def test_flow_schedule_completes_in_order(checker, K, loops, seed, wide):
    out = subprocess.run([checker, str(K), str(loops), str(seed), str(wide)], capture_output=True, text=True)
    assert out.returncode == 0 and out.stdout.startswith("OK"), out.stdout + out.stderr


@pytest.mark.parametrize("traj", ["chess", "euroc"])
@pytest.mark.parametrize("wide", [0, 8, 31])
def test_flow_schedule_on_trajectory_graphs(checker, tmp_path, traj, wide):
    """The C5 / C4 trajectory graphs (K = 256, 2028 directed edges; the edge set does not depend on the image size):
    the launched wide steps and the one-workgroup schedule together factor every column with every update group in
    step order, and the back substitution completes."""
    import sys

    sys.path.insert(0, os.path.join(REPO, "lightweight-mast3r-slam_amd"))
    from m3s.synthetic import chess_poses, euroc_poses, make_traj_graph

    G = make_traj_graph((chess_poses if traj == "chess" else euroc_poses)(256), 24, 32, seed=1)
    f = tmp_path / "edges.txt"
    f.write_text("".join(f"{a} {b}\n" for a, b in zip(G["ii"].tolist(), G["jj"].tolist())))
    out = subprocess.run([checker, "-f", str(f), str(wide)], capture_output=True, text=True)
    assert out.returncode == 0 and out.stdout.startswith("OK"), out.stdout + out.stderr
