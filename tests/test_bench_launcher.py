"""bench.py's N-rank launcher on CPU: `python bench.py --gpus N` without torch.distributed.run
starts N rank processes itself; a mismatch between the launched world and --gpus, or too few devices, is refused
with a non-zero exit instead of a silent 1-GPU line."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "M3S_BENCH_DEVICE")}
    env.update(kw)
    return env


def _json_line(out):
    # stdout holds exactly the one JSON line (gloo's "[Gloo] Rank ..." prints are sent to stderr)
    lines = [ln for ln in out.splitlines() if ln.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), out
    return json.loads(lines[0])


@pytest.mark.timeout(180)
@pytest.mark.parametrize("n", [2, 3])
def test_launcher_starts_n_ranks_over_gloo(n):
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--launch-probe"], env=_env(),
                       capture_output=True, text=True, timeout=170)
    assert r.returncode == 0, r.stderr
    rec = _json_line(r.stdout)
    assert rec["n_gpus"] == n and rec["gpus_arg"] == n
    assert rec["rank_sum"] == n * (n + 1) / 2
    assert rec["launcher"] == "bench.py"


@pytest.mark.timeout(120)
def test_launcher_refuses_without_enough_devices():
    # this container has no GPU: --gpus 2 without the one-device rehearsal must exit non-zero, with no JSON line
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2"], env=_env(HIP_VISIBLE_DEVICES=""),
                       capture_output=True, text=True, timeout=110)
    assert r.returncode != 0
    assert "needs 2 visible GPUs" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


@pytest.mark.timeout(120)
def test_rank_refuses_world_gpus_mismatch():
    # an external launcher started 2 ranks but the line would say --gpus 1: every rank refuses
    r = subprocess.run([sys.executable, BENCH, "--gpus", "1", "--launch-probe"],
                       env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"), capture_output=True, text=True,
                       timeout=110)
    assert r.returncode == 2
    assert "WORLD_SIZE=2 but --gpus 1" in r.stderr
