#!/bin/bash
# round 5: proj_occlusion with the LDS ray-image window (win, the default) vs every corner from global memory (M3S_PROJ_WIN=0): matching + tracking
# GPU tests, then kernel-trace stats and bench frames/s, alternating, 3 reps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05pw
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_matching.py tests/test_gpu_tracking.py tests/test_gpu_configs.py > gpurun_out/r05pw/tests.txt 2>&1 || { tail -40 gpurun_out/r05pw/tests.txt; exit 1; }
tail -2 gpurun_out/r05pw/tests.txt
ARGS="--steps 100 --warmup 10 --no-cpu --no-ba --no-peaks --no-retrieval --no-store --no-kernel-timing"
for rep in 1 2 3; do
for V in 1 0; do
  M3S_PROJ_WIN=$V timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pp2_${V}_$rep -o run -- python3 bench.py $ARGS > gpurun_out/r05pw/${V}_$rep.json 2> gpurun_out/r05pw/${V}_$rep.err || { tail -20 gpurun_out/r05pw/${V}_$rep.err; exit 1; }
  S=$(find /tmp/pp2_${V}_$rep -name "*kernel_stats.csv" | head -1)
  cp "$S" gpurun_out/r05pw/${V}_${rep}_kernel_stats.csv
  python3 - gpurun_out/r05pw/${V}_${rep}_kernel_stats.csv "win=$V $rep" <<'PY'
import csv, sys
r = {}
for row in csv.DictReader(open(sys.argv[1])):
    for k in ("prep_rays", "proj_occ", "refine_tile", "gn_loop", "fuse_kernel"):
        if k in row["Name"]:
            r[k] = float(row["AverageNs"]) / 1e3
print(sys.argv[2], "  ".join("%s %.2f" % kv for kv in r.items()), " sum %.2f" % sum(r.values()))
PY
  M3S_PROJ_WIN=$V timeout -k 10 300 python3 bench.py --steps 200 --warmup 20 --no-cpu --no-ba --no-peaks --no-retrieval --no-store > gpurun_out/r05pw/b_${V}_$rep.json 2> gpurun_out/r05pw/b_${V}_$rep.err || { tail -20 gpurun_out/r05pw/b_${V}_$rep.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r05pw/b_${V}_$rep.json').read().strip().splitlines()[-1]); print('  fps', round(d['value'],1), d['kernels_us'])"
done
done
