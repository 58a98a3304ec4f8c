#!/bin/bash
# round 4: (1) refine with batched column reads: parity + timing; (2) BA subtree phase: parity + solve timings
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
bash scripts/sessions/gpu_r04_e.sh || exit $?
bash scripts/sessions/gpu_r04_f.sh || exit $?
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_tracking.py > gpurun_out/r04g_track_tests.txt 2>&1
rc=$?; tail -4 gpurun_out/r04g_track_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-ba --no-cpu --no-retrieval --no-peaks > gpurun_out/r04g_bench.json 2> gpurun_out/r04g_bench.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r04g_bench.json')); print(d['value'], d['kernels_us'], d['store'])"
