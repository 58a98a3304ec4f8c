#!/bin/bash
# round 4: BA subtree phase (after the LDS-fit fix) + tracking tests + store leg
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
bash scripts/sessions/gpu_r04_f.sh || exit $?
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_tracking.py > gpurun_out/r04h_track_tests.txt 2>&1
rc=$?; tail -4 gpurun_out/r04h_track_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-ba --no-cpu --no-retrieval --no-peaks > gpurun_out/r04h_bench.json 2> gpurun_out/r04h_bench.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r04h_bench.json')); print(d['value'], d['kernels_us'], d['store'])"
