#!/bin/bash
# round 4: sharded refine-bound atomics + separate BA pack by default: matching / refine / BA / tracking tests, then
# the default bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_refine_screen.py tests/test_gpu_matching.py tests/test_gpu_ba.py tests/test_gpu_tracking.py > gpurun_out/r04q_pytest.txt 2>&1
rc=$?; tail -4 gpurun_out/r04q_pytest.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py > gpurun_out/r04q_bench.json 2> gpurun_out/r04q_bench.err || { tail -20 gpurun_out/r04q_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r04q_bench.json')); b=d['ba']; print(d['value'], d['kernels_us'], d['frame']['median_ms'], d['roofline']['frac'], b['ms_solve_per_iter'], b['ms_lin_per_iter'], b['ms_pack'], b['edges_per_s'], b['c4']['edges_per_s'], b['eth3d']['edges_per_s'], d['configs'])"
