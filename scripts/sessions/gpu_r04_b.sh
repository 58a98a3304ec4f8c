#!/bin/bash
# round 4: full GPU suite (new: stall -> RuntimeError) then the default bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests > gpurun_out/r04b_pytest.txt 2>&1
rc=$?; tail -15 gpurun_out/r04b_pytest.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/r04b_bench.json 2> gpurun_out/r04b_bench.err || exit 1
tail -c 3000 gpurun_out/r04b_bench.json
