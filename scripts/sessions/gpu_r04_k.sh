#!/bin/bash
# round 4: full GPU suite, the default bench line, then the round's profiles (kernel traces + PMC passes of the
# tracking bench and the three BA legs, factor stamps)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1500 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests > gpurun_out/r04k_pytest.txt 2>&1
rc=$?; grep -E "passed|failed|FAILED|error" gpurun_out/r04k_pytest.txt | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py > gpurun_out/r04k_bench.json 2> gpurun_out/r04k_bench.err || { tail -20 gpurun_out/r04k_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r04k_bench.json')); print(d['value'], d['kernels_us'], d['ba']['ms_solve_per_iter'], d['ba']['edges_per_s'], d['cpu_baseline']['value'], d['cpu_baseline']['cores'])"

