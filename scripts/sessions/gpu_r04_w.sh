#!/bin/bash
# round 4: full GPU suite, smoke(), the default bench line (final evidence for this round's code)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1500 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests > gpurun_out/r04w_pytest.txt 2>&1
rc=$?; grep -E "passed|failed|FAILED|error" gpurun_out/r04w_pytest.txt | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04w_smoke.txt 2>&1
rc=$?; tail -2 gpurun_out/r04w_smoke.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py > gpurun_out/r04w_bench.json 2> gpurun_out/r04w_bench.err || { tail -20 gpurun_out/r04w_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r04w_bench.json')); b=d['ba']; print(d['value'], d['kernels_us'], d['frame']['median_ms'], d['roofline']['frac'], b['ms_solve_per_iter'], b['ms_lin_per_iter'], b['ms_pack'], b['edges_per_s'], b['c4']['edges_per_s'], b['eth3d']['edges_per_s'], d['configs'], d['cpu_baseline']['value'])"
