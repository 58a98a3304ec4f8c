#!/bin/bash
# Round-3 first GPU pass: VALU issue-rate micro-benchmark, the full GPU test suite, the default bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./scripts/micro/fma_rates > gpurun_out/fma_rates.txt 2>&1
rc=$?; echo "FMA_RATES_RC=$rc"; cat gpurun_out/fma_rates.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "PYTEST_RC=$rc"; tail -8 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "BENCH_RC=$rc"; tail -c 3000 gpurun_out/bench.json; [ $rc -eq 0 ] || { tail -30 gpurun_out/bench.err; exit $rc; }
