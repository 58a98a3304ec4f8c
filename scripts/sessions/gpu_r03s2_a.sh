#!/bin/bash
# Re-entry check of this session: smoke + every GPU test, then the default bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
bash scripts/gpu_check.sh || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
rc=$?; echo "BENCH_RC=$rc"; tail -c 600 gpurun_out/bench_default.json; [ $rc -eq 0 ] || exit $rc
