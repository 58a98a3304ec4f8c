#!/bin/bash
# GPU-box benchmark + rocprofv3 kernel-trace summary. Each step time-limited.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-50}
timeout -k 10 600 python bench.py --steps $STEPS --warmup 10 "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "BENCH_RC=$rc"; tail -5 gpurun_out/bench.err; cat gpurun_out/bench.json
exit $rc
