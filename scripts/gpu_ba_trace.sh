#!/bin/bash
# BA per-iteration timing + rocprofv3 kernel trace of the 256-keyframe solve loop.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ba
export TMPDIR=/tmp
K=${K:-256}
timeout -k 10 300 python scripts/ba_exp.py $K 384 512 10 > gpurun_out/ba/ba_exp.log 2>&1
rc=$?; echo "BA_EXP_RC=$rc"; cat gpurun_out/ba/ba_exp.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ba/trace -o run -- python3 scripts/ba_exp.py $K 384 512 10 > gpurun_out/ba/trace.log 2>&1
rc=$?; echo "BA_TRACE_RC=$rc"
exit $rc
