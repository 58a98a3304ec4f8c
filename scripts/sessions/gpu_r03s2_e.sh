#!/bin/bash
# Shard-scoped keyframe compare (record reuse): the reuse / factor-graph GPU tests, then the 2-rank bench rehearsal
# (gloo on one GPU) for the sharded reuse call, then the dataflow wide-step split sweep
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_factor_graph.py tests/test_gpu_ba.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/reuse_tests.log 2>&1
rc=$?; echo "TESTS_RC=$rc"; tail -3 gpurun_out/reuse_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r03_o.sh || exit $?
bash scripts/gpu_r03s2_d.sh
