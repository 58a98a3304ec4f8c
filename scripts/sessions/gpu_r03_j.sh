#!/bin/bash
# BA record reuse: the new reuse test + every BA / factor-graph test (reuse is FactorGraph's default now)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_factor_graph.py tests/test_gpu_ba.py tests/test_gpu_configs.py -m gpu -v -s -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/reuse_tests.log 2>&1
rc=$?; echo "TESTS_RC=$rc"; grep -E "PASS|FAIL|Error|error|record reuse|replay" gpurun_out/reuse_tests.log | tail -40; exit $rc
