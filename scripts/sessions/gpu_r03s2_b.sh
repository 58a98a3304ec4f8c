#!/bin/bash
# BA solve: dataflow one-workgroup factor + back substitution (default) vs the level-synchronous loops
# (M3S_BA_FLOW=0): solve time and the final-pose hash (bit-identity) on C5 / C4, alternating; then the BA GPU tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for F in 0 1 0 1; do
  echo "== flow $F"
  M3S_BA_FLOW=$F timeout -k 10 200 python3 scripts/ba_exp.py 256 384 512 10 chess calib 2>&1 | grep -E "^rep|rror" || exit 1
  M3S_BA_FLOW=$F timeout -k 10 200 python3 scripts/ba_exp.py 256 320 512 10 euroc rays 2>&1 | grep -E "^rep|rror" || exit 1
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_configs.py tests/test_gpu_factor_graph.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/ba_tests_flow.log 2>&1
rc=$?; echo "TESTS_RC=$rc"; tail -3 gpurun_out/ba_tests_flow.log; exit $rc
