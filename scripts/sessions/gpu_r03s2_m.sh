#!/bin/bash
# (experiment of this session; the wide-launch code was reverted after this measurement, DESIGN.md §4 BA)
# BA wide steps as ONE dataflow launch (default) vs one launch per step (M3S_BA_WIDEFLOW=0): solve time and pose hash
# (bit-identity) on C5 / C4, alternating; then the BA GPU tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for F in 1 0 1 0; do
  echo "== wideflow $F"
  M3S_BA_WIDEFLOW=$F timeout -k 10 120 python3 scripts/ba_exp.py 256 384 512 10 chess calib 2>&1 | grep -E "^rep|rror" || exit 1
  M3S_BA_WIDEFLOW=$F timeout -k 10 120 python3 scripts/ba_exp.py 256 320 512 10 euroc rays 2>&1 | grep -E "^rep|rror" || exit 1
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_configs.py tests/test_gpu_factor_graph.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/ba_tests_wide.log 2>&1
rc=$?; echo "TESTS_RC=$rc"; tail -5 gpurun_out/ba_tests_wide.log; exit $rc
