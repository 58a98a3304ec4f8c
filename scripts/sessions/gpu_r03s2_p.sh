#!/bin/bash
# (experiment of this session; the prefetch was reverted after this measurement, DESIGN.md §4 BA)
# BA dataflow back substitution: each wave's next diagonal block staged in LDS a column ahead (main) vs loaded at the
# column's start (prev): solve time + pose hash (bit-identity), alternating; then the BA GPU tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for V in prev main prev main; do
  if [ "$V" = main ]; then L=lightweight-mast3r-slam_amd/lib/libm3s.so; else L=lightweight-mast3r-slam_amd/lib/exp/libm3s_$V.so; fi
  echo "== $V"
  M3S_LIB=$L timeout -k 10 120 python3 scripts/ba_exp.py 256 384 512 10 chess calib 2>&1 | grep -E "^rep 1|rror" || exit 1
  M3S_LIB=$L timeout -k 10 120 python3 scripts/ba_exp.py 256 320 512 10 euroc rays 2>&1 | grep -E "^rep 1|rror" || exit 1
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_configs.py tests/test_gpu_factor_graph.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/ba_tests_pf.log 2>&1
rc=$?; echo "TESTS_RC=$rc"; tail -3 gpurun_out/ba_tests_pf.log; exit $rc
