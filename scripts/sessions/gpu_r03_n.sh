#!/bin/bash
# BA wide steps with one 32-B task record per launched task (main) vs the table walk (prev): solve time and the
# final-pose hash (bit-identity) on C5 / C4, alternating builds; then the BA GPU tests on main
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for V in prev main prev main; do
  if [ "$V" = main ]; then L=lightweight-mast3r-slam_amd/lib/libm3s.so; else L=lightweight-mast3r-slam_amd/lib/exp/libm3s_$V.so; fi
  echo "== $V"
  M3S_LIB=$L timeout -k 10 200 python3 scripts/ba_exp.py 256 384 512 10 chess calib 2>&1 | grep -E "^rep" || exit 1
  M3S_LIB=$L timeout -k 10 200 python3 scripts/ba_exp.py 256 320 512 10 euroc rays 2>&1 | grep -E "^rep" || exit 1
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_configs.py tests/test_gpu_factor_graph.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/ba_tests_n.log 2>&1
rc=$?; echo "TESTS_RC=$rc"; tail -3 gpurun_out/ba_tests_n.log; exit $rc
