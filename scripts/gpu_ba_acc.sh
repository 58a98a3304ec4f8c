#!/bin/bash
# BA accuracy gate per variant: the ill-conditioned 6-KF fixture + medium graph vs the fp64 truth, then C5/C4 timing.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for V in ${VARIANTS:-main}; do
  if [ "$V" = main ]; then L=lightweight-mast3r-slam_amd/lib/libm3s.so; else L=lightweight-mast3r-slam_amd/lib/exp/libm3s_$V.so; fi
  echo "== $V"
  M3S_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_ba.py -k "factor_graph_matches_reference or medium_graph or gauss_newton_vs_oracle" -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/acc_$V.log 2>&1
  echo "TESTS_RC=$?"; grep -E "passed|failed|Max abs" gpurun_out/acc_$V.log | tail -6
  M3S_LIB=$L timeout -k 10 200 python3 scripts/ba_exp.py 256 384 512 10 chess calib 2>&1 | grep "rep 1" || exit 1
  M3S_LIB=$L timeout -k 10 200 python3 scripts/ba_exp.py 256 320 512 10 euroc rays 2>&1 | grep "rep 1" || exit 1
done
