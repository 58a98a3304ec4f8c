#!/bin/bash
# A/B of the 6-KF factor-graph fixture (test_factor_graph_matches_reference) across libm3s variants: prints the
# max |T - T64| of each (the test's 1e-5 contract) without stopping at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for V in ${VARIANTS:-main}; do
  if [ "$V" = main ]; then L=lightweight-mast3r-slam_amd/lib/libm3s.so; else L=lightweight-mast3r-slam_amd/lib/exp/libm3s_$V.so; fi
  echo "== $V"
  M3S_LIB=$L timeout -k 10 200 python -u -m pytest tests/test_gpu_ba.py -k "factor_graph_matches_reference or medium_graph or full_chunk" -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/fx_$V.log 2>&1
  rc=$?; echo "RC=$rc"; grep -E "Max abs|passed|failed" gpurun_out/fx_$V.log
  [ $rc -le 1 ] || exit $rc
done
