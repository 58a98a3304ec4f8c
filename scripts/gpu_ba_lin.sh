#!/bin/bash
# BA linearisation development: BA parity tests on the shipped library, then C5 (chess calib) and C4-shaped
# (euroc rays) per-iteration times for the shipped library and the lib/exp variants.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_configs.py tests/test_gpu_factor_graph.py -k "ba or BA or gauss or factor or solve or c3" -m gpu -v -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/ba_tests.log 2>&1
rc=$?; echo "BA_TESTS_RC=$rc"; grep -E "PASS|FAIL|Error|error|assert" gpurun_out/ba_tests.log | tail -40
[ $rc -eq 0 ] || exit $rc
for V in ${VARIANTS:-main}; do
  if [ "$V" = main ]; then L=lightweight-mast3r-slam_amd/lib/libm3s.so; else L=lightweight-mast3r-slam_amd/lib/exp/libm3s_$V.so; fi
  echo "== $V"
  M3S_LIB=$L timeout -k 10 200 python3 scripts/ba_exp.py 256 384 512 10 chess calib 2>&1 | grep -v amdgpu.ids || exit 1
  M3S_LIB=$L timeout -k 10 200 python3 scripts/ba_exp.py 256 320 512 10 euroc rays 2>&1 | grep -v amdgpu.ids || exit 1
done
