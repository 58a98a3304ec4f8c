#!/bin/bash
# Refine development: matching parity tests (bit-exact refine) on the shipped library, then refine time per
# variant (lib/exp builds) at 512x512 by dilation_max; the idx checksum must agree across variants.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_matching.py -m gpu -v -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/match_tests.log 2>&1
rc=$?; echo "MATCH_TESTS_RC=$rc"; grep -E "PASS|FAIL|Error|error" gpurun_out/match_tests.log | tail -30
[ $rc -eq 0 ] || exit $rc
for V in ${VARIANTS:-old main}; do
  if [ "$V" = main ]; then L=lightweight-mast3r-slam_amd/lib/libm3s.so; else L=lightweight-mast3r-slam_amd/lib/exp/libm3s_$V.so; fi
  echo "== $V"
  M3S_LIB=$L timeout -k 10 120 python3 scripts/refine_exp.py 2>&1 | grep -v amdgpu.ids || exit 1
done
