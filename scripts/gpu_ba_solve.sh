#!/bin/bash
# BA solve development: BA parity tests, then the C5 graph (chess, calib, K=256) with the multi-workgroup
# factor steps off / default / every step (final poses hashed: must be bit-identical), then phase stamps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_configs.py tests/test_gpu_factor_graph.py -m gpu -v -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/ba_tests.log 2>&1
rc=$?; echo "BA_TESTS_RC=$rc"; grep -E "PASS|FAIL|Error|error" gpurun_out/ba_tests.log | tail -40
[ $rc -eq 0 ] || exit $rc
for W in 1000000 16 0; do
  echo "== M3S_BA_WIDE=$W"
  M3S_BA_WIDE=$W timeout -k 10 200 python scripts/ba_exp.py 256 384 512 10 chess calib 2>&1 | grep -v amdgpu.ids || exit 1
done
echo "== stamps (default)"
M3S_LIB=lightweight-mast3r-slam_amd/lib/exp/libm3s_spst.so timeout -k 10 200 python3 scripts/ba_exp.py 256 384 512 3 chess calib 2>&1 | grep -v amdgpu.ids
echo "== GN stamps (tracking, calib 512x512)"
M3S_LIB=lightweight-mast3r-slam_amd/lib/exp/libm3s_gnst.so timeout -k 10 200 python3 scripts/gn_exp.py 2>&1 | grep -v amdgpu.ids
