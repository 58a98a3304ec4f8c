#!/bin/bash
# BA on round 2's factorisation (+ Newton rays): BA parity tests, solve timings; refine per-block balance
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_configs.py tests/test_gpu_factor_graph.py -m gpu -q -x --timeout 240 --timeout-method thread > gpurun_out/ba_tests.log 2>&1
rc=$?; echo "BA_TESTS_RC=$rc"; tail -4 gpurun_out/ba_tests.log; [ $rc -eq 0 ] || exit $rc
L=lightweight-mast3r-slam_amd/lib/libm3s.so
M3S_LIB=$L timeout -k 10 200 python3 scripts/ba_exp.py 256 384 512 10 chess calib 2>&1 | grep "rep 1" || exit 1
M3S_LIB=$L timeout -k 10 200 python3 scripts/ba_exp.py 256 320 512 10 euroc rays 2>&1 | grep "rep 1" || exit 1
M3S_LIB=lightweight-mast3r-slam_amd/lib/exp/libm3s_rbst.so timeout -k 10 200 python3 scripts/refine_blocks.py 2>&1 | grep -v amdgpu.ids
