#!/bin/bash
# BA solve iteration: parity tests of the BA path, C5/C4 per-iteration timing, factor stamps (M3S_SP_STAMPS)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_configs.py tests/test_gpu_factor_graph.py -m gpu -v --timeout 240 --timeout-method thread > gpurun_out/ba_tests.log 2>&1
rc=$?; echo "BA_TESTS_RC=$rc"; grep -E "FAILED|passed|failed" gpurun_out/ba_tests.log | tail -8; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python3 scripts/ba_exp.py 256 384 512 10 chess calib 2>&1 | grep "rep 1" || exit 1
timeout -k 10 200 python3 scripts/ba_exp.py 256 320 512 10 euroc rays 2>&1 | grep "rep 1" || exit 1
M3S_LIB=lightweight-mast3r-slam_amd/lib/exp/libm3s_spst.so timeout -k 10 200 python3 scripts/ba_exp.py 256 384 512 3 chess calib > gpurun_out/sp_stamps.txt 2>&1
echo "SP_STAMPS_RC=$?"; tail -4 gpurun_out/sp_stamps.txt
