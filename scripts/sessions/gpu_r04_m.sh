#!/bin/bash
# round 4: refine window rework (adaptive columns, packed d=1 window, double-buffered d=2): parity (bit-exact) then
# timing (screen / exact / fill-only / survivor stats)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_refine_screen.py tests/test_gpu_matching.py > gpurun_out/r04m_pytest.txt 2>&1
rc=$?; tail -5 gpurun_out/r04m_pytest.txt; [ $rc -eq 0 ] || exit $rc
L=lightweight-mast3r-slam_amd/lib
{
echo "== screen"; timeout -k 10 120 python3 scripts/refine_exp.py || exit 1
echo "== exact (M3S_REFINE_SCREEN=0)"; M3S_REFINE_SCREEN=0 timeout -k 10 120 python3 scripts/refine_exp.py || exit 1
for V in fillonly stats; do
  echo "== $V"; M3S_LIB=$L/exp/libm3s_$V.so timeout -k 10 120 python3 scripts/refine_exp.py || exit 1
done
} 2>&1 | grep -v amdgpu.ids > gpurun_out/r04m_refine_exp.txt
cat gpurun_out/r04m_refine_exp.txt
