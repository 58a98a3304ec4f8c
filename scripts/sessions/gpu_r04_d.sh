#!/bin/bash
# round 4: refine batched column reads in the screen: parity (bit-exact) then timing (screen / exact)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_refine_screen.py tests/test_gpu_matching.py > gpurun_out/r04e_pytest.txt 2>&1
rc=$?; tail -5 gpurun_out/r04e_pytest.txt; [ $rc -eq 0 ] || exit $rc
{
echo "== screen"; timeout -k 10 120 python3 scripts/refine_exp.py || exit 1
echo "== exact"; M3S_REFINE_SCREEN=0 timeout -k 10 120 python3 scripts/refine_exp.py || exit 1
} 2>&1 | grep -v amdgpu.ids > gpurun_out/r04e_refine_exp.txt
cat gpurun_out/r04e_refine_exp.txt
