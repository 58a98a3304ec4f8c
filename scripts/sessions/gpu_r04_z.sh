#!/bin/bash
# round 4: frontal subtree phase (BA solve): BA GPU tests, then solve timings front vs no front (alternating, one box)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v --timeout 400 --timeout-method thread tests/test_gpu_ba.py tests/test_gpu_configs.py > gpurun_out/r04z_pytest.txt 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/r04z_pytest.txt | tail -12; [ $rc -eq 0 ] || exit $rc
{
for r in 1 2; do
  for F in 0 def; do
    echo "== M3S_BA_FRONT=$F"
    if [ $F = def ]; then unset M3S_BA_FRONT; else export M3S_BA_FRONT=$F; fi
    timeout -k 10 200 python3 scripts/ba_exp.py 256 384 512 10 chess calib 2>&1 | grep "rep 1" || exit 1
    timeout -k 10 200 python3 scripts/ba_exp.py 256 320 512 10 euroc rays 2>&1 | grep "rep 1" || exit 1
  done
done
} > gpurun_out/r04z_ba_exp.txt 2>&1
rc=$?; cat gpurun_out/r04z_ba_exp.txt; [ $rc -eq 0 ] || exit $rc
