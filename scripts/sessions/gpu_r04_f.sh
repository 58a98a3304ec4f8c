#!/bin/bash
# round 4: BA subtree phase — BA parity tests (schedules bit-identical, K=256 truth, full resolution) then solve
# timings per cut (default cost model, legacy launched steps, forced cuts)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_ba.py tests/test_gpu_configs.py -k "ba" -s > gpurun_out/r04f_pytest.txt 2>&1
rc=$?; grep -E "PASS|FAIL|Error|err vs|K=256" gpurun_out/r04f_pytest.txt | tail -40; [ $rc -eq 0 ] || exit $rc
{
for S in def -1 6 10 16 24; do
  echo "== M3S_BA_SUB=$S"
  if [ $S = def ]; then unset M3S_BA_SUB; else export M3S_BA_SUB=$S; fi
  timeout -k 10 200 python3 scripts/ba_exp.py 256 384 512 10 chess calib 2>&1 | grep "rep 1" || exit 1
  timeout -k 10 200 python3 scripts/ba_exp.py 256 320 512 10 euroc rays 2>&1 | grep "rep 1" || exit 1
done
} > gpurun_out/r04f_ba_exp.txt 2>&1
rc=$?; cat gpurun_out/r04f_ba_exp.txt; exit $rc
