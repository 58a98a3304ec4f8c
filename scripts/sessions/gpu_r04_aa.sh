#!/bin/bash
# round 4: BA tests on the final BA code (frontal phase opt-in), then the N=2 rehearsal (gloo, 2 ranks on device 0)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v --timeout 400 --timeout-method thread tests/test_gpu_ba.py tests/test_gpu_configs.py > gpurun_out/r04aa_pytest.txt 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/r04aa_pytest.txt | tail -8; [ $rc -eq 0 ] || exit $rc
bash scripts/sessions/gpu_r04_x.sh
