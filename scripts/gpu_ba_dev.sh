#!/bin/bash
# BA development loop on the GPU box: BA parity tests (unit + K=256 config), then per-iteration timing
# at K=256 on the chess graph (rays, calib) and the circle graph.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_configs.py -k "ba or BA or solve or gauss" -m gpu -v -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/ba_tests.log 2>&1
rc=$?; echo "BA_TESTS_RC=$rc"; grep -E "PASS|FAIL|Error|error" gpurun_out/ba_tests.log | tail -40
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/ba_exp.py ${K:-256} 384 512 10 chess rays 2>&1 | grep -v amdgpu.ids &&
timeout -k 10 200 python scripts/ba_exp.py ${K:-256} 384 512 10 chess calib 2>&1 | grep -v amdgpu.ids &&
timeout -k 10 200 python scripts/ba_exp.py ${K:-256} 384 512 10 circle rays 2>&1 | grep -v amdgpu.ids
