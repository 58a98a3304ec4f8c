#!/bin/bash
# BA development loop on the GPU box: BA parity tests, then per-iteration timing at K=256.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ba.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/ba_tests.log 2>&1
rc=$?; echo "BA_TESTS_RC=$rc"; tail -25 gpurun_out/ba_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/ba_exp.py ${K:-256} 384 512 10 2>&1 | grep -v amdgpu.ids
