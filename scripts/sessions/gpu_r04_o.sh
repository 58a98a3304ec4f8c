#!/bin/bash
# round 4: determinism probe (match repeats, tracker unique-match count separate vs folded setup), then the BA
# factor-graph replay tests after the record-slot layout fix
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 scripts/track_determinism.py > gpurun_out/r04o_determinism.txt 2>&1
rc=$?; cat gpurun_out/r04o_determinism.txt | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_factor_graph.py tests/test_gpu_ba.py > gpurun_out/r04o_pytest.txt 2>&1
rc=$?; tail -6 gpurun_out/r04o_pytest.txt; exit $rc
