#!/bin/bash
# Tracking development: tracking/matching parity tests, GN phase stamps, a short bench (tracking only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_tracking.py tests/test_gpu_configs.py tests/test_gpu_matching.py -m gpu -v -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/track_tests.log 2>&1
rc=$?; echo "TRACK_TESTS_RC=$rc"; grep -E "PASS|FAIL|Error|error" gpurun_out/track_tests.log | tail -40
[ $rc -eq 0 ] || exit $rc
echo "== GN stamps (tracking, calib 512x512)"
M3S_LIB=lightweight-mast3r-slam_amd/lib/exp/libm3s_gnst.so timeout -k 10 200 python3 scripts/gn_exp.py 2>&1 | grep -v amdgpu.ids || exit 1
echo "== bench (tracking only)"
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu --no-ba --no-peaks --no-retrieval > gpurun_out/bench_track.json 2> gpurun_out/bench_track.err
rc=$?; echo "BENCH_RC=$rc"; python3 -c "import json;d=json.loads(open('gpurun_out/bench_track.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['kernels_us'],d['frame'])"
