#!/bin/bash
# GN loop with the setup prologue fused (default) vs the separate track_setup launch (M3S_TRACK_SETUP=kernel):
# tracking/matching/config parity, then an A/B of the tracking bench (alternating, 2 runs each)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_tracking.py tests/test_gpu_configs.py -k "not ba_k256" -m gpu -q -x --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/fused_tests.log 2>&1
rc=$?; echo "TESTS_RC=$rc"; tail -5 gpurun_out/fused_tests.log; [ $rc -eq 0 ] || exit $rc
for V in fused kernel fused kernel; do
  echo "== $V"
  if [ "$V" = kernel ]; then export M3S_TRACK_SETUP=kernel; else unset M3S_TRACK_SETUP; fi
  timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu --no-retrieval --no-peaks --no-ba > gpurun_out/bench_$V.json 2> gpurun_out/bench_$V.err
  rc=$?; echo "BENCH_RC=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_$V.err; exit $rc; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/bench_$V.json').read().strip().splitlines()[-1])
print('value', round(d['value']), 'kernels', d['kernels_us'], 'frame median', round(d['frame']['median_ms'], 4))
"
done
