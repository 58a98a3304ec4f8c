#!/bin/bash
# Refine tail steal (main) vs the separate outlier kernel only (nosteal) + host-side spare match outputs:
# matching/tracking parity, refine_lin time, tracking bench and kernel gaps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/kt
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_matching.py tests/test_gpu_tracking.py tests/test_gpu_configs.py -k "not ba_k256" -m gpu -q -x --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/steal_tests.log 2>&1
rc=$?; echo "TESTS_RC=$rc"; tail -3 gpurun_out/steal_tests.log; [ $rc -eq 0 ] || exit $rc
for V in nosteal main nosteal main; do
  if [ "$V" = main ]; then L=lightweight-mast3r-slam_amd/lib/libm3s.so; else L=lightweight-mast3r-slam_amd/lib/exp/libm3s_$V.so; fi
  echo "== $V"
  M3S_LIB=$L timeout -k 10 120 python3 scripts/refine_exp.py 2>&1 | grep -v amdgpu.ids | grep -v "^8x512" || exit 1
  M3S_LIB=$L timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu --no-retrieval --no-peaks --no-ba > gpurun_out/bench_$V.json 2> gpurun_out/bench_$V.err
  rc=$?; echo "BENCH_RC=$rc"; python3 -c "
import json; d=json.loads(open('gpurun_out/bench_$V.json').read().strip().splitlines()[-1])
print('value', round(d['value']), 'kernels', d['kernels_us'], 'frame median', round(d['frame']['median_ms'], 4))
"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt/t2 -o run -- python3 bench.py --steps 100 --warmup 10 --no-cpu --no-ba --no-peaks --no-retrieval --no-kernel-timing > gpurun_out/kt/bench2.json 2> gpurun_out/kt/bench2.err && python3 scripts/kt_gaps.py gpurun_out/kt/t2 200
find gpurun_out/kt -name "*.csv" -size +2M -delete
