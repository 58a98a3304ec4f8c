#!/bin/bash
# GN block size A/B: tracking tests + per-block stamps + a short tracking-only bench per library
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for V in main gn512; do
  if [ "$V" = main ]; then L=lightweight-mast3r-slam_amd/lib/libm3s.so; S=lightweight-mast3r-slam_amd/lib/exp/libm3s_gnst.so;
  else L=lightweight-mast3r-slam_amd/lib/exp/libm3s_$V.so; S=lightweight-mast3r-slam_amd/lib/exp/libm3s_${V}st.so; fi
  echo "== $V"
  M3S_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_tracking.py tests/test_gpu_configs.py -k "track" -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/track_$V.log 2>&1
  rc=$?; echo "TRACK_TESTS_RC=$rc"; tail -2 gpurun_out/track_$V.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  M3S_LIB=$S timeout -k 10 200 python3 scripts/gn_exp.py 2>&1 | grep -v amdgpu.ids
  M3S_LIB=$L timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu --no-retrieval --no-peaks --no-ba > gpurun_out/bench_$V.json 2> gpurun_out/bench_$V.err
  rc=$?; echo "BENCH_RC=$rc"; python3 -c "
import json; d=json.loads(open('gpurun_out/bench_$V.json').read().strip().splitlines()[-1])
print('value', round(d['value']), 'kernels', d['kernels_us'], 'frame median', round(d['frame']['median_ms'], 4), 'iters', d['config']['gn_iters_mean'])
"; [ $rc -eq 0 ] || exit $rc
done
# BA solve A/B: this tree's factorisation vs round 2's (libm3s_r2: round-2 ba.hip, 16-wave cost model)
for V in main r2; do
  if [ "$V" = main ]; then L=lightweight-mast3r-slam_amd/lib/libm3s.so; S=lightweight-mast3r-slam_amd/lib/exp/libm3s_spst.so;
  else L=lightweight-mast3r-slam_amd/lib/exp/libm3s_$V.so; S=lightweight-mast3r-slam_amd/lib/exp/libm3s_${V}st.so; fi
  echo "== solve $V"
  M3S_LIB=$L timeout -k 10 200 python3 scripts/ba_exp.py 256 384 512 10 chess calib 2>&1 | grep "rep 1" || exit 1
  M3S_LIB=$L timeout -k 10 200 python3 scripts/ba_exp.py 256 320 512 10 euroc rays 2>&1 | grep "rep 1" || exit 1
  M3S_LIB=$S timeout -k 10 200 python3 scripts/ba_exp.py 256 384 512 3 chess calib 2>&1 | grep -E "factor stamps|root-end"
done
