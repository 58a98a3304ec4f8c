#!/bin/bash
# round 4: GN point pairs with fp32 product sums (GN_PAIR=1, shipped) vs fp64 product FMAs (lib/exp/libm3s_gnf64.so):
# tracking parity tests, then the tracking bench A/B (three alternating pairs)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_tracking.py tests/test_gpu_configs.py > gpurun_out/r04v_pytest.txt 2>&1
rc=$?; tail -4 gpurun_out/r04v_pytest.txt; [ $rc -eq 0 ] || exit $rc
L=lightweight-mast3r-slam_amd/lib
A="--steps 100 --warmup 10 --no-ba --no-cpu --no-retrieval --no-store --no-peaks"
for r in 1 2 3; do
  for V in main gnf64; do
    if [ $V = main ]; then LIB=$L/libm3s.so; else LIB=$L/exp/libm3s_$V.so; fi
    M3S_LIB=$LIB timeout -k 10 240 python3 bench.py $A > gpurun_out/r04v_${V}_$r.json 2> gpurun_out/r04v_${V}_$r.err || { tail -20 gpurun_out/r04v_${V}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r04v_${V}_$r.json')); print('$V', round(d['value'],1), round(d['frame']['median_ms']*1e3,1), d['kernels_us'], d['config'].get('gn_iters_mean'))"
  done
done
