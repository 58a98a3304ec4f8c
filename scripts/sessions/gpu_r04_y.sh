#!/bin/bash
# round 4: refine half-chunk double-buffered window (RT_HALF=1, shipped) vs the chunk windows (lib/exp/libm3s_nohalf.so):
# bit-exact parity first, then same-box timings and the tracking bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_refine_screen.py tests/test_gpu_matching.py tests/test_gpu_configs.py > gpurun_out/r04y_pytest.txt 2>&1
rc=$?; tail -3 gpurun_out/r04y_pytest.txt; [ $rc -eq 0 ] || exit $rc
L=lightweight-mast3r-slam_amd/lib
{
for r in 1 2 3; do
  for V in main nohalf; do
    if [ $V = main ]; then LIB=$L/libm3s.so; else LIB=$L/exp/libm3s_$V.so; fi
    echo "== $V"; M3S_LIB=$LIB timeout -k 10 120 python3 scripts/refine_exp.py || exit 1
  done
done
} 2>&1 | grep -v amdgpu.ids > gpurun_out/r04y_refine_exp.txt
cat gpurun_out/r04y_refine_exp.txt | grep -v "8x512"
A="--steps 100 --warmup 10 --no-ba --no-cpu --no-retrieval --no-store --no-peaks"
for r in 1 2; do
  for V in main nohalf; do
    if [ $V = main ]; then LIB=$L/libm3s.so; else LIB=$L/exp/libm3s_$V.so; fi
    M3S_LIB=$LIB timeout -k 10 240 python3 bench.py $A > gpurun_out/r04y_${V}_$r.json 2> gpurun_out/r04y_${V}_$r.err || { tail -20 gpurun_out/r04y_${V}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r04y_${V}_$r.json')); print('$V', round(d['value'],1), round(d['frame']['median_ms']*1e3,1), d['kernels_us'])"
  done
done
