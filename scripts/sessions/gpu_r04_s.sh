#!/bin/bash
# round 4: refine window outliers: hybrid (default: in place up to RT_INPLACE_MAX per wave, else deferred) vs
# pure in place (M3S_REFINE_INPLACE=1: no deferred list, no outlier
# launch) vs the deferred list + refine_outlier_kernel; idx checksum must match; then the tracking bench A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
{
for r in 1 2; do
  for I in 0 1; do
    echo "== inplace=$I"; M3S_REFINE_INPLACE=$I REFINE_EXP_QUICK=1 timeout -k 10 120 python3 scripts/refine_exp.py || exit 1
  done
done
} 2>&1 | grep -v amdgpu.ids > gpurun_out/r04s_refine_exp.txt
cat gpurun_out/r04s_refine_exp.txt
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_matching.py tests/test_gpu_refine_screen.py > gpurun_out/r04s_pytest.txt 2>&1
rc=$?; tail -3 gpurun_out/r04s_pytest.txt; [ $rc -eq 0 ] || exit $rc
A="--steps 100 --warmup 10 --no-ba --no-cpu --no-retrieval --no-store --no-peaks"
for r in 1 2; do
  for I in 0 1; do
    M3S_REFINE_INPLACE=$I timeout -k 10 240 python3 bench.py $A > gpurun_out/r04s_in${I}_$r.json 2> gpurun_out/r04s_in${I}_$r.err || { tail -20 gpurun_out/r04s_in${I}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r04s_in${I}_$r.json')); print('inplace=$I', round(d['value'],1), round(d['frame']['median_ms']*1e3,1), d['kernels_us'])"
  done
done
