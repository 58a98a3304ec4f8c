#!/bin/bash
# round 4: refine sole-sure-winner shortcut (pending running max) + smaller outlier grid: bit-exact parity (refine,
# matching, configs, tracking), timings, tracking bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_refine_screen.py tests/test_gpu_matching.py tests/test_gpu_configs.py tests/test_gpu_tracking.py > gpurun_out/r04t_pytest.txt 2>&1
rc=$?; tail -4 gpurun_out/r04t_pytest.txt; [ $rc -eq 0 ] || exit $rc
{
for r in 1 2; do
  echo "== screen"; timeout -k 10 120 python3 scripts/refine_exp.py || exit 1
done
echo "== exact (M3S_REFINE_SCREEN=0)"; M3S_REFINE_SCREEN=0 REFINE_EXP_QUICK=1 timeout -k 10 120 python3 scripts/refine_exp.py || exit 1
} 2>&1 | grep -v amdgpu.ids > gpurun_out/r04t_refine_exp.txt
cat gpurun_out/r04t_refine_exp.txt
A="--steps 100 --warmup 10 --no-ba --no-cpu --no-retrieval --no-store --no-peaks"
for r in 1 2; do
  timeout -k 10 240 python3 bench.py $A > gpurun_out/r04t_b$r.json 2> gpurun_out/r04t_b$r.err || { tail -20 gpurun_out/r04t_b$r.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r04t_b$r.json')); print(round(d['value'],1), round(d['frame']['median_ms']*1e3,1), d['kernels_us'])"
done
