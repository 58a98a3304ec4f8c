#!/bin/bash
# round 4: the default bench line, the refine window-rework timings (screen / exact / fill-only / survivor stats),
# then a tracking A/B of the separate vs folded setup (two alternating pairs)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python bench.py > gpurun_out/r04p_bench.json 2> gpurun_out/r04p_bench.err || { tail -20 gpurun_out/r04p_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r04p_bench.json')); print(d['value'], d['kernels_us'], d['frame']['median_ms'], d['roofline']['frac'], d['ba']['ms_solve_per_iter'], d['ba']['ms_lin_per_iter'], d['ba']['edges_per_s'], d['cpu_baseline']['value'], d['cpu_baseline']['cores'])"
L=lightweight-mast3r-slam_amd/lib
{
echo "== screen"; timeout -k 10 120 python3 scripts/refine_exp.py || exit 1
echo "== exact (M3S_REFINE_SCREEN=0)"; M3S_REFINE_SCREEN=0 timeout -k 10 120 python3 scripts/refine_exp.py || exit 1
for V in fillonly stats; do
  echo "== $V"; M3S_LIB=$L/exp/libm3s_$V.so timeout -k 10 120 python3 scripts/refine_exp.py || exit 1
done
} 2>&1 | grep -v amdgpu.ids > gpurun_out/r04p_refine_exp.txt
cat gpurun_out/r04p_refine_exp.txt
A="--steps 100 --warmup 10 --no-ba --no-cpu --no-retrieval --no-store --no-peaks"
for r in 1 2; do
  for F in 0 1; do
    M3S_TRACK_FOLD_SETUP=$F timeout -k 10 240 python3 bench.py $A > gpurun_out/r04p_fold${F}_$r.json 2> gpurun_out/r04p_fold${F}_$r.err || { tail -20 gpurun_out/r04p_fold${F}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/r04p_fold${F}_$r.json')); print('fold=$F', round(d['value'],1), round(d['frame']['median_ms']*1e3,1), d['kernels_us'])"
  done
done
