#!/bin/bash
# round 4: folded tracking setup (M3S_TRACK_FOLD_SETUP) bit-identity tests, then an A/B of the tracking bench
# (separate setup launch vs folded), three alternating pairs on one box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_tracking.py > gpurun_out/r04n_pytest.txt 2>&1
rc=$?; tail -5 gpurun_out/r04n_pytest.txt; [ $rc -eq 0 ] || exit $rc
A="--steps 100 --warmup 10 --no-ba --no-cpu --no-retrieval --no-store --no-peaks"
for r in 1 2 3; do
  for F in 0 1; do
    M3S_TRACK_FOLD_SETUP=$F timeout -k 10 240 python3 bench.py $A > gpurun_out/r04n_fold${F}_$r.json 2> gpurun_out/r04n_fold${F}_$r.err || { tail -20 gpurun_out/r04n_fold${F}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/r04n_fold${F}_$r.json')); print('fold=$F', round(d['value'],1), round(d['frame']['median_ms']*1e3,1), d['kernels_us'])"
  done
done
