#!/bin/bash
# round 4: BA solve timings per cut, tracking tests + store leg, refine SQ counters
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
{
for S in def -1 6 10 16 24; do
  echo "== M3S_BA_SUB=$S"
  if [ $S = def ]; then unset M3S_BA_SUB; else export M3S_BA_SUB=$S; fi
  timeout -k 10 200 python3 scripts/ba_exp.py 256 384 512 10 chess calib 2>&1 | grep "rep 1" || exit 1
  timeout -k 10 200 python3 scripts/ba_exp.py 256 320 512 10 euroc rays 2>&1 | grep "rep 1" || exit 1
done
} > gpurun_out/r04j_ba_exp.txt 2>&1
rc=$?; cat gpurun_out/r04j_ba_exp.txt; [ $rc -eq 0 ] || exit $rc
unset M3S_BA_SUB
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_tracking.py > gpurun_out/r04j_track_tests.txt 2>&1
rc=$?; tail -4 gpurun_out/r04j_track_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-ba --no-cpu --no-retrieval --no-peaks > gpurun_out/r04j_bench.json 2> gpurun_out/r04j_bench.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r04j_bench.json')); print(d['value'], d['kernels_us'], d['store'])"
bash scripts/sessions/gpu_r04_i.sh
