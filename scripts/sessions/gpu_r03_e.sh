#!/bin/bash
# Iteration check: all GPU tests, GN-loop per-block stamps, factor stamps, C5/C4 BA timing, a short bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "PYTEST_RC=$rc"; grep -E "FAILED|passed|failed" gpurun_out/pytest_gpu.log | tail -12; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
M3S_LIB=lightweight-mast3r-slam_amd/lib/exp/libm3s_gnst.so timeout -k 10 200 python3 scripts/gn_exp.py > gpurun_out/gn_stamps.txt 2>&1
rc=$?; echo "GN_STAMPS_RC=$rc"; grep -v amdgpu.ids gpurun_out/gn_stamps.txt; [ $rc -eq 0 ] || exit $rc
M3S_LIB=lightweight-mast3r-slam_amd/lib/exp/libm3s_spst.so timeout -k 10 200 python3 scripts/ba_exp.py 256 384 512 3 chess calib > gpurun_out/sp_stamps.txt 2>&1
echo "SP_STAMPS_RC=$?"; tail -4 gpurun_out/sp_stamps.txt
timeout -k 10 200 python3 scripts/ba_exp.py 256 384 512 10 chess calib 2>&1 | grep "rep 1" || exit 1
timeout -k 10 200 python3 scripts/ba_exp.py 256 320 512 10 euroc rays 2>&1 | grep "rep 1" || exit 1
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-cpu --no-retrieval --no-peaks > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "BENCH_RC=$rc"; python3 -c "
import json; d=json.loads(open('gpurun_out/bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'kernels', d['kernels_us'], 'frame', d['frame']['median_ms'])
b=d['ba']; print('C5', {x: b[x] for x in ('edges_per_s','ms_per_call','ms_setup','ms_pack','ms_plan_host','ms_lin_per_iter','ms_solve_per_iter')}, b['roofline']['frac'])
c=b['c4']; print('C4', {x: c[x] for x in ('edges_per_s','ms_per_call','ms_setup','ms_lin_per_iter','ms_solve_per_iter')}, c['roofline']['frac'])
"; [ $rc -eq 0 ] || { tail -30 gpurun_out/bench.err; exit $rc; }
for V in ${VARIANTS}; do
  L=lightweight-mast3r-slam_amd/lib/exp/libm3s_$V.so; echo "== $V"
  M3S_LIB=$L timeout -k 10 400 python3 -u scripts/ba_acc.py > gpurun_out/acc_$V.json 2> gpurun_out/acc_$V.err
  echo "ACC_RC=$?"; cat gpurun_out/acc_$V.json
  M3S_LIB=$L timeout -k 10 200 python3 scripts/ba_exp.py 256 320 512 10 euroc rays 2>&1 | grep "rep 1"
done
