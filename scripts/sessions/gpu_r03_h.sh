#!/bin/bash
# Refine add-encoding A/B (main: hand-picked VOP2 + SDWA adds; rnoslp: the compiler's scalar adds; rold: the
# compiler's paired v_pk_add_f16) + matching parity on main; one SQ counter pass of refine on main
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/rpmc
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_matching.py -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/match_tests.log 2>&1
rc=$?; echo "MATCH_TESTS_RC=$rc"; tail -2 gpurun_out/match_tests.log; [ $rc -eq 0 ] || exit $rc
for V in rold rnoslp main rold main; do
  if [ "$V" = main ]; then L=lightweight-mast3r-slam_amd/lib/libm3s.so; else L=lightweight-mast3r-slam_amd/lib/exp/libm3s_$V.so; fi
  echo "== $V"
  M3S_LIB=$L timeout -k 10 120 python3 scripts/refine_exp.py 2>&1 | grep -v amdgpu.ids || exit 1
done
for V in rold main; do
  if [ "$V" = main ]; then L=lightweight-mast3r-slam_amd/lib/libm3s.so; else L=lightweight-mast3r-slam_amd/lib/exp/libm3s_$V.so; fi
  M3S_LIB=$L timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS --kernel-include-regex refine_tile --kernel-trace --output-format csv -d gpurun_out/rpmc/$V -o run -- python3 scripts/refine_exp.py > gpurun_out/rpmc/$V.log 2>&1
  rc=$?; echo "PMC_$V=$rc"; [ $rc -eq 0 ] || exit $rc
done
# BA: the solve replayed as a captured graph (default) vs direct launches
timeout -k 10 400 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_configs.py -k "ba" -m gpu -q -x --timeout 240 --timeout-method thread > gpurun_out/ba_tests.log 2>&1
rc=$?; echo "BA_TESTS_RC=$rc"; tail -2 gpurun_out/ba_tests.log; [ $rc -eq 0 ] || exit $rc
for G in 1 0 1; do
  echo "== M3S_BA_GRAPH=$G"
  M3S_BA_GRAPH=$G timeout -k 10 200 python3 scripts/ba_exp.py 256 384 512 10 chess calib 2>&1 | grep "rep 1" || exit 1
  M3S_BA_GRAPH=$G timeout -k 10 200 python3 scripts/ba_exp.py 256 320 512 10 euroc rays 2>&1 | grep "rep 1" || exit 1
done
