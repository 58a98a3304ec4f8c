#!/bin/bash
# BA accumulation-order variants: accuracy census (scripts/ba_acc.py) + C5/C4 timing per library; tracking tests;
# VALU issue rates with the wall-clock calibration.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
[ -n "$SKIP_FMA" ] || timeout -k 10 120 ./scripts/micro/fma_rates > gpurun_out/fma_rates.txt 2>&1
rc=$?; echo "FMA_RATES_RC=$rc"; cat gpurun_out/fma_rates.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_tracking.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/track_tests.log 2>&1
rc=$?; echo "TRACK_TESTS_RC=$rc"; tail -3 gpurun_out/track_tests.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for V in main ${VARIANTS}; do
  if [ "$V" = main ]; then L=lightweight-mast3r-slam_amd/lib/libm3s.so; else L=lightweight-mast3r-slam_amd/lib/exp/libm3s_$V.so; fi
  echo "== $V"
  M3S_LIB=$L timeout -k 10 400 python3 -u scripts/ba_acc.py > gpurun_out/acc_$V.json 2> gpurun_out/acc_$V.err
  rc=$?; echo "ACC_RC=$rc"; cat gpurun_out/acc_$V.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/acc_$V.err; exit $rc; }
  M3S_LIB=$L timeout -k 10 200 python3 scripts/ba_exp.py 256 384 512 10 chess calib 2>&1 | grep "rep 1" || exit 1
  M3S_LIB=$L timeout -k 10 200 python3 scripts/ba_exp.py 256 320 512 10 euroc rays 2>&1 | grep "rep 1" || exit 1
done
