#!/bin/bash
# round 5: contraction and rays Newton variants of the BA linearisation — accuracy census vs the fp64 truth,
# then C5 / C4 linearisation time
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for V in main fast nonewton fastnn; do
  if [ "$V" = main ]; then L=lightweight-mast3r-slam_amd/lib/libm3s.so; else L=lightweight-mast3r-slam_amd/lib/ab/libm3s_$V.so; fi
  echo "== $V accuracy" && M3S_LIB=$L timeout -k 10 400 python3 scripts/ba_acc.py 2>&1 | grep -v amdgpu.ids | tail -3 || exit 1
done
for rep in 1 2; do
for V in main fast nonewton fastnn; do
  if [ "$V" = main ]; then L=lightweight-mast3r-slam_amd/lib/libm3s.so; else L=lightweight-mast3r-slam_amd/lib/ab/libm3s_$V.so; fi
  echo "== $V C5" && M3S_LIB=$L timeout -k 10 200 python3 scripts/ba_exp.py 256 384 512 10 chess calib 2>&1 | grep "rep 1" || exit 1
  echo "== $V C4" && M3S_LIB=$L timeout -k 10 200 python3 scripts/ba_exp.py 256 320 512 10 euroc rays 2>&1 | grep "rep 1" || exit 1
done
done
