#!/bin/bash
# BA fp32 run length 32 (run32 build) vs the shipped 16 after the D-form transform: accuracy census + C5 / C4 time
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for V in run32 main run32 main; do
  if [ "$V" = main ]; then L=lightweight-mast3r-slam_amd/lib/libm3s.so; else L=lightweight-mast3r-slam_amd/lib/exp/libm3s_$V.so; fi
  echo "== $V"
  [ "$V" = run32 ] && { M3S_LIB=$L timeout -k 10 300 python3 scripts/ba_acc.py 2>&1 | grep -E "^\{" || exit 1; }
  M3S_LIB=$L timeout -k 10 200 python3 scripts/ba_exp.py 256 384 512 10 chess calib 2>&1 | grep -E "^rep 1|rror" || exit 1
  M3S_LIB=$L timeout -k 10 200 python3 scripts/ba_exp.py 256 320 512 10 euroc rays 2>&1 | grep -E "^rep 1|rror" || exit 1
done
