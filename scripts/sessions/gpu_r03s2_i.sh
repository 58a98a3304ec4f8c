#!/bin/bash
# BA linearisation accuracy / time: X + (D X + t) with D = sR - I (main: + row FMAs; nofma: transform only) vs the
# quaternion expression (quat): the fp64-truth error of every BA fixture (scripts/ba_acc.py), then C5 / C4 lin time
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for V in quat nofma main; do
  if [ "$V" = main ]; then L=lightweight-mast3r-slam_amd/lib/libm3s.so; else L=lightweight-mast3r-slam_amd/lib/exp/libm3s_$V.so; fi
  echo "== $V"
  M3S_LIB=$L timeout -k 10 300 python3 scripts/ba_acc.py 2>&1 | grep -vE "amdgpu.ids" | tail -12 || exit 1
  M3S_LIB=$L timeout -k 10 200 python3 scripts/ba_exp.py 256 384 512 10 chess calib 2>&1 | grep -E "^rep 1|rror" || exit 1
  M3S_LIB=$L timeout -k 10 200 python3 scripts/ba_exp.py 256 320 512 10 euroc rays 2>&1 | grep -E "^rep 1|rror" || exit 1
done
