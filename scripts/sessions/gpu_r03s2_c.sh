#!/bin/bash
# BA solve phase stamps (M3S_SP_STAMPS build): dataflow vs level-synchronous, C5 and C4
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
L=lightweight-mast3r-slam_amd/lib/exp/libm3s_stamps.so
for F in 0 1; do
  echo "== flow $F"
  M3S_LIB=$L M3S_BA_FLOW=$F timeout -k 10 200 python3 scripts/ba_exp.py 256 384 512 4 chess calib 2>&1 | grep -vE "amdgpu.ids|^graph" || exit 1
  M3S_LIB=$L M3S_BA_FLOW=$F timeout -k 10 200 python3 scripts/ba_exp.py 256 320 512 4 euroc rays 2>&1 | grep -vE "amdgpu.ids|^graph" || exit 1
done
