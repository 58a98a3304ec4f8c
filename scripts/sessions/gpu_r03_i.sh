#!/bin/bash
# Refine: candidate-chain interleave A/B (lib/exp/libm3s_ilvN: N chains of a column interleaved channel by channel)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for V in main ilv2 ilv3 ilv4 ilv7 main ilv2; do
  if [ "$V" = main ]; then L=lightweight-mast3r-slam_amd/lib/libm3s.so; else L=lightweight-mast3r-slam_amd/lib/exp/libm3s_$V.so; fi
  echo "== $V"
  M3S_LIB=$L timeout -k 10 120 python3 scripts/refine_exp.py 2>&1 | grep -v amdgpu.ids | grep -v "^8x512" || exit 1
done
