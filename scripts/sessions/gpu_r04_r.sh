#!/bin/bash
# round 4: refine register-pressure variants (spills): 3 blocks per CU (148 VGPRs, no spill), column read batches of
# 4 / 3 (fewer live candidate loads), against the shipped build; timings only (results are identical by construction)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
L=lightweight-mast3r-slam_amd/lib
{
for V in main occ3 cb4 cb3 occ3cb4 main; do
  if [ $V = main ]; then LIB=$L/libm3s.so; else LIB=$L/exp/libm3s_$V.so; fi
  echo "== $V"; M3S_LIB=$LIB REFINE_EXP_QUICK=1 timeout -k 10 120 python3 scripts/refine_exp.py || exit 1
done
} 2>&1 | grep -v amdgpu.ids > gpurun_out/r04r_refine_exp.txt
cat gpurun_out/r04r_refine_exp.txt
