#!/bin/bash
# round 4: same-box A/B of the refine sole-sure-winner shortcut (shipped) vs without it (lib/exp/libm3s_nopend.so)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
L=lightweight-mast3r-slam_amd/lib
{
for r in 1 2 3; do
  for V in main nopend; do
    if [ $V = main ]; then LIB=$L/libm3s.so; else LIB=$L/exp/libm3s_$V.so; fi
    echo "== $V"; M3S_LIB=$LIB REFINE_EXP_QUICK=1 timeout -k 10 120 python3 scripts/refine_exp.py || exit 1
  done
done
} 2>&1 | grep -v amdgpu.ids > gpurun_out/r04u_refine_exp.txt
cat gpurun_out/r04u_refine_exp.txt
