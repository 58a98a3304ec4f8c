#!/bin/bash
# round 4: refine screen breakdown (experiment builds; timings only, the shipped library first for the checksum)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
L=lightweight-mast3r-slam_amd/lib
{
echo "== main (screen)"; timeout -k 10 120 python3 scripts/refine_exp.py || exit 1
echo "== main exact (M3S_REFINE_SCREEN=0)"; M3S_REFINE_SCREEN=0 timeout -k 10 120 python3 scripts/refine_exp.py || exit 1
for V in nosurv noload nocomp fillonly stats; do
  echo "== $V"; M3S_LIB=$L/exp/libm3s_$V.so timeout -k 10 120 python3 scripts/refine_exp.py || exit 1
done
} 2>&1 | grep -v amdgpu.ids > gpurun_out/r04c_refine_exp.txt
cat gpurun_out/r04c_refine_exp.txt
