#!/bin/bash
# round 4: kernel trace of the BA solve with the frontal phase on (plan's cut) and off (C5 chess calib, 384x512)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for F in def 0 12; do
  if [ $F = def ]; then unset M3S_BA_FRONT; else export M3S_BA_FRONT=$F; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04z2_$F -o run -- python3 scripts/ba_exp.py 256 384 512 4 chess calib > gpurun_out/r04z2_$F.log 2>&1 || { tail -5 gpurun_out/r04z2_$F.log; exit 1; }
  grep "rep 1" gpurun_out/r04z2_$F.log
  f=$(find gpurun_out/r04z2_$F -name "*kernel_stats.csv" | head -1)
  echo "== $F"; grep -E "ba_front|ba_sparse|ba_assemble|ba_subtree" "$f" | cut -d, -f1-8
  cp "$f" gpurun_out/r04z2_${F}_stats.csv && rm -rf gpurun_out/r04z2_$F
done
