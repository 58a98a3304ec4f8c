#!/bin/bash
# round 5: kernel-trace stats of the tracking bench, new vs head (lib/ab), alternating, 2 reps: prep_rays and
# fuse_kernel durations (the bench spans do not time the fuse launch)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05pp
export TMPDIR=/tmp
ARGS="--steps 60 --warmup 10 --no-cpu --no-ba --no-peaks --no-retrieval --no-store --no-kernel-timing"
for rep in 1 2; do
for V in new head; do
  if [ "$V" = new ]; then L=lightweight-mast3r-slam_amd/lib/libm3s.so; else L=lightweight-mast3r-slam_amd/lib/ab/libm3s_$V.so; fi
  M3S_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pp_${V}_$rep -o run -- python3 bench.py $ARGS > gpurun_out/r05pp/${V}_$rep.json 2> gpurun_out/r05pp/${V}_$rep.err || { tail -20 gpurun_out/r05pp/${V}_$rep.err; exit 1; }
  S=$(find /tmp/pp_${V}_$rep -name "*kernel_stats.csv" | head -1)
  cp "$S" gpurun_out/r05pp/${V}_${rep}_kernel_stats.csv
  echo "== $V $rep"; cut -d, -f1-4 "$S" | head -8
done
done
