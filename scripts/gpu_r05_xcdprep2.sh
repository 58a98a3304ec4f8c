#!/bin/bash
# round 5: XCD-banded prep_rays A/B, more repetitions: kernel-trace stats (4 reps, alternating) + bench frames/s
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05xq
export TMPDIR=/tmp
ARGS="--steps 100 --warmup 10 --no-cpu --no-ba --no-peaks --no-retrieval --no-store --no-kernel-timing"
for rep in 1 2 3 4; do
for V in new head; do
  if [ "$V" = new ]; then L=lightweight-mast3r-slam_amd/lib/libm3s.so; else L=lightweight-mast3r-slam_amd/lib/ab/libm3s_$V.so; fi
  M3S_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/xq_${V}_$rep -o run -- python3 bench.py $ARGS > gpurun_out/r05xq/${V}_$rep.json 2> gpurun_out/r05xq/${V}_$rep.err || { tail -20 gpurun_out/r05xq/${V}_$rep.err; exit 1; }
  S=$(find /tmp/xq_${V}_$rep -name "*kernel_stats.csv" | head -1)
  cp "$S" gpurun_out/r05xq/${V}_${rep}_kernel_stats.csv
  python3 - gpurun_out/r05xq/${V}_${rep}_kernel_stats.csv "$V $rep" <<'PY'
import csv, sys
r = {}
for row in csv.DictReader(open(sys.argv[1])):
    for k in ("prep_rays", "proj_occ", "refine_tile", "gn_loop", "fuse_kernel"):
        if k in row["Name"]:
            r[k] = float(row["AverageNs"]) / 1e3
print(sys.argv[2], "  ".join("%s %.2f" % kv for kv in r.items()), " sum %.2f" % sum(r.values()))
PY
  M3S_LIB=$L timeout -k 10 300 python3 bench.py --steps 200 --warmup 20 --no-cpu --no-ba --no-peaks --no-retrieval --no-store > gpurun_out/r05xq/b_${V}_$rep.json 2> gpurun_out/r05xq/b_${V}_$rep.err || { tail -20 gpurun_out/r05xq/b_${V}_$rep.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r05xq/b_${V}_$rep.json').read().strip().splitlines()[-1]); print('  fps', round(d['value'],1))"
done
done
