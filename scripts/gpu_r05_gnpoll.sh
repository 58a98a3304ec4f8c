#!/bin/bash
# round 5: GN hand-off polls and the shard counters read with all loads issued first ("new") vs
# the committed kernel
# ("head", lib/ab):
# tracker outputs bit for bit (scripts/track_dump.py), then kernel-trace stats and bench frames/s alternating (3 reps)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05gp
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_tracking.py > gpurun_out/r05gp/tests.txt 2>&1 || { tail -30 gpurun_out/r05gp/tests.txt; exit 1; }
tail -2 gpurun_out/r05gp/tests.txt
timeout -k 10 200 python3 -u scripts/track_dump.py /tmp/r05gp_new.npz > gpurun_out/r05gp/dump_new.txt 2>&1 || { tail -20 gpurun_out/r05gp/dump_new.txt; exit 1; }
M3S_LIB=lightweight-mast3r-slam_amd/lib/ab/libm3s_head.so timeout -k 10 200 python3 -u scripts/track_dump.py /tmp/r05gp_head.npz > gpurun_out/r05gp/dump_head.txt 2>&1 || { tail -20 gpurun_out/r05gp/dump_head.txt; exit 1; }
python3 - <<'PY'
import numpy as np
a, b = np.load("/tmp/r05gp_new.npz"), np.load("/tmp/r05gp_head.npz")
bad = [k for k in a.files if not np.array_equal(a[k], b[k])]
print("bit-identical:", not bad, "arrays", len(a.files), "differing", bad[:10])
PY
ARGS="--steps 100 --warmup 10 --no-cpu --no-ba --no-peaks --no-retrieval --no-store --no-kernel-timing"
for rep in 1 2 3; do
for V in head new; do
  if [ "$V" = new ]; then L=lightweight-mast3r-slam_amd/lib/libm3s.so; else L=lightweight-mast3r-slam_amd/lib/ab/libm3s_$V.so; fi
  M3S_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/gs_${V}_$rep -o run -- python3 bench.py $ARGS > gpurun_out/r05gp/${V}_$rep.json 2> gpurun_out/r05gp/${V}_$rep.err || { tail -20 gpurun_out/r05gp/${V}_$rep.err; exit 1; }
  S=$(find /tmp/gs_${V}_$rep -name "*kernel_stats.csv" | head -1)
  cp "$S" gpurun_out/r05gp/${V}_${rep}_kernel_stats.csv
  python3 - gpurun_out/r05gp/${V}_${rep}_kernel_stats.csv "$V $rep" <<'PY'
import csv, sys
r = {}
for row in csv.DictReader(open(sys.argv[1])):
    for k in ("prep_rays", "proj_occ", "refine_tile", "gn_loop", "fuse_kernel"):
        if k in row["Name"]:
            r[k] = float(row["AverageNs"]) / 1e3
print(sys.argv[2], "  ".join("%s %.2f" % kv for kv in r.items()), " sum %.2f" % sum(r.values()))
PY
  M3S_LIB=$L timeout -k 10 300 python3 bench.py --steps 200 --warmup 20 --no-cpu --no-ba --no-peaks --no-retrieval --no-store > gpurun_out/r05gp/b_${V}_$rep.json 2> gpurun_out/r05gp/b_${V}_$rep.err || { tail -20 gpurun_out/r05gp/b_${V}_$rep.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r05gp/b_${V}_$rep.json').read().strip().splitlines()[-1]); print('  fps', round(d['value'],1), d['kernels_us'])"
done
done
