#!/bin/bash
# Round 6 A/B of tracking builds on one box: the tracker's outputs bit for bit (scripts/track_dump.py) and, alternating,
# rocprofv3 kernel stats + the bench's frames/s. LIBS="head new" (lightweight-mast3r-slam_amd/lib/exp/libm3s_<name>.so;
# "new" = the in-tree lib/libm3s.so). OUT=gpurun_out/<tag>.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/ab}
LIBS=${LIBS:-head new}
REPS=${REPS:-2}
mkdir -p $OUT
libpath() { if [ "$1" = new ]; then echo lightweight-mast3r-slam_amd/lib/libm3s.so; else echo lightweight-mast3r-slam_amd/lib/exp/libm3s_$1.so; fi; }
for L in $LIBS; do
  M3S_LIB=$(libpath $L) timeout -k 10 200 python3 scripts/track_dump.py $OUT/dump_$L.npz > $OUT/dump_$L.log 2>&1
  rc=$?; echo "DUMP_$L=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/dump_$L.log; exit $rc; }
  M3S_LIB=$(libpath $L) timeout -k 10 200 python3 scripts/match_dump.py $OUT/mdump_$L.npz > $OUT/mdump_$L.log 2>&1
  rc=$?; echo "MDUMP_$L=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/mdump_$L.log; exit $rc; }
done
python3 - "$OUT" $LIBS <<'PY'
import sys, numpy as np
out, libs = sys.argv[1], sys.argv[2:]
for pre in ("dump", "mdump"):
    ref = np.load(f"{out}/{pre}_{libs[0]}.npz")
    for L in libs[1:]:
        d = np.load(f"{out}/{pre}_{L}.npz")
        bad = [k for k in ref.files if not np.array_equal(ref[k], d[k], equal_nan=True)]
        print(f"{pre} bit-identical {libs[0]} vs {L}: {not bad} arrays {len(ref.files)} differing {bad[:8]}")
PY
rm -f $OUT/dump_*.npz $OUT/mdump_*.npz  # ~100 MB: the copy-back limit is 64 MiB
for r in $(seq 1 $REPS); do
  for L in $LIBS; do
    D=$OUT/prof_${L}_$r
    M3S_LIB=$(libpath $L) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 bench.py --steps 60 --warmup 10 --no-cpu --no-ba --no-peaks --no-retrieval --no-store > $D.json 2> $D.err
    rc=$?; [ $rc -eq 0 ] || { echo "PROF_$L rc=$rc"; tail -5 $D.err; exit $rc; }
    f=$(find $D -name "run_kernel_stats.csv" | head -1)
    python3 - "$f" "$D.json" "$L" "$r" <<'PY'
import csv, json, sys
f, j, L, r = sys.argv[1:]
rows = {x["Name"]: float(x["AverageNs"]) / 1e3 for x in csv.DictReader(open(f))}
short = {"refine_tile": "refine", "gn_loop": "gn", "proj_occlusion": "proj", "prep_rays": "prep", "fuse_kernel": "fuse"}
got = {}
for name, us in rows.items():
    for k, v in short.items():
        if k in name:
            got[v] = got.get(v, 0) + us
d = json.load(open(j))
print(f"{L} {r}: " + "  ".join(f"{k} {v:.2f}" for k, v in got.items()) + f"  sum {sum(got.values()):.2f}  fps(traced) {d['value']:.0f}")
PY
    find $D -name "run_kernel_trace.csv" -delete
    M3S_LIB=$(libpath $L) timeout -k 10 200 python3 bench.py --no-cpu --no-ba --no-peaks --no-retrieval --no-store > $OUT/bench_${L}_$r.json 2>/dev/null
    python3 -c "import json;d=json.load(open('$OUT/bench_${L}_$r.json'));print('   $L $r fps', round(d['value']), 'median_ms', round(d['frame']['median_ms'],4), d['kernels_us'])"
  done
done
