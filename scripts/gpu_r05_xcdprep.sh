#!/bin/bash
# round 5: prep_rays tiles XCD-banded like proj_occlusion / refine (their L2 then holds what prep wrote) vs the
# previous build (lib/ab head): matching + tracking GPU tests on new, then kernel-trace stats (2 reps, alternating)
# and one TCC hit / miss PMC pass per variant
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05xp
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_matching.py tests/test_gpu_tracking.py tests/test_gpu_refine_screen.py > gpurun_out/r05xp/tests.txt 2>&1 || { tail -30 gpurun_out/r05xp/tests.txt; exit 1; }
tail -2 gpurun_out/r05xp/tests.txt
ARGS="--steps 60 --warmup 10 --no-cpu --no-ba --no-peaks --no-retrieval --no-store --no-kernel-timing"
for rep in 1 2; do
for V in new head; do
  if [ "$V" = new ]; then L=lightweight-mast3r-slam_amd/lib/libm3s.so; else L=lightweight-mast3r-slam_amd/lib/ab/libm3s_$V.so; fi
  M3S_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/xp_${V}_$rep -o run -- python3 bench.py $ARGS > gpurun_out/r05xp/${V}_$rep.json 2> gpurun_out/r05xp/${V}_$rep.err || { tail -20 gpurun_out/r05xp/${V}_$rep.err; exit 1; }
  S=$(find /tmp/xp_${V}_$rep -name "*kernel_stats.csv" | head -1)
  cp "$S" gpurun_out/r05xp/${V}_${rep}_kernel_stats.csv
  python3 - gpurun_out/r05xp/${V}_${rep}_kernel_stats.csv "$V $rep" <<'PY'
import csv, sys
r = {}
for row in csv.DictReader(open(sys.argv[1])):
    for k in ("prep_rays", "proj_occ", "refine_tile", "gn_loop", "fuse_kernel"):
        if k in row["Name"]:
            r[k] = float(row["AverageNs"]) / 1e3
print(sys.argv[2], "  ".join("%s %.2f" % kv for kv in r.items()))
PY
done
done
for V in new head; do
  if [ "$V" = new ]; then L=lightweight-mast3r-slam_amd/lib/libm3s.so; else L=lightweight-mast3r-slam_amd/lib/ab/libm3s_$V.so; fi
  M3S_LIB=$L timeout -k 10 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d /tmp/xpp_$V -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-ba --no-peaks --no-retrieval --no-store --no-kernel-timing > /dev/null 2> gpurun_out/r05xp/pmc_$V.err || { tail -20 gpurun_out/r05xp/pmc_$V.err; exit 1; }
  S=$(find /tmp/xpp_$V -name "*counter_collection.csv" | head -1)
  python3 - "$S" "$V" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for row in csv.DictReader(open(sys.argv[1])):
    for k in ("prep_rays", "proj_occ", "refine_tile", "gn_loop", "fuse_kernel"):
        if k in row["Kernel_Name"]:
            acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, d in acc.items():
    h = sum(d["TCC_HIT_sum"]) / max(len(d["TCC_HIT_sum"]), 1)
    m = sum(d["TCC_MISS_sum"]) / max(len(d["TCC_MISS_sum"]), 1)
    print(sys.argv[2], "%-12s hit %.0f miss %.0f  hit rate %.3f" % (k, h, m, h / max(h + m, 1)))
PY
done
