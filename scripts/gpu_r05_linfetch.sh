#!/bin/bash
# round 5: ba_lin_kernel with the first round's records and X_j fetched before the relative-pose math ("new") vs the
# committed kernel ("head",
# lib/ab): the BA GPU tests on new, the C5 loop's kernel-trace stats for both (scripts/ba_exp.py), poses compared
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05lf
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ba.py tests/test_gpu_ba_top.py > gpurun_out/r05lf/tests.txt 2>&1 || { tail -40 gpurun_out/r05lf/tests.txt; exit 1; }
tail -2 gpurun_out/r05lf/tests.txt
for rep in 1 2 3; do
for V in new head; do
  if [ "$V" = new ]; then L=lightweight-mast3r-slam_amd/lib/libm3s.so; else L=lightweight-mast3r-slam_amd/lib/ab/libm3s_$V.so; fi
  M3S_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/be_${V}_$rep -o run -- python3 scripts/ba_exp.py 256 384 512 3 chess calib > gpurun_out/r05lf/${V}_$rep.log 2>&1 || { tail -20 gpurun_out/r05lf/${V}_$rep.log; exit 1; }
  S=$(find /tmp/be_${V}_$rep -name "*kernel_stats.csv" | head -1)
  cp "$S" gpurun_out/r05lf/${V}_${rep}_kernel_stats.csv
  python3 - gpurun_out/r05lf/${V}_${rep}_kernel_stats.csv "$V $rep" <<'PY'
import csv, sys
r = {}
for row in csv.DictReader(open(sys.argv[1])):
    for k in ("ba_edge_kernel", "ba_lin_kernel", "ba_sparse_factor", "ba_pack_kernel"):
        if k in row["Name"]:
            r[k] = r.get(k, 0) + float(row["TotalDurationNs"]) / 1e3 / max(int(row["Calls"]), 1)
print(sys.argv[2], "  ".join("%s %.2f" % kv for kv in r.items()))
PY
  grep -i "pose\|Twc\|sha\|hash" gpurun_out/r05lf/${V}_$rep.log | head -3
done
done
