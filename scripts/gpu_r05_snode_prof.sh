#!/bin/bash
# round 5: kernel split of the supernodal solve (rocprofv3 kernel trace, C5 and C4)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for G in "384 512 10 chess calib" "320 512 10 euroc rays"; do
  set -- $G
  M3S_BA_SOLVER=snode timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r05d_$4 -o prof -- python3 scripts/ba_exp.py 256 $1 $2 $3 $4 $5 > /tmp/r05d_$4.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob
for f in sorted(glob.glob("/tmp/r05d_*/**/*kernel_stats.csv", recursive=True)):
    print("==", f)
    for r in csv.DictReader(open(f)):
        print(f"{r['Name'][:70]:70s} calls {r['Calls']:>6s} avg_us {float(r['AverageNs'])/1e3:9.2f} total_ms {float(r['TotalDurationNs'])/1e6:8.2f}")
PY
