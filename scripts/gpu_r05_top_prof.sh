#!/bin/bash
# round 5: kernel-trace stats of the C5 BA loop with the dense top phase (M3S_BA_TOP=25) and without, + the split's
# fixed cost at M3S_BA_TOP=2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r05v
for TOP in 0 25; do
  M3S_BA_TOP=$TOP timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r05v_$TOP -o run -- python3 scripts/ba_exp.py 256 384 512 3 chess calib > gpurun_out/r05v/exp_$TOP.txt 2>&1 || { tail -20 gpurun_out/r05v/exp_$TOP.txt; exit 1; }
  f=$(find /tmp/r05v_$TOP -name "run_kernel_stats.csv" | head -1)
  echo "== top $TOP"; grep "rep 1" gpurun_out/r05v/exp_$TOP.txt
  python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if "sparse" in n or "dense_top" in n or "assemble" in n or "step_kernel" in n:
        print(f"  {n[:70]:70s} calls {r['Calls']:>6s} avg {float(r['AverageNs'])/1e3:8.1f} us")
PY
done
for TOP in 0 2 0 2; do echo "== top $TOP"; M3S_BA_TOP=$TOP timeout -k 10 200 python3 scripts/ba_exp.py 256 384 512 10 chess calib 2>&1 | grep "rep 1" || exit 1; done
