#!/bin/bash
# Round 6: tracking bench (default 100 steps, no BA / store / CPU legs) and its rocprofv3 kernel-trace stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r06}
mkdir -p gpurun_out/$TAG
ARGS=${ARGS:---no-cpu --no-ba --no-peaks --no-retrieval --no-store}
for k in 1 2; do
  timeout -k 10 300 python3 bench.py $ARGS > gpurun_out/$TAG/bench_$k.json 2> gpurun_out/$TAG/bench_$k.err
  rc=$?; echo "BENCH_RC=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/$TAG/bench_$k.err; exit $rc; }
  python3 -c "import json;d=json.load(open('gpurun_out/$TAG/bench_$k.json'));print(round(d['value']),d['frame']['median_ms'],d['kernels_us'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/trace -o run -- python3 bench.py --steps 40 --warmup 5 $ARGS > gpurun_out/$TAG/trace_bench.json 2> gpurun_out/$TAG/trace.err
rc=$?; echo "TRACE_RC=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/$TAG/trace -name "run_kernel_stats.csv" | head -1); cp "$f" gpurun_out/$TAG/kernel_stats.csv
find gpurun_out/$TAG/trace -name "run_kernel_trace.csv" -delete
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/$TAG/kernel_stats.csv')):
    print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,2))
"
