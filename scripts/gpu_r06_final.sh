#!/bin/bash
# Round-6 closing evidence: smoke + every GPU test (-s: the printed parity rates), the default bench line, the same
# line at the driver's 20 / 5 steps, then the tracking bench's kernel-trace stats and PMC passes (gpu_prof.sh),
# summarised by profile_summary.py into gpurun_out/summ (copied into profiles/ afterwards).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/summ
export TMPDIR=/tmp
TAG=${TAG:-r06}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/summ/${TAG}_smoke.txt 2>&1
rc=$?; echo "SMOKE_RC=$rc"; tail -2 gpurun_out/summ/${TAG}_smoke.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/summ/${TAG}_pytest_gpu.txt 2>&1
rc=$?; echo "PYTEST_RC=$rc"; tail -2 gpurun_out/summ/${TAG}_pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py > gpurun_out/summ/${TAG}_bench.json 2> gpurun_out/summ/${TAG}_bench.err
rc=$?; echo "BENCH_RC=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/summ/${TAG}_bench.err; exit $rc; }
python3 -c "import json;d=json.load(open('gpurun_out/summ/${TAG}_bench.json'));print(round(d['value']),d['frame']['median_ms'],d['kernels_us'],d['ba']['edges_per_s'],d['ba']['ms_solve_per_iter'])"
for k in 1 2 3; do
  timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-retrieval --no-store --no-peaks > gpurun_out/summ/${TAG}_bench_s20_$k.json 2>/dev/null
  python3 -c "import json;d=json.load(open('gpurun_out/summ/${TAG}_bench_s20_$k.json'));f=d['frame'];print('s20', round(d['value']),round(f['median_ms'],4),round(f['mean_ms'],4),round(f['max_ms'],4),f['first_ms'])"
done
ARGS="--steps 20 --warmup 5 --no-cpu --no-ba --no-peaks --no-retrieval --no-store" TAG=$TAG bash scripts/gpu_prof.sh || exit $?
PROF_OUT=gpurun_out/summ python3 scripts/profile_summary.py gpurun_out/prof $TAG || exit $?
find gpurun_out/prof -name "run_kernel_trace.csv" -delete 2>/dev/null
find gpurun_out/prof -name "run_counter_collection.csv" -size +4M -delete 2>/dev/null
du -sh gpurun_out
