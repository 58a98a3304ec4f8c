#!/bin/bash
# Round-5 closing evidence: smoke + every GPU test, the default bench line, then the tracking bench's kernel-trace
# stats and PMC passes (gpu_prof.sh, summarised by profile_summary.py). The BA kernels are unchanged since the
# round-5 BA profiles (profiles/r05_ba*), so their passes are not repeated.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/summ
export TMPDIR=/tmp
bash scripts/gpu_check.sh || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
rc=$?; echo "BENCH_RC=$rc"; tail -c 400 gpurun_out/bench_default.json; [ $rc -eq 0 ] || exit $rc
ARGS="--steps 20 --warmup 5 --no-cpu --no-ba --no-peaks --no-retrieval --no-store" bash scripts/gpu_prof.sh || exit $?
PROF_OUT=gpurun_out/summ python3 scripts/profile_summary.py gpurun_out/prof ${TAG:-r05f} || exit $?
find gpurun_out/prof -name "run_kernel_trace.csv" -delete 2>/dev/null
find gpurun_out/prof -name "run_counter_collection.csv" -size +4M -delete 2>/dev/null
du -sh gpurun_out
