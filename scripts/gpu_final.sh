#!/bin/bash
# Round-end evidence in one call: smoke + every GPU test, the default bench line, then the profiles
# (gpu_prof_round.sh: kernel-trace stats + PMC passes of the tracking bench and of the C5 BA loop).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/gpu_check.sh || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
rc=$?; echo "BENCH_RC=$rc"; tail -c 400 gpurun_out/bench_default.json; [ $rc -eq 0 ] || exit $rc
TAG=${TAG:-r03} bash scripts/gpu_prof_round.sh
