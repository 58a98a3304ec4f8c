#!/bin/bash
# Retrieval quantization: kernel-trace stats + HBM traffic (FETCH_SIZE / WRITE_SIZE passes) of scripts/rq_exp.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/rqprof
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rqprof/trace -o run -- python3 scripts/rq_exp.py 65536 1024 300 5 20 > gpurun_out/rqprof/trace.log 2>&1 || exit 1
for P in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d gpurun_out/rqprof/pmc_$P -o run -- python3 scripts/rq_exp.py 65536 1024 300 5 5 > /dev/null 2>&1 || exit 1
done
echo RQPROF_OK
