#!/bin/bash
# rocprofv3 kernel-trace stats + separate PMC passes (never combined with sys/runtime traces).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
TAG=${TAG:-r01}
ARGS=${ARGS:---steps 20 --warmup 5 --no-cpu --no-ba --no-peaks --no-retrieval}
rocprofv3 -L > gpurun_out/prof/counters_list.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace -o run -- python3 bench.py $ARGS > gpurun_out/prof/trace_bench.json 2> gpurun_out/prof/trace.err
echo "TRACE_RC=$?"
for P in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum" ; do
  N=$(echo $P | tr ' ' '_' | cut -c1-40)
  timeout -k 10 300 rocprofv3 --pmc $P --kernel-trace --output-format csv -d gpurun_out/prof/pmc_$N -o run -- python3 bench.py $ARGS > /dev/null 2> gpurun_out/prof/pmc_$N.err
  echo "PMC $N RC=$?"
done
find gpurun_out/prof -name "*.csv" | head -50
