#!/bin/bash
# rocprofv3 kernel trace (+ --stats) and PMC passes (one counter group per run, kernel trace only) of the
# C5 BA loop (256-keyframe chess graph, calib, 384x512): HBM bytes, VALU / memory instruction counts.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/ba_pmc}
mkdir -p $OUT
export TMPDIR=/tmp
ARGS=${ARGS:-"256 384 512 3 chess calib"}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 scripts/ba_exp.py $ARGS > $OUT/trace.log 2>&1
echo "TRACE RC=$?"
for P in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_TRANS_F32" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"; do
  N=$(echo $P | tr ' ' '_' | cut -c1-40)
  timeout -k 10 -s KILL 200 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $OUT/$N -o run -- python3 scripts/ba_exp.py $ARGS > $OUT/$N.log 2>&1
  echo "PMC $N RC=$?"
done
python3 scripts/pmc_summary.py $OUT > $OUT/summary.txt 2>&1; grep -A3 "ba_lin\|==" $OUT/summary.txt | head -60
