#!/bin/bash
# PMC passes (one counter group per run) over the BA experiment: HBM bytes and VALU/memory instruction counts of ba_lin.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ba_pmc
export TMPDIR=/tmp
K=${K:-256}
for P in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_TRANS_F32" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"; do
  N=$(echo $P | tr ' ' '_' | cut -c1-40)
  timeout -k 10 -s KILL 200 rocprofv3 --pmc $P --kernel-trace --output-format csv -d gpurun_out/ba_pmc/$N -o run -- python3 scripts/ba_exp.py $K 384 512 3 > gpurun_out/ba_pmc/$N.log 2>&1
  echo "PMC $N RC=$?"
done
