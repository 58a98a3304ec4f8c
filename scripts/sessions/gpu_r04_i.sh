#!/bin/bash
# round 4: SQ counters of the screened refine tile kernel (two passes, kernel-trace only)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/rpmc4
export TMPDIR=/tmp
N=0
for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_LDS_ADDR_CONFLICT SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_ANY"; do
  N=$((N+1))
  REFINE_EXP_QUICK=1 timeout -k 10 -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex refine_tile --kernel-trace --output-format csv -d gpurun_out/rpmc4/p$N -o run -- python3 scripts/refine_exp.py > gpurun_out/rpmc4/p$N.log 2>&1
  rc=$?; echo "PMC_$N=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/rpmc4/p$N.log; exit $rc; }
done
python3 scripts/pmc_summary.py gpurun_out/rpmc4 > gpurun_out/r04i_refine_pmc.txt; cat gpurun_out/r04i_refine_pmc.txt
find gpurun_out/rpmc4 -name "*.csv" -size +2M -delete
