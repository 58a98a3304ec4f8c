#!/bin/bash
# Round evidence on one GPU box: smoke, GPU parity tests, the default bench line, rocprofv3 kernel-trace
# stats + separate PMC passes of the tracking bench (gpu_prof.sh) and of the 256-keyframe BA loop.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof_ba
export TMPDIR=/tmp
bash scripts/gpu_check.sh || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
rc=$?; echo "BENCH_RC=$rc"; tail -c 600 gpurun_out/bench_default.json; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_prof.sh || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ba/trace -o run -- python3 scripts/ba_exp.py 256 384 512 3 > gpurun_out/prof_ba/trace.log 2>&1
echo "BA_TRACE_RC=$?"
for P in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_CVT SQ_INSTS_MFMA"; do
  N=$(echo $P | tr ' ' '_' | cut -c1-40)
  timeout -k 10 -s KILL 200 rocprofv3 --pmc $P --kernel-trace --output-format csv -d gpurun_out/prof_ba/pmc_$N -o run -- python3 scripts/ba_exp.py 256 384 512 3 > gpurun_out/prof_ba/pmc_$N.log 2>&1
  echo "BA PMC $N RC=$?"
done
