#!/bin/bash
# Round-6 BA profiles: the three BA legs' kernel traces and PMC passes (the loop of scripts/ba_exp.py), summarised by
# profile_summary.py into gpurun_out/summ (TAG r06_ba, r06_ba_c4, r06_ba_eth3d).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r06}
export TMPDIR=/tmp
mkdir -p gpurun_out/summ
for LEG in c5 c4 eth3d; do
  if [ $LEG = c5 ]; then BA="python3 scripts/ba_exp.py 256 384 512 3 chess calib"; D=gpurun_out/prof_ba; T=${TAG}_ba;
  elif [ $LEG = c4 ]; then BA="python3 scripts/ba_exp.py 256 320 512 3 euroc rays"; D=gpurun_out/prof_ba_c4; T=${TAG}_ba_c4;
  else BA="python3 scripts/ba_exp.py 256 304 512 3 chess calib"; D=gpurun_out/prof_ba_eth3d; T=${TAG}_ba_eth3d; fi
  rm -rf $D; mkdir -p $D
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- $BA > $D/trace.log 2>&1
  rc=$?; echo "BA_${LEG}_TRACE_RC=$rc"; [ $rc -eq 0 ] || { tail -20 $D/trace.log; exit $rc; }
  for P in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"; do
    N=$(echo $P | tr ' ' '_' | cut -c1-40)
    timeout -k 10 -s KILL 200 rocprofv3 --pmc $P --kernel-include-regex m3s --kernel-trace --output-format csv -d $D/pmc_$N -o run -- $BA > $D/pmc_$N.log 2>&1
    rc=$?; echo "BA_${LEG} PMC $N RC=$rc"; [ $rc -eq 0 ] || { tail -20 $D/pmc_$N.log; exit $rc; }
  done
  grep "sha1" $D/trace.log | tail -1
  PROF_OUT=gpurun_out/summ python3 scripts/profile_summary.py $D $T || exit $?
  find $D -name "run_kernel_trace.csv" -delete
  find $D -name "run_counter_collection.csv" -size +4M -delete
done
du -sh gpurun_out
