#!/bin/bash
# Round profile evidence on one GPU box, kept under gpurun_out/ (<64 MiB): rocprofv3 kernel-trace stats and
# separate PMC passes of the tracking bench (gpu_prof.sh) and of the C5 BA loop (chess, calib, K=256),
# summarised on the box by profile_summary.py into gpurun_out/summ/ (copied into profiles/ afterwards).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r04}
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_ba gpurun_out/summ
# keep the copy-back small whatever happens: the per-dispatch traces are summarised on the box
cleanup() {
  find gpurun_out/prof gpurun_out/prof_ba gpurun_out/prof_ba_c4 gpurun_out/prof_ba_eth3d -name "run_kernel_trace.csv" -delete 2>/dev/null
  find gpurun_out/prof gpurun_out/prof_ba gpurun_out/prof_ba_c4 gpurun_out/prof_ba_eth3d -name "run_counter_collection.csv" -size +4M -delete 2>/dev/null
  du -sh gpurun_out
}
trap cleanup EXIT
ARGS="--steps 20 --warmup 5 --no-cpu --no-ba --no-peaks --no-retrieval --no-store" bash scripts/gpu_prof.sh || exit $?
PROF_OUT=gpurun_out/summ python3 scripts/profile_summary.py gpurun_out/prof $TAG || exit $?
# the two BA legs of the bench, each with its own trace and PMC passes: C5 (chess, calib, 384x512) and C4
# (EuRoC MH_02, rays, 320x512), K = 256
for LEG in c5 c4 eth3d; do
  if [ $LEG = c5 ]; then BA="python3 scripts/ba_exp.py 256 384 512 3 chess calib"; D=gpurun_out/prof_ba; T=${TAG}_ba;
  elif [ $LEG = c4 ]; then BA="python3 scripts/ba_exp.py 256 320 512 3 euroc rays"; D=gpurun_out/prof_ba_c4; T=${TAG}_ba_c4;
  else BA="python3 scripts/ba_exp.py 256 304 512 3 chess calib"; D=gpurun_out/prof_ba_eth3d; T=${TAG}_ba_eth3d; fi
  mkdir -p $D
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- $BA > $D/trace.log 2>&1
  rc=$?; echo "BA_${LEG}_TRACE_RC=$rc"; [ $rc -eq 0 ] || { tail -20 $D/trace.log; exit $rc; }
  for P in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"; do
    N=$(echo $P | tr ' ' '_' | cut -c1-40)
    timeout -k 10 -s KILL 200 rocprofv3 --pmc $P --kernel-include-regex m3s --kernel-trace --output-format csv -d $D/pmc_$N -o run -- $BA > $D/pmc_$N.log 2>&1
    rc=$?; echo "BA_${LEG} PMC $N RC=$rc"; [ $rc -eq 0 ] || { tail -20 $D/pmc_$N.log; exit $rc; }
  done
  PROF_OUT=gpurun_out/summ python3 scripts/profile_summary.py $D $T || exit $?
done
# factor-kernel phase stamps (M3S_SP_STAMPS variant built by build_variant.sh spst), not profiled
if [ -f lightweight-mast3r-slam_amd/lib/exp/libm3s_spst.so ]; then
  M3S_LIB=lightweight-mast3r-slam_amd/lib/exp/libm3s_spst.so timeout -k 10 200 python3 scripts/ba_exp.py 256 384 512 3 chess calib > gpurun_out/summ/sp_stamps.log 2>&1
  echo "SP_STAMPS_RC=$?"; tail -4 gpurun_out/summ/sp_stamps.log
fi
exit 0
