#!/bin/bash
# BA linearisation A/B across libm3s variants (lib/exp, built by build_variant.sh): the 6-KF fixture and
# medium-graph accuracy tests (max |T - T64| printed), then C5 / C4-shaped per-iteration times.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
VARIANTS="${VARIANTS:-main}" bash scripts/gpu_ba_fixture_ab.sh || exit $?
for V in ${VARIANTS:-main}; do
  if [ "$V" = main ]; then L=lightweight-mast3r-slam_amd/lib/libm3s.so; else L=lightweight-mast3r-slam_amd/lib/exp/libm3s_$V.so; fi
  echo "== $V timing"
  M3S_LIB=$L timeout -k 10 200 python3 scripts/ba_exp.py 256 384 512 10 chess calib 2>&1 | grep "rep 1" || exit 1
  M3S_LIB=$L timeout -k 10 200 python3 scripts/ba_exp.py 256 320 512 10 euroc rays 2>&1 | grep "rep 1" || exit 1
done
