#!/bin/bash
# round 5: refine without spills (straight-line levels) — matching/refine parity, then A/B refine time vs the old build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_matching.py tests/test_gpu_refine_screen.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r05f_tests.txt 2>&1
rc=$?; echo "PYTEST_RC=$rc" >> gpurun_out/r05f_tests.txt; if [ $rc -gt 1 ]; then exit $rc; fi
for rep in 1 2 3; do
  for L in lightweight-mast3r-slam_amd/lib/ab/libm3s_refold.so lightweight-mast3r-slam_amd/lib/libm3s.so; do
    echo "== $L" && M3S_LIB=$L timeout -k 10 120 python3 scripts/refine_exp.py 2>&1 | tail -4 || exit 1
  done
done
