#!/bin/bash
# round 5: the dense top phase of the BA factorisation (M3S_BA_TOP=t): GPU tests, then the C5 / C4 solve time per
# iteration (scripts/ba_exp.py spans) without it and at t = 8, 16, 25, alternating, twice
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ba_top.py tests/test_gpu_ba.py > gpurun_out/r05u_tests.txt 2>&1 || { tail -40 gpurun_out/r05u_tests.txt; exit 1; }
grep -E "top|passed|failed" gpurun_out/r05u_tests.txt | tail -12
for rep in 1 2; do
for TOP in 0 8 16 25; do
  echo "== top $TOP C5" && M3S_BA_TOP=$TOP timeout -k 10 200 python3 scripts/ba_exp.py 256 384 512 10 chess calib 2>&1 | grep "rep 1" || exit 1
  echo "== top $TOP C4" && M3S_BA_TOP=$TOP timeout -k 10 200 python3 scripts/ba_exp.py 256 320 512 10 euroc rays 2>&1 | grep "rep 1" || exit 1
done
done
