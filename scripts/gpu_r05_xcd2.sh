#!/bin/bash
# round 5: XCD-0 affinity of the BA solve (assembly + wide steps + one-workgroup kernel) — BA tests, then A/B timing
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_configs.py tests/test_gpu_factor_graph.py -m gpu -q --timeout 250 --timeout-method thread > gpurun_out/r05h_tests.txt 2>&1
rc=$?; echo "PYTEST_RC=$rc" >> gpurun_out/r05h_tests.txt; if [ $rc -gt 1 ]; then exit $rc; fi
for rep in 1 2; do
for X in 0 1; do
  echo "== XCD0=$X C5" && M3S_BA_XCD0=$X timeout -k 10 200 python3 scripts/ba_exp.py 256 384 512 10 chess calib 2>&1 | grep "rep 1" || exit 1
  echo "== XCD0=$X C4" && M3S_BA_XCD0=$X timeout -k 10 200 python3 scripts/ba_exp.py 256 320 512 10 euroc rays 2>&1 | grep "rep 1" || exit 1
done
done
