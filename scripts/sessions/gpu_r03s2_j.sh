#!/bin/bash
# BA linearisation X + (D X + t) + calib-row FMAs (shipped): accuracy census, C5 / C4 time vs the quaternion build,
# then the BA GPU tests and the full-size batched match test
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 scripts/ba_acc.py 2>&1 | grep -vE "amdgpu.ids" | tail -3 || exit 1
for V in quat main quat main; do
  if [ "$V" = main ]; then L=lightweight-mast3r-slam_amd/lib/libm3s.so; else L=lightweight-mast3r-slam_amd/lib/exp/libm3s_$V.so; fi
  echo "== $V"
  M3S_LIB=$L timeout -k 10 200 python3 scripts/ba_exp.py 256 384 512 10 chess calib 2>&1 | grep -E "^rep 1|rror" || exit 1
  M3S_LIB=$L timeout -k 10 200 python3 scripts/ba_exp.py 256 320 512 10 euroc rays 2>&1 | grep -E "^rep 1|rror" || exit 1
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_configs.py tests/test_gpu_factor_graph.py -m gpu -v -s -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/ba_tests_mat.log 2>&1
rc=$?; echo "TESTS_RC=$rc"; grep -E "err|mismatch|passed|failed|FAIL" gpurun_out/ba_tests_mat.log | cut -c1-200 | tail -45; exit $rc
