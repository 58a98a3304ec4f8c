#!/bin/bash
# round 5: supernodal BA solver — parity tests, then per-iteration solve time vs the column-task solver (C5, C4)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ba_snode.py -q -s --timeout 250 --timeout-method thread > gpurun_out/r05c_snode_test.txt 2>&1
rc=$?
echo "PYTEST_RC=$rc" >> gpurun_out/r05c_snode_test.txt
if [ $rc -gt 1 ]; then exit $rc; fi
for S in sparse snode; do
  echo "== $S C5" && M3S_BA_SOLVER=$S timeout -k 10 200 python3 scripts/ba_exp.py 256 384 512 10 chess calib || exit 1
  echo "== $S C4" && M3S_BA_SOLVER=$S timeout -k 10 200 python3 scripts/ba_exp.py 256 320 512 10 euroc rays || exit 1
done
