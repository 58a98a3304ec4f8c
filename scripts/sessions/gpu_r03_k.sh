#!/bin/bash
# BA solve: the wide-step split by task-count threshold (M3S_BA_WIDE=t: every step up to the last one with more
# than t tasks launches multi-workgroup) against the cost model's own choice (unset)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for T in model 4 8 12 16 24 32; do
  echo "== wide threshold $T"
  if [ $T = model ]; then unset M3S_BA_WIDE; else export M3S_BA_WIDE=$T; fi
  timeout -k 10 200 python3 scripts/ba_exp.py 256 384 512 10 chess calib 2>&1 | grep -E "rep 1|wide" || exit 1
  timeout -k 10 200 python3 scripts/ba_exp.py 256 320 512 10 euroc rays 2>&1 | grep -E "rep 1|wide" || exit 1
done
