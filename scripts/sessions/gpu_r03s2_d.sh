#!/bin/bash
# BA dataflow: split between launched wide steps and the one-workgroup part (M3S_BA_WIDE=t: launch every step up to
# the last one with more than t tasks; unset = the cost model), C5 and C4 solve time and pose hash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for T in default 1000 64 40 24 16; do
  echo "== wide threshold $T"
  if [ "$T" = default ]; then unset M3S_BA_WIDE; else export M3S_BA_WIDE=$T; fi
  timeout -k 10 200 python3 scripts/ba_exp.py 256 384 512 10 chess calib 2>&1 | grep -E "^rep 1|rror" || exit 1
  timeout -k 10 200 python3 scripts/ba_exp.py 256 320 512 10 euroc rays 2>&1 | grep -E "^rep 1|rror" || exit 1
done
