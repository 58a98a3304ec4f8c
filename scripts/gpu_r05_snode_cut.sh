#!/bin/bash
# round 5: supernodal solve time vs the supernodal cut (C5): 0 = one workgroup does everything
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for C in 0 1 2 3 4 6 8; do
  echo "== cut $C" && M3S_BA_SOLVER=snode M3S_BA_SN_CUT=$C timeout -k 10 200 python3 scripts/ba_exp.py 256 384 512 10 chess calib 2>&1 | grep "rep 1" || exit 1
done
