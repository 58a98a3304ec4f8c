#!/bin/bash
# round 5 experiment: wide factor steps + one-workgroup kernel pinned to XCD 0 (M3S_BA_XCD0=1) vs spread
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
for X in 0 1; do
  echo "== XCD0=$X C5" && M3S_BA_XCD0=$X timeout -k 10 200 python3 scripts/ba_exp.py 256 384 512 10 chess calib 2>&1 | grep "rep 1" || exit 1
  echo "== XCD0=$X C4" && M3S_BA_XCD0=$X timeout -k 10 200 python3 scripts/ba_exp.py 256 320 512 10 euroc rays 2>&1 | grep "rep 1" || exit 1
done
done
