#!/bin/bash
# round 5: BA linearisation chunk length (M3S_BA_CHUNK_POINTS; default 24576 = 48 rounds of 512 points per block, one
# fp32 run flush per block) against 32768 (64 rounds) and 49152 (96: two flushes), C5 / C4, alternating, twice
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
for CP in 24576 32768 49152; do
  echo "== chunk $CP C5" && M3S_BA_CHUNK_POINTS=$CP timeout -k 10 200 python3 scripts/ba_exp.py 256 384 512 10 chess calib 2>&1 | grep "rep 1" || exit 1
  echo "== chunk $CP C4" && M3S_BA_CHUNK_POINTS=$CP timeout -k 10 200 python3 scripts/ba_exp.py 256 320 512 10 euroc rays 2>&1 | grep "rep 1" || exit 1
done
done
