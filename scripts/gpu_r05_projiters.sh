#!/bin/bash
# proj_occlusion time vs LM iterations, windowed and global-gather kernels (scripts/proj_iters_exp.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u scripts/proj_iters_exp.py > gpurun_out/r05_proj_iters.txt 2>&1; rc=$?; cat gpurun_out/r05_proj_iters.txt; exit $rc
