#!/bin/bash
# Round-end evidence of this session: smoke + GPU suite + default bench + rocprofv3 stats/PMC (gpu_final.sh), then
# the 2-rank rehearsal (gloo on one GPU)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=r03 bash scripts/gpu_final.sh || exit $?
bash scripts/gpu_r03_o.sh > gpurun_out/n2_rehearsal.txt 2>&1; echo "N2_RC=$?"; tail -4 gpurun_out/n2_rehearsal.txt
