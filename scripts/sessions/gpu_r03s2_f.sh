#!/bin/bash
# dataflow back substitution without waits on parent-chain columns: A/B + BA tests, then the stamps build
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash scripts/gpu_r03s2_b.sh || exit $?
bash scripts/gpu_r03s2_c.sh
