#!/bin/bash
# round 4: the round's profiles (kernel traces + PMC passes of the tracking bench and the three BA legs, stamps)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=r04 timeout -k 10 1100 bash scripts/gpu_prof_round.sh
