#!/bin/bash
# round 4: grouped BA pack order (keyframe-i groups, chunk-major, XCD-contiguous) vs the plain grid-stride order:
# BA GPU tests, then two alternating bench pairs (BA legs: ms_pack, fresh-call edges/s)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v --timeout 400 --timeout-method thread tests/test_gpu_ba.py tests/test_gpu_configs.py tests/test_gpu_factor_graph.py > gpurun_out/r04ab_pytest.txt 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/r04ab_pytest.txt | tail -8; [ $rc -eq 0 ] || exit $rc
A="--steps 20 --warmup 5 --no-cpu --no-retrieval --no-store --no-peaks"
for r in 1 2; do
  for G in 0 1; do
    M3S_BA_PACK_GROUPED=$G timeout -k 10 400 python3 bench.py $A > gpurun_out/r04ab_g${G}_$r.json 2> gpurun_out/r04ab_g${G}_$r.err || { tail -20 gpurun_out/r04ab_g${G}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r04ab_g${G}_$r.json')); b=d['ba']; print('grouped=$G', 'C5 pack', round(b['ms_pack'],3), round(b['pack']['GBps']), b['ms_per_call'], round(b['edges_per_s']), 'C4 pack', round(b['c4']['ms_pack'],3), round(b['c4']['edges_per_s']), 'eth3d pack', round(b['eth3d']['ms_pack'],3), round(b['eth3d']['edges_per_s']))"
  done
done
