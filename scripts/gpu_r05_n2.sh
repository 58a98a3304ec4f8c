#!/bin/bash
# round 5: rehearsal of the N-rank bench on a 1-GPU box: 2 ranks on device 0 over gloo (the driver's multi-GPU runs use one
# GPU per rank over RCCL), every leg incl. the sharded BA with record reuse
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
M3S_BENCH_DEVICE=0 M3S_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29527 bench.py --gpus 2 --steps 50 --warmup 5 --no-cpu --no-retrieval --no-peaks --no-store \
  > gpurun_out/r05t_bench_n2.json 2> gpurun_out/r05t_bench_n2.err
rc=$?; echo "BENCH_N2_RC=$rc"; tail -5 gpurun_out/r05t_bench_n2.err; [ $rc -eq 0 ] || exit $rc
python3 -c "
import json; d=json.loads(open('gpurun_out/r05t_bench_n2.json').read().strip().splitlines()[-1])
print('n_gpus', d['n_gpus'], 'value', round(d['value']), 'config', d['config']['parallelism'])
b=d['ba']; print('C5', round(b['edges_per_s']), b['ms_per_call'], 'reuse', b['reuse']); print('C4', round(b['c4']['edges_per_s']), b['c4']['reuse'])
"
