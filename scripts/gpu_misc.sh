#!/bin/bash
# Tracking parity tests + a short tracking bench, then the N=2 bench path rehearsed on one GPU (gloo).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_matching.py tests/test_gpu_tracking.py tests/test_gpu_configs.py -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/track_tests.log 2>&1
rc=$?; echo "TRACK_TESTS_RC=$rc"; tail -3 gpurun_out/track_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu --no-ba --no-peaks --no-retrieval > gpurun_out/bench_track.json 2> gpurun_out/bench_track.err
rc=$?; echo "BENCH_RC=$rc"; [ $rc -eq 0 ] || exit $rc
python3 -c "import json;d=json.loads(open('gpurun_out/bench_track.json').read().strip().splitlines()[-1]);print(d['value'],d['kernels_us'],d['frame']['median_ms'])"
M3S_BENCH_DEVICE=0 M3S_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 50 --warmup 5 --no-cpu > gpurun_out/bench_n2.json 2> gpurun_out/bench_n2.err
rc=$?; echo "N2_RC=$rc"; tail -3 gpurun_out/bench_n2.err
python3 -c "import json;d=json.loads(open('gpurun_out/bench_n2.json').read().strip().splitlines()[-1]);print(d['value'],d['n_gpus'],d['ba']['edges_per_s'],d['ba']['n_gpus'],d['ba']['c4']['edges_per_s'])"
