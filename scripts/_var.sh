set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -m pytest tests/test_gpu_matching.py tests/test_gpu_tracking.py -q -x -p no:cacheprovider 2>&1 | tail -2 || exit 1
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu --no-ba 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['kernels_us'])"
