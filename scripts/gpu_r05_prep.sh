#!/bin/bash
# round 5: prep_rays and fuse_kernel with their loads issued up front ("new") against the previous build ("head",
# lib/ab): matching + tracking GPU tests on new, the tracking bench kernel spans alternating (3 reps), then the
# SharedKeyframes store A/B (scripts/store_ab.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_matching.py tests/test_gpu_tracking.py > gpurun_out/r05p_tests.txt 2>&1 || { tail -30 gpurun_out/r05p_tests.txt; exit 1; }
tail -2 gpurun_out/r05p_tests.txt
for rep in 1 2 3; do
for V in new head; do
  if [ "$V" = new ]; then L=lightweight-mast3r-slam_amd/lib/libm3s.so; else L=lightweight-mast3r-slam_amd/lib/ab/libm3s_$V.so; fi
  M3S_LIB=$L timeout -k 10 300 python3 bench.py --steps 100 --warmup 10 --no-ba --no-cpu --no-retrieval --no-store --no-peaks > gpurun_out/r05p_bench_$V.json 2> gpurun_out/r05p_bench_$V.err || { tail -20 gpurun_out/r05p_bench_$V.err; exit 1; }
  python3 - "$V" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/r05p_bench_{sys.argv[1]}.json").read().strip().splitlines()[-1])
print(sys.argv[1], round(d["value"], 1), d["kernels_us"])
PY
done
done
timeout -k 10 300 python -u scripts/store_ab.py > gpurun_out/r05_store_ab.txt 2>&1 || { tail -30 gpurun_out/r05_store_ab.txt; exit 1; }
cat gpurun_out/r05_store_ab.txt
