#!/bin/bash
# round 5: proj_occlusion LM loop with select-based accept / reject and 32-bit gather offsets ("new"), the same
# without SLP vectorisation of matching.hip ("noslp"), and the previous build ("head"): matching + refine GPU tests
# on new and noslp, the new ragged-tile BA pack test, then the tracking bench's kernel spans, alternating, 3 reps
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_matching.py tests/test_gpu_tracking.py "tests/test_gpu_ba.py::test_pack_tiles_with_ragged_last_tile" > gpurun_out/r05s_tests.txt 2>&1 || { tail -30 gpurun_out/r05s_tests.txt; exit 1; }
tail -2 gpurun_out/r05s_tests.txt
M3S_LIB=lightweight-mast3r-slam_amd/lib/ab/libm3s_noslp.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_matching.py > gpurun_out/r05s_tests_noslp.txt 2>&1 || { tail -30 gpurun_out/r05s_tests_noslp.txt; exit 1; }
tail -2 gpurun_out/r05s_tests_noslp.txt
for rep in 1 2 3; do
for V in new head noslp; do
  if [ "$V" = new ]; then L=lightweight-mast3r-slam_amd/lib/libm3s.so; else L=lightweight-mast3r-slam_amd/lib/ab/libm3s_$V.so; fi
  M3S_LIB=$L timeout -k 10 300 python3 bench.py --steps 100 --warmup 10 --no-ba --no-cpu --no-retrieval --no-store --no-peaks > gpurun_out/r05s_bench_$V.json 2> gpurun_out/r05s_bench_$V.err || { tail -20 gpurun_out/r05s_bench_$V.err; exit 1; }
  python3 - "$V" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/r05s_bench_{sys.argv[1]}.json").read().strip().splitlines()[-1])
print(sys.argv[1], round(d["value"], 1), d["kernels_us"], d.get("configs"))
PY
done
done
