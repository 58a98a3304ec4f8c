#!/bin/bash
# round 5 BA pack / linearisation A/B: BA GPU tests on the new library, then the bench BA legs (ms_pack,
# ms_lin_per_iter, ms_per_call) for each variant library under lightweight-mast3r-slam_amd/lib/ab, twice
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ba.py > gpurun_out/r05p_tests.txt 2>&1 || { tail -30 gpurun_out/r05p_tests.txt; exit 1; }
tail -3 gpurun_out/r05p_tests.txt
for rep in 1 2; do
for V in new head tiled2 tiled8k; do
  if [ "$V" = new ]; then L=lightweight-mast3r-slam_amd/lib/libm3s.so; else L=lightweight-mast3r-slam_amd/lib/ab/libm3s_$V.so; fi
  M3S_LIB=$L timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu --no-retrieval --no-store --no-peaks --no-kernel-timing > gpurun_out/r05p_bench_$V.json 2> gpurun_out/r05p_bench_$V.err || { tail -20 gpurun_out/r05p_bench_$V.err; exit 1; }
  python3 - "$V" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/r05p_bench_{sys.argv[1]}.json").read().strip().splitlines()[-1])
b = d["ba"]
print(sys.argv[1], {k: (round(v["ms_pack"], 3), round(v["ms_lin_per_iter"], 3), round(v["ms_per_call"], 2)) for k, v in (("c5", b), ("c4", b["c4"]), ("eth3d", b["eth3d"]))})
PY
done
done
