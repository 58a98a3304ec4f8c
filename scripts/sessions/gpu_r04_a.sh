#!/bin/bash
# round 4: screened refine — parity (screen vs exact, oracle) then tracking-bench A/B (screen off / on)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_refine_screen.py tests/test_gpu_matching.py > gpurun_out/r04a_pytest.txt 2>&1
rc=$?; tail -30 gpurun_out/r04a_pytest.txt; [ $rc -eq 0 ] || exit $rc
for s in 0 1 0 1; do
  M3S_REFINE_SCREEN=$s timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-ba --no-cpu --no-retrieval --no-peaks > gpurun_out/r04a_bench_s$s.json 2> gpurun_out/r04a_bench_s$s.err || exit 1
  python - <<PY
import json; d=json.load(open("gpurun_out/r04a_bench_s$s.json"))
print("screen=$s", d["value"], d["ms_per_step"], {k: round(v,1) for k,v in d.get("kernels_us",{}).items()})
PY
done
