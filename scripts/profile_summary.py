"""Turn a gpu_prof.sh run (gpurun_out/prof) into the committed round summaries under profiles/.

Writes  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (bench.py command)
        profiles/<tag>_pmc.json           per-kernel HBM traffic per launch from FETCH_SIZE / WRITE_SIZE,
                                          corrected as MI355X_MICROARCH.md §HBM prescribes (FETCH_SIZE
                                          is reported in KiB and counts half of a 16-B/lane streaming
                                          read on gfx950: x2; WRITE_SIZE exact), plus the other counters
        profiles/<tag>_pmc_summary.txt    human-readable counter means and profiled durations
usage: python scripts/profile_summary.py gpurun_out/prof r01
"""
import collections
import csv
import glob
import json
import os
import shutil
import subprocess
import sys

src, tag = sys.argv[1], sys.argv[2]
repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
out = os.environ.get("PROF_OUT", os.path.join(repo, "profiles"))
os.makedirs(out, exist_ok=True)
shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(out, f"{tag}_kernel_stats.csv"))

counters = collections.defaultdict(lambda: collections.defaultdict(list))
durations = collections.defaultdict(list)
for f in glob.glob(f"{src}/pmc_*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        counters[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_trace.csv"))):
    durations[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)

res = {}
for k, cs in counters.items():
    if "m3s" not in k:
        continue
    mean = {c: sum(v) / len(v) for c, v in cs.items()}
    fetch = 2.0 * mean.get("FETCH_SIZE", 0.0) * 1024.0
    write = mean.get("WRITE_SIZE", 0.0) * 1024.0
    d = durations.get(k, [])
    res[k] = {"hbm_read_bytes": fetch, "hbm_write_bytes": write, "traffic_bytes": fetch + write,
              "avg_duration_us": 1e6 * sum(d) / len(d) if d else None, "launches": len(d),
              "counters": mean}
json.dump(res, open(os.path.join(out, f"{tag}_pmc.json"), "w"), indent=1)
txt = subprocess.run([sys.executable, os.path.join(repo, "scripts", "pmc_summary.py"), src], capture_output=True,
                     text=True).stdout
open(os.path.join(out, f"{tag}_pmc_summary.txt"), "w").write(txt)
for k, v in res.items():
    print(f"{k[:60]:60s} traffic {v['traffic_bytes'] / 1e6:8.2f} MB  {v['avg_duration_us'] or 0:8.1f} us")
