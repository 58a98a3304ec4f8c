"""Summarise rocprofv3 counter-collection CSVs: mean counter value and mean duration per kernel."""
import collections
import csv
import glob
import sys

root = sys.argv[1]
for f in sorted(glob.glob(f"{root}/**/run_counter_collection.csv", recursive=True)):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"][:48]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print("==", f)
    for k, v in agg.items():
        if "m3s" not in k:
            continue
        print(" ", k, {c: round(sum(x) / len(x), 1) for c, x in v.items()})
for f in sorted(glob.glob(f"{root}/**/run_kernel_trace.csv", recursive=True))[:1]:
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        d[r["Kernel_Name"][:48]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print("== durations (us, profiled)", f)
    for k, v in d.items():
        if "m3s" in k:
            print(" ", k, round(sum(v) / len(v), 1), len(v))
