"""Summarise a rocprofv3 kernel trace: per-kernel count / mean / total duration and the mean gap
between consecutive kernels. usage: python scripts/kt_summary.py <dir containing *_kernel_trace.csv> [filter]"""
import collections
import csv
import glob
import sys

f = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
d = collections.defaultdict(list)
gaps = []
prev_end = None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if flt in r["Kernel_Name"]:
        d[r["Kernel_Name"][:70]].append((e - s) / 1e3)
        if prev_end is not None and s - prev_end < 100000:
            gaps.append((s - prev_end) / 1e3)
        prev_end = e
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    print(f"{k:70s} n={len(v):6d} mean={sum(v) / len(v):8.2f} us  total={sum(v) / 1e3:8.2f} ms  max={max(v):8.2f}")
if gaps:
    print(f"gaps between consecutive kernels: n={len(gaps)} mean={sum(gaps) / len(gaps):.2f} us")
