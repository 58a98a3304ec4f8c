"""Print a kernel timeline window (start offset, duration, gap before) from a rocprofv3 kernel trace.
usage: python scripts/kt_timeline.py <dir> [skip] [count]"""
import csv
import glob
import sys

f = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
skip = int(sys.argv[2]) if len(sys.argv) > 2 else 200
cnt = int(sys.argv[3]) if len(sys.argv) > 3 else 30
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))[skip:skip + cnt]
t0 = int(rows[0]["Start_Timestamp"])
prev = None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev is not None else 0.0
    print(f"{(s - t0) / 1e3:9.2f} us  dur {(e - s) / 1e3:8.2f}  gap {gap:7.2f}  {r['Kernel_Name'][:60]}")
    prev = e
