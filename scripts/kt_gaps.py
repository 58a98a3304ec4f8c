"""Median idle gap before each kernel of the tracking loop, from a rocprofv3 kernel trace (the gap before
prep_rays is the host's time between one frame's publish and the next frame's first launch).
usage: python scripts/kt_gaps.py <dir containing *_kernel_trace.csv> [skip]"""
import collections
import csv
import glob
import sys

import numpy as np

f = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
skip = int(sys.argv[2]) if len(sys.argv) > 2 else 100
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))[skip:]
gap, dur = collections.defaultdict(list), collections.defaultdict(list)
prev_end = None
for r in rows:
    name = r["Kernel_Name"]
    short = next((k for k in ("prep_rays", "proj_occlusion", "refine_tile", "refine_outlier", "track_setup",
                              "gn_loop", "fuse_kernel", "track_init") if k in name), name[:30])
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if prev_end is not None:
        gap[short].append((s - prev_end) / 1e3)
    dur[short].append((e - s) / 1e3)
    prev_end = e
tot_g = tot_d = 0.0
for k in dur:
    g = np.median(gap[k]) if gap[k] else 0.0
    d = np.median(dur[k])
    tot_g += g
    tot_d += d
    print(f"{k:16s} n={len(dur[k]):5d}  median duration {d:8.2f} us  median gap before {g:7.2f} us")
print(f"sum of medians: kernels {tot_d:.1f} us, gaps {tot_g:.1f} us")
