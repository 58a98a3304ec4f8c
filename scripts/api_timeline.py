"""Merge a rocprofv3 kernel trace and HIP API trace into one host/device timeline window.
usage: python scripts/api_timeline.py <dir> [skip_kernels] [count_kernels]

Prints, in time order, each HIP API call (host thread, start offset, duration) and each kernel (device
start, duration), so the gaps between a frame's last kernel, the host's return from its sync and the next
frame's first launch can be read off directly."""
import csv
import glob
import sys

d = sys.argv[1]
skip = int(sys.argv[2]) if len(sys.argv) > 2 else 200
cnt = int(sys.argv[3]) if len(sys.argv) > 3 else 30
kf = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
af = glob.glob(f"{d}/**/*hip_api_trace.csv", recursive=True)[0]
ks = sorted(csv.DictReader(open(kf)), key=lambda r: int(r["Start_Timestamp"]))[skip:skip + cnt]
t0, t1 = int(ks[0]["Start_Timestamp"]), int(ks[-1]["End_Timestamp"])
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K", r["Kernel_Name"][:50]) for r in ks]
for r in csv.DictReader(open(af)):
    s = int(r["Start_Timestamp"])
    if t0 - 100000 <= s <= t1:
        name = r["Function"]
        if name in ("hipGetDevice", "hipGetLastError", "hipDeviceGetAttribute", "hipPeekAtLastError"):
            continue
        ev.append((s, int(r["End_Timestamp"]), "A", name[:50]))
ev.sort()
for s, e, kind, name in ev:
    ind = "" if kind == "A" else "                              "
    print(f"{(s - t0) / 1e3:9.2f} us {ind}{kind} {name:<50s} dur {(e - s) / 1e3:8.2f}  end {(e - t0) / 1e3:9.2f}")
