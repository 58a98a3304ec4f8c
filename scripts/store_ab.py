"""A/B of the SharedKeyframes per-frame overhead (bench `store` leg): the tracker's one-hold slot read (slot_frame)
against the store's own __getitem__ inside the hold (slot_frame disabled), alternated. One JSON line per run."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    # spawn (the store's Manager) re-imports this file: everything runs under the __main__ guard
    sys.argv = [sys.argv[0], "--no-ba", "--no-cpu"]
    import bench
    import m3s.tracker as T

    args = bench.parse()
    keep = T.slot_frame
    res = []
    for rep in range(2):
        for variant in ("getitem", "slot_frame"):
            T.slot_frame = (lambda *a: None) if variant == "getitem" else keep
            r = bench.bench_store(args, "cuda")
            res.append({"variant": variant, "rep": rep, **r["median_ms"]})
            print(json.dumps(res[-1]), flush=True)


if __name__ == "__main__":
    main()
