"""Build-time check (csrc/Makefile): the named kernels of a gfx950 assembly file spill no VGPR.

usage: python3 isa_check_spills.py <file.s> <kernel substring> [...]
Every kernel whose symbol contains one of the substrings must report `.vgpr_spill_count: 0` in the AMDGPU metadata
(refine_tile_kernel spilled 19 VGPRs, 80 B of scratch per lane). Exit 1 names the offenders."""
import re
import sys


def main():
    path, names = sys.argv[1], sys.argv[2:]
    text = open(path).read()
    # metadata entries: "- .args: ... .name: <sym> ... .vgpr_spill_count: N" per kernel (order-independent search)
    found, bad = 0, []
    for block in re.split(r"\n\s+- \.", text):
        m = re.search(r"\.name:\s+(\S+)", block)
        sp = re.search(r"\.vgpr_spill_count:\s+(\d+)", block)
        if not m or not sp or not any(n in m.group(1) for n in names):
            continue
        found += 1
        if int(sp.group(1)) != 0:
            bad.append(f"{m.group(1)}: {sp.group(1)} spilled VGPRs")
    if found == 0:
        print(f"isa_check_spills: no kernel matching {names} in {path}")
        return 1
    if bad:
        print("isa_check_spills: VGPR spills\n  " + "\n  ".join(bad))
        return 1
    print(f"ISA check ok: {found} kernels matching {names}, no VGPR spills")
    return 0


if __name__ == "__main__":
    sys.exit(main())
