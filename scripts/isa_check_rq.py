#!/usr/bin/env python3
"""Build-time ISA check of rq_gemm_topk_kernel's hand-ordered K loop (csrc/retrieval.hip).

The kernel streams the codebook into a 3-slot register ring with inline-asm `global_load_dwordx4` and retires
those loads with its own `s_waitcnt vmcnt(4)`: the compiler cannot see that the ring registers are still in
flight, so correctness rests on no instruction touching a ring register before the wait that retires its load.
This script checks exactly that on the compiled gfx950 assembly (`hipcc --cuda-device-only -S`, the Makefile's
build/retrieval.s): it walks each instantiation from the kernel entry through the K loop in issue order, keeps
the queue of outstanding vector-memory operations (gfx9 `vmcnt` counts loads and stores in issue order;
`s_waitcnt vmcnt(N)` retires all but the N most recent), runs the loop body twice so the back edge's carried
loads are seen, and fails if any instruction reads or writes a VGPR whose load is still outstanding.
Straight-line issue order is assumed through the body's forward skips (every step taken), which is the
steady state of the loop.

usage: isa_check_rq.py build/retrieval.s   (exit 1 and a listing of the hazards on failure)
"""
import re
import sys

KERNEL_RE = re.compile(r"^(_ZN3m3s19rq_gemm_topk_kernel\w*):")
VREG_RE = re.compile(r"\bv(?:\[(\d+):(\d+)\]|(\d+)\b)")
VM_OPS = ("global_", "buffer_", "flat_", "scratch_")


def vregs(text):
    out = set()
    for a, b, c in VREG_RE.findall(text):
        if c:
            out.add(int(c))
        else:
            out.update(range(int(a), int(b) + 1))
    return out


def instructions(lines):
    for ln in lines:
        s = ln.split(";", 1)[0].strip()
        if not s or s.startswith(".") or s.endswith(":"):
            continue
        yield s


def check_kernel(name, body):
    """body: the kernel's lines. Returns a list of hazard strings."""
    try:
        head = next(i for i, l in enumerate(body) if "This Loop Header: Depth=1" in l)
    except StopIteration:
        return [f"{name}: K-loop header not found"]
    label = body[head].split(":", 1)[0]
    try:
        tail = next(i for i in range(head + 1, len(body)) if re.search(r"s_c?branch\w*\s+" + re.escape(label) + r"\b", body[i]))
    except StopIteration:
        return [f"{name}: K-loop back edge to {label} not found"]
    queue = []  # outstanding vector-memory ops in issue order: (dest vregs, text)
    hazards = []
    ring_loads = 0
    waits = 0

    def walk(lines, tag):
        nonlocal ring_loads, waits
        for ins in instructions(lines):
            op = ins.split(None, 1)[0]
            operands = ins[len(op):]
            if op == "s_waitcnt":
                m = re.search(r"vmcnt\((\d+)\)", operands)
                if m:
                    waits += tag == "body1"
                    n = int(m.group(1))
                    while len(queue) > n:
                        queue.pop(0)
                continue
            pending = set().union(*(d for d, _ in queue)) if queue else set()
            if op.startswith(VM_OPS):
                parts = [p.strip() for p in operands.split(",")]
                is_load = "load" in op and not op.startswith("global_load_lds") and not op.startswith("buffer_load_lds")
                dest = vregs(parts[0]) if is_load else set()
                srcs = vregs(",".join(parts[1:] if is_load else parts))
                if (srcs | dest) & pending:
                    hazards.append(f"{name} [{tag}]: '{ins}' touches in-flight VGPRs {sorted((srcs | dest) & pending)}")
                queue.append((dest, ins))
                if op == "global_load_dwordx4" and tag == "body1":
                    ring_loads += 1
                continue
            touched = vregs(operands)
            if touched & pending:
                hard = [t for d, t in queue if d & touched]
                hazards.append(f"{name} [{tag}]: '{ins}' touches in-flight VGPRs {sorted(touched & pending)} of {hard}")

    walk(body[:head], "prologue")
    walk(body[head:tail + 1], "body1")
    walk(body[head:tail + 1], "body2")  # the state carried across the back edge
    if ring_loads < 4 or waits < 1:
        hazards.append(f"{name}: unexpected K-loop shape ({ring_loads} dwordx4 loads, {waits} vmcnt waits)")
    return hazards


def check_file(path):
    with open(path) as f:
        lines = f.read().splitlines()
    kernels = []
    for i, l in enumerate(lines):
        m = KERNEL_RE.match(l)
        if m:
            end = next(j for j in range(i, len(lines)) if "s_endpgm" in lines[j])
            kernels.append((m.group(1), lines[i + 1:end]))
    if not kernels:
        return 0, [f"{path}: no rq_gemm_topk_kernel instantiation found"]
    hazards = []
    for name, body in kernels:
        hazards += check_kernel(name, body)
    return len(kernels), hazards


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else "lightweight-mast3r-slam_amd/csrc/build/retrieval.s"
    n, hazards = check_file(path)
    if hazards:
        print("\n".join(hazards[:40]))
        print(f"ISA check FAILED: {len(hazards)} hazard(s) in {n} rq_gemm_topk_kernel instantiation(s)")
        sys.exit(1)
    print(f"ISA check ok: {n} rq_gemm_topk_kernel instantiations, no VGPR touched while its load is in flight")


if __name__ == "__main__":
    main()
