"""CPU: the build-time ISA check of the retrieval GEMM's hand-retired codebook ring (scripts/isa_check_rq.py).

The checker itself is exercised on small hand-written loops (a correct two-deep ring, a ring read one wait too
early, a ring register clobbered in flight); the real gfx950 assembly that `make` emits is checked when present."""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "scripts"))
import isa_check_rq as C  # noqa: E402

HEAD = "_ZN3m3s19rq_gemm_topk_kernelILi5EEEvPK15HIP_vector_typeIjLj4EEPKfS4_S6_iPy:"


def _kernel(loop_body, prologue=None):
    prologue = prologue or [
        "global_load_dwordx4 v[10:13], v[2:3], off",
        "global_load_dwordx4 v[20:23], v[2:3], off",
        "s_waitcnt vmcnt(0)",
    ]
    lines = [HEAD] + ["\t" + p for p in prologue]
    lines += [".LBB1_4:                                ; =>This Loop Header: Depth=1"]
    lines += ["\t" + b for b in loop_body] + ["\ts_branch .LBB1_4", "\ts_endpgm"]
    return lines


def _ring(wait):
    """3-slot ring, 2 steps ahead, 4 loads per step as in rq_gemm_topk_kernel (one load per slot here)."""
    body = []
    slots = ["v[10:13]", "v[20:23]", "v[30:33]"]
    for s in range(6):  # the 6-step unrolled body (lcm of 3 slots and 2 LDS images)
        cur, nxt = slots[s % 3], slots[(s + 2) % 3]
        body += ["global_load_lds_dwordx4 v[4:5], off", f"global_load_dwordx4 {nxt}, v[2:3], off"]
        body += ["global_store_dword v[2:3], v41, off"] * 3  # pad: 4 vm ops after the ring load per step
        body += [f"v_mfma_f32_16x16x32_bf16 v[60:63], {cur}, v[50:53], v[60:63]", f"s_waitcnt vmcnt({wait}) lgkmcnt(0)"]
    return body


def _check(lines):
    name = HEAD[:-1]
    return C.check_kernel(name, lines[1:-1])


def test_correct_ring_passes():
    assert _check(_kernel(_ring(4))) == []


def test_ring_read_before_its_wait_is_flagged():
    hz = _check(_kernel(_ring(9)))  # keeps the previous step's load in flight into the next step
    assert hz and all("touches in-flight VGPRs" in h for h in hz)


def test_ring_register_clobbered_in_flight_is_flagged():
    body = _ring(4)
    body.insert(2, "v_mov_b32_e32 v30, 0")  # writes the slot its own step just started loading
    assert any("v_mov_b32_e32 v30, 0" in h for h in _check(_kernel(body)))


def test_missing_loop_is_reported():
    lines = [HEAD, "\ts_endpgm"]
    assert _check(lines) == [f"{HEAD[:-1]}: K-loop header not found"]


def test_built_retrieval_assembly_has_no_ring_hazard():
    path = os.path.join(REPO, "lightweight-mast3r-slam_amd", "csrc", "build", "retrieval.s")
    if not os.path.exists(path):
        pytest.skip("build/retrieval.s not built (make -C lightweight-mast3r-slam_amd/csrc emits it)")
    n, hazards = C.check_file(path)
    assert n == 8 and hazards == [], hazards[:5]
