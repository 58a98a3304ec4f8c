"""Time m3s_quantize at the reference's retrieval shapes (64k x 1024 codebook, 300 features, k=5)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lightweight-mast3r-slam_amd"))
from m3s import _lib  # noqa: E402
from m3s.retrieval import Codebook  # noqa: E402

C, D, M, k = (int(x) for x in (sys.argv[1:5] if len(sys.argv) > 4 else (65536, 1024, 300, 5)))
reps = int(sys.argv[5]) if len(sys.argv) > 5 else 50
g = torch.Generator(device="cuda").manual_seed(0)
c = torch.nn.functional.normalize(torch.randn(C, D, device="cuda", generator=g), dim=1)
q = torch.nn.functional.normalize(torch.randn(M, D, device="cuda", generator=g), dim=1)
cb = Codebook(c)
for _ in range(5):
    cb.quantize(q, k)
torch.cuda.synchronize()
lib = _lib.load()
lib.m3s_timing_enable(1)
lib.m3s_timing_reset()
t0 = time.perf_counter()
for _ in range(reps):
    cb.quantize(q, k)
torch.cuda.synchronize()
el = (time.perf_counter() - t0) / reps
ms, cnt = _lib.c_double(), _lib.c_int()
lib.m3s_timing_query(b"quantize_topk", ms, cnt)
lib.m3s_timing_enable(0)
tk = ms.value / max(cnt.value, 1)
fl = 2.0 * M * C * D
print(f"quantize C={C} D={D} M={M} k={k}: wall {el * 1e3:.3f} ms/call, gemm+topk+merge {tk:.3f} ms "
      f"({fl / tk / 1e9:.0f} alg TFLOP/s, {3 * ((M + 303) // 304 * 304) * C * D * 2 / tk / 1e9:.0f} MFMA TFLOP/s, "
      f"{C * D * 4 / tk / 1e6:.0f} GB/s codebook)")
# torch fp32 reference formulation on the same device, for context
t0 = time.perf_counter()
for _ in range(reps):
    l2 = torch.sum(q ** 2, dim=1)[:, None] + torch.sum(c ** 2, dim=1)[None, :] - 2 * (q @ c.mT)
    torch.topk(l2, k, dim=1, largest=False)
torch.cuda.synchronize()
print(f"torch fp32 (reference formulation, hipBLASLt + topk): {(time.perf_counter() - t0) / reps * 1e3:.3f} ms/call")
