"""``import lietorch`` for the reference glue on ROCm (lietorch itself is CUDA-only and absent).

Exposes the lietorch-compatible ``Sim3`` of ``m3s.sim3`` — the group the tracking / BA path uses
(``tracker.py``, ``frame.py``, ``global_opt.py``, ``main.py``). ``SE3`` appears only in the
trajectory export (``lietorch_utils.py:7-12``, evaluation — out of scope) and is not provided.
"""
from m3s.sim3 import Sim3  # noqa: F401

__all__ = ["Sim3"]
