"""``import lietorch`` for the reference glue on ROCm (lietorch itself is CUDA-only and absent).

Exposes the lietorch-compatible ``Sim3`` of ``m3s.sim3`` — the group the tracking / BA path uses
(``tracker.py``, ``frame.py``, ``global_opt.py``, ``main.py``) — and ``SE3`` for the trajectory
export (``lietorch_utils.py:6-13``).
"""
from m3s.sim3 import SE3, Sim3, as_SE3  # noqa: F401

__all__ = ["Sim3", "SE3", "as_SE3"]
