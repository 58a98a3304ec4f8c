"""m3s — MI355X-native MASt3R-SLAM tracking hot path (host side over libm3s.so).

Modules: matching (fused dense matcher), tracker (FrameTracker), global_opt (FactorGraph),
dist_ba (edge-sharded multi-GPU BA), sim3 (lietorch-compatible Sim3), frame, config, synthetic.
The drop-in operator module is the sibling package ``mast3r_slam_backends``.
"""
import os
import sys

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if PKG_ROOT not in sys.path:
    sys.path.insert(0, PKG_ROOT)

__version__ = "0.1.0"
