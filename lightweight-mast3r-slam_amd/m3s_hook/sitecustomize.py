"""Start-up hook: with this directory (and lightweight-mast3r-slam_amd/) on PYTHONPATH, the reference's unchanged
main.py builds the fused MI355X FrameTracker / FactorGraph (m3s/hook.py). Chains to the next sitecustomize."""
import importlib.util
import os
import sys

_here = os.path.dirname(os.path.abspath(__file__))
_pkg = os.path.dirname(_here)
if _pkg not in sys.path:
    sys.path.insert(0, _pkg)
try:
    from m3s import hook as _hook

    _hook.install()
except Exception as _e:  # never break interpreter start-up
    print(f"m3s_hook: not installed ({_e})", file=sys.stderr)

# the site module imports only the first sitecustomize on sys.path: run the next one too
for _p in sys.path:
    _f = os.path.join(_p, "sitecustomize.py")
    if _p and os.path.abspath(_p) != _here and os.path.isfile(_f):
        _spec = importlib.util.spec_from_file_location("_next_sitecustomize", _f)
        _spec.loader.exec_module(importlib.util.module_from_spec(_spec))
        break
