"""Run the reference's ``main.py`` UNCHANGED on the fused MI355X tracker and factor graph.

``lightweight-mast3r-slam_amd/m3s_hook/sitecustomize.py`` calls :func:`install` at interpreter start-up in every
process that has that directory on ``PYTHONPATH`` (the frontend and, through ``PYTHONPATH`` inheritance, the
spawned backend process of ``main.py``):

* when ``mast3r_slam.tracker`` / ``mast3r_slam.global_opt`` finish importing, their ``FrameTracker`` /
  ``FactorGraph`` are replaced by ``m3s.tracker.FrameTracker`` / ``m3s.global_opt.FactorGraph`` (same
  constructors, methods and returns), so ``from mast3r_slam.tracker import FrameTracker`` in ``main.py:29`` (and
  ``:17``) binds the fused classes;
* ``mast3r_slam.config.config`` becomes ``m3s.config.config`` (one dict, which the reference's ``load_config``
  updates in place: ``config.py:41-44``), so the fused classes read the YAML the run was started with.

Nothing of the reference is copied or edited; without the hook directory on the path nothing changes.
"""
import importlib
import importlib.abc
import sys

PATCHES = {"mast3r_slam.config": ("config", "m3s.config"),
           "mast3r_slam.tracker": ("FrameTracker", "m3s.tracker"),
           "mast3r_slam.global_opt": ("FactorGraph", "m3s.global_opt")}


class _PatchingFinder(importlib.abc.MetaPathFinder):
    def find_spec(self, name, path, target=None):
        if name not in PATCHES:
            return None
        for finder in sys.meta_path:
            if finder is self or not hasattr(finder, "find_spec"):
                continue
            spec = finder.find_spec(name, path, target)
            if spec is not None:
                break
        else:
            return None
        attr, src = PATCHES[name]
        loader = spec.loader
        orig_exec = loader.exec_module

        class _Loader(importlib.abc.Loader):
            def create_module(self, spec_):
                return loader.create_module(spec_)

            def exec_module(self, module):
                orig_exec(module)
                setattr(module, attr, getattr(importlib.import_module(src), attr))
                setattr(module, "_m3s_original_" + attr, True)

        spec.loader = _Loader()
        return spec


def install():
    """Idempotent: put the patching finder first on sys.meta_path."""
    if not any(isinstance(f, _PatchingFinder) for f in sys.meta_path):
        sys.meta_path.insert(0, _PatchingFinder())
