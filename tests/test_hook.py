"""The start-up hook that lets the reference's unchanged main.py build the fused tracker / factor graph
(m3s/hook.py, m3s_hook/sitecustomize.py), on a stand-in `mast3r_slam` package (host test, no GPU)."""
import os
import subprocess
import sys
import textwrap

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "lightweight-mast3r-slam_amd")


def test_hook_swaps_classes_and_shares_config(tmp_path):
    ref = tmp_path / "ref" / "mast3r_slam"
    ref.mkdir(parents=True)
    (ref / "__init__.py").write_text("")
    (ref / "config.py").write_text(textwrap.dedent("""
        config = {}
        def set_global_config(cfg):
            global config
            config.update(cfg)
            return config
    """))
    (ref / "tracker.py").write_text("from mast3r_slam.config import config\nclass FrameTracker:\n    pass\n")
    (ref / "global_opt.py").write_text("class FactorGraph:\n    pass\n")
    main = tmp_path / "main.py"  # a main.py that imports like the reference's (main.py:17-29), unchanged
    main.write_text(textwrap.dedent("""
        from mast3r_slam.global_opt import FactorGraph
        from mast3r_slam.config import config, set_global_config
        from mast3r_slam.tracker import FrameTracker
        set_global_config({"use_calib": True, "tracking": {"max_iters": 7}})
        import m3s.config, m3s.tracker, m3s.global_opt
        assert FrameTracker is m3s.tracker.FrameTracker, FrameTracker
        assert FactorGraph is m3s.global_opt.FactorGraph, FactorGraph
        assert m3s.config.config is config and config["use_calib"] is True
        assert m3s.tracker.config is config and m3s.tracker.config["tracking"]["max_iters"] == 7
        print("HOOK_OK")
    """))
    env = dict(os.environ, PYTHONPATH=os.pathsep.join([os.path.join(PKG, "m3s_hook"), PKG, str(tmp_path / "ref")]))
    r = subprocess.run([sys.executable, str(main)], env=env, capture_output=True, text=True, timeout=120, cwd=tmp_path)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "HOOK_OK" in r.stdout
    # without the hook directory nothing changes
    env["PYTHONPATH"] = os.pathsep.join([PKG, str(tmp_path / "ref")])
    r = subprocess.run([sys.executable, str(main)], env=env, capture_output=True, text=True, timeout=120, cwd=tmp_path)
    assert r.returncode != 0 and "AssertionError" in r.stderr
