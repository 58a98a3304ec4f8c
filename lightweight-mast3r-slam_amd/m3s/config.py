"""Configuration with the reference's keys, defaults and ``inherit`` chains.

Mirrors ``/root/reference/mast3r_slam/config.py:7-48`` (YAML with ``inherit``, a float-friendly
SafeLoader, a global mutable ``config`` dict) and carries the path's defaults from
``config/base.yaml:8-50`` so the package works without the reference's config files. Only the
sections the hot path reads are required: ``matching``, ``tracking``, ``local_opt``, ``use_calib``.
"""
import copy
import re

import yaml

DEFAULTS = {
    "use_calib": False,
    "single_thread": False,
    "dataset": {"subsample": 1, "img_downsample": 1, "center_principle_point": True},
    "matching": {"max_iter": 10, "lambda_init": 1e-8, "convergence_thresh": 1e-6, "dist_thresh": 1e-1,
                 "radius": 3, "dilation_max": 5},
    "tracking": {"min_match_frac": 0.05, "max_iters": 50, "C_conf": 0.0, "Q_conf": 1.5, "rel_error": 1e-3,
                 "delta_norm": 1e-3, "huber": 1.345, "match_frac_thresh": 0.333, "sigma_ray": 0.003,
                 "sigma_dist": 1e1, "sigma_pixel": 1.0, "sigma_depth": 1e1, "sigma_point": 0.05,
                 "pixel_border": -10, "depth_eps": 1e-6, "filtering_mode": "weighted_pointmap",
                 "filtering_score": "median"},
    "local_opt": {"pin": 1, "window_size": 1e6, "C_conf": 0.0, "Q_conf": 1.5, "min_match_frac": 0.1,
                  "pixel_border": -10, "depth_eps": 1e-6, "max_iters": 10, "sigma_ray": 0.003, "sigma_dist": 1e1,
                  "sigma_pixel": 1.0, "sigma_depth": 1e1, "sigma_point": 0.05, "delta_norm": 1e-8,
                  "use_cuda": True},
    "retrieval": {"k": 3, "min_thresh": 5e-3},
    "reloc": {"min_match_frac": 0.3, "strict": True},
}

config = copy.deepcopy(DEFAULTS)


def _loader():
    loader = yaml.SafeLoader
    loader.add_implicit_resolver(
        "tag:yaml.org,2002:float",
        re.compile(r"""^(?:[-+]?(?:[0-9][0-9_]*)\.[0-9_]*(?:[eE][-+]?[0-9]+)?
                    |[-+]?(?:[0-9][0-9_]*)(?:[eE][-+]?[0-9]+)
                    |\.[0-9_]+(?:[eE][-+][0-9]+)?
                    |[-+]?[0-9][0-9_]*(?::[0-5]?[0-9])+\.[0-9_]*
                    |[-+]?\.(?:inf|Inf|INF)
                    |\.(?:nan|NaN|NAN))$""", re.X),
        list("-+0123456789."),
    )
    return loader


def merge_config(dict1, dict2):
    for k, v in dict2.items():
        if isinstance(v, dict):
            dict1.setdefault(k, {})
            merge_config(dict1[k], v)
        else:
            dict1[k] = v
    return dict1


def load_config(path, is_parent=False):
    """config.py:7-37: load YAML, resolve ``inherit`` (paths relative to the CWD like the reference)."""
    with open(path, "r") as f:
        cfg = yaml.load(f, Loader=_loader()) or {}
    inherit = cfg.get("inherit")
    parent = load_config(inherit, is_parent=True) if inherit is not None else copy.deepcopy(DEFAULTS)
    cfg = merge_config(parent, cfg)
    if is_parent:
        return cfg
    set_global_config(cfg)
    return config


def set_global_config(cfg):
    config.clear()
    config.update(merge_config(copy.deepcopy(DEFAULTS), cfg))
    return config


def reset_config():
    return set_global_config({})
