"""Pixel-ray helpers for the torch glue around the fused kernels.

Only what the glue itself needs: the calibrated-mode constraint of a pointmap to its pixel rays
(``constrain_points_to_ray``, ``get_pixel_coords``, ``backproject`` — reference
``mast3r_slam/geometry.py:37-42, 107-123``), used by ``FrameTracker.get_points_poses`` and
``FactorGraph.solve_GN_calib``. The residual / Jacobian math of ``point_to_ray_dist``,
``act_Sim3`` and ``project_calib`` lives in the HIP kernels (track.hip, ba.hip).
"""
import torch


def get_pixel_coords(b, img_size, device, dtype):
    """(b, H, W, 2) grid of (u, v) = (column, row)."""
    h, w = int(img_size[0]), int(img_size[1])
    vv, uu = torch.meshgrid(torch.arange(h, device=device), torch.arange(w, device=device), indexing="ij")
    return torch.stack((uu, vv), dim=-1).to(dtype).expand(b, h, w, 2).contiguous()


def backproject(p, z, K):
    """P = z * [(u - cx) / fx, (v - cy) / fy, 1]; p (..., 2), z (..., 1)."""
    x = (p[..., 0] - K[0, 2]) / K[0, 0]
    y = (p[..., 1] - K[1, 2]) / K[1, 1]
    ray = torch.stack((x, y, torch.ones_like(x)), dim=-1).to(K.dtype)
    return z * ray


def constrain_points_to_ray(img_size, Xs, K):
    """Replace every point of Xs (B, H*W, 3) by the point at its own depth on its pixel's ray."""
    uv = get_pixel_coords(Xs.shape[0], img_size, Xs.device, Xs.dtype).view(*Xs.shape[:-1], 2)
    return backproject(uv, Xs[..., 2:3], K)
