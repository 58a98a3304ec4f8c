"""Synthetic post-ViT inputs for tests and benchmarks (no network: no checkpoints, no datasets).

* ``make_pair``: one frame/keyframe pair as MASt3R would return it (SURVEY.md §8d "Synthetic pair"):
  a smooth depth surface back-projected with K, a known sub-pixel flow + in-plane rotation between
  the two images, L2-normalised smooth 24-channel descriptors, confidences 1 + Exp(mean 4), and
  the keyframe's canonical pointmap = T_gt * (keyframe points seen from the frame) + noise.
* ``SyntheticModel``: the ``asymmetric_inference(frame_i, frame_j)`` provider the tracker calls in
  place of the ViT, cycling through a ring of pairs kept resident on the device.
* ``make_graph``: a keyframe factor graph inside a box-shaped room (ray-cast pointmaps, so matched
  points are geometrically consistent), consecutive + loop edges, GT-reprojection matches with
  outliers, perturbed initial Sim(3) poses (SURVEY.md §8d "C4/C5 synthetic factor graph").
"""
import math

import numpy as np
import torch
import torch.nn.functional as F


def intrinsics(H, W, device="cpu"):
    f = 0.8 * W
    return torch.tensor([[f, 0.0, W / 2.0], [0.0, f, H / 2.0], [0.0, 0.0, 1.0]], dtype=torch.float32, device=device)


def _depth(u, v, H, W, g):
    z = torch.full_like(u, 2.0)
    for _ in range(3):
        fu, fv = (torch.rand(2, generator=g) * 2 - 1) * (2 * math.pi / (0.6 * max(H, W)))
        ph = torch.rand(1, generator=g) * 2 * math.pi
        z = z + (0.5 / 3) * torch.sin(fu * u + fv * v + ph)
    return z


def _smooth_desc(H, W, Fd, g, sigma=2.0):
    n = torch.randn(1, Fd, H, W, generator=g)
    r = int(3 * sigma)
    k = torch.exp(-0.5 * (torch.arange(-r, r + 1, dtype=torch.float32) / sigma) ** 2)
    k = k / k.sum()
    n = F.conv2d(F.pad(n, (r, r, 0, 0), mode="reflect"), k.view(1, 1, 1, -1).repeat(Fd, 1, 1, 1), groups=Fd)
    n = F.conv2d(F.pad(n, (0, 0, r, r), mode="reflect"), k.view(1, 1, -1, 1).repeat(Fd, 1, 1, 1), groups=Fd)
    return F.normalize(n[0].permute(1, 2, 0), dim=-1)  # (H, W, F)


def _bilinear(img, u, v):
    """img (H,W,C) sampled at float (u,v) with border clamping."""
    H, W, _ = img.shape
    grid = torch.stack((u / (W - 1) * 2 - 1, v / (H - 1) * 2 - 1), dim=-1)[None]
    out = F.grid_sample(img.permute(2, 0, 1)[None], grid, mode="bilinear", padding_mode="border", align_corners=True)
    return out[0].permute(1, 2, 0)


def quat_from_axis_angle(axis, angle):
    axis = torch.as_tensor(axis, dtype=torch.float32)
    axis = axis / axis.norm()
    return torch.cat((axis * math.sin(angle / 2), torch.tensor([math.cos(angle / 2)])))


def make_pair(H=64, W=64, Fd=24, seed=0, flow=(3.3, -2.7), rot_deg=1.0, noise=0.002, desc_noise=0.05,
              t_gt=(0.01, -0.005, 0.004), rot_gt_deg=0.5, scale_gt=1.01):
    """Returns dict with X (2,H,W,3), C (2,H,W), D (2,H,W,F), Q (2,H,W), Xk (H*W,3), Ck (H*W,1),
    K (3,3), T_gt (8) — all float32 CPU tensors."""
    g = torch.Generator().manual_seed(seed)
    K = intrinsics(H, W)
    fx, fy, cx, cy = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
    vv, uu = torch.meshgrid(torch.arange(H, dtype=torch.float32), torch.arange(W, dtype=torch.float32), indexing="ij")
    zfun = lambda u, v, gg=g.get_state(): _depth(u, v, H, W, torch.Generator().set_state(gg))
    z1 = zfun(uu, vv)
    X11 = torch.stack(((uu - cx) / fx * z1, (vv - cy) / fy * z1, z1), dim=-1)
    th = math.radians(rot_deg)
    du, dv = uu - cx, vv - cy
    u1 = math.cos(th) * du - math.sin(th) * dv + cx + flow[0]
    v1 = math.sin(th) * du + math.cos(th) * dv + cy + flow[1]
    z21 = zfun(u1, v1)
    X21c = torch.stack(((u1 - cx) / fx * z21, (v1 - cy) / fy * z21, z21), dim=-1)
    X21 = X21c + noise * torch.randn(H, W, 3, generator=g)
    D11 = _smooth_desc(H, W, Fd, g)
    D21 = _bilinear(D11, u1, v1) + desc_noise * torch.randn(H, W, Fd, generator=g)
    D21 = F.normalize(D21, dim=-1)
    C = 1.0 + torch.empty(2, H, W).exponential_(0.25, generator=g)
    Q = 1.0 + torch.empty(2, H, W).exponential_(0.25, generator=g)
    q = quat_from_axis_angle((0.3, -0.5, 0.8), math.radians(rot_gt_deg))
    T_gt = torch.cat((torch.tensor(t_gt, dtype=torch.float32), q, torch.tensor([scale_gt])))
    from m3s.sim3 import Sim3

    Xk = Sim3(T_gt.view(1, 8)).act(X21c.reshape(-1, 3)) + noise * torch.randn(H * W, 3, generator=g)
    Ck = (1.0 + torch.empty(H * W, 1).exponential_(0.25, generator=g))
    return dict(X=torch.stack((X11, X21)), C=C, D=torch.stack((D11, D21)), Q=Q, Xk=Xk.float(), Ck=Ck, K=K,
                T_gt=T_gt, flow=(u1, v1))


class SyntheticModel:
    """Stands in for MASt3R's asymmetric decoder: returns a ring of resident synthetic outputs."""

    def __init__(self, pairs, device):
        self.pairs = [{k: (v.to(device) if torch.is_tensor(v) else v) for k, v in p.items() if k != "flow"}
                      for p in pairs]
        self.step = 0

    def asymmetric_inference(self, frame_i, frame_j):
        p = self.pairs[self.step % len(self.pairs)]
        self.step += 1
        return p["X"], p["C"], p["D"], p["Q"]


# ------------------------------------------------------------------------------------------------
# factor graph
# ------------------------------------------------------------------------------------------------
def _raycast_box(origin, dirs, half=3.0):
    """Distance along unit dirs (N,3) from origin (3,) to the inside wall of [-half, half]^3."""
    with torch.no_grad():
        t = torch.full(dirs.shape[:-1], float("inf"), device=dirs.device)
        for a in range(3):
            d = dirs[..., a]
            for wall in (-half, half):
                ta = (wall - origin[a]) / torch.where(d.abs() < 1e-9, torch.full_like(d, 1e-9), d)
                t = torch.where(ta > 0, torch.minimum(t, ta), t)
    return t


def make_graph(n_kf=8, H=48, W=64, loops_per_kf=3, seed=1, outlier_frac=0.05, valid_prob=0.8,
               pose_noise=(0.02, 1.0, 0.01), device="cpu"):
    """Returns dict: Twc_gt (K,8), Twc0 (K,8) perturbed (kf 0 exact: pinned), Xs (K,N,3), Cs (K,N,1),
    ii, jj (E,) undirected edges, idx (E,N) i->j matches (for each pixel of j its pixel in i),
    valid (E,N,1), Q (E,N,1), K (3,3). Two-way edges are built by the caller (prep_two_way_edges)."""
    from m3s.sim3 import Sim3

    g = torch.Generator().manual_seed(seed)
    N = H * W
    K = intrinsics(H, W)
    fx, fy, cx, cy = [float(x) for x in (K[0, 0], K[1, 1], K[0, 2], K[1, 2])]
    # smooth camera path inside the room
    ts, qs = [], []
    for k in range(n_kf):
        a = 2 * math.pi * k / max(n_kf, 1)
        ts.append(torch.tensor([0.8 * math.cos(a), 0.3 * math.sin(2 * a), 0.8 * math.sin(a)]))
        qs.append(quat_from_axis_angle((0.05, 1.0, 0.02), -a + 0.15 * math.sin(3 * a)))
    Twc_gt = torch.cat((torch.stack(ts), torch.stack(qs), torch.ones(n_kf, 1)), dim=1)
    vv, uu = torch.meshgrid(torch.arange(H, dtype=torch.float32), torch.arange(W, dtype=torch.float32), indexing="ij")
    rays_c = torch.stack(((uu - cx) / fx, (vv - cy) / fy, torch.ones_like(uu)), dim=-1).reshape(-1, 3)
    Xs = []
    for k in range(n_kf):
        T = Sim3(Twc_gt[k].view(1, 8))
        dirs_w = T.act(rays_c) - Twc_gt[k, :3]
        dist = _raycast_box(Twc_gt[k, :3], F.normalize(dirs_w, dim=-1))
        z = dist / rays_c.norm(dim=-1)  # depth along the optical axis
        Xs.append(rays_c * z[:, None])
    Xs = torch.stack(Xs)  # canonical (camera) coordinates
    Cs = 1.0 + torch.empty(n_kf, N, 1).exponential_(0.25, generator=g)
    edges = [(k - 1, k) for k in range(1, n_kf)]
    for k in range(4, n_kf):
        cands = torch.randperm(k - 1, generator=g)[:loops_per_kf].tolist()
        edges += [(c, k) for c in cands if (c, k) not in edges]
    ii = torch.tensor([e[0] for e in edges], dtype=torch.int64)
    jj = torch.tensor([e[1] for e in edges], dtype=torch.int64)
    E = len(edges)
    idx = torch.zeros(E, N, dtype=torch.int64)
    valid = torch.zeros(E, N, 1, dtype=torch.bool)
    for e, (i, j) in enumerate(edges):
        Ti, Tj = Sim3(Twc_gt[i].view(1, 8)), Sim3(Twc_gt[j].view(1, 8))
        Xi = (Ti.inv() * Tj).act(Xs[j])
        z = Xi[:, 2]
        u = fx * Xi[:, 0] / z + cx
        v = fy * Xi[:, 1] / z + cy
        inb = (z > 0.1) & (u >= 0) & (u <= W - 1) & (v >= 0) & (v <= H - 1)
        ui = u.round().clamp(0, W - 1).long()
        vi = v.round().clamp(0, H - 1).long()
        lin = ui + W * vi
        out = torch.rand(N, generator=g) < outlier_frac
        lin = torch.where(out, torch.randint(0, N, (N,), generator=g), lin)
        idx[e] = lin
        valid[e, :, 0] = inb & (torch.rand(N, generator=g) < valid_prob)
    Q = 1.0 + torch.empty(E, N, 1).exponential_(0.25, generator=g)
    t_n, r_n, s_n = pose_noise
    Twc0 = Twc_gt.clone()
    for k in range(1, n_kf):
        dq = quat_from_axis_angle(torch.randn(3, generator=g).tolist(), math.radians(r_n) * float(torch.randn(1, generator=g)))
        T = Sim3(torch.cat((t_n * torch.randn(3, generator=g), dq, torch.tensor([1.0 + s_n * float(torch.randn(1, generator=g))]))).view(1, 8))
        Twc0[k] = (T * Sim3(Twc_gt[k].view(1, 8))).data[0]
    out = dict(Twc_gt=Twc_gt, Twc0=Twc0, Xs=Xs.float(), Cs=Cs, ii=ii, jj=jj, idx=idx, valid=valid, Q=Q, K=K, H=H, W=W)
    return {k: (v.to(device) if torch.is_tensor(v) else v) for k, v in out.items()}


def two_way(G):
    """global_opt.py:106-112 prep_two_way_edges on the undirected synthetic graph (needs j->i maps,
    built here from the i->j maps' GT geometry by reprojection in the other direction)."""
    from m3s.sim3 import Sim3

    H, W = G["H"], G["W"]
    K = G["K"].cpu()
    fx, fy, cx, cy = [float(x) for x in (K[0, 0], K[1, 1], K[0, 2], K[1, 2])]
    idx_r, valid_r = [], []
    Xs = G["Xs"].cpu()
    Tg = G["Twc_gt"].cpu()
    g = torch.Generator().manual_seed(7)
    for i, j in zip(G["ii"].tolist(), G["jj"].tolist()):
        X = (Sim3(Tg[j].view(1, 8)).inv() * Sim3(Tg[i].view(1, 8))).act(Xs[i])
        z = X[:, 2]
        u = fx * X[:, 0] / z + cx
        v = fy * X[:, 1] / z + cy
        inb = (z > 0.1) & (u >= 0) & (u <= W - 1) & (v >= 0) & (v <= H - 1)
        lin = u.round().clamp(0, W - 1).long() + W * v.round().clamp(0, H - 1).long()
        idx_r.append(lin)
        valid_r.append((inb & (torch.rand(lin.shape[0], generator=g) < 0.8))[:, None])
    dev = G["ii"].device
    ii = torch.cat((G["ii"], G["jj"]))
    jj = torch.cat((G["jj"], G["ii"]))
    idx = torch.cat((G["idx"], torch.stack(idx_r).to(dev)))
    valid = torch.cat((G["valid"], torch.stack(valid_r).to(dev)))
    Q = torch.cat((G["Q"], G["Q"].flip(1)))
    return ii, jj, idx, valid, Q


def retrieval_inputs(seed, C, D, M):
    """Unit-norm fp32 codebook centroids (C, D) and local features (M, D), ASMK-like, from a numpy seed
    (the retrieval golden fixtures store only the seed, shapes and a checksum)."""
    rng = np.random.default_rng(seed)
    c = rng.standard_normal((C, D)).astype(np.float32)
    c /= np.linalg.norm(c, axis=1, keepdims=True)
    q = rng.standard_normal((M, D)).astype(np.float32)
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    return c, q
