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


def tum_fr1_intrinsics(H=384, W=512):
    """TUM freiburg1 calibration (dataloader.py:78-81, 640x480) scaled to the MASt3R frame like
    Intrinsics.from_calib's K_frame (dataloader.py:289-293): 640x480 -> 512x384 is a 1.25 downscale, no crop."""
    s = 640.0 / W
    assert abs(480.0 / H - s) < 1e-9, "TUM frames keep the 4:3 aspect"
    fx, fy, cx, cy = 517.3 / s, 516.5 / s, 318.6 / s, 255.3 / s
    return torch.tensor([[fx, 0.0, cx], [0.0, fy, cy], [0.0, 0.0, 1.0]], dtype=torch.float32)


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
              t_gt=(0.01, -0.005, 0.004), rot_gt_deg=0.5, scale_gt=1.01, K=None):
    """Returns dict with X (2,H,W,3), C (2,H,W), D (2,H,W,F), Q (2,H,W), Xk (H*W,3), Ck (H*W,1),
    K (3,3), T_gt (8) — all float32 CPU tensors. K: camera intrinsics (default `intrinsics(H, W)`)."""
    g = torch.Generator().manual_seed(seed)
    K = intrinsics(H, W) if K is None else torch.as_tensor(K, dtype=torch.float32)
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


def make_warm_batch(H, W, seeds, K=None):
    """A batch of pairs (one per seed) with a warm-start idx_1_to_2_init like a tracker's previous matches
    (matching.py:25-49 prep's idx path): a shifted identity, with some entries out of range on both sides so that
    lin_to_pixel's floor semantics and the clamp are exercised. Returns X11, X21 (B,H,W,3), D11, D21 (B,H,W,F),
    idx_init (B,H*W) int64 (CPU tensors)."""
    P = [make_pair(H, W, seed=s, K=K) for s in seeds]
    X11 = torch.stack([p["X"][0] for p in P])
    X21 = torch.stack([p["X"][1] for p in P])
    D11 = torch.stack([p["D"][0] for p in P])
    D21 = torch.stack([p["D"][1] for p in P])
    vv, uu = torch.meshgrid(torch.arange(H), torch.arange(W), indexing="ij")
    idx = []
    for b in range(len(seeds)):
        u = (uu - 3 + b).clamp(0, W - 1)
        v = (vv + 2 - b).clamp(0, H - 1)
        i = (v * W + u).reshape(-1).to(torch.int64)
        i[::997] = -5 - b  # before the image: v = -1 -> clamped to row 1
        i[1::991] = H * W + 7 + b  # past the image: v = H -> clamped to row H - 2
        idx.append(i)
    return X11, X21, D11, D21, torch.stack(idx)


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


# ------------------------------------------------------------------------------------------------
# C4/C5 factor graphs on a recorded trajectory
# ------------------------------------------------------------------------------------------------
def _traj(name, K):
    import os

    P = np.loadtxt(os.path.join(os.path.dirname(__file__), "data", name))
    assert K <= len(P), f"{name} holds {len(P)} poses"
    return P[:K]


def chess_poses(K=256):
    """The first K of 256 7-Scenes chess ground-truth poses (m3s/data/chess_kf256.txt, written by
    scripts/make_traj_poses.py from groundtruths/7-scenes/chess.txt), (K,8) float64 [t, q xyzw, s]."""
    return _traj("chess_kf256.txt", K)


def euroc_poses(K=256):
    """The first K of 256 EuRoC MH_02_easy ground-truth poses (m3s/data/euroc_mh02_kf256.txt, written by
    scripts/make_traj_poses.py), (K,8) float64 [t, q xyzw, s]: the C4-shaped (EuRoC) BA graph."""
    return _traj("euroc_mh02_kf256.txt", K)


def _act(T, X):
    """Sim(3) rows T (...,8) acting on points X (...,N,3) (T broadcast over N)."""
    t, q, s = T[..., None, 0:3], T[..., None, 3:7], T[..., None, 7:8]
    uv = 2.0 * torch.cross(q[..., :3].expand_as(X), X, dim=-1)
    return s * (X + q[..., 3:4] * uv + torch.cross(q[..., :3].expand_as(X), uv, dim=-1)) + t


def _inv(T):
    q = torch.cat((-T[..., 3:6], T[..., 6:7]), -1)
    s = 1.0 / T[..., 7:8]
    Ti = torch.cat((torch.zeros_like(T[..., :3]), q, s), -1)
    t = -_act(Ti, T[..., None, 0:3])[..., 0, :]
    return torch.cat((t, q, s), -1)


def _mul(A, B):
    """Sim(3) composition A * B of rows (...,8)."""
    qa, qb = A[..., 3:7], B[..., 3:7]
    xyz = qa[..., 3:4] * qb[..., :3] + qb[..., 3:4] * qa[..., :3] + torch.cross(qa[..., :3], qb[..., :3], dim=-1)
    w = qa[..., 3:4] * qb[..., 3:4] - (qa[..., :3] * qb[..., :3]).sum(-1, keepdim=True)
    t = _act(A, B[..., None, 0:3])[..., 0, :]
    return torch.cat((t, xyz, w, A[..., 7:8] * B[..., 7:8]), -1)


def make_traj_graph(poses, H, W, loops_per_kf=3, seed=1, outlier_frac=0.05, valid_prob=0.8,
                    pose_noise=(0.02, 1.0, 0.01), device="cpu", covis_grid=(12, 16)):
    """SURVEY.md §8(d) C4/C5 synthetic factor graph on a recorded trajectory (e.g. `chess_poses()`).

    Keyframe k gets the consecutive edge (k-1, k) (main.py:116-120, n_consec = 1) and up to `loops_per_kf`
    retrieval-like edges (main.py:121-131, retrieval k = 3, base.yaml:53): the earlier keyframes i < k-1 that
    see most of keyframe k's view (ground-truth co-visibility on a coarse pixel grid, which is what the image
    retrieval ranks by), kept when at least 5 % of the grid is co-visible. The pointmaps are ray-cast into a
    box room around the trajectory, the matches are GT reprojections with `outlier_frac` random outliers, and
    both directions of every edge are built the way FactorGraph.add_factors stores them (global_opt.py:32-101:
    ii = [i, j], jj = [j, i], idx_ii2jj for each direction). Everything is computed on `device`.

    Returns dict: Twc_gt, Twc0 (K,8) f32 (kf 0 exact), Xs (K,N,3), Cs (K,N,1), ii, jj (E_dir,) i64,
    idx (E_dir,N) i64, valid (E_dir,N,1) bool, Q (E_dir,N,1) f32, K (3,3), H, W, E_und."""
    dev = torch.device(device)
    g = torch.Generator(device=dev).manual_seed(seed)
    P = torch.as_tensor(np.asarray(poses), dtype=torch.float64)
    n_kf = P.shape[0]
    centre = P[:, :3].mean(0)
    half = float((P[:, :3] - centre).abs().max()) + 1.5
    P[:, :3] -= centre  # the room is the box [-half, half]^3 around the trajectory
    Twc_gt = P.float().to(dev)
    N = H * W
    Kc = intrinsics(H, W, device=dev)
    fx, fy, cx, cy = [float(x) for x in (Kc[0, 0], Kc[1, 1], Kc[0, 2], Kc[1, 2])]

    def rays(h, w):
        vv, uu = torch.meshgrid(torch.linspace(0, H - 1, h, device=dev), torch.linspace(0, W - 1, w, device=dev),
                                indexing="ij")
        return torch.stack(((uu - cx) / fx, (vv - cy) / fy, torch.ones_like(uu)), -1).reshape(-1, 3)

    def pointmaps(rc, Ts):
        dirs = _act(Ts, rc.expand(Ts.shape[0], -1, -1)) - Ts[:, None, :3]
        out = []
        for k in range(Ts.shape[0]):
            d = _raycast_box(Ts[k, :3], F.normalize(dirs[k], dim=-1), half)
            out.append(rc * (d / rc.norm(dim=-1))[:, None])
        return torch.stack(out)

    def project(Tij, Xj):
        Xi = _act(Tij, Xj)
        z = Xi[..., 2]
        return fx * Xi[..., 0] / z + cx, fy * Xi[..., 1] / z + cy, z

    # retrieval-like loop candidates from coarse GT co-visibility
    Xg = pointmaps(rays(*covis_grid), Twc_gt)
    edges = [(k - 1, k) for k in range(1, n_kf)]
    inv_all = _inv(Twc_gt)
    for k in range(2, n_kf):
        Tik = _mul(inv_all[: k - 1], Twc_gt[k].expand(k - 1, 8))
        u, v, z = project(Tik, Xg[k].expand(k - 1, -1, -1))
        score = ((z > 0.1) & (u >= 0) & (u <= W - 1) & (v >= 0) & (v <= H - 1)).float().mean(1)
        top = torch.topk(score, min(loops_per_kf, k - 1))
        edges += [(int(i), k) for s, i in zip(top.values.tolist(), top.indices.tolist()) if s >= 0.05]
    E_und = len(edges)
    Xs = pointmaps(rays(H, W), Twc_gt)
    ii_u = torch.tensor([e[0] for e in edges], dtype=torch.int64, device=dev)
    jj_u = torch.tensor([e[1] for e in edges], dtype=torch.int64, device=dev)
    ii = torch.cat((ii_u, jj_u))
    jj = torch.cat((jj_u, ii_u))
    E = ii.shape[0]
    idx = torch.empty(E, N, dtype=torch.int64, device=dev)
    valid = torch.empty(E, N, 1, dtype=torch.bool, device=dev)
    for e in range(E):  # idx_ii2jj: for each pixel of j its pixel in i
        i, j = int(ii[e]), int(jj[e])
        u, v, z = project(_mul(inv_all[i], Twc_gt[j]), Xs[j])
        inb = (z > 0.1) & (u >= 0) & (u <= W - 1) & (v >= 0) & (v <= H - 1)
        lin = u.round().clamp(0, W - 1).long() + W * v.round().clamp(0, H - 1).long()
        out = torch.rand(N, generator=g, device=dev) < outlier_frac
        idx[e] = torch.where(out, torch.randint(0, N, (N,), generator=g, device=dev), lin)
        valid[e, :, 0] = inb & (torch.rand(N, generator=g, device=dev) < valid_prob)
    Cs = 1.0 + torch.empty(n_kf, N, 1, device=dev).exponential_(0.25, generator=g)
    Q = 1.0 + torch.empty(E, N, 1, device=dev).exponential_(0.25, generator=g)
    t_n, r_n, s_n = pose_noise
    gc = torch.Generator().manual_seed(seed)  # pose noise on the host: identical on every device
    Twc0 = Twc_gt.cpu().clone()
    for k in range(1, n_kf):
        dq = quat_from_axis_angle(torch.randn(3, generator=gc).tolist(), math.radians(r_n) * float(torch.randn(1, generator=gc)))
        dT = torch.cat((t_n * torch.randn(3, generator=gc), dq, torch.tensor([1.0 + s_n * float(torch.randn(1, generator=gc))])))
        Twc0[k] = _mul(dT, Twc0[k])
    return dict(Twc_gt=Twc_gt, Twc0=Twc0.to(dev), Xs=Xs.float(), Cs=Cs, ii=ii, jj=jj, idx=idx, valid=valid, Q=Q,
                K=Kc, H=H, W=W, E_und=E_und)


# ------------------------------------------------------------------------------------------------
# backend replay (C3 / C4): a keyframe sequence with decoder outputs for any keyframe pair
# ------------------------------------------------------------------------------------------------
def _stable_seed(*key):
    """A seed from a key tuple that does not depend on the interpreter's string-hash randomisation."""
    import zlib

    return zlib.crc32(repr(key).encode())


class SceneReplay:
    """Stands in for MASt3R + the retrieval model over a recorded trajectory, for replaying the backend loop
    (main.py:116-165: retrieval -> add_factors -> solve_GN_* per new keyframe) without a checkpoint.

    The world is the box room of ``make_traj_graph``. Keyframe k sees it from the ground-truth pose ``Twc_gt[k]``
    (ray-cast pointmap, camera coordinates, + N(0, noise^2)); its initial pose ``Twc0[k]`` is the ground truth
    perturbed (what tracking would hand the backend; keyframe 0 exact). Descriptors are a smooth 24-channel field
    of the WORLD point (sums of random plane waves, L2-normalised), so the same surface point carries the same
    descriptor in every view and the fused matcher finds the geometric correspondences.

    * ``symmetric_inference(kfs_i, kfs_j)``: X, C, D, Q (4, b, H, W, ...) ordered (ii, ji, jj, ij) like
      ``mast3r_decode_symmetric_batch`` (mast3r_utils.py:117-146): X_ji = T_i^-1 T_j X_j with ground-truth
      poses, descriptors of the pixels' world points (+ noise).
    * ``features(k)``: M local retrieval features of keyframe k (128-D, unit norm): a random unit vector per
      coarse world voxel (0.5 m) that keyframe sees at M fixed pixels, + noise — the input of
      ``RetrievalDatabase.quantize_custom``. The scoring around it (ASMK) is out of scope; ``retrieve`` ranks
      earlier keyframes by shared visual words instead.
    Keyframe ids are the frames' ``frame_id``."""

    def __init__(self, poses, H, W, K=None, Fd=24, seed=3, noise=0.003, desc_noise=0.03,
                 pose_noise=(0.01, 0.5, 0.005), n_feat=64, feat_dim=128, device="cpu"):
        from m3s.sim3 import Sim3

        dev = torch.device(device)
        g = torch.Generator().manual_seed(seed)
        P = torch.as_tensor(np.asarray(poses), dtype=torch.float64)
        n_kf = P.shape[0]
        centre = P[:, :3].mean(0)
        self.half = float((P[:, :3] - centre).abs().max()) + 1.5
        P[:, :3] -= centre
        self.Twc_gt = P.float().to(dev)
        self.H, self.W, self.N, self.dev = H, W, H * W, dev
        self.K = (intrinsics(H, W) if K is None else torch.as_tensor(K, dtype=torch.float32)).to(dev)
        fx, fy, cx, cy = [float(x) for x in (self.K[0, 0], self.K[1, 1], self.K[0, 2], self.K[1, 2])]
        vv, uu = torch.meshgrid(torch.arange(H, dtype=torch.float32, device=dev),
                                torch.arange(W, dtype=torch.float32, device=dev), indexing="ij")
        rays = torch.stack(((uu - cx) / fx, (vv - cy) / fy, torch.ones_like(uu)), -1).reshape(-1, 3)
        self.Xc, self.Xw = [], []
        for k in range(n_kf):
            T = Sim3(self.Twc_gt[k].view(1, 8))
            d = _raycast_box(self.Twc_gt[k, :3], F.normalize(T.act(rays) - self.Twc_gt[k, :3], dim=-1), self.half)
            Xc = rays * (d / rays.norm(dim=-1))[:, None]
            self.Xc.append(Xc)
            self.Xw.append(T.act(Xc))
        # descriptor field: Fd channels, each a sum of 4 plane waves of 0.25-0.6 m wavelength
        nw = 4
        dirs = F.normalize(torch.randn(Fd, nw, 3, generator=g), dim=-1)
        lam = 0.25 + 0.35 * torch.rand(Fd, nw, generator=g)
        self.wave_k = (2 * math.pi * dirs / lam[..., None]).to(dev)
        self.wave_ph = (2 * math.pi * torch.rand(Fd, nw, generator=g)).to(dev)
        self.noise, self.desc_noise = noise, desc_noise
        self.seed = seed
        # per-keyframe confidences and pointmap noise (fixed per keyframe and view role)
        self.C = [(1.0 + torch.empty(self.N).exponential_(0.25, generator=g)).to(dev) for _ in range(n_kf)]
        t_n, r_n, s_n = pose_noise
        Twc0 = self.Twc_gt.cpu().clone()
        for k in range(1, n_kf):
            dq = quat_from_axis_angle(torch.randn(3, generator=g).tolist(),
                                      math.radians(r_n) * float(torch.randn(1, generator=g)))
            dT = torch.cat((t_n * torch.randn(3, generator=g), dq,
                            torch.tensor([1.0 + s_n * float(torch.randn(1, generator=g))])))
            Twc0[k] = _mul(dT, Twc0[k])
        self.Twc0 = Twc0.to(dev)
        # retrieval features
        self.n_feat, self.feat_dim = n_feat, feat_dim
        self.feat_px = [torch.randperm(self.N, generator=g)[:n_feat].to(dev) for _ in range(n_kf)]

    def _gen(self, *key):
        return torch.Generator(device=self.dev).manual_seed(_stable_seed(self.seed, *key))

    def descriptors(self, Xw, g):
        ph = torch.einsum("fwc,nc->nfw", self.wave_k, Xw) + self.wave_ph[None]
        D = torch.sin(ph).sum(-1)
        D = D + self.desc_noise * torch.randn(D.shape, generator=g, device=self.dev)
        return F.normalize(D, dim=-1)

    def pointmap(self, k, role):
        """Keyframe k's own pointmap as a decoder output of `role` (its own camera), with fresh noise."""
        g = self._gen(k, role, "X")
        return self.Xc[k] + self.noise * torch.randn(self.Xc[k].shape, generator=g, device=self.dev)

    def keyframe(self, k):
        """(X_canon (N,3), C (N,1)) the keyframe enters the backend with (its tracking-time canonical pointmap)."""
        return self.pointmap(k, "kf"), self.C[k][:, None].clone()

    def _rel(self, i, j, Xj):
        from m3s.sim3 import Sim3

        Tij = Sim3(self.Twc_gt[i].view(1, 8)).inv() * Sim3(self.Twc_gt[j].view(1, 8))
        return Tij.act(Xj)

    def symmetric_inference(self, kfs_i, kfs_j):
        H, W = self.H, self.W
        out = {n: [] for n in "XCDQ"}
        for fi, fj in zip(kfs_i, kfs_j):
            i, j = int(fi.frame_id), int(fj.frame_id)
            Xii, Xjj = self.pointmap(i, ("ii", j)), self.pointmap(j, ("jj", i))
            Xji = self._rel(i, j, self.pointmap(j, ("ji", i)))
            Xij = self._rel(j, i, self.pointmap(i, ("ij", j)))
            g = self._gen(i, j, "DQ")
            Dii, Dji = self.descriptors(self.Xw[i], g), self.descriptors(self.Xw[j], g)
            Djj, Dij = self.descriptors(self.Xw[j], g), self.descriptors(self.Xw[i], g)
            for name, vals in (("X", (Xii, Xji, Xjj, Xij)), ("D", (Dii, Dji, Djj, Dij))):
                out[name].append(torch.stack([v.reshape(H, W, -1) for v in vals]))
            for name in "CQ":
                out[name].append((1.0 + torch.empty(4, H, W, device=self.dev).exponential_(0.25, generator=g)))
        return tuple(torch.stack(out[n], dim=1) for n in "XCDQ")

    def features(self, k):
        Xw = self.Xw[k][self.feat_px[k]]
        cells = torch.floor(Xw / 0.5).long().cpu().tolist()
        f = torch.stack([torch.randn(self.feat_dim, generator=torch.Generator().manual_seed(
            _stable_seed(self.seed, "cell", *c))) for c in cells]).to(self.dev)
        f = F.normalize(f, dim=-1)
        g = self._gen(k, "feat")
        return F.normalize(f + 0.1 * torch.randn(f.shape, generator=g, device=self.dev) / math.sqrt(self.feat_dim),
                           dim=-1)


def retrieve(words, k, n_best=3, min_thresh=5e-3):
    """Earlier keyframes ranked by the fraction of keyframe k's visual words (quantize ids, (M, a)) they share
    (a bag-of-words stand-in for the ASMK similarity of retrieval_database.py:106-170, which is out of scope);
    the n_best with a score above min_thresh (main.py:121-126: retrieval k, min_thresh)."""
    mine = set(np.asarray(words[k]).reshape(-1).tolist())
    scores = [(len(mine & set(np.asarray(words[i]).reshape(-1).tolist())) / max(len(mine), 1), i) for i in range(k)]
    scores.sort(key=lambda s: (-s[0], s[1]))
    return [i for s, i in scores[:n_best] if s > min_thresh]
