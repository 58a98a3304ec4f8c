"""CPU estimate of the survivor counts of a bound-screened refine (experiment script, no GPU).

For the bench's synthetic 512x512 pair: per level, candidates whose fp64 score s_c satisfies
s_c + B > max(ms, max_c(s_c - B)) survive the screen and need the exact c10::Half chain.
Prints per-level mean survivors per pixel and the mean of the per-wave (32x2 pixels) maximum.
"""
import sys, os
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "lightweight-mast3r-slam_amd"))
from m3s.synthetic import make_pair

H = W = int(sys.argv[1]) if len(sys.argv) > 1 else 512
Bfac = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0125
P = make_pair(H, W, seed=0)
D11 = P["D"][0].half().double().numpy()
D21 = P["D"][1].half().double().numpy().reshape(-1, 24)
u1, v1 = P["flow"]
cu = np.clip(u1.numpy().astype(np.int64).reshape(-1), 0, W - 1)
cv = np.clip(v1.numpy().astype(np.int64).reshape(-1), 0, H - 1)
nq = np.linalg.norm(D21, axis=1)
cmax = np.linalg.norm(D11, axis=2).max()
B = Bfac * nq * cmax + 2.0 ** -19
ms = np.zeros(H * W)
has = np.zeros(H * W, bool)
pix = np.arange(H * W)
tu, tv = pix % W, pix // W
wave = (tv // 8) * (W // 32) * 4 + (tu // 32) * 4 + (tv % 8) // 2  # 32x2 pixel waves
for d in range(8, 0, -1):
    S = np.full((H * W, 49), -np.inf)
    ok = np.zeros((H * W, 49), bool)
    for i in range(7):
        for j in range(7):
            u = cu - 3 * d + i * d
            v = cv - 3 * d + j * d
            m = (u >= 0) & (u < W) & (v >= 0) & (v < H)
            c = i * 7 + j
            ok[:, c] = m
            uu, vv = np.clip(u, 0, W - 1), np.clip(v, 0, H - 1)
            S[:, c] = np.where(m, np.einsum("nk,nk->n", D21, D11[vv, uu]), -np.inf)
    L = np.maximum(ms, np.max(np.where(ok, S - B[:, None], -np.inf), axis=1))
    surv = ok & (S + B[:, None] > ms[:, None]) & (S + B[:, None] >= L[:, None])
    surv[has, 24] = False  # the centre holds the running max exactly
    ns = surv.sum(1)
    wmax = np.zeros(wave.max() + 1)
    np.maximum.at(wmax, wave, ns)
    best = np.argmax(S, axis=1)
    bv = S[pix, best]
    upd = bv > ms
    ms = np.where(upd, bv, ms)
    has |= upd
    cu = np.where(upd, cu - 3 * d + (best // 7) * d, cu)
    cv = np.where(upd, cv - 3 * d + (best % 7) * d, cv)
    print(f"d={d}: survivors/pixel mean {ns.mean():.2f} p99 {np.percentile(ns, 99):.0f}; wave max mean {wmax.mean():.2f} p90 {np.percentile(wmax, 90):.0f}")
