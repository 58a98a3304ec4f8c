"""Window-size statistics of the refine tile kernel's levels (CPU only; sizing study for csrc/refine.hip).

For the synthetic 512x512 pair (bench C1 shape) this runs the oracle's iter_proj, then replays the refine levels
d = 5..1 in numpy fp32 (scores approximate the c10::Half chain: the centre path can differ from the exact kernel on
near-ties, which does not matter for window sizes) and reports, per level, the distribution over 32x8 tiles of the
window the kernel's placement rule needs: rows = (max v - min v) + 6d + 1 and cols = (max u - min u) + 6d + 1 over
the tile's inlier centres (within 16 px of the tile's mean initial displacement, refine.hip refine_level).

    python scripts/refine_window_stats.py [H W]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "lightweight-mast3r-slam_amd"))

from oracle import oracle as O  # noqa: E402  (test infrastructure: the reference restatement)
from m3s import synthetic  # noqa: E402

TW, TH = 32, int(os.environ.get("RT_TH", "8"))


def main():
    H, W = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (512, 512)
    p = synthetic.make_pair(H, W, seed=0)
    X = p["X"].numpy()
    D = p["D"].numpy().astype(np.float16).astype(np.float32)
    rays, pts, p_init = O.prep_for_iter_proj(X[:1], X[1:2])
    p_new, _ = O.iter_proj(rays, pts, p_init, 10, 1e-8, 1e-6)
    p1 = p_new.astype(np.int64)[0]  # (N, 2) u, v
    D11 = D[0]
    q = D[1].reshape(H * W, -1)
    cu, cv = p1[:, 0].copy(), p1[:, 1].copy()
    best = np.zeros(H * W, np.float32)
    vv, uu = np.divmod(np.arange(H * W), W)
    ty, tx = vv // TH, uu // TW
    tile = ty * ((W + TW - 1) // TW) + tx
    ntiles = tile.max() + 1
    cnt = np.bincount(tile, minlength=ntiles)
    fu = np.bincount(tile, cu - uu, ntiles) / cnt
    fv = np.bincount(tile, cv - vv, ntiles) / cnt
    fu, fv = np.trunc(fu).astype(np.int64), np.trunc(fv).astype(np.int64)
    print(f"{H}x{W}: {ntiles} tiles")
    for d in range(5, 0, -1):
        inl = (np.abs(cu - uu - fu[tile]) <= 16) & (np.abs(cv - vv - fv[tile]) <= 16)
        big = 1 << 30
        mnu = np.full(ntiles, big)
        mxu = np.full(ntiles, -big)
        mnv = np.full(ntiles, big)
        mxv = np.full(ntiles, -big)
        np.minimum.at(mnu, tile[inl], cu[inl])
        np.maximum.at(mxu, tile[inl], cu[inl])
        np.minimum.at(mnv, tile[inl], cv[inl])
        np.maximum.at(mxv, tile[inl], cv[inl])
        rows = mxv - mnv + 6 * d + 1
        cols = mxu - mnu + 6 * d + 1
        pr = np.percentile(rows, [50, 90, 99, 100])
        pc = np.percentile(cols, [50, 90, 99, 100])
        print(f"d={d}: rows p50/p90/p99/max {pr.astype(int).tolist()}  cols {pc.astype(int).tolist()}  "
              f"non-inlier px {int((~inl).sum())}")
        for rlim, clim in ((17, 48), (26, 48), (20, 64), (40, 64)):
            print(f"      fits rows<={rlim} cols<={clim}: {np.mean((rows <= rlim) & (cols <= clim)) * 100:.1f}% of tiles")
        # deferred lanes of the 40 x 64 window when the cover does not fit, by placement rule: bbox middle (shipped),
        # mean inlier centre, tile centre + flow estimate
        RD = 3 * d
        x_lo, x_hi, y_lo, y_hi = mnu - RD, mxu + RD, mnv - RD, mxv + RD
        cntin = np.bincount(tile[inl], minlength=ntiles).clip(1)
        mu = np.bincount(tile[inl], cu[inl], ntiles) / cntin
        mv = np.bincount(tile[inl], cv[inl], ntiles) / cntin
        tcu = (np.arange(ntiles) % ((W + TW - 1) // TW)) * TW + TW // 2 + fu
        tcv = (np.arange(ntiles) // ((W + TW - 1) // TW)) * TH + TH // 2 + fv
        for name, cx, cy in (("bbox-mid", (x_lo + x_hi) >> 1, (y_lo + y_hi) >> 1),
                             ("mean", np.round(mu).astype(np.int64), np.round(mv).astype(np.int64)),
                             ("flow", tcu, tcv)):
            wx0 = np.where(x_hi - x_lo + 1 <= 64, x_lo, cx - 32)
            wy0 = np.where(y_hi - y_lo + 1 <= 40, y_lo, cy - 20)
            bx = cu - RD - wx0[tile]
            by = cv - RD - wy0[tile]
            lin = (bx >= 0) & (bx + 2 * RD < 64) & (by >= 0) & (by + 2 * RD < 40)
            print(f"      placement {name:8s}: deferred lanes {int((~lin).sum())}")
        # one level (fp32 scores; scan order u outer, v inner; strict '>')
        off = np.arange(-3, 4) * d
        cand_u = np.clip(cu[:, None, None] + off[:, None, None].T.reshape(1, 7, 1), 0, W - 1)
        cand_v = np.clip(cv[:, None, None] + off.reshape(1, 1, 7), 0, H - 1)
        okm = ((cu[:, None, None] + off.reshape(1, 7, 1) >= 0) & (cu[:, None, None] + off.reshape(1, 7, 1) < W)
               & (cv[:, None, None] + off.reshape(1, 1, 7) >= 0) & (cv[:, None, None] + off.reshape(1, 1, 7) < H))
        cand_u = np.broadcast_to(cand_u, (H * W, 7, 7))
        cand_v = np.broadcast_to(cand_v, (H * W, 7, 7))
        s = np.einsum("nijk,nk->nij", D11[cand_v, cand_u], q).reshape(H * W, 49)
        s = np.where(okm.reshape(H * W, 49), s, -np.inf)
        k = np.argmax(s, axis=1)
        m = s[np.arange(H * W), k]
        win = m > best
        best = np.where(win, m, best)
        cu = np.where(win, cu - 3 * d + (k // 7) * d, cu)
        cv = np.where(win, cv - 3 * d + (k % 7) * d, cv)


if __name__ == "__main__":
    main()
