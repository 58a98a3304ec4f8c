"""The tracker chain on the oracle (test infrastructure, CPU): tracker.py:28-114 with O.match, the fp64 opt_pose_*
restatement and the weighted_pointmap fusion. Shared by the CPU pin against the reference run
(tests/test_oracle.py) and the GPU config-size tests (tests/test_gpu_configs.py)."""
import numpy as np

import oracle.oracle as O

I8 = np.array([0, 0, 0, 0, 0, 0, 1, 1.0])


def oracle_track(P, mode, H, W):
    """tracker.py:28-114 on the oracle: match, Qk, valid_opt, opt_pose_* (fp64), keyframe fusion."""
    X, C, D, Q = (P[k].numpy() for k in ("X", "C", "D", "Q"))
    Xk, Ck, K = P["Xk"].numpy(), P["Ck"].numpy()[:, 0], P["K"].numpy()
    idx, valid = O.match(X[:1], X[1:], D[:1], D[1:])
    i, vm = idx[0], valid[0, :, 0]
    Qk = np.sqrt(Q[0].reshape(-1)[i] * Q[1].reshape(-1))
    v = vm & (C[0].reshape(-1)[i] > 0.0) & (Ck > 0.0) & (Qk > 1.5)
    if mode == "rays":
        Tf, Tr, it = O.track_rays(X[0].reshape(-1, 3)[i], Xk, I8, I8, Qk, v)
    else:
        Xf = O.backproject_constrain(X[0].reshape(1, -1, 3), K, (H, W))[0][i]
        z = O.backproject_constrain(Xk[None], K, (H, W))[0][:, 2]
        u, vv = np.meshgrid(np.arange(W, dtype=np.float32), np.arange(H, dtype=np.float32), indexing="xy")
        vmk = z > 1e-6
        meas = np.stack((u.reshape(-1), vv.reshape(-1), np.log(np.where(vmk, z, 1.0))), -1) * vmk[:, None]
        Tf, Tr, it = O.track_calib(Xf, Xk, I8, I8, Qk, v, meas, vmk, K, (H, W))
    Xkk = O.sim3_act(Tr, X[1].reshape(-1, 3).astype(np.float64))
    Ckf = C[1].reshape(-1, 1).astype(np.float64)
    kX = (Ck[:, None] * Xk + Ckf * Xkk) / (Ck[:, None] + Ckf)
    return idx, valid, Tf, kX, it


def oracle_track_seq(pairs, H, W, mode="calib"):
    """tracker.py:28-114 over a sequence of frames against one keyframe (calib or rays mode) on the oracle: each frame
    matched from the previous frame's idx_f2k (reset on new_kf), started at the previous frame's pose, the keyframe
    fused by weighted_pointmap after every frame (frame.py:74-77: X <- (C X + C' X') / (C + C'), C <- C + C',
    N <- N + 1; the tracker's Ck is the average C / N). Returns [(T_WCf, iters, new_kf)] per frame and the final
    keyframe (X, C, N)."""
    P0 = pairs[0]
    K = P0["K"].numpy()
    kX = P0["Xk"].numpy().astype(np.float64)
    kC = P0["Ck"].numpy()[:, 0].astype(np.float64)
    kN = 1
    T = I8.copy()
    idx_prev = None
    out = []
    u, vv = np.meshgrid(np.arange(W, dtype=np.float32), np.arange(H, dtype=np.float32), indexing="xy")
    for P in pairs:
        X, C, D, Q = (P[k].numpy() for k in ("X", "C", "D", "Q"))
        idx, valid = O.match(X[:1], X[1:], D[:1], D[1:], idx_prev)
        i, vm = idx[0], valid[0, :, 0]
        Qk = np.sqrt(Q[0].reshape(-1)[i] * Q[1].reshape(-1))
        Ck = (kC / kN).astype(np.float32)
        v = vm & (C[0].reshape(-1)[i] > 0.0) & (Ck > 0.0) & (Qk > 1.5)
        Xk32 = kX.astype(np.float32)
        if mode == "rays":
            Tf, Tr, it = O.track_rays(X[0].reshape(-1, 3)[i], Xk32, T, I8, Qk, v)
        else:
            Xf = O.backproject_constrain(X[0].reshape(1, -1, 3), K, (H, W))[0][i]
            z = O.backproject_constrain(Xk32[None], K, (H, W))[0][:, 2]
            vmk = z > 1e-6
            meas = np.stack((u.reshape(-1), vv.reshape(-1), np.log(np.where(vmk, z, 1.0))), -1) * vmk[:, None]
            Tf, Tr, it = O.track_calib(Xf, Xk32, T, I8, Qk, v, meas, vmk, K, (H, W))
        valid_kf = vm & (Qk > 1.5)
        n_unique = np.unique(i[vm]).size
        new_kf = min(valid_kf.sum() / i.size, n_unique / i.size) < 0.333
        Xkk = O.sim3_act(Tr, X[1].reshape(-1, 3).astype(np.float64))
        Cf1 = C[1].reshape(-1).astype(np.float64)
        kX = (kC[:, None] * kX + Cf1[:, None] * Xkk) / (kC + Cf1)[:, None]
        kC = kC + Cf1
        kN += 1
        out.append((Tf, it, bool(new_kf)))
        T = Tf.astype(np.float32).astype(np.float64)  # the next frame starts at this frame's (fp32) pose
        idx_prev = None if new_kf else idx
    return out, kX, kC, kN
