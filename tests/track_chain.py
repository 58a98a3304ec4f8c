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
