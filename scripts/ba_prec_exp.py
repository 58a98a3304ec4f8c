"""Which fp32 stage of the rays-mode BA rows carries the C4 error? CPU experiment.

Builds the bench's C4 graph (EuRoC MH_02 trajectory, K=256, 320x512, m3s.synthetic.make_traj_graph seed 1, the graph
of tests/test_gpu_configs.py::test_ba_k256_full_resolution_vs_fp64_truth), runs 2 GN iterations with the
linearisation of scripts/ba_prec_lin.c under several stage-precision masks (fp64 assembly + dense Cholesky), and
prints each mask's pose / dx distance from the oracle's fp64 truth (oracle/liboracle_m3s_f64.so).

  gcc -O2 -fopenmp -fPIC -shared -ffp-contract=off scripts/ba_prec_lin.c -o /tmp/libbaprec.so -lm
  python scripts/ba_prec_exp.py [--H 320 --W 512 --K 256] [--masks all,-REL,...]
"""
import argparse
import ctypes
import os
import sys
import time

import numpy as np
import scipy.linalg as sla

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "lightweight-mast3r-slam_amd")]

from oracle import oracle as O  # noqa: E402

BITS = {"POSE": 1, "REL": 2, "MAP": 4, "REC": 8, "NRM": 16, "ERR": 32, "JAC": 64, "WGT": 128, "PROD": 256, "ADJ": 512,
        "RETR": 1024}  # RETR: dx rounded to fp32 and the retraction (expSim3 + compose) in fp32 (host side here)
ALL = sum(BITS.values())


def parse_mask(s):
    if s == "all":
        return ALL
    if s == "none":
        return 0
    m = ALL if s.startswith("-") else 0
    for tok in s.replace("-", " -").replace("+", " +").split():
        if tok.startswith("-"):
            m &= ~BITS[tok[1:]]
        else:
            m |= BITS[tok.lstrip("+")]
    return m


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--H", type=int, default=320)
    ap.add_argument("--W", type=int, default=512)
    ap.add_argument("--K", type=int, default=256)
    ap.add_argument("--iters", type=int, default=2)
    ap.add_argument("--chunk", type=int, default=24576)
    ap.add_argument("--masks", default="none,all,-REL,-MAP,-REC,-NRM,-ERR,-JAC,-WGT,-PROD,-ADJ,-POSE")
    a = ap.parse_args()
    import torch

    from m3s.synthetic import euroc_poses, make_traj_graph

    torch.set_num_threads(8)
    t0 = time.time()
    G = make_traj_graph(euroc_poses(a.K), a.H, a.W, seed=1, device="cpu")
    n = lambda t: np.ascontiguousarray(t.numpy())
    Twc0, Xs, Cs = n(G["Twc0"]), n(G["Xs"]), np.ascontiguousarray(n(G["Cs"])[..., 0])
    ii, jj, idx = n(G["ii"]), n(G["jj"]), n(G["idx"])
    valid = np.ascontiguousarray(n(G["valid"])[..., 0]).astype(np.uint8)
    Q = np.ascontiguousarray(n(G["Q"])[..., 0])
    del G
    K, N = Xs.shape[0], Xs.shape[1]
    E = ii.shape[0]
    print(f"graph K={K} N={N} E={E} built in {time.time() - t0:.1f}s", flush=True)
    sa, sb = 0.003, 10.0
    p = O.ba_params("rays", sa, sb, 0.0, 1.5)
    O.set_threads(8)
    t0 = time.time()
    T_ref, dx_ref, _ = O.gauss_newton_f64("rays", Twc0, Xs, Cs, ii, jj, idx, valid, Q, p, a.iters, 0.0)
    print(f"fp64 truth in {time.time() - t0:.1f}s", flush=True)

    L = ctypes.CDLL("/tmp/libbaprec.so")
    dp, fp, ip, up = (ctypes.POINTER(t) for t in (ctypes.c_double, ctypes.c_float, ctypes.c_int64, ctypes.c_uint8))
    L.prec_lin_rays.argtypes = [ctypes.c_int, dp, fp, fp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ip, ip, ip, up,
                                fp, ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_double, dp, dp]
    P = lambda x, t: x.ctypes.data_as(t)
    u = np.unique(np.concatenate((ii, jj)))
    ie, je = np.searchsorted(u, ii).astype(np.int64), np.searchsorted(u, jj).astype(np.int64)
    L64 = O.lib64()
    L64.m3o_pose_retr.argtypes = [dp, dp, ctypes.c_int, ctypes.c_int]
    L32 = O.lib()
    L32.m3o_pose_retr.argtypes = [fp, fp, ctypes.c_int, ctypes.c_int]
    nopt = K - 1
    nv = nopt * 7
    for ms in a.masks.split(","):
        m = parse_mask(ms)
        T = Twc0.astype(np.float64).copy()
        t0 = time.time()
        for it in range(a.iters):
            Hs = np.zeros((4, E, 49))
            gs = np.zeros((2, E, 7))
            L.prec_lin_rays(m, P(T, dp), P(Xs, fp), P(Cs, fp), N, E, a.chunk, P(ie, ip), P(je, ip), P(idx, ip),
                            P(valid, up), P(Q, fp), sa, sb, 0.0, 1.5, P(Hs, dp), P(gs, dp))
            A = np.zeros((nv, nv))
            b = np.zeros(nv)
            for blk, (rr, cc) in enumerate(((ie, ie), (ie, je), (je, ie), (je, je))):
                for e in range(E):
                    r, c = rr[e] - 1, cc[e] - 1
                    if r >= 0 and c >= 0:
                        A[r * 7:r * 7 + 7, c * 7:c * 7 + 7] += Hs[blk, e].reshape(7, 7)
            for e in range(E):
                if ie[e] >= 1:
                    b[(ie[e] - 1) * 7:(ie[e] - 1) * 7 + 7] += gs[0, e]
                if je[e] >= 1:
                    b[(je[e] - 1) * 7:(je[e] - 1) * 7 + 7] += gs[1, e]
            dx = -sla.cho_solve(sla.cho_factor(A, lower=True), b)
            if m & BITS["RETR"]:
                dxf = dx.astype(np.float32)
                Tf = T.astype(np.float32)
                L32.m3o_pose_retr(P(Tf, fp), P(dxf, fp), K, 1)
                T, dx = Tf.astype(np.float64), dxf.astype(np.float64)
            else:
                L64.m3o_pose_retr(P(T, dp), P(dx, dp), K, 1)
            if m & BITS["POSE"]:  # the poses are stored as float between iterations
                T = T.astype(np.float32).astype(np.float64)
        pe = np.abs(T - T_ref).max()
        de = np.abs(dx.reshape(-1, 7) - dx_ref.reshape(-1, 7)).max()
        print(f"mask {ms:>10s} ({m:4d}): pose err {pe:.3e}  dx err {de:.3e}   [{time.time() - t0:.1f}s]", flush=True)


if __name__ == "__main__":
    main()
