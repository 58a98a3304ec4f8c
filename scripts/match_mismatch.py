"""Census of the fused match's idx / valid mismatches against the oracle.

For every config-size case of tests/test_gpu_configs.py it runs the oracle's match with its intermediates
(O.match_diag: p_new, the truncated p1, conv, the occlusion distance, the LM margins), the fused HIP match (default
radius, and radius 0, whose idx is the kernel's own truncated p1) and the reference iter_proj op on the oracle's own
rays (isolates LM arithmetic from prep), and prints, per case, the mismatch counts and for each mismatched pixel the
facts that classify it. Usage: python scripts/match_mismatch.py [out.json]
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "lightweight-mast3r-slam_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle.oracle as O  # noqa: E402


def cases():
    from m3s.synthetic import make_pair, tum_fr1_intrinsics

    P = make_pair(512, 512, seed=11)
    yield "C1-512x512", P["X"].numpy()[:1], P["X"].numpy()[1:], P["D"].numpy()[:1], P["D"].numpy()[1:], None
    P = make_pair(384, 512, seed=11, K=tum_fr1_intrinsics(384, 512))
    yield "C2-384x512", P["X"].numpy()[:1], P["X"].numpy()[1:], P["D"].numpy()[:1], P["D"].numpy()[1:], None
    P = make_pair(512, 512, seed=12)
    X, D = P["X"].numpy(), P["D"].numpy()
    idx0, _ = O.match(X[:1], X[1:], D[:1], D[1:])
    init = idx0.copy()
    init[:, ::7] = np.clip(init[:, ::7] + 1, 0, 512 * 512 - 1)
    yield "C1-warm", X[:1], X[1:], D[:1], D[1:], init
    Ps = [make_pair(384, 512, seed=s, K=tum_fr1_intrinsics(384, 512)) for s in (21, 22)]
    X11 = np.concatenate([np.stack((P["X"][0], P["X"][1])) for P in Ps])
    X21 = np.concatenate([np.stack((P["X"][1], P["X"][0])) for P in Ps])
    D11 = np.concatenate([np.stack((P["D"][0], P["D"][1])) for P in Ps])
    D21 = np.concatenate([np.stack((P["D"][1], P["D"][0])) for P in Ps])
    yield "C3-batched", X11, X21, D11, D21, None


def hip_match(X11, X21, D11, D21, init, radius=None):
    from m3s.config import config
    from m3s.matching import match

    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    saved = config["matching"]["radius"]
    if radius is not None:
        config["matching"]["radius"] = radius
    try:
        i, v = match(t(X11), t(X21), t(D11), t(D21), idx_1_to_2_init=None if init is None else t(init))
        torch.cuda.synchronize()
        return i.cpu().numpy(), v.cpu().numpy()[..., 0]
    finally:
        config["matching"]["radius"] = saved


def census(name, X11, X21, D11, D21, init):
    import mast3r_slam_backends as B

    r = O.match_diag(X11, X21, D11, D21, idx_init=init)
    g_idx, g_valid = hip_match(X11, X21, D11, D21, init)
    g_p1, g_valid0 = hip_match(X11, X21, D11, D21, init, radius=0)
    b, h, w = X21.shape[:3]
    rays, pts, p_init = O.prep_for_iter_proj(X11, X21, init)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    pn_op, conv_op = B.iter_proj(t(rays), t(pts), t(p_init), 10, 1e-8, 1e-6)
    pn_op, conv_op = pn_op.cpu().numpy(), conv_op.cpu().numpy()
    r_valid = r["valid"][..., 0]
    out = {"case": name, "pixels": int(r["idx"].size),
           "idx_mismatch": int((g_idx != r["idx"]).sum()), "valid_mismatch": int((g_valid != r_valid).sum()),
           "p1_mismatch": int((g_p1 != r["p1"]).sum()), "valid_r0_equals_valid": bool((g_valid0 == g_valid).all()),
           "op_pnew_maxdiff": float(np.abs(pn_op - r["p_new"]).max()),
           "op_pnew_p99": float(np.percentile(np.abs(pn_op - r["p_new"]), 99.99)),
           "op_conv_mismatch": int((conv_op != r["conv"]).sum()), "pixels_detail": []}
    bad = np.argwhere((g_idx != r["idx"]) | (g_valid != r_valid) | (g_p1 != r["p1"]))
    for bi, n in bad[:200]:
        pn = r["p_new"][bi, n]
        gp = np.array([g_p1[bi, n] % w, g_p1[bi, n] // w])
        rp = np.array([r["p1"][bi, n] % w, r["p1"][bi, n] // w])
        frac_dist = np.abs(pn - np.round(pn))
        out["pixels_detail"].append({
            "b": int(bi), "n": int(n), "idx_diff": bool(g_idx[bi, n] != r["idx"][bi, n]),
            "valid_diff": bool(g_valid[bi, n] != r_valid[bi, n]), "p1_hip": gp.tolist(), "p1_oracle": rp.tolist(),
            "p_new_oracle": pn.tolist(), "p_new_op": pn_op[bi, n].tolist(),
            "int_dist": frac_dist.tolist(), "accept_margin": float(r["accept_margin"][bi, n]),
            "conv_margin": float(r["conv_margin"][bi, n]), "conv": bool(r["conv"][bi, n]),
            "conv_op": bool(conv_op[bi, n]), "d_minus_thresh": float(r["d"][bi, n] - 0.1)})
    return out


def main():
    res = []
    for c in cases():
        o = census(*c)
        print(json.dumps({k: v for k, v in o.items() if k != "pixels_detail"}), flush=True)
        for p in o["pixels_detail"][:40]:
            print("   ", json.dumps(p), flush=True)
        res.append(o)
    if len(sys.argv) > 1:
        json.dump(res, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
