"""GPU parity: the bound-screened refine (refine.hip SCREEN path) equals the exact scan bit for bit.

The screen scores every candidate with an fp32 dot of the half operands and runs the exact c10::Half chain
(matching_kernels.cu:47-77 semantics) only on candidates within the rounding bound of the level's best. Its
result must be the sequential scan's: the unscreened tile path (M3S_REFINE_SCREEN=0, itself bit-exact against the
oracle in test_gpu_matching.py) on the same inputs, and the oracle where the inputs allow a direct refine check.
Cases: the bench's synthetic pairs at 512x512 and 512x384, and adversarial descriptors (exact ties everywhere,
few-level quantised values, random non-smooth vectors, subnormal products, norms past the screen's overflow
guard, NaN pixels, zero queries).
"""
import numpy as np
import pytest
import torch

import oracle.oracle as O

pytestmark = pytest.mark.gpu


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _match_both(monkeypatch, X11, X21, D11, D21, idx_init=None):
    from m3s.matching import match

    args = [_dev(X11), _dev(X21), _dev(D11), _dev(D21)]
    if idx_init is not None:
        args.append(_dev(idx_init))
    monkeypatch.setenv("M3S_REFINE_SCREEN", "0")
    idx0, valid0 = match(*args)
    torch.cuda.synchronize()
    idx0, valid0 = idx0.cpu().numpy().copy(), valid0.cpu().numpy().copy()
    monkeypatch.setenv("M3S_REFINE_SCREEN", "1")
    idx1, valid1 = match(*args)
    torch.cuda.synchronize()
    return idx0, valid0, idx1.cpu().numpy(), valid1.cpu().numpy()


def _pair(H, W, seed):
    from m3s.synthetic import make_pair

    P = make_pair(H, W, seed=seed)
    return (P["X"][0].numpy()[None], P["X"][1].numpy()[None], P["D"][0].numpy()[None], P["D"][1].numpy()[None])


@pytest.mark.parametrize("H,W", [(512, 512), (384, 512), (50, 70)])
def test_screen_equals_exact_on_synthetic_pairs(monkeypatch, H, W):
    X11, X21, D11, D21 = _pair(H, W, seed=7)
    idx0, valid0, idx1, valid1 = _match_both(monkeypatch, X11, X21, D11, D21)
    np.testing.assert_array_equal(idx1, idx0)
    np.testing.assert_array_equal(valid1, valid0)


def _adversarial(kind, D11, D21, rng):
    D11, D21 = D11.copy(), D21.copy()
    if kind == "all_ties":  # one descriptor everywhere: every candidate ties, the first in scan order wins
        D11[:] = D11[0, 0, 0]
        D21[:] = D11[0, 0, 0]
    elif kind == "quantised":  # three levels: many exact ties among near-best candidates
        D11 = np.sign(np.round(D11 * 3)) / np.sqrt(24)
        D21 = np.sign(np.round(D21 * 3)) / np.sqrt(24)
    elif kind == "random":  # white (non-smooth) unit descriptors
        D11 = rng.standard_normal(D11.shape).astype(np.float32)
        D11 /= np.linalg.norm(D11, axis=-1, keepdims=True)
        D21 = rng.standard_normal(D21.shape).astype(np.float32)
        D21 /= np.linalg.norm(D21, axis=-1, keepdims=True)
    elif kind == "tiny":  # products in the half subnormal range
        D11 *= 2e-3
        D21 *= 3e-3
    elif kind == "huge":  # |q| cmax past the overflow guard: exact scoring for every candidate, inf ties
        D11 *= 300.0
        D21 *= 300.0
    elif kind == "nan":  # a NaN pixel makes the norm bound NaN: the screen switches off
        D11[0, 5, 7, 3] = np.nan
    elif kind == "zero_queries":  # q = 0: every score is +0 and never beats the running max
        D21[0, ::3] = 0.0
    return D11.astype(np.float32), D21.astype(np.float32)


@pytest.mark.parametrize("kind", ["all_ties", "quantised", "random", "tiny", "huge", "nan", "zero_queries"])
def test_screen_equals_exact_adversarial(monkeypatch, kind):
    rng = np.random.default_rng(11)
    X11, X21, D11, D21 = _pair(96, 128, seed=3)
    D11, D21 = _adversarial(kind, D11, D21, rng)
    idx0, valid0, idx1, valid1 = _match_both(monkeypatch, X11, X21, D11, D21)
    np.testing.assert_array_equal(idx1, idx0)
    np.testing.assert_array_equal(valid1, valid0)


@pytest.mark.parametrize("kind", ["quantised", "random", "tiny"])
def test_screen_matches_oracle_refine(monkeypatch, kind):
    """Direct oracle check of the refine stage: with radius 3 / dilation 5 the fused idx equals the oracle's
    refine (c10::Half restatement) started from the GPU's own projection (radius 0 gives p1 = idx exactly)."""
    from m3s.config import config
    from m3s.matching import match

    rng = np.random.default_rng(5)
    X11, X21, D11, D21 = _pair(64, 96, seed=9)
    D11, D21 = _adversarial(kind, D11, D21, rng)
    H, W = 64, 96
    config["matching"]["radius"] = 0
    idx_p, _ = match(_dev(X11), _dev(X21), _dev(D11), _dev(D21))
    lin = idx_p.cpu().numpy().reshape(1, -1)
    p1 = np.stack((lin % W, lin // W), -1).astype(np.int64)
    config["matching"]["radius"] = 3
    monkeypatch.setenv("M3S_REFINE_SCREEN", "1")
    idx, _ = match(_dev(X11), _dev(X21), _dev(D11), _dev(D21))
    ref = O.refine_matches(O.to_half_bits(D11), O.to_half_bits(D21.reshape(1, H * W, 24)), p1, 3, 5)
    ref_lin = ref[..., 0] + W * ref[..., 1]
    np.testing.assert_array_equal(idx.cpu().numpy().reshape(1, -1), ref_lin)
