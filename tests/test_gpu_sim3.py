"""the lietorch-compatible Sim3 / SE3 surface on device tensors.

Every op the reference glue calls on GPU poses (frame.py, tracker.py, global_opt.py, lietorch_utils.py:6-13) —
Identity, exp, inv, *, act, retr, matrix, indexing/clone, and as_SE3 — run on CUDA tensors and are checked
against the oracle shim (oracle/lietorch_shim.py, torch-CPU) and the fp64 closed forms of oracle/oracle.py
(sim3_mul / sim3_inv / sim3_act / sim3_exp). lietorch itself is absent, so its parity stays unpinned
(SURVEY §8c); these checks pin the class to the group law and to gn_kernels.cu's expSim3.
"""
import numpy as np
import pytest
import torch

import oracle.lietorch_shim as shim
import oracle.oracle as O

pytestmark = pytest.mark.gpu


def _poses(n=32, seed=0):
    g = torch.Generator().manual_seed(seed)
    xi = torch.randn(n, 7, generator=g) * torch.tensor([0.4, 0.4, 0.4, 0.6, 0.6, 0.6, 0.2])
    xi[0] = 0
    xi[1, 3:6] = 1e-5  # small-angle branch
    xi[2, 6] = 1e-8  # |sigma| < EPS branch
    return xi, torch.randn(n, 9, 3, generator=g)


def test_sim3_device_ops_match_shim_and_fp64():
    from m3s.sim3 import Sim3

    xi, p = _poses()
    dxi, dp = xi.cuda(), p.cuda()
    T = Sim3.exp(dxi)
    assert T.device.type == "cuda" and T.shape == (32,) and T.data.dtype == torch.float32
    Ts = shim.Sim3.exp(xi)
    np.testing.assert_allclose(T.data.cpu().numpy(), Ts.data.numpy(), atol=2e-6)
    Td = T.data.cpu().double().numpy()
    for k in range(32):
        np.testing.assert_allclose(Td[k], O.exp_sim3_f32(xi[k].numpy()), atol=2e-6)
    # inv, compose, act against the fp64 closed forms (on the same fp32 inputs)
    U = Sim3.exp(dxi.flip(0) * 0.7)
    Ud = U.data.cpu().double().numpy()
    Ti, TU, act = T.inv().data.cpu().numpy(), (T * U).data.cpu().numpy(), T.act(dp).cpu().numpy()
    for k in range(32):
        np.testing.assert_allclose(Ti[k], O.sim3_inv(Td[k]), atol=1e-5, rtol=1e-5)
        np.testing.assert_allclose(TU[k], O.sim3_mul(Td[k], Ud[k]), atol=1e-5, rtol=1e-5)
        np.testing.assert_allclose(act[k], O.sim3_act(Td[k], p[k].double().numpy()), atol=2e-5, rtol=1e-5)
    np.testing.assert_allclose((T * U).data.cpu().numpy(), (Ts * shim.Sim3(U.data.cpu())).data.numpy(), atol=2e-6)
    # group identities on device
    I = Sim3.Identity(32, device="cuda")
    np.testing.assert_allclose((T.inv() * T).data.cpu().numpy(), I.data.cpu().numpy(), atol=2e-6)
    np.testing.assert_allclose((T * U).act(dp).cpu().numpy(), T.act(U.act(dp)).cpu().numpy(), atol=3e-5)
    # retr = exp(a) * T (left retraction, gn_kernels.cu:392-413)
    a = dxi.flip(0) * 0.3
    np.testing.assert_allclose(T.retr(a).data.cpu().numpy(), (Sim3.exp(a) * T).data.cpu().numpy(), atol=1e-6)
    np.testing.assert_allclose(T.retr(a).data.cpu().numpy(), Ts.retr(a.cpu()).data.numpy(), atol=3e-6)
    # matrix acts like act on homogeneous points
    M = T.matrix()
    assert M.device.type == "cuda" and M.shape == (32, 4, 4)
    ph = torch.cat((dp, torch.ones(32, 9, 1, device="cuda")), -1)
    np.testing.assert_allclose((M[:, None] @ ph[..., None])[..., :3, 0].cpu().numpy(), T.act(dp).cpu().numpy(),
                               atol=3e-5)
    np.testing.assert_allclose(M.cpu().numpy(), Ts.matrix().numpy(), atol=3e-6)
    # indexing / clone / batch shapes the glue uses (frame.py T_WC (1,8) rows, global_opt.py T_WCs[pin:])
    row = T[3:4]
    assert row.shape == (1,) and torch.equal(row.data, T.data[3:4])
    c = T.clone()
    c.data[0, 0] += 1.0
    assert not torch.equal(c.data, T.data)


def test_se3_and_as_se3_on_device():
    from m3s.sim3 import SE3, Sim3, as_SE3

    xi, p = _poses(8, seed=3)
    T = Sim3.exp(xi.cuda())
    S = as_SE3(T)  # lietorch_utils.py:6-13: Sim3 -> host SE3 [t, q], scale dropped
    assert isinstance(S, SE3) and S.data.shape == (8, 7) and S.data.device.type == "cpu"
    assert torch.equal(S.data, T.data.cpu()[:, :7])
    assert as_SE3(S) is S
    T2 = Sim3(T.data.view(8, 1, 8))  # (..., 8) batches flatten
    assert as_SE3(T2).data.shape == (8, 7)
    Sd = SE3(T.data[:, :7])
    unit = Sim3(torch.cat((T.data[:, :7], torch.ones(8, 1, device="cuda")), -1))
    np.testing.assert_allclose(Sd.act(p.cuda()).cpu().numpy(), unit.act(p.cuda()).cpu().numpy(), atol=1e-6)
    np.testing.assert_allclose((Sd.inv() * Sd).data.cpu().numpy(), SE3.Identity(8).data.numpy(), atol=2e-6)
    assert torch.equal(Sd.translation(), T.data[:, :3])
