"""ORACLE — test infrastructure only.

A torch-CPU restatement of the subset of lietorch's ``Sim3`` that the reference's Python glue calls
(``Identity``, ``inv``, ``*``, ``act``, ``retr``, ``exp``, ``data``, ``matrix``, indexing).  It is
injected as ``sys.modules['lietorch']`` only by ``tests/golden/make_golden.py`` so the reference's
own ``tracker.py`` / ``geometry.py`` / ``global_opt.py`` can run here to produce golden vectors.

lietorch itself is a third-party dependency that is NOT in /root/reference
(``pyproject.toml:15``: ``lietorch @ git+https://github.com/princeton-vl/lietorch.git``, unpinned;
the only pin-like citation is commit 0fa9ce8f… in ``gn_kernels.cu:344``).  Its published algorithm
is restated here:

* data layout ``[t(3), q(4, xyzw), s]``; tangent layout ``[tau(3), phi(3), sigma]``;
* ``act(p) = s * R(q) p + t``; ``a * b = (q_a q_b, s_a s_b, t_a + s_a R_a t_b)`` with the product
  quaternion re-normalised (lietorch's RxSO3 constructor normalises — unverifiable here, recorded
  as parity hazard a-notes 11 in SURVEY.md);
* ``inv = (q^-1, 1/s, -(1/s) R^-1 t)``;
* ``exp`` = SO3 exp (Taylor below ``theta^2 < 1e-6``) with the Sim3 ``W = C I + A Phi + B Phi^2``
  (same closed form the reference restates in ``gn_kernels.cu:323-390``);
* ``retr(a) = exp(a) * self`` (left retraction, as ``gn_kernels.cu:392-413``).

Parity of this shim against lietorch itself is unpinned (no lietorch test vectors exist here).
"""
import torch

_EPS = 1e-6


def _quat_mul(a, b):
    ax, ay, az, aw = a.unbind(-1)
    bx, by, bz, bw = b.unbind(-1)
    return torch.stack(
        (
            aw * bx + ax * bw + ay * bz - az * by,
            aw * by - ax * bz + ay * bw + az * bx,
            aw * bz + ax * by - ay * bx + az * bw,
            aw * bw - ax * bx - ay * by - az * bz,
        ),
        dim=-1,
    )


def _quat_rot(q, p):
    qv = q[..., :3]
    w = q[..., 3:4]
    uv = 2.0 * torch.cross(qv.expand_as(p), p, dim=-1)
    return p + w * uv + torch.cross(qv.expand_as(uv), uv, dim=-1)


def _exp(xi):
    tau, phi, sigma = xi[..., :3], xi[..., 3:6], xi[..., 6]
    theta_sq = (phi * phi).sum(-1)
    theta = torch.sqrt(theta_sq)
    small = theta_sq < _EPS
    theta_p4 = theta_sq * theta_sq
    safe_theta = torch.where(small, torch.ones_like(theta), theta)
    imag = torch.where(small, 0.5 - theta_sq / 48.0 + theta_p4 / 3840.0, torch.sin(0.5 * safe_theta) / safe_theta)
    real = torch.where(small, 1.0 - theta_sq / 8.0 + theta_p4 / 384.0, torch.cos(0.5 * safe_theta))
    q = torch.cat((imag[..., None] * phi, real[..., None]), dim=-1)
    scale = torch.exp(sigma)

    s_small = sigma.abs() < _EPS
    t_small = theta < _EPS
    one = torch.ones_like(sigma)
    th2 = torch.where(t_small, one, theta_sq)
    th = torch.where(t_small, one, theta)
    sg = torch.where(s_small, one, sigma)
    A0 = torch.where(t_small, 0.5 * one, (1.0 - torch.cos(th)) / th2)
    B0 = torch.where(t_small, one / 6.0, (th - torch.sin(th)) / (th2 * th))
    C1 = (scale - 1.0) / sg
    sg2 = sg * sg
    A1s = ((sg - 1.0) * scale + 1.0) / sg2
    B1s = (scale * 0.5 * sg2 + scale - 1.0 - sg * scale) / (sg2 * sg)
    a = scale * torch.sin(th)
    b = scale * torch.cos(th)
    c = th2 + sg2
    A1 = (a * sg + (1.0 - b) * th) / (th * c)
    B1 = (C1 - ((b - 1.0) * sg + a * th) / c) / th2
    A = torch.where(s_small, A0, torch.where(t_small, A1s, A1))
    B = torch.where(s_small, B0, torch.where(t_small, B1s, B1))
    C = torch.where(s_small, one, C1)
    pxt = torch.cross(phi, tau, dim=-1)
    ppxt = torch.cross(phi, pxt, dim=-1)
    t = C[..., None] * tau + A[..., None] * pxt + B[..., None] * ppxt
    return torch.cat((t, q, scale[..., None]), dim=-1)


class Sim3:
    embedded_dim = 8
    manifold_dim = 7

    def __init__(self, data):
        if isinstance(data, Sim3):
            data = data.data
        self.data = data

    # --- constructors ---
    @classmethod
    def Identity(cls, *batch, device=None, dtype=torch.float32):
        d = torch.zeros(*batch, 8, device=device, dtype=dtype)
        d[..., 6] = 1.0
        d[..., 7] = 1.0
        return cls(d)

    @classmethod
    def exp(cls, xi):
        return cls(_exp(xi))

    # --- accessors ---
    @property
    def shape(self):
        return self.data.shape[:-1]

    @property
    def device(self):
        return self.data.device

    @property
    def dtype(self):
        return self.data.dtype

    def __getitem__(self, index):
        return Sim3(self.data[index])

    def __len__(self):
        return self.data.shape[0]

    def _split(self):
        return self.data[..., :3], self.data[..., 3:7], self.data[..., 7:8]

    # --- group ops ---
    def inv(self):
        t, q, s = self._split()
        qi = q * torch.tensor([-1.0, -1.0, -1.0, 1.0], dtype=q.dtype, device=q.device)
        si = 1.0 / s
        ti = -si * _quat_rot(qi, t)
        return Sim3(torch.cat((ti, qi, si), dim=-1))

    def __mul__(self, other):
        if not isinstance(other, Sim3):
            raise TypeError("Sim3 * Sim3 only")
        t1, q1, s1 = self._split()
        t2, q2, s2 = other._split()
        q = _quat_mul(q1, q2)
        q = q / torch.linalg.norm(q, dim=-1, keepdim=True)
        t = t1 + s1 * _quat_rot(q1, t2)
        return Sim3(torch.cat((t, q, s1 * s2), dim=-1))

    def act(self, p):
        t, q, s = self._split()
        while t.dim() < p.dim():
            t, q, s = t.unsqueeze(-2), q.unsqueeze(-2), s.unsqueeze(-2)
        return s * _quat_rot(q, p) + t

    def retr(self, a):
        return Sim3.exp(a) * self

    def matrix(self):
        t, q, s = self._split()
        eye = torch.eye(3, dtype=self.data.dtype, device=self.data.device).expand(*self.shape, 3, 3)
        R = torch.stack([_quat_rot(q, eye[..., :, k]) for k in range(3)], dim=-1)
        M = torch.zeros(*self.shape, 4, 4, dtype=self.data.dtype, device=self.data.device)
        M[..., :3, :3] = s[..., None] * R
        M[..., :3, 3] = t
        M[..., 3, 3] = 1.0
        return M

    def __repr__(self):
        return f"Sim3({self.data})"


class SE3(Sim3):
    pass
