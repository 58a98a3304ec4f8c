"""lietorch-compatible ``Sim3`` on torch tensors (the subset the SLAM glue uses).

lietorch is a CUDA-only third-party dependency of the reference (``pyproject.toml:15``) and is absent
on ROCm, so the tracker / factor graph need this stand-in for ``Identity``, ``inv``, ``*``, ``act``,
``retr``, ``exp``, ``data``, ``matrix`` and indexing (call sites
``tracker.py:98,180,195,212``, ``frame.py:24``, ``global_opt.py:117``). Small pose batches are plain
torch ops on the pose's device; the per-pixel ``act`` of the tracking path runs inside the fused HIP
kernels instead (track.hip), so this class is never on the per-pixel hot path.

Semantics (lietorch's published Sim3): data ``[t(3), q(4, xyzw), s]``, tangent ``[tau, phi, sigma]``,
``retr(a) = Exp(a) * X``; group products re-normalise the quaternion (lietorch's RxSO3 ctor).
"""
import torch

_EPS = 1e-6


def _qmul(a, b):
    ax, ay, az, aw = a.unbind(-1)
    bx, by, bz, bw = b.unbind(-1)
    return torch.stack((aw * bx + ax * bw + ay * bz - az * by,
                        aw * by - ax * bz + ay * bw + az * bx,
                        aw * bz + ax * by - ay * bx + az * bw,
                        aw * bw - ax * bx - ay * by - az * bz), dim=-1)


def _qrot(q, p):
    qv, w = q[..., :3], q[..., 3:4]
    qv = qv.expand_as(p)
    uv = 2.0 * torch.cross(qv, p, dim=-1)
    return p + w * uv + torch.cross(qv, uv, dim=-1)


def _exp(xi):
    tau, phi, sigma = xi[..., :3], xi[..., 3:6], xi[..., 6]
    th2 = (phi * phi).sum(-1)
    th = th2.sqrt()
    one = torch.ones_like(sigma)
    small_q = th2 < _EPS
    ths = torch.where(small_q, one, th)
    imag = torch.where(small_q, 0.5 - th2 / 48.0 + th2 * th2 / 3840.0, torch.sin(0.5 * ths) / ths)
    real = torch.where(small_q, 1.0 - th2 / 8.0 + th2 * th2 / 384.0, torch.cos(0.5 * ths))
    S = torch.exp(sigma)
    s_small, t_small = sigma.abs() < _EPS, th < _EPS
    t2 = torch.where(t_small, one, th2)
    t1 = torch.where(t_small, one, th)
    sg = torch.where(s_small, one, sigma)
    C1 = (S - 1.0) / sg
    a, b, c = S * torch.sin(t1), S * torch.cos(t1), t2 + sg * sg
    A = torch.where(s_small, torch.where(t_small, 0.5 * one, (1.0 - torch.cos(t1)) / t2),
                    torch.where(t_small, ((sg - 1.0) * S + 1.0) / (sg * sg), (a * sg + (1.0 - b) * t1) / (t1 * c)))
    B = torch.where(s_small, torch.where(t_small, one / 6.0, (t1 - torch.sin(t1)) / (t2 * t1)),
                    torch.where(t_small, (S * 0.5 * sg * sg + S - 1.0 - sg * S) / (sg * sg * sg),
                                (C1 - ((b - 1.0) * sg + a * t1) / c) / t2))
    C = torch.where(s_small, one, C1)
    pxt = torch.cross(phi, tau, dim=-1)
    t = C[..., None] * tau + A[..., None] * pxt + B[..., None] * torch.cross(phi, pxt, dim=-1)
    return torch.cat((t, imag[..., None] * phi, real[..., None], S[..., None]), dim=-1)


class Sim3:
    embedded_dim = 8
    manifold_dim = 7

    def __init__(self, data):
        self.data = data.data if isinstance(data, Sim3) else data

    @classmethod
    def Identity(cls, *batch, device=None, dtype=torch.float32):
        d = torch.zeros(*batch, 8, device=device, dtype=dtype)
        d[..., 6] = 1.0
        d[..., 7] = 1.0
        return cls(d)

    @classmethod
    def exp(cls, xi):
        return cls(_exp(xi))

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

    def clone(self):
        return Sim3(self.data.clone())

    def to(self, *args, **kwargs):
        return Sim3(self.data.to(*args, **kwargs))

    def cpu(self):
        return Sim3(self.data.cpu())

    def inv(self):
        t, q, s = self.data[..., :3], self.data[..., 3:7], self.data[..., 7:8]
        qi = torch.cat((-q[..., :3], q[..., 3:]), dim=-1)
        si = 1.0 / s
        return Sim3(torch.cat((-si * _qrot(qi, t), qi, si), dim=-1))

    def __mul__(self, other):
        if not isinstance(other, Sim3):
            return NotImplemented
        t1, q1, s1 = self.data[..., :3], self.data[..., 3:7], self.data[..., 7:8]
        t2, q2, s2 = other.data[..., :3], other.data[..., 3:7], other.data[..., 7:8]
        q = _qmul(q1, q2)
        q = q / torch.linalg.norm(q, dim=-1, keepdim=True)
        return Sim3(torch.cat((t1 + s1 * _qrot(q1, t2), q, s1 * s2), dim=-1))

    def act(self, p):
        t, q, s = self.data[..., :3], self.data[..., 3:7], self.data[..., 7:8]
        while t.dim() < p.dim():
            t, q, s = t.unsqueeze(-2), q.unsqueeze(-2), s.unsqueeze(-2)
        return s * _qrot(q, p) + t

    def retr(self, a):
        return Sim3.exp(a) * self

    def matrix(self):
        t, q, s = self.data[..., :3], self.data[..., 3:7], self.data[..., 7:8]
        eye = torch.eye(3, dtype=self.dtype, device=self.device).expand(*self.shape, 3, 3)
        R = torch.stack([_qrot(q, eye[..., :, k]) for k in range(3)], dim=-1)
        M = torch.zeros(*self.shape, 4, 4, dtype=self.dtype, device=self.device)
        M[..., :3, :3] = s[..., None] * R
        M[..., :3, 3] = t
        M[..., 3, 3] = 1.0
        return M

    def __repr__(self):
        return f"Sim3({self.data})"


class SE3:
    """lietorch-compatible SE3 (data [t(3), q(4) xyzw]) for the reference's trajectory export
    (``lietorch_utils.py:6-13`` ``as_SE3``, ``evaluate.py``, ``visualization.py``): the Sim(3) group
    with the scale fixed to 1."""

    embedded_dim = 7
    manifold_dim = 6

    def __init__(self, data):
        self.data = data.data if isinstance(data, SE3) else data

    def _sim3(self):
        return Sim3(torch.cat((self.data, torch.ones_like(self.data[..., :1])), dim=-1))

    @classmethod
    def _from_sim3(cls, T):
        return cls(T.data[..., :7])

    @classmethod
    def Identity(cls, *batch, device=None, dtype=torch.float32):
        return cls._from_sim3(Sim3.Identity(*batch, device=device, dtype=dtype))

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
        return SE3(self.data[index])

    def __len__(self):
        return self.data.shape[0]

    def clone(self):
        return SE3(self.data.clone())

    def to(self, *args, **kwargs):
        return SE3(self.data.to(*args, **kwargs))

    def cpu(self):
        return SE3(self.data.cpu())

    def inv(self):
        return SE3._from_sim3(self._sim3().inv())

    def __mul__(self, other):
        if not isinstance(other, SE3):
            return NotImplemented
        return SE3._from_sim3(self._sim3() * other._sim3())

    def act(self, p):
        return self._sim3().act(p)

    def translation(self):
        return self.data[..., :3]

    def matrix(self):
        return self._sim3().matrix()

    def __repr__(self):
        return f"SE3({self.data})"


def as_SE3(X):
    """``lietorch_utils.as_SE3`` (``lietorch_utils.py:6-13``): an SE3 passes through; a Sim3 (any batch shape)
    becomes a flat (M,) SE3 of its [t, q] on the host, the scale dropped."""
    if isinstance(X, SE3):
        return X
    d = X.data.detach().cpu()
    t, q, _ = d.reshape(-1, d.shape[-1]).split([3, 4, 1], -1)
    return SE3(torch.cat([t, q], dim=-1))
