"""Frame / keyframe containers used by the tracker (subset of ``mast3r_slam/frame.py``).

``Frame.update_pointmap`` and ``get_average_conf`` follow ``frame.py:41-108``. The reference's
multi-process ``SharedKeyframes`` (CUDA-IPC buffers behind a Manager lock, ``frame.py:220-327``) is
out of scope; ``Keyframes`` keeps the same indexing surface in one process.
"""
import dataclasses
from typing import Optional

import torch

from m3s.config import config
from m3s.sim3 import Sim3


@dataclasses.dataclass
class Frame:
    frame_id: int
    img_size: tuple  # (H, W) of the pointmap (reference: frame.img.shape[-2:])
    T_WC: Sim3 = None
    X_canon: Optional[torch.Tensor] = None  # (H*W, 3)
    C: Optional[torch.Tensor] = None  # (H*W, 1) confidence sum
    feat: Optional[torch.Tensor] = None
    pos: Optional[torch.Tensor] = None
    N: int = 0
    N_updates: int = 0
    K: Optional[torch.Tensor] = None
    score: Optional[torch.Tensor] = None
    shared: bool = dataclasses.field(default=False, repr=False)  # X_canon / C alias a caller's buffer

    def __post_init__(self):
        if self.T_WC is None:
            self.T_WC = Sim3.Identity(1)

    def get_score(self, C):
        if config["tracking"]["filtering_score"] == "median":
            return torch.median(C)
        return torch.mean(C)

    def update_pointmap(self, X, C, own=False):
        """frame.py:41-105. ``own``: the caller hands over X / C (fresh model outputs nothing else
        writes), so the first assignment keeps them without the reference's clone; the one in-place
        mode (indep_conf) copies them before writing."""
        mode = config["tracking"]["filtering_mode"]
        if self.N == 0:
            if own:
                self.X_canon, self.C, self.shared = X, C, True
            else:
                self.X_canon, self.C, self.shared = X.clone(), C.clone(), False
            self.N, self.N_updates = 1, 1
            if mode == "best_score":
                self.score = self.get_score(C)
            return
        if mode == "first":
            if self.N_updates == 1:
                self.X_canon, self.C, self.N, self.shared = X.clone(), C.clone(), 1, False
        elif mode == "recent":
            self.X_canon, self.C, self.N, self.shared = X.clone(), C.clone(), 1, False
        elif mode == "best_score":
            s = self.get_score(C)
            if s > self.score:
                self.X_canon, self.C, self.N, self.score, self.shared = X.clone(), C.clone(), 1, s, False
        elif mode == "indep_conf":
            if self.shared:  # copy on write: never modify a buffer the frame does not own
                self.X_canon, self.C, self.shared = self.X_canon.clone(), self.C.clone(), False
            m = C > self.C
            self.X_canon[m.repeat(1, 3)] = X[m.repeat(1, 3)]
            self.C[m] = C[m]
            self.N = 1
        elif mode == "weighted_pointmap":
            self.X_canon = ((self.C * self.X_canon) + (C * X)) / (self.C + C)
            self.C = self.C + C
            self.N += 1
            self.shared = False
        elif mode == "weighted_spherical":
            def to_sph(P):
                r = torch.linalg.norm(P, dim=-1, keepdim=True)
                x, y, z = torch.tensor_split(P, 3, dim=-1)
                return torch.cat((r, torch.atan2(y, x), torch.acos(z / r)), dim=-1)

            def to_cart(S):
                r, phi, th = torch.tensor_split(S, 3, dim=-1)
                return torch.cat((r * torch.sin(th) * torch.cos(phi), r * torch.sin(th) * torch.sin(phi),
                                  r * torch.cos(th)), dim=-1)

            S = ((self.C * to_sph(self.X_canon)) + (C * to_sph(X))) / (self.C + C)
            self.X_canon = to_cart(S)
            self.C = self.C + C
            self.N += 1
            self.shared = False
        self.N_updates += 1

    def get_average_conf(self):
        return self.C / self.N if self.C is not None else None


class Keyframes:
    """Single-process keyframe store with the SharedKeyframes indexing surface."""

    def __init__(self):
        self._kfs = []

    def __len__(self):
        return len(self._kfs)

    def __getitem__(self, idx):
        return self._kfs[int(idx)]

    def __setitem__(self, idx, frame):
        self._kfs[int(idx)] = frame

    def append(self, frame):
        self._kfs.append(frame)

    def pop_last(self):
        self._kfs.pop()

    def last_keyframe(self):
        return self._kfs[-1] if self._kfs else None

    def update_T_WCs(self, T_WCs, idx):
        """frame.py SharedKeyframes.update_T_WCs: T_WCs (K',1) or (K',) Sim3 for keyframe ids idx."""
        data = T_WCs.data.reshape(-1, 8)
        for k, i in enumerate(idx.tolist() if torch.is_tensor(idx) else idx):
            self._kfs[int(i)].T_WC = Sim3(data[k].reshape(1, 8).clone())
