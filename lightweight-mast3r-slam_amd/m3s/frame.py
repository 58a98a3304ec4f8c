"""Frame / keyframe containers used by the tracker (subset of ``mast3r_slam/frame.py``).

``Frame.update_pointmap`` and ``get_average_conf`` follow ``frame.py:41-108``. ``Keyframes`` keeps the
reference store's indexing surface in one process; ``SharedKeyframes`` is the reference's multi-process store
(``frame.py:220-327``: ``share_memory_`` buffers per slot behind a Manager ``RLock``) with the same surface, which
the fused tracker writes its fused keyframe into IN PLACE (``FrameTracker.track``: the fusion kernel stores X / C
and the slot counters straight into the slot) instead of the reference's full-record ``__setitem__`` copy.
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
    # the image fields of the reference Frame (frame.py:14-30), carried by SharedKeyframes records
    img: Optional[torch.Tensor] = None
    uimg: Optional[torch.Tensor] = None
    img_shape: Optional[torch.Tensor] = None
    img_true_shape: Optional[torch.Tensor] = None

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


class SharedKeyframes:
    """The reference's multi-process keyframe store (``frame.py:220-327``), same surface and semantics: per-slot
    ``share_memory_`` buffers (X, C, N, N_updates, T_WC, img, uimg on the host, feat, pos, ...) behind a Manager
    ``RLock``; ``__getitem__`` returns a Frame whose X_canon / C / feat / pos are VIEWS of the slot, ``__setitem__``
    copies a whole record back and marks the slot dirty. ``FrameTracker.track`` recognises the buffers (``slot_rows``)
    and fuses into the slot in place, which leaves img / uimg / feat / pos / T_WC untouched (a track changes only
    X, C, N, N_updates and the dirty flag), so the reference's full-record copy at tracker.py:101 is not needed."""

    def __init__(self, manager, h, w, buffer=512, dtype=torch.float32, device="cuda", feat_dim=1024):
        self.lock = manager.RLock()
        self.n_size = manager.Value("i", 0)
        self.h, self.w = h, w
        self.buffer = buffer
        self.dtype = dtype
        self.device = device
        self.feat_dim = feat_dim
        self.num_patches = h * w // (16 * 16)
        z = lambda *shape, dt=dtype, dev=device: torch.zeros(*shape, device=dev, dtype=dt).share_memory_()
        self.dataset_idx = z(buffer, dt=torch.int)
        self.img = z(buffer, 3, h, w)
        self.uimg = z(buffer, h, w, 3, dev="cpu")
        self.img_shape = z(buffer, 1, 2, dt=torch.int)
        self.img_true_shape = z(buffer, 1, 2, dt=torch.int)
        self.T_WC = z(buffer, 1, 8)
        self.X = z(buffer, h * w, 3)
        self.C = z(buffer, h * w, 1)
        self.N = z(buffer, dt=torch.int)
        self.N_updates = z(buffer, dt=torch.int)
        self.feat = z(buffer, 1, self.num_patches, feat_dim)
        self.pos = z(buffer, 1, self.num_patches, 2, dt=torch.long)
        self.is_dirty = z(buffer, 1, dt=torch.bool)
        self.K = z(3, 3)

    def __getitem__(self, idx) -> Frame:
        with self.lock:
            kf = Frame(int(self.dataset_idx[idx]), (self.h, self.w), T_WC=Sim3(self.T_WC[idx]))
            kf.img, kf.uimg = self.img[idx], self.uimg[idx]
            kf.img_shape, kf.img_true_shape = self.img_shape[idx], self.img_true_shape[idx]
            kf.X_canon = self.X[idx]
            kf.C = self.C[idx]
            kf.feat = self.feat[idx]
            kf.pos = self.pos[idx]
            kf.N = int(self.N[idx])
            kf.N_updates = int(self.N_updates[idx])
            kf.shared = True  # the slot's buffers: update_pointmap copies before any in-place write
            if config["use_calib"]:
                kf.K = self.K
            return kf

    def __setitem__(self, idx, value: Frame) -> None:
        with self.lock:
            self.n_size.value = max(idx + 1, self.n_size.value)
            self.dataset_idx[idx] = value.frame_id
            if value.img is not None:
                self.img[idx] = value.img
            if value.uimg is not None:
                self.uimg[idx] = value.uimg
            if value.img_shape is not None:
                self.img_shape[idx] = value.img_shape
            if value.img_true_shape is not None:
                self.img_true_shape[idx] = value.img_true_shape
            self.T_WC[idx] = value.T_WC.data.reshape(1, 8)
            self.X[idx] = value.X_canon.reshape(-1, 3)
            self.C[idx] = value.C.reshape(-1, 1)
            if value.feat is not None:
                self.feat[idx] = value.feat
            if value.pos is not None:
                self.pos[idx] = value.pos
            self.N[idx] = value.N
            self.N_updates[idx] = value.N_updates
            self.is_dirty[idx] = True
            return idx

    def __len__(self):
        with self.lock:
            return self.n_size.value

    def append(self, value: Frame):
        with self.lock:
            self[self.n_size.value] = value

    def pop_last(self):
        with self.lock:
            self.n_size.value -= 1

    def last_keyframe(self) -> Optional[Frame]:
        with self.lock:
            if self.n_size.value == 0:
                return None
            return self[self.n_size.value - 1]

    def update_T_WCs(self, T_WCs, idx) -> None:
        with self.lock:
            self.T_WC[idx] = T_WCs.data.reshape(-1, 1, 8)

    def get_dirty_idx(self):
        with self.lock:
            idx = torch.where(self.is_dirty)[0]
            self.is_dirty[:] = False
            return idx

    def set_intrinsics(self, K):
        assert config["use_calib"]
        with self.lock:
            self.K[:] = K

    def get_intrinsics(self):
        assert config["use_calib"]
        with self.lock:
            return self.K


_SLOT_BUFFERS = ("dataset_idx", "img", "uimg", "img_shape", "img_true_shape", "T_WC", "X", "C", "N", "N_updates",
                 "feat", "pos", "is_dirty", "K")


def slot_frame(store, idx):
    """store[idx] of a buffer-backed keyframe store (this module's SharedKeyframes or the reference's,
    frame.py:248-267) for a caller that already holds store.lock: the same record of slot views, with the three
    scalar reads (dataset_idx, N, N_updates: int(...) on device tensors, one synchronising D2H copy each in
    __getitem__) done as ONE copy, and without __getitem__'s own (nested, one Manager round trip per acquire and
    release) lock hold. None when the store is not buffer-backed."""
    if not all(torch.is_tensor(getattr(store, a, None)) for a in _SLOT_BUFFERS):
        return None
    if not all(getattr(store, a).dtype == torch.int32 for a in ("dataset_idx", "N", "N_updates")):
        return None
    fid, n, nu = torch.stack((store.dataset_idx[idx], store.N[idx], store.N_updates[idx])).tolist()
    kf = Frame(fid, (store.h, store.w), T_WC=Sim3(store.T_WC[idx]))
    kf.img, kf.uimg = store.img[idx], store.uimg[idx]
    kf.img_shape, kf.img_true_shape = store.img_shape[idx], store.img_true_shape[idx]
    kf.X_canon, kf.C = store.X[idx], store.C[idx]
    kf.feat, kf.pos = store.feat[idx], store.pos[idx]
    kf.N, kf.N_updates = n, nu
    kf.shared = True
    if config["use_calib"]:
        kf.K = store.K
    return kf


def slot_rows(store, keyframe, idx):
    """(X row, C row, N, N_updates, is_dirty) device views of slot idx of a buffer-backed keyframe store (this
    module's SharedKeyframes or the reference's, frame.py:220-245) when `keyframe` is that slot's record (its X_canon
    / C are the slot's own rows), else None."""
    X, C = getattr(store, "X", None), getattr(store, "C", None)
    Nt, Nu, dirty = getattr(store, "N", None), getattr(store, "N_updates", None), getattr(store, "is_dirty", None)
    if not all(torch.is_tensor(t) for t in (X, C, Nt, Nu, dirty)) or not X.is_cuda:
        return None
    if not (0 <= idx < X.shape[0]) or Nt.dtype != torch.int32 or Nu.dtype != torch.int32 or dirty.dtype != torch.bool:
        return None
    Xr, Cr = X[idx], C[idx]
    xk, ck = getattr(keyframe, "X_canon", None), getattr(keyframe, "C", None)
    if xk is None or ck is None or xk.data_ptr() != Xr.data_ptr() or ck.data_ptr() != Cr.data_ptr():
        return None
    if not (Xr.is_contiguous() and Cr.is_contiguous() and Xr.dtype == torch.float32 and Cr.dtype == torch.float32):
        return None
    return Xr, Cr, Nt[idx:idx + 1], Nu[idx:idx + 1], dirty[idx:idx + 1]
