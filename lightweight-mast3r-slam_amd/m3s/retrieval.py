"""Retrieval codebook quantization on the MI355X matrix cores.

The hot op of the reference's ``RetrievalDatabase`` is ``quantize_custom``
(``/root/reference/mast3r_slam/retrieval_database.py:96-105``): the squared distances of the M local
features of a keyframe to every codebook centroid, ``(|q|^2 + |c|^2) - 2 q c^T``, and the indices of
the k nearest (``torch.topk(..., largest=False).indices``). It is called once per query
(``accumulate_scores``, ``:119``, k = ``multiple_assignment`` of ``query_ivf``) and once per database
add without a previous query (``add_to_ivf_custom``, ``:151-153``).

``Codebook`` arranges the centroids once for the matrix cores (the reference moves them to the device
once, ``:20-22``); ``Codebook.quantize`` is one asynchronous C call (``m3s_quantize``: fragment prep
of the queries, the fused GEMM + block top-k kernel, the final merge) on torch's current stream.
``QuantizeMixin`` gives a ``RetrievalDatabase`` subclass the drop-in ``quantize_custom``. The ASMK
inverted-file scoring around it (numpy, ``asmk``) is out of the north-star scope.
"""
import torch

from m3s import _lib


class Codebook:
    """The (C, D) fp32 centroids, prepared once for ``m3s_quantize`` on their device."""

    def __init__(self, centroids, device=None):
        c = torch.as_tensor(centroids)
        device = torch.device(device) if device is not None else (c.device if c.is_cuda else torch.device("cuda"))
        c = c.to(device=device, dtype=torch.float32).contiguous()
        if c.dim() != 2 or c.shape[0] < 1 or c.shape[1] < 1:
            raise RuntimeError(f"codebook: centroids must be (C, D), got {tuple(c.shape)}")
        lib = _lib.load()
        _lib.require_cuda("codebook", c)
        self.centroids = c
        self.C, self.D = int(c.shape[0]), int(c.shape[1])
        nbytes = lib.m3s_codebook_size(self.C, self.D)
        self._buf = torch.empty(nbytes, dtype=torch.uint8, device=device)
        _lib.check(lib.m3s_codebook_prepare(_lib.ptr(c), self.C, self.D, _lib.ptr(self._buf), nbytes,
                                            _lib.stream_ptr(device)))

    @property
    def device(self):
        return self.centroids.device

    def quantize(self, qvecs, k):
        """(M, k) int64 indices of the k nearest centroids per row of ``qvecs`` (ascending distance)."""
        lib = _lib.load()
        q = torch.as_tensor(qvecs)
        if q.dim() != 2 or q.shape[1] != self.D:
            raise RuntimeError(f"quantize: qvecs must be (M, {self.D}), got {tuple(q.shape)}")
        q = q.to(device=self.device, dtype=torch.float32).contiguous()
        M, k = int(q.shape[0]), int(k)
        out = torch.empty((M, k), dtype=torch.int64, device=self.device)
        if M == 0:
            return out
        if not 1 <= k <= 8 or k > self.C:
            raise RuntimeError(f"quantize: multiple_assignment k={k} must be in 1..min(8, C={self.C})")
        nbytes = lib.m3s_quantize_workspace_size(self.C, self.D, M, k)
        st = _lib.stream_ptr(self.device)
        ws = _lib.workspace("quantize", nbytes, self.device, st)
        _lib.check(lib.m3s_quantize(_lib.ptr(self._buf), self.C, self.D, _lib.ptr(q), M, k, _lib.ptr(out),
                                    _lib.ptr(ws), nbytes, st))
        return out


class QuantizeMixin:
    """Mix into the reference's ``RetrievalDatabase`` (before it in the bases) to route
    ``quantize_custom`` through the matrix-core kernel; ``self.centroids`` is used as the codebook."""

    def quantize_custom(self, qvecs, params):
        cb = getattr(self, "_m3s_codebook", None)
        if cb is None or cb.centroids.data_ptr() != self.centroids.data_ptr():
            cb = Codebook(self.centroids)
            self._m3s_codebook = cb
        k = params["quantize"]["multiple_assignment"]
        return cb.quantize(qvecs, k)


def quantize_custom(centroids, qvecs, params):
    """Functional form of ``RetrievalDatabase.quantize_custom`` (prepares the codebook per call)."""
    cb = centroids if isinstance(centroids, Codebook) else Codebook(centroids)
    return cb.quantize(qvecs, params["quantize"]["multiple_assignment"])
