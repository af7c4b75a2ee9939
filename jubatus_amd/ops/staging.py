"""Small-transfer staging for the latency paths (row engines, LOF).

A request on these paths moves a handful of tiny arrays each way (a query
CSR up, k neighbours down). As separate pageable ``torch.from_numpy(..).to()``
/ ``.cpu()`` copies each is a blocking round trip (~10-20 us); ``Stager``
packs all uploads of a step into ONE async H2D from a pinned ring, and all
downloads into ONE D2H into a pinned buffer followed by one stream sync.

Ring discipline: a ring region is rewritten only after the stream has
passed the copy out of it - ``fetch`` (which syncs) rewinds the ring; a
wrap-around syncs first.
"""
from __future__ import annotations

import numpy as np
import torch

_T = {np.dtype(np.int32): torch.int32, np.dtype(np.int64): torch.int64,
      np.dtype(np.float32): torch.float32, np.dtype(np.float64): torch.float64,
      np.dtype(np.uint8): torch.uint8}


class Stager:
    def __init__(self, device, nbytes: int = 1 << 20):
        self.device = torch.device(device)
        self._alloc_up(nbytes)
        self._down_h = torch.empty(1 << 16, dtype=torch.uint8, pin_memory=True)
        self._down_d = torch.empty(1 << 16, dtype=torch.uint8, device=self.device)
        self._pos = 0

    def _alloc_up(self, n: int) -> None:
        self._up_h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
        self._up_d = torch.empty(n, dtype=torch.uint8, device=self.device)

    def _stream(self):
        return torch.cuda.current_stream(self.device)

    def put(self, *arrays: np.ndarray) -> list[torch.Tensor]:
        """host arrays -> device tensors (same dtype/shape), one async H2D"""
        arrays = [np.ascontiguousarray(a) for a in arrays]
        sizes = [(a.nbytes + 15) // 16 * 16 for a in arrays]
        total = max(16, sum(sizes))
        if self._pos + total > self._up_h.numel():
            self._stream().synchronize()
            self._pos = 0
            if total > self._up_h.numel():
                self._alloc_up(1 << (total - 1).bit_length())
        hb = self._up_h.numpy()
        base = off = self._pos
        spans = []
        for a, sz in zip(arrays, sizes):
            hb[off:off + a.nbytes] = a.view(np.uint8).reshape(-1)
            spans.append((off, a))
            off += sz
        self._up_d[base:off].copy_(self._up_h[base:off], non_blocking=True)
        self._pos = off
        out = []
        for o, a in spans:
            t = self._up_d[o:o + a.nbytes].view(_T[a.dtype])
            out.append(t.view(a.shape) if a.ndim != 1 else t)
        return out

    def fetch(self, *tensors: torch.Tensor) -> list[np.ndarray]:
        """device tensors -> host numpy copies: gathered on the device into
        one buffer, one D2H, one sync"""
        flat = [t.contiguous().view(-1).view(torch.uint8) for t in tensors]
        sizes = [(f.numel() + 15) // 16 * 16 for f in flat]
        total = max(16, sum(sizes))
        if total > self._down_h.numel():
            n = 1 << (total - 1).bit_length()
            self._down_h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
            self._down_d = torch.empty(n, dtype=torch.uint8, device=self.device)
        off = 0
        for f, sz in zip(flat, sizes):
            self._down_d[off:off + f.numel()].copy_(f)
            off += sz
        self._down_h[:off].copy_(self._down_d[:off], non_blocking=True)
        self._stream().synchronize()
        self._pos = 0
        hb = self._down_h.numpy()
        out, off = [], 0
        for t, f, sz in zip(tensors, flat, sizes):
            dt = {torch.int32: np.int32, torch.int64: np.int64, torch.float32: np.float32,
                  torch.float64: np.float64, torch.uint8: np.uint8}[t.dtype]
            out.append(hb[off:off + f.numel()].view(dt).reshape(tuple(t.shape)).copy())
            off += sz
        return out

    def synced(self) -> None:
        """the caller synchronised the stream: the ring may be rewound"""
        self._pos = 0
