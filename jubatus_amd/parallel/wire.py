"""Host objects over tensor collectives, msgpack-encoded (no pickling).

The model plane moves its bulk data as tensors (RCCL over xGMI on GPUs,
gloo on hosts); the small structured parts of a MIX - label lists, a
driver's diff of dicts, a model-handover header - travel here as msgpack
bytes in a uint8 tensor: sizes first (one tiny all-gather), then the padded
payload. The reference ships the same objects as msgpack over its RPC
(linear_mixer.cpp:422-544 get_diff / put_diff), so the encodings agree in
what they can carry: maps, arrays, strings, numbers, bytes (tuples arrive as
lists; numpy scalars and arrays are converted).
"""
from __future__ import annotations

from typing import Any

import msgpack
import numpy as np
import torch
import torch.distributed as dist


def _default(o: Any):
    if isinstance(o, np.generic):
        return o.item()
    if isinstance(o, np.ndarray):
        return o.tolist()
    if isinstance(o, (set, frozenset)):
        return sorted(o)
    raise TypeError(f"cannot encode {type(o).__name__} for the model plane")


def encode(obj: Any) -> bytes:
    return msgpack.packb(obj, use_bin_type=True, default=_default)


def decode(b: bytes) -> Any:
    return msgpack.unpackb(b, raw=False, strict_map_key=False)


def _device(group) -> torch.device:
    if str(dist.get_backend(group)) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def _tensor(b: bytes, n: int, dev: torch.device) -> torch.Tensor:
    t = torch.zeros(max(n, 1), dtype=torch.uint8)
    if b:
        t[:len(b)] = torch.frombuffer(bytearray(b), dtype=torch.uint8)
    return t.to(dev)


def all_gather(obj: Any, group=None) -> list:
    """every rank's object, in rank order"""
    if not (dist.is_available() and dist.is_initialized()):
        return [obj]
    dev = _device(group)
    b = encode(obj)
    n = dist.get_world_size(group)
    size = torch.tensor([len(b)], dtype=torch.int64, device=dev)
    sizes = [torch.empty_like(size) for _ in range(n)]
    dist.all_gather(sizes, size, group=group)
    sizes = [int(s.item()) for s in sizes]
    mx = max(max(sizes), 1)
    bufs = [torch.empty(mx, dtype=torch.uint8, device=dev) for _ in range(n)]
    dist.all_gather(bufs, _tensor(b, mx, dev), group=group)
    return [decode(bytes(t[:s].cpu().numpy())) for t, s in zip(bufs, sizes)]


def broadcast(obj: Any, src: int, group=None) -> Any:
    """rank ``src``'s object on every rank"""
    if not (dist.is_available() and dist.is_initialized()):
        return obj
    dev = _device(group)
    me = dist.get_rank()
    b = encode(obj) if me == src else b""
    size = torch.tensor([len(b)], dtype=torch.int64, device=dev)
    dist.broadcast(size, src=src, group=group)
    n = int(size.item())
    t = _tensor(b, n, dev)
    dist.broadcast(t, src=src, group=group)
    return obj if me == src else decode(bytes(t[:n].cpu().numpy()))


def exchange(obj: Any, peer: int, group=None) -> Any:
    """symmetric swap with one peer (the lower rank sends first)"""
    dev = _device(group)
    me = dist.get_rank()
    b = encode(obj)
    mine = torch.tensor([len(b)], dtype=torch.int64, device=dev)
    theirs = torch.empty_like(mine)
    if me < peer:
        dist.send(mine, peer, group=group)
        dist.recv(theirs, peer, group=group)
    else:
        dist.recv(theirs, peer, group=group)
        dist.send(mine, peer, group=group)
    n = int(theirs.item())
    out = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
    data = _tensor(b, len(b), dev)
    if me < peer:
        dist.send(data, peer, group=group)
        dist.recv(out, peer, group=group)
    else:
        dist.recv(out, peer, group=group)
        dist.send(data, peer, group=group)
    return decode(bytes(out[:n].cpu().numpy()))
