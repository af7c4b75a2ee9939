"""Model-plane collectives over RCCL (torch.distributed backend "nccl" on ROCm).

The reference MIXes models by a master-driven gather (get_diff) -> fold
(mixable->mix) -> scatter (put_diff) over msgpack-RPC
(jubatus/server/framework/mixer/linear_mixer.cpp:422-544). On one MI355X node
the same averaging is a single all-reduce over xGMI: every rank contributes
its dense hashed tables and receives the cluster mean.

Bucketing: tensors are all-reduced in buckets of ``bucket_bytes`` (default
256 MiB: large messages keep all 7 xGMI links of a rank busy; the models are
HBM-resident, so no staging copy is made - each bucket is a view).
"""
from __future__ import annotations

import hashlib
import os
from typing import Iterable, Sequence

import torch
import torch.distributed as dist

DEFAULT_BUCKET_BYTES = int(os.environ.get("JUBATUS_MIX_BUCKET_BYTES", 256 << 20))


def is_dist() -> bool:
    return dist.is_available() and dist.is_initialized()


def backend(group=None) -> str:
    return str(dist.get_backend(group))


def world() -> int:
    return dist.get_world_size() if is_dist() else 1


def rank() -> int:
    return dist.get_rank() if is_dist() else 0


def _chunks(t: torch.Tensor, bucket_elems: int) -> Iterable[torch.Tensor]:
    flat = t.view(-1)
    for i in range(0, flat.numel(), bucket_elems):
        yield flat[i:i + bucket_elems]


def allreduce_mean_(tensors: Sequence[torch.Tensor], group=None,
                    bucket_bytes: int = DEFAULT_BUCKET_BYTES) -> None:
    """In-place cluster mean of every tensor (sum all-reduce, then 1/N scale
    fused into one elementwise pass per tensor on the HIP stream)."""
    n = dist.get_world_size(group) if is_dist() else 1
    if n == 1:
        return
    from ..ops import hip
    for t in tensors:
        if not t.is_contiguous():
            raise ValueError("mix tensors must be contiguous")
        elems = max(1, bucket_bytes // t.element_size())
        for c in _chunks(t, elems):
            dist.all_reduce(c, op=dist.ReduceOp.SUM, group=group)
        if t.dtype == torch.float32 and t.is_cuda:
            hip.scale_(t, 1.0 / n)
        else:
            t.div_(n)


def allreduce_sum_(tensors: Sequence[torch.Tensor], group=None,
                   bucket_bytes: int = DEFAULT_BUCKET_BYTES) -> None:
    if not is_dist():
        return
    for t in tensors:
        elems = max(1, bucket_bytes // t.element_size())
        for c in _chunks(t, elems):
            dist.all_reduce(c, op=dist.ReduceOp.SUM, group=group)


def allreduce_sum_async(tensors: Sequence[torch.Tensor], group=None,
                        bucket_bytes: int = DEFAULT_BUCKET_BYTES) -> list:
    """Launch in-place SUM all-reduces without blocking; returns the work
    handles. On RCCL the collective runs on the communicator's stream after
    the work already queued on the current stream; ``work.wait()`` makes the
    current stream (not the host) wait for it."""
    if not is_dist():
        return []
    works = []
    for t in tensors:
        elems = max(1, bucket_bytes // t.element_size())
        for c in _chunks(t, elems):
            works.append(dist.all_reduce(c, op=dist.ReduceOp.SUM, group=group, async_op=True))
    return works


def fingerprint(strings: Sequence[str]) -> int:
    h = hashlib.blake2b("\x00".join(strings).encode(), digest_size=7).digest()
    return int.from_bytes(h, "little")


def all_equal(value: int, device: torch.device | None = None, group=None) -> bool:
    """True iff every rank passed the same 56-bit value (two tiny all-reduces)."""
    if not is_dist():
        return True
    dev = device if device is not None else (torch.device("cuda", torch.cuda.current_device())
                                             if dist.get_backend(group) == "nccl"
                                             else torch.device("cpu"))
    t = torch.tensor([value, -value], dtype=torch.int64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return int(t[0]) == value and int(t[1]) == -value


def all_gather_object(obj, group=None) -> list:
    """every rank's (msgpack-encodable) object, no pickling (parallel/wire.py)"""
    from . import wire
    return wire.all_gather(obj, group)
