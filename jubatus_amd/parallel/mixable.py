"""How a driver takes part in a MIX (the reference's linear_mixable /
push_mixable, jubatus_core EXTERNAL; used at linear_mixer.cpp:438-480 and
push_mixer.cpp:410-472).

A driver supports one of:

* ``mix()`` - a collective over the current process group (dense models on
  the GPU: label/row reconciliation + RCCL all-reduce mean of the HBM
  tables; models/classifier.py);
* ``get_diff() / mix_diff(a, b) / put_diff(m)`` - the reference's
  linear_mixable protocol, run as an all-gather of the msgpack-encoded diffs
  (parallel/wire.py: bytes in a tensor, no pickling), a fold in rank order
  (the reference folds in arrival order, linear_mixer.cpp:455-485; rank
  order makes it deterministic) and a local put_diff. Row engines use their
  own tensor MIX (parallel/row_mix.py).

Model hand-over to an obsolete (newly joined) member: ``broadcast_from(src)``
if the driver has it, else ``pack()`` / ``unpack()`` through a broadcast of
the packed object.
"""
from __future__ import annotations

import time
from typing import Any

from ..framework.mixer import UnsupportedMixables


def _dist():
    import torch.distributed as dist
    return dist


def linear_mix(driver: Any) -> dict:
    """Run one MIX on the current process group; returns stats."""
    t0 = time.perf_counter()
    nbytes = 0
    if hasattr(driver, "mix"):
        nbytes = int(driver.mix() or 0)
    elif hasattr(driver, "get_diff"):
        from . import wire
        diff = driver.get_diff()
        diffs = wire.all_gather(diff)          # msgpack bytes over the collective
        mixed = diffs[0]
        for d in diffs[1:]:
            mixed = driver.mix_diff(mixed, d)
        driver.put_diff(mixed)
        nbytes = len(wire.encode(diff))
    else:
        raise UnsupportedMixables(f"{type(driver).__name__} is not mixable")
    return {"bytes": nbytes, "seconds": time.perf_counter() - t0}


def broadcast_model(driver: Any, src: int, apply: bool = True) -> None:
    """rank ``src`` hands its model to the group; members with apply=False
    (up to date) take part in the collective but keep their own model"""
    dist = _dist()
    if hasattr(driver, "broadcast_from"):
        driver.broadcast_from(src, apply=apply)
        return
    from . import wire
    model = wire.broadcast(driver.pack() if dist.get_rank() == src else None, src)
    if dist.get_rank() != src and apply:
        driver.unpack(model)


def pair_exchange(driver: Any, peer: int) -> None:
    """Symmetric pairwise MIX with one peer (push_mixer's pull/push in both
    directions, push_mixer.cpp:354-388): both sides end with the same model
    (the mean of the two for tensor drivers, mix_diff of the two diffs
    otherwise)."""
    dist = _dist()
    me = dist.get_rank()
    if hasattr(driver, "pair_mix"):
        driver.pair_mix(peer)
        return
    if not hasattr(driver, "get_diff"):
        raise UnsupportedMixables(f"{type(driver).__name__} is not push-mixable")
    from . import wire
    mine = driver.get_diff()
    theirs = wire.exchange(mine, peer)     # lower rank sends first
    mixed = driver.mix_diff(mine, theirs) if me < peer else driver.mix_diff(theirs, mine)
    driver.put_diff(mixed)
