"""push_mixer family: pairwise (gossip) MIX schedules (reference C24:
jubatus/server/framework/mixer/{push_mixer,random_mixer,broadcast_mixer,skip_mixer}.hpp).

Reference: each node picks candidate peers (filter_candidates) and runs a
symmetric pull/push exchange with each, over msgpack-RPC, with no lock
(push_mixer.cpp:335-408). Here the exchanges are point-to-point
send/recv on the cluster process group (RCCL p2p over xGMI on GPUs), with a
schedule every rank derives identically from (epoch, mix round):

* random_mixer    one random perfect matching of the ranks per round
                  (an odd rank out skips the round)
* broadcast_mixer every pair, in a round-robin tournament order
* skip_mixer      recursive doubling: strides N/2, N/4, ..., 1
                  (skip_mixer.hpp:46-57); for N a power of two, pairwise
                  averaging along this butterfly yields the exact mean

The trigger agreement is the same as linear_mixer (one all-reduce per tick).
"""
from __future__ import annotations

import random

from .linear_mixer import CollectiveMixer
from .mixable import pair_exchange
from ..utils import fault, trace


def skip_strides(n: int) -> list[int]:
    """N/2, N/4, ..., 1 (reference skip_mixer.hpp:46-57 picks the peers at
    these distances from self)."""
    out = []
    s = n // 2
    while s >= 1:
        out.append(s)
        s //= 2
    return out


def skip_peers(rank: int, n: int) -> list[int]:
    """Peers of ``rank`` per stride, butterfly pairing (rank xor stride for
    powers of two; the +stride ring peer otherwise)."""
    peers = []
    for s in skip_strides(n):
        if n & (n - 1) == 0:
            peers.append(rank ^ s)
        else:
            peers.append((rank + s) % n)
    return peers


def random_matching(n: int, seed: int) -> dict[int, int]:
    order = list(range(n))
    random.Random(seed).shuffle(order)
    m = {}
    for i in range(0, n - 1, 2):
        a, b = order[i], order[i + 1]
        m[a], m[b] = b, a
    return m


def round_robin(n: int) -> list[dict[int, int]]:
    """Tournament rounds covering every pair once (circle method)."""
    players = list(range(n)) + ([None] if n % 2 else [])
    k = len(players)
    rounds = []
    for _ in range(k - 1):
        m = {}
        for i in range(k // 2):
            a, b = players[i], players[k - 1 - i]
            if a is not None and b is not None:
                m[a], m[b] = b, a
        rounds.append(m)
        players = [players[0]] + [players[-1]] + players[1:-1]
    return rounds


class PushMixer(CollectiveMixer):
    def __init__(self, strategy: str, argv, coord, rw_mutex, server_type: str,
                 protocol_version: int = 1, backend: str | None = None):
        super().__init__(argv, coord, rw_mutex, server_type, protocol_version, backend)
        if strategy not in ("random_mixer", "broadcast_mixer", "skip_mixer"):
            raise ValueError(f"unknown push mixer: {strategy}")
        self.kind = strategy

    def schedule(self, rank: int, n: int, round_no: int) -> list[int]:
        if n <= 1:
            return []
        if self.kind == "random_mixer":
            peer = random_matching(n, seed=(self.group.epoch << 20) ^ round_no).get(rank)
            return [] if peer is None else [peer]
        if self.kind == "broadcast_mixer":
            return [r[rank] for r in round_robin(n) if rank in r]
        # skip_mixer: strides that pair up symmetrically
        if n & (n - 1) == 0:
            return skip_peers(rank, n)
        # non power of two: fall back to the tournament restricted to log2 rounds
        rounds = round_robin(n)
        return [r[rank] for r in rounds[:max(1, len(skip_strides(n)))] if rank in r]

    def mix_once(self) -> dict:
        import time
        t0 = time.perf_counter()
        g = self.group
        for peer in self.schedule(g.rank, g.world, getattr(self, "round_no", self.mix_count)):
            fault.on_mix("pair")
            with trace.span("mix.pair"):
                pair_exchange(self.driver, peer)
        return {"bytes": 0, "seconds": time.perf_counter() - t0}
