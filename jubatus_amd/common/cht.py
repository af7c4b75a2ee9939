"""Consistent hash table (reference C9: jubatus/server/common/cht.{hpp,cpp}).

Each server registers NUM_VSERV = 8 virtual nodes; vnode i is the ephemeral
node ``<actor>/cht/<md5hex(ip_port[_i])>`` with payload ``ip_port``.
``find(key, n)``: md5(key), lower_bound in the sorted hash list, then n
consecutive vnodes with wrap-around. Like the reference it does not dedupe
physical hosts (a host can be returned twice). MD5 is computed natively
(csrc/native/jb_hash.hpp).
"""
from __future__ import annotations

import bisect

from .._native import native
from .lock_service import LockService
from .membership import build_actor_path, build_loc_str, revert

NUM_VSERV = 8


def make_hash(key: str) -> str:
    return native().md5_hex(key)


class CHT:
    def __init__(self, ls: LockService, type_: str, name: str):
        self.ls, self.type, self.name = ls, type_, name
        self.path = build_actor_path(type_, name) + "/cht"

    @staticmethod
    def setup_cht_dir(ls: LockService, type_: str, name: str) -> None:
        base = build_actor_path(type_, name)
        if not (ls.create(base) and ls.create(base + "/cht")):
            raise RuntimeError(f"Failed to create cht directory: {base}/cht")

    def register_node(self, ip: str, port: int) -> None:
        for i in range(NUM_VSERV):
            hp = f"{self.path}/{make_hash(build_loc_str(ip, port, i))}"
            if not self.ls.create(hp, build_loc_str(ip, port), True):
                raise RuntimeError(f"Failed to register cht node: {hp}")

    def unregister_node(self, ip: str, port: int) -> None:
        for i in range(NUM_VSERV):
            self.ls.remove(f"{self.path}/{make_hash(build_loc_str(ip, port, i))}")

    def find(self, key: str, n: int) -> list[tuple[str, int]]:
        hlist = sorted(self.ls.list(self.path))
        if not hlist:
            raise LookupError(f"failed to fetch list of CHT entry: {key}")
        h = make_hash(key)
        idx = bisect.bisect_left(hlist, h) % len(hlist)
        out = []
        for _ in range(n):
            loc = self.ls.read(f"{self.path}/{hlist[idx]}")
            if loc is None:
                raise LookupError(f"failed to read CHT entry: {self.path}")
            out.append(revert(loc))
            idx = (idx + 1) % len(hlist)
        return out

    def find_host(self, host: str, port: int, n: int) -> list[tuple[str, int]]:
        return self.find(build_loc_str(host, port), n)
