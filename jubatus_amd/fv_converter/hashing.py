"""Feature hashing shared by the host converter, the native runtime and the
GPU fast path: FNV-1a/64 over the UTF-8 feature name, then a multiply-high
range reduction into ``[0, hash_max_size)``.

Twins: csrc/native/jb_hash.hpp (host C++) and csrc/hip/jb_device.hpp (GPU).
"""
from __future__ import annotations

from functools import lru_cache

_MASK = (1 << 64) - 1
FNV_OFFSET = 0xCBF29CE484222325
FNV_PRIME = 0x100000001B3


def fnv1a64(data: bytes, h: int = FNV_OFFSET) -> int:
    for c in data:
        h ^= c
        h = (h * FNV_PRIME) & _MASK
    return h


def hash_to_index(h: int, H: int) -> int:
    h ^= h >> 29
    h = (h * 0xBF58476D1CE4E5B9) & _MASK
    h ^= h >> 32
    return (h * H) >> 64


@lru_cache(maxsize=1 << 16)
def feature_index(name: str, H: int) -> int:
    return hash_to_index(fnv1a64(name.encode("utf-8", errors="surrogateescape")), H)
