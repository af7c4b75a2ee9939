"""The datum type: the unit of input of every engine.

Wire layout (reference: jubatus/client/common/datum.hpp:42-46)::

    [ [[key, string]...], [[key, double]...], [[key, raw]...] ]
"""
from __future__ import annotations

from typing import Any, Iterable

from ..common.exceptions import ArgumentError


class Datum:
    __slots__ = ("string_values", "num_values", "binary_values")

    def __init__(self, values: dict | None = None):
        self.string_values: list[tuple[str, str]] = []
        self.num_values: list[tuple[str, float]] = []
        self.binary_values: list[tuple[str, bytes]] = []
        if values:
            for k, v in values.items():
                self.add(k, v)

    # builder API (mirrors the reference clients: add_string/add_number/add_binary)
    def add(self, key: str, value: Any) -> "Datum":
        if isinstance(value, (bytes, bytearray, memoryview)):
            self.binary_values.append((key, bytes(value)))
        elif isinstance(value, str):
            self.string_values.append((key, value))
        elif isinstance(value, bool):
            self.num_values.append((key, float(value)))
        elif isinstance(value, (int, float)):
            self.num_values.append((key, float(value)))
        else:
            raise ArgumentError(f"unsupported datum value type {type(value)!r} for key {key!r}")
        return self

    add_string = add
    add_number = add
    add_binary = add

    def to_msgpack(self) -> list:
        return [[[k, v] for k, v in self.string_values],
                [[k, float(v)] for k, v in self.num_values],
                [[k, v] for k, v in self.binary_values]]

    @classmethod
    def from_msgpack(cls, obj: Any) -> "Datum":
        d = cls()
        if isinstance(obj, Datum):
            return obj
        if not isinstance(obj, (list, tuple)) or len(obj) < 2:
            raise ArgumentError("datum must be an array [string_values, num_values, binary_values]")
        try:
            return cls._parse(obj, d)
        except (ValueError, TypeError) as e:
            raise ArgumentError(f"malformed datum: {e}") from e

    @classmethod
    def _parse(cls, obj: Any, d: "Datum") -> "Datum":
        for kv in obj[0]:
            k, v = kv
            d.string_values.append((_s(k), _s(v)))
        for kv in obj[1]:
            k, v = kv
            if isinstance(v, bool) or not isinstance(v, (int, float)):
                raise ArgumentError("num_values value must be a number")
            d.num_values.append((_s(k), float(v)))
        if len(obj) >= 3:
            for kv in obj[2]:
                k, v = kv
                d.binary_values.append((_s(k), v if isinstance(v, bytes) else _b(v)))
        return d

    def __eq__(self, other: object) -> bool:
        return isinstance(other, Datum) and self.to_msgpack() == other.to_msgpack()

    def __repr__(self) -> str:
        return (f"Datum(string_values={self.string_values!r}, num_values={self.num_values!r}, "
                f"binary_values={self.binary_values!r})")


def _s(x: Any) -> str:
    if isinstance(x, str):
        return x
    if isinstance(x, (bytes, bytearray)):
        return bytes(x).decode("utf-8", errors="surrogateescape")
    raise ArgumentError(f"expected string, got {type(x)!r}")


def _b(x: Any) -> bytes:
    if isinstance(x, (bytes, bytearray)):
        return bytes(x)
    if isinstance(x, str):
        return x.encode("utf-8", errors="surrogateescape")
    raise ArgumentError(f"expected raw, got {type(x)!r}")


def as_datum(x: Any) -> Datum:
    if isinstance(x, Datum):
        return x
    if isinstance(x, dict):
        return Datum(x)
    return Datum.from_msgpack(x)


def datums(xs: Iterable[Any]) -> list[Datum]:
    return [as_datum(x) for x in xs]
