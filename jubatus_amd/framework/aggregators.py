"""Result aggregators of broadcast / cht proxy calls (reference
jubatus/server/framework/aggregators.hpp:27-63)."""
from __future__ import annotations

from typing import Any, Callable


def merge(a: dict, b: dict) -> dict:
    out = dict(a)
    out.update(b)
    return out


def concat(a: list, b: list) -> list:
    return list(a) + list(b)


def pass_(a: Any, b: Any) -> Any:
    return a


def add(a: Any, b: Any) -> Any:
    return a + b


def all_and(a: bool, b: bool) -> bool:
    return bool(a) and bool(b)


def all_or(a: bool, b: bool) -> bool:
    return bool(a) or bool(b)


AGGREGATORS: dict[str, Callable[[Any, Any], Any]] = {
    "merge": merge, "concat": concat, "pass": pass_, "add": add, "all_and": all_and,
    "all_or": all_or, "ignore": pass_,
}
