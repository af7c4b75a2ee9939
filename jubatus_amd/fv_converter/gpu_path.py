"""GPU fv_converter fast path (host half).

Decides whether a converter config runs on the GPU and packs its rules
into the device rule tables.

* fast path (``fast_eligible``, csrc/hip/fv_hash.hip + scan.hip, one slot
  per (value, rule)): no filters, no binary or combination rules; every
  string rule is of built-in type ``str`` with global weight ``bin``; every
  num rule is ``num`` or ``log``; key matchers ``*``, prefix, suffix, exact;
* wide rule set (``wide_eligible``, csrc/hip/fv_wide.hip and the native host
  twin csrc/native/jb_hostfv_wide.hpp): adds the ``space`` / ``ngram``
  splitters, tf / log_tf with idf / bm25 global weights and add / mul
  combinations.

``gpu_eligible`` is either; regex matchers, filters and plug-ins keep the
host converter.
"""
from __future__ import annotations

import math
import struct

import numpy as np

from .converter import DatumToFvConverter

_RULE = struct.Struct("<iiiiiifi")  # mirrors jb::GpuRule
_KIND = {"all": 0, "prefix": 1, "suffix": 2, "exact": 3}


def fast_eligible(conv: DatumToFvConverter) -> bool:
    """the fixed-slot fast path (fv_hash.hip / scan.hip): one slot per
    (value, rule), constant string weights"""
    if conv.string_filters or conv.num_filters or conv.binary_rules or conv.combination_rules:
        return False
    for r in conv.string_rules:
        if r.type_name != "str" or r.splitter is not None or r.gw != "bin":
            return False
        if r.matcher.kind not in _KIND:
            return False
    for r in conv.num_rules:
        if r.type_name not in ("num", "log") or r.matcher.kind not in _KIND:
            return False
    return True


class GpuRuleTable:
    """Packed rule tables: (string rules, num rules, byte blob)."""

    def __init__(self, conv: DatumToFvConverter):
        if not fast_eligible(conv):
            raise ValueError("converter config is not eligible for the GPU fast path")
        blob = bytearray()

        def put(b: bytes) -> tuple[int, int]:
            off = len(blob)
            blob.extend(b)
            return off, len(b)

        srows = []
        for r in conv.string_rules:
            mo, ml = put(r.matcher.arg.encode())
            so, sl = put(r.suffix.encode())
            w = {"bin": 1.0, "tf": 1.0, "log_tf": math.log(2.0)}[r.sw]
            srows.append(_RULE.pack(_KIND[r.matcher.kind], mo, ml, so, sl, 0, w, 0))
        nrows = []
        for r in conv.num_rules:
            mo, ml = put(r.matcher.arg.encode())
            so, sl = put(f"@{r.type_name}".encode())
            nrows.append(_RULE.pack(_KIND[r.matcher.kind], mo, ml, so, sl,
                                    1 if r.type_name == "log" else 0, 0.0, 0))
        self.n_srules = len(srows)
        self.n_nrules = len(nrows)
        self.srules = np.frombuffer(b"".join(srows) or b"\0" * _RULE.size, dtype=np.uint8).copy()
        self.nrules = np.frombuffer(b"".join(nrows) or b"\0" * _RULE.size, dtype=np.uint8).copy()
        self.blob = np.frombuffer(bytes(blob) or b"\0", dtype=np.uint8).copy()
        self.H = conv.hash_max_size


# ------------------------------------------------------------- wide rule set
# string rule value_kind = splitter | sample_weight << 4 | global_weight << 8
# (csrc/native/jb_hostfv_wide.hpp, csrc/hip/fv_wide.hip); pad = ngram length
_SPLIT = {"str": 0, "ngram": 1, "space": 2}
_SW = {"bin": 0, "tf": 1, "log_tf": 2}
_GW = {"bin": 0, "idf": 1, "bm25": 2}
_COMB = {"add": 0, "mul": 1}


def wide_eligible(conv: DatumToFvConverter) -> bool:
    """configs the wide native / GPU converter reproduces exactly: str /
    space / ngram splitters, every sample and global weight, num / log num
    types, add / mul combinations; no filters, plug-ins or regex matchers"""
    if conv.string_filters or conv.num_filters or conv.binary_rules:
        return False
    for r in conv.string_rules:
        if r.split_kind not in _SPLIT or r.matcher.kind not in _KIND:
            return False
        if r.split_kind == "ngram" and r.split_n <= 0:
            return False
    for r in conv.num_rules:
        if r.kind not in ("num", "log") or r.matcher.kind not in _KIND:
            return False
    for ml, mr, tname, _ in conv.combination_rules:
        if conv.combination_methods.get(tname) not in _COMB:
            return False
        if ml.kind not in _KIND or mr.kind not in _KIND:
            return False
    return True


class WideRuleTable:
    """Packed wide rule tables: string rules, num rules, combination rules
    (two entries each: left matcher + "/type" suffix + op, right matcher)."""

    def __init__(self, conv: DatumToFvConverter):
        if not wide_eligible(conv):
            raise ValueError("converter config is not eligible for the wide native path")
        blob = bytearray()

        def put(b: bytes) -> tuple[int, int]:
            off = len(blob)
            blob.extend(b)
            return off, len(b)

        srows = []
        for r in conv.string_rules:
            mo, ml = put(r.matcher.arg.encode())
            so, sl = put(r.suffix.encode())
            vk = _SPLIT[r.split_kind] | _SW[r.sw] << 4 | _GW[r.gw] << 8
            srows.append(_RULE.pack(_KIND[r.matcher.kind], mo, ml, so, sl, vk, 0.0, r.split_n))
        nrows = []
        for r in conv.num_rules:
            mo, ml = put(r.matcher.arg.encode())
            so, sl = put(f"@{r.type_name}".encode())
            nrows.append(_RULE.pack(_KIND[r.matcher.kind], mo, ml, so, sl,
                                    1 if r.kind == "log" else 0, 0.0, 0))
        crows = []
        for ml_, mr_, tname, _ in conv.combination_rules:
            lo, ll = put(ml_.arg.encode())
            so, sl = put(f"/{tname}".encode())
            ro, rl = put(mr_.arg.encode())
            crows.append(_RULE.pack(_KIND[ml_.kind], lo, ll, so, sl,
                                    _COMB[conv.combination_methods[tname]], 0.0, 0))
            crows.append(_RULE.pack(_KIND[mr_.kind], ro, rl, 0, 0, 0, 0.0, 0))
        self.n_srules = len(srows)
        self.n_nrules = len(nrows)
        self.n_crules = len(crows) // 2
        self.srules = np.frombuffer(b"".join(srows) or b"\0" * _RULE.size, dtype=np.uint8).copy()
        self.nrules = np.frombuffer(b"".join(nrows) or b"\0" * _RULE.size, dtype=np.uint8).copy()
        self.crules = np.frombuffer(b"".join(crows) or b"\0" * _RULE.size, dtype=np.uint8).copy()
        self.blob = np.frombuffer(bytes(blob) or b"\0", dtype=np.uint8).copy()
        self.H = conv.hash_max_size
        self.global_weights = conv.uses_global_weight


def gpu_eligible(conv: DatumToFvConverter) -> bool:
    """the GPU converts this config: the fixed-slot fast path or the wide
    rule-set kernels (csrc/hip/fv_wide.hip: ngram / space, tf / idf / bm25 with
    the DF table in HBM, combinations)"""
    return fast_eligible(conv) or wide_eligible(conv)
