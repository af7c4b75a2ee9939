"""datum -> sparse feature vector conversion (host reference path).

Implements the ``converter`` section of every engine config (reference
contract: config/*/*.json; conversion itself lives in jubatus_core,
EXTERNAL, called at jubatus/server/server/classifier_serv.cpp:111 and
jubatus/server/cmd/jubaconv.cpp:91-96).

Feature-name scheme (our own, documented; the GPU fast path in
csrc/hip/fv_hash.hip produces byte-identical names for the subset it
supports)::

    string rule   <key>$<token>@<type>#<sample_weight>/<global_weight>
    num rule      <key>@<type>              (num, log, user types)
                  <key>$<value>@str         (num type "str")
    binary rule   <key>$<token>@<type>      (plugins)
    combination   <left>&<right>/<type>

Feature names are mapped to model indices by ``feature_index`` (FNV-1a/64 +
range reduction into ``hash_max_size``); engines that keep names (weight,
jubaconv) use the names directly.

Supported pieces:
  key matchers   ``*``, ``prefix*``, ``*suffix``, ``/regex/``, exact
  string filters regexp (pattern, replace)
  num filters    add (value), linear_normalization (min, max, truncate),
                 gaussian_normalization (average, standard_deviation),
                 sigmoid_normalization (gain, bias)
  string types   str, space, ngram (char_num), regexp (pattern, group),
                 dynamic (plugin)
  num types      num, log, str, add (value), dynamic (plugin)
  binary types   dynamic (plugin)
  weights        sample: bin, tf, log_tf; global: bin, idf, bm25
  combination    add, mul
"""
from __future__ import annotations

import math
import re
import threading
from collections import OrderedDict
from typing import Any, Callable

from .datum import Datum, as_datum

DEFAULT_HASH_MAX_SIZE = 1 << 20


def device_hash_max_size() -> int:
    """Feature-table height of the GPU linear models (classifier,
    regression) when the configuration gives no ``hash_max_size``: the host
    default 2^20 on every backend, so model files interchange between GPU
    and --cpu servers and mixed members agree on the height.
    JUBATUS_DEVICE_HASH_BITS opts into an HBM-sized table (e.g. 24: AROW at
    64 labels is 8 GiB of W + P on a 288 GB device); feature indices are
    int32, so at most 31 bits. Native twin: csrc/server/jb_server_common.hpp."""
    import os
    bits = 20
    try:
        b = int(os.environ.get("JUBATUS_DEVICE_HASH_BITS", "20"))
        if 10 <= b <= 31:
            bits = b
    except ValueError:
        pass
    return 1 << bits


class ConverterError(ValueError):
    pass


# ------------------------------------------------------------------ matchers
class KeyMatcher:
    __slots__ = ("kind", "arg", "_re", "spec")

    def __init__(self, spec: str):
        self.spec = spec
        self._re = None
        if spec == "*" or spec == "":
            self.kind, self.arg = "all", ""
        elif len(spec) >= 2 and spec.startswith("/") and spec.endswith("/"):
            self.kind, self.arg = "regex", spec[1:-1]
            self._re = re.compile(self.arg)
        elif spec.endswith("*"):
            self.kind, self.arg = "prefix", spec[:-1]
        elif spec.startswith("*"):
            self.kind, self.arg = "suffix", spec[1:]
        else:
            self.kind, self.arg = "exact", spec

    def match(self, key: str) -> bool:
        k = self.kind
        if k == "all":
            return True
        if k == "prefix":
            return key.startswith(self.arg)
        if k == "suffix":
            return key.endswith(self.arg)
        if k == "exact":
            return key == self.arg
        return self._re.search(key) is not None


# ------------------------------------------------------------------ splitters
def _ngram(n: int) -> Callable[[str], list[str]]:
    def split(text: str) -> list[str]:
        if n <= 0:
            raise ConverterError("char_num must be positive")
        return [text[i:i + n] for i in range(0, len(text) - n + 1)]
    return split


def _regexp_splitter(pattern: str, group: int) -> Callable[[str], list[str]]:
    rx = re.compile(pattern)

    def split(text: str) -> list[str]:
        return [m.group(group) for m in rx.finditer(text)]
    return split


def _space(text: str) -> list[str]:
    return [t for t in text.split(" ") if t]


def _params(d: dict) -> dict:
    return {k: v for k, v in d.items() if k != "method"}


class WeightManager:
    """Document-frequency statistics for the idf / bm25 global weights.

    The statistics are keyed by the hashed feature index (``feature_index``
    of the feature name into ``[0, H)``) - the same index space as the
    models - and held as dense int64 arrays: the native host hasher
    (csrc/native/jb_hostfv.hpp) and the GPU fv path (ops/fv_wide.py) update
    and read these very arrays; two names only share statistics when they
    share a model index.

    Mixable: ``get_diff`` / ``put_diff`` exchange the (doc_count, total
    length, df) deltas since the last MIX as sparse (index, count) records.
    """

    BM25_K1 = 1.2
    BM25_B = 0.75

    def __init__(self, H: int = DEFAULT_HASH_MAX_SIZE):
        import numpy as np
        self._np = np
        self._lock = threading.RLock()
        self.H = int(H)
        # [doc_count, total_len, diff_docs, diff_len]
        self.counts = np.zeros(4, np.int64)
        self.df = None           # int64[H], allocated on first use
        self.diff = None         # int64[H]: df delta since the last MIX
        self.device_table = None  # ops/fv_wide.DeviceDf when a GPU path owns a copy

    # ---------------------------------------------------------- storage
    def arrays(self):
        """(df, diff, counts) - allocated on first use"""
        if self.df is None:
            self.df = self._np.zeros(self.H, self._np.int64)
            self.diff = self._np.zeros(self.H, self._np.int64)
        if self.device_table is not None:
            self.device_table.pull(self)
        return self.df, self.diff, self.counts

    # the counts are always current on the host (a device batch updates
    # them there); df / diff may sit in HBM (ops/fv_wide.py DeviceDf)
    @property
    def doc_count(self) -> int:
        return int(self.counts[0])

    @property
    def total_len(self) -> int:
        return int(self.counts[1])

    def update_idx(self, idx: list[int]) -> None:
        """one document whose non-bin-weighted features have these indices
        (duplicates count toward the length, once toward df)"""
        with self._lock:
            df, diff, c = self.arrays()
            c[0] += 1
            c[2] += 1
            c[1] += len(idx)
            c[3] += len(idx)
            for i in set(idx):
                df[i] += 1
                diff[i] += 1
            if self.device_table is not None:
                self.device_table.host_changed()

    def df_of(self, i: int) -> int:
        if self.df is None:
            return 0
        df, _, _ = self.arrays()
        return int(df[i])

    def idf_idx(self, i: int) -> float:
        df = self.df_of(i)
        n = self.doc_count
        if df <= 0 or n <= 0:
            return 0.0
        return math.log(n / df)

    def avg_len(self) -> float:
        n = self.doc_count
        return self.total_len / n if n else 1.0

    def clear(self) -> None:
        with self._lock:
            if self.device_table is not None:
                self.device_table.clear()
            self.counts[:] = 0
            if self.df is not None:
                self.df[:] = 0
                self.diff[:] = 0

    # MIX
    def get_diff(self) -> dict:
        with self._lock:
            df, diff, c = self.arrays()
            nz = self._np.flatnonzero(diff)
            return {"docs": int(c[2]), "len": int(c[3]), "idx": nz.tolist(),
                    "df": diff[nz].tolist()}

    @staticmethod
    def mix(a: dict, b: dict) -> dict:
        acc: dict[int, int] = dict(zip(a["idx"], a["df"]))
        for i, v in zip(b["idx"], b["df"]):
            acc[i] = acc.get(i, 0) + v
        ks = sorted(acc)
        return {"docs": a["docs"] + b["docs"], "len": a["len"] + b["len"], "idx": ks,
                "df": [acc[k] for k in ks]}

    def put_diff(self, mixed: dict) -> None:
        with self._lock:
            np = self._np
            df, diff, c = self.arrays()
            # replace own contribution by the cluster-wide one
            c[0] += mixed["docs"] - c[2]
            c[1] += mixed["len"] - c[3]
            df -= diff
            if mixed["idx"]:
                np.add.at(df, np.asarray(mixed["idx"], np.int64), np.asarray(mixed["df"], np.int64))
            np.maximum(df, 0, out=df)
            diff[:] = 0
            c[2] = c[3] = 0
            if self.device_table is not None:
                self.device_table.host_changed()

    def pack(self) -> list:
        with self._lock:
            c = self.counts
            if self.df is None:
                return [int(c[0]), int(c[1]), {"idx": [], "df": []}]
            df, _, _ = self.arrays()
            nz = self._np.flatnonzero(df)
            return [int(c[0]), int(c[1]), {"idx": nz.tolist(), "df": df[nz].tolist()}]

    def unpack(self, obj: list) -> None:
        from .hashing import feature_index
        with self._lock:
            np = self._np
            self.clear()
            df, diff, c = self.arrays()
            c[0], c[1] = int(obj[0]), int(obj[1])
            tab = obj[2]
            tab = {(k.decode() if isinstance(k, bytes) else k): v for k, v in tab.items()}
            if "idx" in tab and isinstance(tab.get("idx"), list):
                if tab["idx"]:
                    np.add.at(df, np.asarray(tab["idx"], np.int64), np.asarray(tab["df"], np.int64))
            else:   # name-keyed statistics (older models)
                for name, v in tab.items():
                    df[feature_index(name, self.H)] += int(v)
            if self.device_table is not None:
                self.device_table.host_changed()


class _StringRule:
    def __init__(self, matcher, type_name, splitter, sw, gw, split=("str", 0)):
        self.matcher, self.type_name, self.splitter = matcher, type_name, splitter
        self.sw, self.gw = sw, gw
        self.split_kind, self.split_n = split      # str / space / ngram(n) / regexp / dynamic
        self.suffix = f"@{type_name}#{sw}/{gw}"


class _NumRule:
    def __init__(self, matcher, type_name, fn, kind="num"):
        self.matcher, self.type_name, self.fn = matcher, type_name, fn
        self.kind = kind                           # num / log / str / add / dynamic


class DatumToFvConverter:
    SAMPLE_WEIGHTS = ("bin", "tf", "log_tf")
    GLOBAL_WEIGHTS = ("bin", "idf", "bm25")

    def __init__(self, config: dict | None, plugin_loader=None,
                 default_hash_max_size: int | None = None):
        config = dict(config or {})
        self.config = config
        self.hash_max_size = int(config.get("hash_max_size") or default_hash_max_size
                                 or DEFAULT_HASH_MAX_SIZE)
        if self.hash_max_size <= 0:
            raise ConverterError("hash_max_size must be positive")
        self.weights = WeightManager(self.hash_max_size)
        self._plugins = plugin_loader
        self._build(config)

    # ---------------------------------------------------------------- build
    def _plugin(self, kind: str, params: dict):
        if self._plugins is None:
            from .plugin import PluginLoader
            self._plugins = PluginLoader()
        return self._plugins.create(kind, params)

    def _build(self, c: dict) -> None:
        # string filters
        sf_types = {}
        for name, p in (c.get("string_filter_types") or {}).items():
            m = p.get("method")
            if m == "regexp":
                rx = re.compile(p["pattern"])
                rep = p.get("replace", "")
                sf_types[name] = (lambda rx, rep: lambda s: rx.sub(rep, s))(rx, rep)
            elif m == "dynamic":
                sf_types[name] = self._plugin("string_filter", _params(p))
            else:
                raise ConverterError(f"unknown string filter method: {m}")
        self.string_filters = []
        for r in c.get("string_filter_rules") or []:
            if r["type"] not in sf_types:
                raise ConverterError(f"unknown string filter type: {r['type']}")
            self.string_filters.append((KeyMatcher(r["key"]), sf_types[r["type"]], r["suffix"]))
        # num filters
        nf_types = {}
        for name, p in (c.get("num_filter_types") or {}).items():
            m = p.get("method")
            if m == "add":
                v = float(p["value"])
                nf_types[name] = (lambda v: lambda x: x + v)(v)
            elif m == "linear_normalization":
                lo, hi = float(p["min"]), float(p["max"])
                trunc = str(p.get("truncate", "true")).lower() != "false"
                if hi <= lo:
                    raise ConverterError("linear_normalization: max must exceed min")

                def lin(x, lo=lo, hi=hi, trunc=trunc):
                    y = (x - lo) / (hi - lo)
                    return min(1.0, max(0.0, y)) if trunc else y
                nf_types[name] = lin
            elif m == "gaussian_normalization":
                avg, sd = float(p["average"]), float(p["standard_deviation"])
                if sd <= 0:
                    raise ConverterError("gaussian_normalization: standard_deviation must be > 0")
                nf_types[name] = (lambda a, s: lambda x: (x - a) / s)(avg, sd)
            elif m == "sigmoid_normalization":
                gain, bias = float(p["gain"]), float(p["bias"])
                nf_types[name] = (lambda g, b: lambda x: 1.0 / (1.0 + math.exp(-g * (x - b))))(gain, bias)
            elif m == "dynamic":
                nf_types[name] = self._plugin("num_filter", _params(p))
            else:
                raise ConverterError(f"unknown num filter method: {m}")
        self.num_filters = []
        for r in c.get("num_filter_rules") or []:
            if r["type"] not in nf_types:
                raise ConverterError(f"unknown num filter type: {r['type']}")
            self.num_filters.append((KeyMatcher(r["key"]), nf_types[r["type"]], r["suffix"]))
        # string types
        st = {"str": None, "space": _space}
        split_meta = {"str": ("str", 0), "space": ("space", 0)}
        for name, p in (c.get("string_types") or {}).items():
            m = p.get("method")
            if m == "ngram":
                st[name] = _ngram(int(p["char_num"]))
                split_meta[name] = ("ngram", int(p["char_num"]))
            elif m == "regexp":
                st[name] = _regexp_splitter(p["pattern"], int(p.get("group", 0)))
                split_meta[name] = ("regexp", 0)
            elif m == "dynamic":
                st[name] = self._plugin("string_feature", _params(p))
                split_meta[name] = ("dynamic", 0)
            else:
                raise ConverterError(f"unknown string type method: {m}")
        self.string_rules = []
        for r in c.get("string_rules") or []:
            t = r["type"]
            if t not in st:
                raise ConverterError(f"unknown string type: {t}")
            sw = r.get("sample_weight", "bin")
            gw = r.get("global_weight", "bin")
            if sw not in self.SAMPLE_WEIGHTS:
                raise ConverterError(f"unknown sample_weight: {sw}")
            if gw not in self.GLOBAL_WEIGHTS:
                raise ConverterError(f"unknown global_weight: {gw}")
            self.string_rules.append(_StringRule(KeyMatcher(r["key"]), t, st[t], sw, gw,
                                                 split_meta[t]))
        # num types
        nt: dict[str, Any] = {"num": lambda k, x: [(f"{k}@num", x)],
                              "log": lambda k, x: [(f"{k}@log", math.log(max(1.0, x)))],
                              "str": lambda k, x: [(f"{k}${_num_str(x)}@str", 1.0)]}
        num_meta = {"num": "num", "log": "log", "str": "str"}
        for name, p in (c.get("num_types") or {}).items():
            m = p.get("method")
            if m == "add":
                v = float(p["value"])
                nt[name] = (lambda n, v: lambda k, x: [(f"{k}@{n}", x + v)])(name, v)
            elif m == "dynamic":
                plug = self._plugin("num_feature", _params(p))
                nt[name] = (lambda plug: lambda k, x: list(plug(k, x)))(plug)
            elif m == "num":       # a user type is named after itself (key@<type>), as the GPU rules
                nt[name] = (lambda n: lambda k, x: [(f"{k}@{n}", x)])(name)
            elif m == "log":
                nt[name] = (lambda n: lambda k, x: [(f"{k}@{n}", math.log(max(1.0, x)))])(name)
            elif m == "str":
                nt[name] = (lambda n: lambda k, x: [(f"{k}${_num_str(x)}@{n}", 1.0)])(name)
            else:
                raise ConverterError(f"unknown num type method: {m}")
            num_meta[name] = m
        self.num_rules = []
        for r in c.get("num_rules") or []:
            t = r["type"]
            if t not in nt:
                raise ConverterError(f"unknown num type: {t}")
            self.num_rules.append(_NumRule(KeyMatcher(r["key"]), t, nt[t], num_meta[t]))
        # binary types
        bt = {}
        for name, p in (c.get("binary_types") or {}).items():
            if p.get("method") != "dynamic":
                raise ConverterError(f"unknown binary type method: {p.get('method')}")
            bt[name] = self._plugin("binary_feature", _params(p))
        self.binary_rules = []
        for r in c.get("binary_rules") or []:
            if r["type"] not in bt:
                raise ConverterError(f"unknown binary type: {r['type']}")
            self.binary_rules.append((KeyMatcher(r["key"]), r["type"], bt[r["type"]]))
        # combination
        ct = {"add": lambda a, b: a + b, "mul": lambda a, b: a * b}
        self.combination_methods = {"add": "add", "mul": "mul"}
        for name, p in (c.get("combination_types") or {}).items():
            m = p.get("method")
            self.combination_methods[name] = m
            if m in ("add", "mul"):
                ct[name] = ct[m]
            elif m == "dynamic":
                ct[name] = self._plugin("combination_feature", _params(p))
            else:
                raise ConverterError(f"unknown combination method: {m}")
        self.combination_rules = []
        for r in c.get("combination_rules") or []:
            if r["type"] not in ct:
                raise ConverterError(f"unknown combination type: {r['type']}")
            self.combination_rules.append((KeyMatcher(r["key_left"]), KeyMatcher(r["key_right"]),
                                           r["type"], ct[r["type"]]))
        self.uses_global_weight = any(r.gw != "bin" for r in self.string_rules)
        # the common "every number as itself" config (clustering, anomaly,
        # regression defaults): conversion is one comprehension
        self._num_only = (not self.string_filters and not self.num_filters and
                          not self.string_rules and not self.binary_rules and
                          not self.combination_rules and len(self.num_rules) == 1 and
                          self.num_rules[0].matcher.kind == "all" and
                          self.num_rules[0].kind == "num" and self.num_rules[0].type_name == "num")

    # -------------------------------------------------------------- convert
    def _filtered(self, d: Datum) -> tuple[list, list]:
        sv = list(d.string_values)
        for m, f, suffix in self.string_filters:
            for k, v in list(sv):
                if m.match(k):
                    sv.append((k + suffix, f(v)))
        nv = list(d.num_values)
        for m, f, suffix in self.num_filters:
            for k, v in list(nv):
                if m.match(k):
                    nv.append((k + suffix, float(f(v))))
        return sv, nv

    def _string_features(self, sv) -> list[tuple[str, float, str]]:
        """-> (name, sample-weighted value, global weight kind)"""
        out = []
        for k, v in sv:
            for r in self.string_rules:
                if not r.matcher.match(k):
                    continue
                if r.splitter is None:
                    toks = [v]
                else:
                    toks = r.splitter(v)
                counts: "OrderedDict[str, int]" = OrderedDict()
                for t in toks:
                    counts[t] = counts.get(t, 0) + 1
                for t, tf in counts.items():
                    if r.sw == "bin":
                        w = 1.0
                    elif r.sw == "tf":
                        w = float(tf)
                    else:
                        w = math.log(1.0 + tf)
                    out.append((f"{k}${t}{r.suffix}", w, r.gw))
        return out

    def _convert(self, datum: Any, update: bool) -> list[tuple[str, float]]:
        d = as_datum(datum)
        if self._num_only:
            return [(f"{k}@num", x) for k, x in d.num_values]
        sv, nv = self._filtered(d)
        sfeat = self._string_features(sv)
        fv: list[tuple[str, float]] = []
        if self.uses_global_weight:
            from .hashing import feature_index
            H = self.hash_max_size
            gidx = [feature_index(n, H) if gw != "bin" else -1 for n, _, gw in sfeat]
            wm = self.weights
            if update:
                wm.update_idx([i for i in gidx if i >= 0])
            n_docs = wm.doc_count
            avg_len = wm.avg_len()
            doc_len = sum(1 for i in gidx if i >= 0)
            for (name, w, gw), i in zip(sfeat, gidx):
                if gw != "bin":
                    df = wm.df_of(i)
                    idf = math.log(n_docs / df) if df > 0 and n_docs > 0 else 0.0
                    if gw == "idf":
                        w *= idf
                    else:
                        k1, b = WeightManager.BM25_K1, WeightManager.BM25_B
                        w = idf * (w * (k1 + 1)) / (w + k1 * (1 - b + b * doc_len / max(avg_len, 1e-9)))
                fv.append((name, w))
        else:
            fv.extend((name, w) for name, w, _ in sfeat)
        for k, x in nv:
            for r in self.num_rules:
                if r.matcher.match(k):
                    fv.extend(r.fn(k, x))
        for k, v in d.binary_values:
            for m, tname, plug in self.binary_rules:
                if m.match(k):
                    for tok, w in plug(k, v):
                        fv.append((f"{k}${tok}@{tname}", float(w)))
        if self.combination_rules:
            base = list(fv)
            for ml, mr, tname, fn in self.combination_rules:
                for i in range(len(base)):
                    ni, vi = base[i]
                    if not ml.match(ni):
                        continue
                    for j in range(i + 1, len(base)):
                        nj, vj = base[j]
                        if mr.match(nj):
                            fv.append((f"{ni}&{nj}/{tname}", float(fn(vi, vj))))
        return fv

    def convert(self, datum: Any) -> list[tuple[str, float]]:
        return self._convert(datum, update=False)

    def convert_and_update_weight(self, datum: Any) -> list[tuple[str, float]]:
        return self._convert(datum, update=True)

    def hashed(self, fv: list[tuple[str, float]]) -> tuple[list[int], list[float]]:
        from .hashing import feature_index
        H = self.hash_max_size
        return [feature_index(n, H) for n, _ in fv], [float(v) for _, v in fv]


def _num_str(x: float) -> str:
    if float(x).is_integer() and abs(x) < 1e16:
        return str(int(x))
    return format(x, ".17g")
