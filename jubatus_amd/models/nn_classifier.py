"""Nearest-neighbor classifiers: NN (LSH family), cosine, euclidean.

Reference: classifier configs config/classifier/{nn,cosine,euclidean}.json
(jubatus/server/server/classifier_serv.cpp:91-117 builds jubatus_core's
nearest_neighbor_classifier / inverted-index classifiers, EXTERNAL).
Parameters: ``nearest_neighbor_num`` (k), ``local_sensitivity`` (alpha),
for NN also ``method`` (lsh / euclid_lsh / minhash) + ``parameter``
(hash_num), optional ``unlearner`` / ``unlearner_parameter``.

Training stores each example as a row (id = a per-server sequence) tagged
with its label; classification queries the k nearest rows on the row
engine (GPU XOR-popcount / sparse scan kernels, models/similarity.py) and
scores each label by sum exp(-alpha * distance) over its neighbours (NN,
euclidean) or by the summed cosine similarity (cosine). Every known label is
reported (0 when no neighbour carries it). MIX: the versioned rows (row
engine) plus label counts.
"""
from __future__ import annotations

import math
import threading
import uuid
from typing import Any, Sequence

from ..fv_converter.converter import DatumToFvConverter
from ..fv_converter.datum import as_datum
from .row_engine import LSH_METHODS, RowEngine


class NNClassifier:
    def __init__(self, method: str, parameter: dict, converter: DatumToFvConverter, device: Any = None):
        p = dict(parameter or {})
        self.method = method
        self.k = int(p.get("nearest_neighbor_num", 128))
        self.alpha = float(p.get("local_sensitivity", 1.0))
        if self.k <= 0 or self.alpha < 0:
            raise ValueError("nearest_neighbor_num must be positive, local_sensitivity >= 0")
        if method in ("NN", "nearest_neighbor"):
            idx_method = p.get("method", "lsh")
            if idx_method not in LSH_METHODS:
                raise ValueError(f"unknown nearest neighbor method: {idx_method}")
            idx_param = p.get("parameter") or {}
            self.similar = False
        elif method == "cosine":
            idx_method, idx_param, self.similar = "inverted_index", {}, True
        elif method == "euclidean":
            idx_method, idx_param, self.similar = "inverted_index_euclid", {}, False
        else:
            raise ValueError(f"unsupported nn classifier method: {method}")
        self.engine = RowEngine(idx_method, idx_param, converter, device,
                                p.get("unlearner"), p.get("unlearner_parameter"))
        self.device = device
        self.prefix = uuid.uuid4().hex[:8]
        self._lock = threading.RLock()
        self.clear()

    def clear(self) -> None:
        with self._lock:
            self.engine.clear()
            self.row_label: dict[str, str] = {}
            self.labels: dict[str, int] = {}
            self.seq = 0

    # --------------------------------------------------------------- train
    def train(self, data: Sequence[tuple[str, Any]]) -> int:
        with self._lock:
            for label, d in data:
                rid = f"{self.prefix}-{self.seq}"
                self.seq += 1
                self.engine.set_row(rid, as_datum(d))
                self.row_label[rid] = label
                self.labels[label] = self.labels.get(label, 0) + 1
            self._gc()
            return len(data)

    def _gc(self) -> None:
        """drop labels of rows the unlearner evicted"""
        if self.engine.unlearner.kind:
            live = set(self.engine.rows.slot_of)
            for rid in [r for r in self.row_label if r not in live]:
                del self.row_label[rid]

    def _score(self, neighbors: list[tuple[str, float]]) -> dict[str, float]:
        sc = {lab: 0.0 for lab in self.labels}
        for rid, v in neighbors:
            lab = self.row_label.get(rid)
            if lab is None:
                continue
            sc[lab] = sc.get(lab, 0.0) + (v if self.similar else math.exp(-self.alpha * v))
        return sc

    def classify(self, data: Sequence[Any]) -> list[list[tuple[str, float]]]:
        with self._lock:
            out = []
            for d in data:
                nb = self.engine.query_datum(as_datum(d), self.k, self.similar)
                out.append(list(self._score(nb).items()))
            return out

    # -------------------------------------------------------------- labels
    def get_labels(self) -> dict[str, int]:
        with self._lock:
            return dict(self.labels)

    def set_label(self, label: str) -> bool:
        with self._lock:
            if label in self.labels:
                return False
            self.labels[label] = 0
            return True

    def delete_label(self, label: str) -> bool:
        with self._lock:
            if label not in self.labels:
                return False
            for rid in [r for r, lab in self.row_label.items() if lab == label]:
                self.engine.clear_row(rid)
                del self.row_label[rid]
            del self.labels[label]
            return True

    # ----------------------------------------------------------------- MIX
    def get_diff(self) -> dict:
        with self._lock:
            rows = self.engine.get_diff()
            tagged = {rid: self.row_label.get(rid) for rid in rows["rows"]}
            return {"rows": rows, "tags": tagged, "labels": dict(self.labels)}

    @staticmethod
    def mix_diff(a: dict, b: dict) -> dict:
        tags = dict(a["tags"])
        tags.update(b["tags"])
        labels = dict(a["labels"])
        for k, v in b["labels"].items():
            labels[k] = max(labels.get(k, 0), v)
        return {"rows": RowEngine.mix_diff(a["rows"], b["rows"]), "tags": tags, "labels": labels}

    def put_diff(self, mixed: dict) -> bool:
        with self._lock:
            self.engine.put_diff(mixed["rows"])
            for rid, lab in mixed["tags"].items():
                if lab is not None:
                    self.row_label[rid] = lab
            for rid in mixed["rows"]["removed"]:
                self.row_label.pop(rid, None)
            counts: dict[str, int] = {lab: 0 for lab in mixed["labels"]}
            counts.update({lab: 0 for lab in self.labels})
            for lab in self.row_label.values():
                counts[lab] = counts.get(lab, 0) + 1
            self.labels = counts
            return True

    def pack(self) -> dict:
        with self._lock:
            return {"method": self.method, "engine": self.engine.pack(), "row_label": self.row_label,
                    "labels": self.labels, "seq": self.seq}

    def unpack(self, obj: dict) -> None:
        with self._lock:
            self.engine.unpack(obj["engine"])
            self.row_label = dict(obj["row_label"])
            self.labels = {k: int(v) for k, v in obj["labels"].items()}
            self.seq = int(obj["seq"])

    def get_status(self) -> dict[str, str]:
        st = {"method": self.method, "num_labels": str(len(self.labels)),
              "nearest_neighbor_num": str(self.k), "local_sensitivity": str(self.alpha)}
        st.update({f"nn.{k}": v for k, v in self.engine.get_status().items()})
        return st
