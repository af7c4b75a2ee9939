"""jubaclassifier server glue (reference C28: jubatus/server/server/classifier_serv.cpp).

Config: {"method", "parameter", "converter"} (classifier_serv.cpp:56-65,91-117).
Linear methods (perceptron, PA, PA1, PA2, CW, AROW, NHERD) run on the
hashed-table driver (models/classifier.py); NN / cosine / euclidean run on
the nearest-neighbor classifier (models/nn_classifier.py).

RPC methods (classifier.idl): train, classify, get_labels, set_label, clear,
delete_label; all NOLOCK at the dispatcher with a brief write lock to bump
the update counter (classifier_serv.cpp:131-134).
"""
from __future__ import annotations

import json
import os
import math
import time

from ..common.exceptions import ArgumentError, ConfigNotSet
from ..common.mprpc import name_and_rest, split_params
from ..framework.device import select_device
from ..framework.batching import MicroBatcher, msgpack_array_len
from ..framework.server_base import ServerBase
from ..fv_converter.converter import DatumToFvConverter, device_hash_max_size
from ..fv_converter.datum import Datum
from ..models.classifier import LINEAR_METHODS, LinearClassifier
from ..utils import logger, trace

log = logger.get_logger("classifier")

NN_METHODS = ("NN", "nearest_neighbor", "cosine", "euclidean")


def build_classifier(cfg: dict, device):
    method = cfg.get("method")
    if not isinstance(method, str):
        raise ValueError("config: 'method' is required")
    param = cfg.get("parameter")
    if method in LINEAR_METHODS:
        # HBM-sized feature table on a GPU when the config names no
        # hash_max_size (the native server picks the same height)
        conv = DatumToFvConverter(cfg.get("converter") or {},
                                  default_hash_max_size=device_hash_max_size() if device is not None else None)
        # how concurrent train requests update the model: serial-equivalent by
        # default; JUBATUS_UPDATE_MODE=atomic opts into lock-free streams (the
        # native server reads the same variable)
        mode = os.environ.get("JUBATUS_UPDATE_MODE", "exact")
        # W storage: fp32 (default) or bf16 (JUBATUS_WEIGHT_DTYPE=bf16; GPU only)
        wdt = os.environ.get("JUBATUS_WEIGHT_DTYPE", "fp32")
        return LinearClassifier(method, param, conv, device=device,
                                concurrent_update=mode if mode in ("exact", "atomic", "hogwild") else "exact",
                                weight_dtype=wdt if wdt in ("fp32", "bf16") else "fp32")
    conv = DatumToFvConverter(cfg.get("converter") or {})
    if method in NN_METHODS:
        from ..models.nn_classifier import NNClassifier
        return NNClassifier(method, param or {}, conv, device=device)
    raise ValueError(f"unsupported classifier method: {method}")


def labeled_data(data) -> list[tuple[str, Datum]]:
    if not isinstance(data, list):
        raise ArgumentError("train: data must be a list")
    out = []
    for item in data:
        if not isinstance(item, (list, tuple)) or len(item) != 2 or not isinstance(item[0], str):
            raise ArgumentError("labeled_datum must be [label, datum]")
        out.append((item[0], Datum.from_msgpack(item[1])))
    return out


class ClassifierServ(ServerBase):
    type_name = "classifier"

    def __init__(self, argv, coord=None):
        super().__init__(argv, coord)
        self.clf = None
        self.config = None
        self._train_batcher = self._classify_batcher = None
        self._batch_stats = {"train": [0, 0], "classify": [0, 0]}
        self.device = select_device(argv)

    def check_set_config(self) -> None:
        if self.clf is None:
            raise ConfigNotSet()

    # ------------------------------------------------------------- config
    def set_config(self, config: str) -> None:
        cfg = json.loads(config)
        self.clf = build_classifier(cfg, self.device)
        self._train_batcher = self._classify_batcher = None
        if getattr(self.clf, "gpu", False) and hasattr(self.clf, "train_requests"):
            clf = self.clf

            def train_many(bodies):
                clf.train_requests(list(bodies))       # one launch, one stream per request
                return [max(0, msgpack_array_len(b)) for b in bodies]

            def classify_many(bodies):
                flat = clf.classify_requests(list(bodies))
                out, k = [], 0
                for b in bodies:
                    n = max(0, msgpack_array_len(b))
                    out.append(flat[k:k + n])
                    k += n
                return out
            self._train_batcher = MicroBatcher(train_many)
            self._classify_batcher = MicroBatcher(classify_many)
        self.config = config
        if self.mixer is not None:
            self.mixer.set_driver(self.clf)
        log.info("config loaded: %s", cfg.get("method"))

    def get_config(self) -> str:
        self.check_set_config()
        return self.config

    def get_driver(self):
        self.check_set_config()
        return self.clf

    # ---------------------------------------------------------------- RPC
    def _bump(self) -> None:
        with self.rw_mutex.write():
            self.event_model_updated()

    def train(self, data) -> int:
        self.check_set_config()
        items = labeled_data(data)
        self._bump()
        return self.clf.train(items)

    def raw_train(self, params: bytes) -> int:
        """zero-copy path: the list<labeled_datum> bytes go straight to the
        GPU pipeline (native scan -> pinned staging -> fv_hash -> update)."""
        self.check_set_config()
        parts = split_params(params)
        if len(parts) != 2:
            raise ArgumentError("train: expected 2 arguments")
        self._bump()
        if self._train_batcher is not None:
            try:
                return self._train_batcher.submit(parts[1])
            except TypeError as e:
                raise ArgumentError(str(e)) from e
        if hasattr(self.clf, "train_requests"):
            try:
                return self.clf.train_requests([parts[1]])
            except TypeError as e:
                raise ArgumentError(str(e)) from e
        from ..common.mprpc import unpackb
        return self.clf.train(labeled_data(unpackb(bytes(parts[1]))))

    def classify(self, data) -> list:
        self.check_set_config()
        if not isinstance(data, list):
            raise ArgumentError("classify: data must be a list")
        res = self.clf.classify([Datum.from_msgpack(d) for d in data])
        out = []
        for row in res:
            r = []
            for label, score in row:
                if not math.isfinite(score):
                    log.warning("score is infinite: %s = %s", label, score)
                r.append([label, float(score)])
            out.append(r)
        return out

    def raw_classify(self, params: bytes) -> list:
        """zero-copy classify: the list<datum> bytes go straight to the
        latency path (native hashing + one kernel launch) or the GPU batch
        pipeline, without building Python datums"""
        self.check_set_config()
        if not (hasattr(self.clf, "classify_requests") and getattr(self.clf, "gpu", False)):
            from ..common.mprpc import unpackb
            parts = split_params(params)
            if len(parts) != 2:
                raise ArgumentError("classify: expected 2 arguments")
            return self.classify(unpackb(bytes(parts[1])))
        parts = split_params(params)
        if len(parts) != 2:
            raise ArgumentError("classify: expected 2 arguments")
        try:
            res = self._classify_batcher.submit(parts[1]) if self._classify_batcher is not None \
                else self.clf.classify_requests([parts[1]])
        except TypeError as e:
            raise ArgumentError(str(e)) from e
        for row in res:
            for label, score in row:
                if not math.isfinite(score):
                    log.warning("score is infinite: %s = %s", label, score)
        return res

    # ------------------------------------------------ transport batching
    def batched_methods(self) -> dict:
        """GPU engines: concurrent train / classify RPCs are served in
        batches by the transport (one GPU launch per batch)"""
        if not (getattr(self.clf, "gpu", False) and hasattr(self.clf, "train_requests")):
            return {}
        return {"train": self.batch_train, "classify": self.batch_classify}

    def _split_bodies(self, params_list: list, what: str):
        bodies, idx, out = [], [], [None] * len(params_list)
        for i, p in enumerate(params_list):
            try:
                bodies.append(name_and_rest(p))   # O(1): the scanner validates the data
                idx.append(i)
            except ArgumentError as e:
                out[i] = ArgumentError(f"{what}: {e}")
        return bodies, idx, out

    def batch_train(self, params_list: list) -> list:
        self.check_set_config()
        t0 = time.perf_counter_ns()
        bodies, idx, out = self._split_bodies(params_list, "train")
        with self.rw_mutex.write():
            self.event_model_updated(len(bodies))
        trace.record("batch.train.split", time.perf_counter_ns() - t0)
        self._batch_stats["train"][0] += len(bodies)
        self._batch_stats["train"][1] += 1
        try:
            t1 = time.perf_counter_ns()
            self.clf.train_requests(bodies)          # one launch, one stream per request
            trace.record("batch.train.submit", time.perf_counter_ns() - t1)
            for i, b in zip(idx, bodies):
                out[i] = max(0, msgpack_array_len(b))
        except TypeError:
            for i, b in zip(idx, bodies):            # isolate the malformed request(s)
                try:
                    out[i] = self.clf.train_requests([b])
                except TypeError as e:
                    out[i] = ArgumentError(str(e))
        return out

    def batch_classify(self, params_list: list) -> list:
        self.check_set_config()
        bodies, idx, out = self._split_bodies(params_list, "classify")
        self._batch_stats["classify"][0] += len(bodies)
        self._batch_stats["classify"][1] += 1
        try:
            flat = self.clf.classify_requests(bodies)
            k = 0
            for i, b in zip(idx, bodies):
                n = max(0, msgpack_array_len(b))
                out[i] = flat[k:k + n]
                k += n
        except TypeError:
            for i, b in zip(idx, bodies):
                try:
                    out[i] = self.clf.classify_requests([b])
                except TypeError as e:
                    out[i] = ArgumentError(str(e))
        return out

    def arena_methods(self) -> dict:
        """train on the GPU pipeline straight from the transport's pinned
        arena (no Python per request, no host scan; see RpcServer.set_arena)"""
        clf = self.clf
        if not (getattr(clf, "gpu", False) and getattr(clf.pipe, "fast", False)):
            return {}
        import torch
        from ..ops.feature_pipeline import RequestArena
        mb = int(os.environ.get("JUBATUS_TRAIN_ARENA_MB", "32"))
        nslots = int(os.environ.get("JUBATUS_ARENA_THREADS", "2")) + 2
        self._arena_slots = [torch.empty(mb << 20, dtype=torch.uint8, pin_memory=True)
                             for _ in range(nslots)]
        views = [RequestArena.over(t, [], []) for t in self._arena_slots]

        def serve(slot, offs, lens):
            self.check_set_config()
            self._batch_stats["train"][0] += len(offs)
            self._batch_stats["train"][1] += 1
            return self.clf.train_arena_sync(views[slot], offs, lens)
        return {"train": ([t.data_ptr() for t in self._arena_slots], mb << 20, serve)}

    def get_labels(self) -> dict:
        self.check_set_config()
        return self.clf.get_labels()

    def set_label(self, label: str) -> bool:
        self.check_set_config()
        self._bump()
        return self.clf.set_label(label)

    def clear(self) -> bool:
        self.check_set_config()
        self._bump()
        self.clf.clear()
        log.info("model cleared: %s", self.argv().name)
        return True

    def delete_label(self, label: str) -> bool:
        self.check_set_config()
        self._bump()
        return self.clf.delete_label(label)

    def get_status(self, status: dict) -> None:
        if self.clf is not None:
            status.update(self.clf.get_status())
        if self.device is not None:
            import torch
            status["device"] = str(self.device)
            status["hbm_allocated_bytes"] = str(torch.cuda.memory_allocated(self.device))
        for k, b in (("train", self._train_batcher), ("classify", self._classify_batcher)):
            calls, launches = self._batch_stats[k]
            if b is not None:
                calls, launches = calls + b.calls, launches + b.batches
            if calls:
                status[f"batching.{k}.calls"] = str(calls)
                status[f"batching.{k}.launches"] = str(launches)
