"""jubaclustering glue (reference jubatus/server/server/clustering_serv.cpp:71-151).

push(list<datum>) [update], get_revision, get_core_members, get_k_center,
get_nearest_center(datum), get_nearest_members(datum) [analysis], clear
(clustering.idl:26-44). ``weighted_datum`` travels as [weight, datum].
Queries before the first clustering raise "clustering is not performed yet"
(the reference's not_performed exception).
"""
from __future__ import annotations

import msgpack

from ..common.exceptions import ArgumentError
from ..common.mprpc import split_params
from ..framework.engine_serv import EngineServ
from ..fv_converter.converter import DatumToFvConverter
from ..fv_converter.datum import Datum
from ..models.clustering import Clustering


class ClusteringServ(EngineServ):
    type_name = "clustering"

    def build_driver(self, cfg: dict):
        return Clustering(cfg.get("method"), cfg.get("parameter"),
                          DatumToFvConverter(cfg.get("converter") or {}), device=self.device)

    def push(self, points) -> bool:
        self.check_set_config()
        if not isinstance(points, list):
            raise ArgumentError("push: points must be a list")
        return self.driver.push([Datum.from_msgpack(p) for p in points])

    def raw_push(self, params: bytes) -> bool:
        """zero-copy path: the list<datum> bytes go to the native named
        converter in one call (models/clustering.py push_body)"""
        self.check_set_config()
        parts = split_params(params)
        if len(parts) != 2:
            raise ArgumentError("push: expected 2 arguments")
        if getattr(self.driver, "_native", None) is None:
            return self.push(msgpack.unpackb(parts[1], raw=False))
        return self.driver.push_body(parts[1])

    def get_revision(self) -> int:
        self.check_set_config()
        return self.driver.get_revision()

    def get_core_members(self):
        self.check_set_config()
        return [[[w, d.to_msgpack()] for w, d in members]
                for members in self.driver.get_core_members()]

    def get_k_center(self):
        self.check_set_config()
        return [d.to_msgpack() for d in self.driver.get_k_center()]

    def get_nearest_center(self, point):
        self.check_set_config()
        return self.driver.get_nearest_center(Datum.from_msgpack(point)).to_msgpack()

    def get_nearest_members(self, point):
        self.check_set_config()
        return [[w, d.to_msgpack()]
                for w, d in self.driver.get_nearest_members(Datum.from_msgpack(point))]
