"""jubanearest_neighbor glue (reference nearest_neighbor_serv.cpp:96-178)."""
from __future__ import annotations

from ..framework.engine_serv import EngineServ
from ..fv_converter.converter import DatumToFvConverter
from ..fv_converter.datum import Datum
from ..models.recommender import NearestNeighbor


def _pairs(res):
    return [[rid, float(s)] for rid, s in res]


class NearestNeighborServ(EngineServ):
    type_name = "nearest_neighbor"

    def build_driver(self, cfg: dict):
        return NearestNeighbor(cfg.get("method"), cfg.get("parameter"),
                               DatumToFvConverter(cfg.get("converter") or {}), device=self.device)

    def clear(self) -> bool:
        self.check_set_config()
        self.driver.clear()
        return True

    def set_row(self, rid: str, d) -> bool:
        self.check_set_config()
        return self.driver.set_row(rid, Datum.from_msgpack(d))

    def neighbor_row_from_id(self, rid: str, size: int):
        self.check_set_config()
        return _pairs(self.driver.neighbor_row_from_id(rid, size))

    def neighbor_row_from_datum(self, d, size: int):
        self.check_set_config()
        return _pairs(self.driver.neighbor_row_from_datum(Datum.from_msgpack(d), size))

    def similar_row_from_id(self, rid: str, n: int):
        self.check_set_config()
        return _pairs(self.driver.similar_row_from_id(rid, n))

    def similar_row_from_datum(self, d, n: int):
        self.check_set_config()
        return _pairs(self.driver.similar_row_from_datum(Datum.from_msgpack(d), n))

    def get_all_rows(self):
        self.check_set_config()
        return self.driver.get_all_rows()
