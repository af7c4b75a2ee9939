"""jubarecommender glue (reference recommender_serv.cpp:105-224)."""
from __future__ import annotations

from ..framework.engine_serv import EngineServ
from ..fv_converter.converter import DatumToFvConverter
from ..fv_converter.datum import Datum
from ..models.recommender import Recommender


class RecommenderServ(EngineServ):
    type_name = "recommender"

    def __init__(self, argv, coord=None):
        super().__init__(argv, coord)
        self.clear_row_cnt = 0
        self.update_row_cnt = 0

    def build_driver(self, cfg: dict):
        return Recommender(cfg.get("method"), cfg.get("parameter"),
                           DatumToFvConverter(cfg.get("converter") or {}), device=self.device)

    def clear_row(self, rid: str) -> bool:
        self.check_set_config()
        self.clear_row_cnt += 1
        return self.driver.clear_row(rid)

    def update_row(self, rid: str, d) -> bool:
        self.check_set_config()
        self.update_row_cnt += 1
        return self.driver.update_row(rid, Datum.from_msgpack(d))

    def clear(self) -> bool:
        self.check_set_config()
        self.clear_row_cnt = 0
        self.update_row_cnt = 0
        self.driver.clear()
        return True

    def complete_row_from_id(self, rid: str):
        self.check_set_config()
        return self.driver.complete_row_from_id(rid).to_msgpack()

    def complete_row_from_datum(self, d):
        self.check_set_config()
        return self.driver.complete_row_from_datum(Datum.from_msgpack(d)).to_msgpack()

    def similar_row_from_id(self, rid: str, size: int):
        self.check_set_config()
        return [[r, float(s)] for r, s in self.driver.similar_row_from_id(rid, size)]

    def similar_row_from_datum(self, d, size: int):
        self.check_set_config()
        return [[r, float(s)] for r, s in self.driver.similar_row_from_datum(Datum.from_msgpack(d), size)]

    def decode_row(self, rid: str):
        self.check_set_config()
        return self.driver.decode_row(rid).to_msgpack()

    def get_all_rows(self):
        self.check_set_config()
        return self.driver.get_all_rows()

    def calc_similarity(self, lhs, rhs) -> float:
        self.check_set_config()
        return float(self.driver.calc_similarity(Datum.from_msgpack(lhs), Datum.from_msgpack(rhs)))

    def calc_l2norm(self, d) -> float:
        self.check_set_config()
        return float(self.driver.calc_l2norm(Datum.from_msgpack(d)))

    def get_status(self, status: dict) -> None:
        super().get_status(status)
        status["clear_row_cnt"] = str(self.clear_row_cnt)
        status["update_row_cnt"] = str(self.update_row_cnt)
