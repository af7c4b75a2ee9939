"""jubaweight glue (reference jubatus/server/server/weight_serv.cpp:30-110).

update(datum) / calc_weight(datum) -> list<feature> [nolock], clear
(weight.idl:24-30). ``method`` / ``parameter`` are accepted and ignored.
"""
from __future__ import annotations

from ..framework.engine_serv import EngineServ
from ..fv_converter.converter import DatumToFvConverter
from ..fv_converter.datum import Datum
from ..models.weight import Weight


class WeightServ(EngineServ):
    type_name = "weight"

    def uses_gpu(self) -> bool:
        return False

    def build_driver(self, cfg: dict):
        if "converter" not in cfg:
            raise ValueError("weight config requires converter")
        return Weight(DatumToFvConverter(cfg["converter"]))

    def update(self, d):
        self.check_set_config()
        self.bump()
        return [[k, v] for k, v in self.driver.update(Datum.from_msgpack(d))]

    def calc_weight(self, d):
        self.check_set_config()
        return [[k, v] for k, v in self.driver.calc_weight(Datum.from_msgpack(d))]

    def clear(self) -> bool:
        self.check_set_config()
        self.bump()
        self.driver.clear()
        return True
