"""jubastat glue (reference jubatus/server/server/stat_serv.cpp:51-106).

push(key, value) [update], sum / stddev / max / min / entropy / moment
[analysis], clear (stat.idl:20-36). Config: {"window_size": N}. Host-only
engine (per-key scalar bookkeeping: nothing here is worth a kernel launch).
"""
from __future__ import annotations

from ..framework.engine_serv import EngineServ
from ..models.stat import Stat


class StatServ(EngineServ):
    type_name = "stat"

    def uses_gpu(self) -> bool:
        return False

    def build_driver(self, cfg: dict):
        if "window_size" not in cfg:
            raise ValueError("stat config requires window_size")
        return Stat(int(cfg["window_size"]))

    def push(self, key: str, value: float) -> bool:
        self.check_set_config()
        return self.driver.push(key, float(value))

    def sum(self, key: str) -> float:
        self.check_set_config()
        return self.driver.sum(key)

    def stddev(self, key: str) -> float:
        self.check_set_config()
        return self.driver.stddev(key)

    def max(self, key: str) -> float:
        self.check_set_config()
        return self.driver.max(key)

    def min(self, key: str) -> float:
        self.check_set_config()
        return self.driver.min(key)

    def entropy(self, key: str) -> float:
        self.check_set_config()
        return self.driver.entropy()        # key is ignored (stat_serv.cpp:89-91)

    def moment(self, key: str, degree: int, center: float) -> float:
        self.check_set_config()
        return self.driver.moment(key, int(degree), float(center))
