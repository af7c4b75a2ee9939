"""jubaburst glue (reference jubatus/server/server/burst_serv.cpp:44-246).

add_documents(list<document>) -> number accepted (results recomputed when
any was accepted), get_result / get_result_at / get_all_bursted_results(_at),
get_all_keywords, add_keyword / remove_keyword / remove_all_keywords, clear
(burst.idl:42-69). In a cluster each keyword is processed by its two CHT
owners (``will_process``, replication level 2); the processed set is
re-derived whenever the membership changes (the reference's child watcher on
the actor's nodes, burst_serv.cpp:200-246) and the other servers receive the
results through MIX.
"""
from __future__ import annotations

from ..common.exceptions import ArgumentError
from ..framework.engine_serv import EngineServ
from ..models.burst import Burst

REPLICATION = 2


def _window(res) -> list:
    start, batches = res
    return [float(start), [[int(d), int(r), float(w)] for d, r, w in batches]]


class BurstServ(EngineServ):
    type_name = "burst"

    def __init__(self, argv, coord=None):
        super().__init__(argv, coord)
        self._members_seen: tuple | None = None

    def uses_gpu(self) -> bool:
        return False

    def build_driver(self, cfg: dict):
        return Burst(cfg.get("method"), cfg.get("parameter"))

    # --------------------------------------------------- keyword ownership
    def will_process(self, kw: str) -> bool:
        a = self.argv()
        if a.is_standalone():
            return True
        from ..common.cht import CHT
        owners = CHT(self.coord, self.type_name, a.name).find(kw, REPLICATION)
        return (a.eth, a.port) in [(h, p) for h, p in owners]

    def _rehash_if_needed(self) -> None:
        a = self.argv()
        if a.is_standalone():
            return
        from ..common.membership import get_all_nodes
        members = tuple(sorted(get_all_nodes(self.coord, self.type_name, a.name)))
        if members != self._members_seen:
            self._members_seen = members
            self.driver.set_processed_keywords(
                [k for k, _, _ in self.driver.get_all_keywords() if self.will_process(k)])

    # --------------------------------------------------------------- API
    def add_documents(self, data) -> int:
        self.check_set_config()
        if not isinstance(data, list):
            raise ArgumentError("add_documents: data must be a list")
        self._rehash_if_needed()
        n = 0
        for doc in data:
            pos, text = doc[0], doc[1]
            if isinstance(text, bytes):
                text = text.decode()
            if self.driver.add_document(text, float(pos)):
                n += 1
        if n:
            self.driver.calculate_results()
        return n

    def get_result(self, keyword: str):
        self.check_set_config()
        return _window(self.driver.get_result(keyword))

    def get_result_at(self, keyword: str, pos: float):
        self.check_set_config()
        return _window(self.driver.get_result_at(keyword, float(pos)))

    def get_all_bursted_results(self):
        self.check_set_config()
        return {k: _window(v) for k, v in self.driver.get_all_bursted_results().items()}

    def get_all_bursted_results_at(self, pos: float):
        self.check_set_config()
        return {k: _window(v) for k, v in self.driver.get_all_bursted_results_at(float(pos)).items()}

    def get_all_keywords(self):
        self.check_set_config()
        return [[k, s, g] for k, s, g in self.driver.get_all_keywords()]

    def add_keyword(self, keyword) -> bool:
        self.check_set_config()
        kw, scaling, gamma = keyword[0], float(keyword[1]), float(keyword[2])
        return self.driver.add_keyword(kw, scaling, gamma, self.will_process(kw))

    def remove_keyword(self, keyword: str) -> bool:
        self.check_set_config()
        return self.driver.remove_keyword(keyword)

    def remove_all_keywords(self) -> bool:
        self.check_set_config()
        return self.driver.remove_all_keywords()
