"""jubaanomaly glue (reference anomaly_serv.cpp:126-320).

``add``: a new id from the global id generator; standalone inserts locally
under the write lock; distributed mode sends the row to its two CHT owners
(``selective_update``: local call when the owner is this server, else a
server-to-server ``update`` RPC; the primary must succeed, the replica is
best effort). ``load`` resets the standalone id counter to
``find_max_int_id() + 1`` (anomaly_serv.cpp:299-320).
"""
from __future__ import annotations

from ..common.idgen import create_id_generator
from ..common.mprpc import RpcClient
from ..framework.engine_serv import EngineServ
from ..fv_converter.converter import DatumToFvConverter
from ..fv_converter.datum import Datum
from ..models.anomaly import LOF
from ..utils import logger

log = logger.get_logger("anomaly")


class AnomalyServ(EngineServ):
    type_name = "anomaly"

    def __init__(self, argv, coord=None):
        super().__init__(argv, coord)
        self.idgen = create_id_generator(argv, coord)

    def build_driver(self, cfg: dict):
        return LOF(cfg.get("method"), cfg.get("parameter"),
                   DatumToFvConverter(cfg.get("converter") or {}), device=self.device)

    def clear_row(self, rid: str) -> bool:
        self.check_set_config()
        return self.driver.clear_row(rid)

    def add(self, d):
        self.check_set_config()
        rid = str(self.idgen.generate())
        datum = Datum.from_msgpack(d)
        if self.argv().is_standalone():
            with self.rw_mutex.write():
                self.event_model_updated()
                return [rid, float(self.driver.add(rid, datum))]
        from ..common.cht import CHT
        owners = CHT(self.coord, self.type_name, self.argv().name).find(rid, 2)
        if not owners:
            raise RuntimeError(f"no server found in cht: {self.argv().name}")
        score = self._selective_update(owners[0], rid, datum)
        for o in owners[1:]:
            try:
                self._selective_update(o, rid, datum)
            except Exception as e:  # noqa: BLE001 - replica is best effort
                log.warning("cannot create replica (%s): %s:%d", e, o[0], o[1])
        return [rid, float(score)]

    def _selective_update(self, owner, rid: str, datum: Datum) -> float:
        host, port = owner
        a = self.argv()
        if host == a.eth and port == a.port:
            with self.rw_mutex.write():
                self.event_model_updated()
                return self.driver.update(rid, datum)
        with RpcClient(host, port, a.interconnect_timeout) as c:
            return float(c.call("update", a.name, rid, datum.to_msgpack()))

    def update(self, rid: str, d) -> float:
        self.check_set_config()
        return float(self.driver.update(rid, Datum.from_msgpack(d)))

    def overwrite(self, rid: str, d) -> float:
        self.check_set_config()
        return float(self.driver.overwrite(rid, Datum.from_msgpack(d)))

    def calc_score(self, d) -> float:
        self.check_set_config()
        return float(self.driver.calc_score(Datum.from_msgpack(d)))

    def get_all_rows(self):
        self.check_set_config()
        return self.driver.get_all_rows()

    def _reset_idgen(self) -> None:
        if self.argv().is_standalone():
            self.idgen.set_next(self.driver.find_max_int_id() + 1)

    def load(self, model_id: str) -> bool:
        ok = super().load(model_id)
        self._reset_idgen()
        return ok

    def load_file(self, path: str) -> None:
        super().load_file(path)
        self._reset_idgen()
