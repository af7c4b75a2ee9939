"""jubaregression server glue (reference jubatus/server/server/regression_serv.cpp).

train(list<scored_datum>) [update], estimate(list<datum>) [analysis],
clear() [update] (regression.idl:25-31).
"""
from __future__ import annotations

from ..common.exceptions import ArgumentError
from ..common.mprpc import split_params
from ..framework.engine_serv import EngineServ
from ..fv_converter.converter import DatumToFvConverter, device_hash_max_size
from ..models.regression import PARegression


class RegressionServ(EngineServ):
    type_name = "regression"

    def build_driver(self, cfg: dict):
        return PARegression(cfg.get("method"), cfg.get("parameter"),
                            DatumToFvConverter(cfg.get("converter") or {},
                                               default_hash_max_size=(device_hash_max_size()
                                                                      if self.device is not None else None)),
                            device=self.device)

    def train(self, data) -> int:
        self.check_set_config()
        if not isinstance(data, list):
            raise ArgumentError("train: data must be a list")
        return self.driver.train(data)

    def raw_train(self, params: bytes) -> int:
        """zero-copy path (GPU fv_hash) for list<scored_datum> bodies"""
        self.check_set_config()
        parts = split_params(params)
        if len(parts) != 2:
            raise ArgumentError("train: expected 2 arguments")
        try:
            return self.driver.train_requests([parts[1]])
        except TypeError as e:
            raise ArgumentError(str(e)) from e

    def estimate(self, data) -> list[float]:
        self.check_set_config()
        if not isinstance(data, list):
            raise ArgumentError("estimate: data must be a list")
        return self.driver.estimate(data)
