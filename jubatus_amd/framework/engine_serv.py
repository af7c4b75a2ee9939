"""Common glue of the engine servers (the shared parts of every
jubatus/server/server/*_serv.cpp): config parsing, driver construction,
mixer wiring, ``check_set_config`` and the brief write lock that bumps the
update counter for NOLOCK mutators."""
from __future__ import annotations

import json
from typing import Any

from ..common.exceptions import ConfigNotSet
from ..utils import logger
from .device import select_device
from .server_base import ServerBase

log = logger.get_logger("engine")


class EngineServ(ServerBase):
    type_name = ""

    def __init__(self, argv, coord=None):
        super().__init__(argv, coord)
        self.driver: Any = None
        self.config: str | None = None
        self.device = select_device(argv) if self.uses_gpu() else None

    # engines that run on the host only override this
    def uses_gpu(self) -> bool:
        return True

    def build_driver(self, cfg: dict) -> Any:
        raise NotImplementedError

    def check_set_config(self) -> None:
        if self.driver is None:
            raise ConfigNotSet()

    def set_config(self, config: str) -> None:
        cfg = json.loads(config)
        if not isinstance(cfg, dict):
            raise ValueError("config must be a JSON object")
        self.driver = self.build_driver(cfg)
        self.config = config
        if self.mixer is not None:
            self.mixer.set_driver(self.driver)
        log.info("config loaded (%s)", self.type_name)

    def get_config(self) -> str:
        self.check_set_config()
        return self.config

    def get_driver(self):
        self.check_set_config()
        return self.driver

    def bump(self) -> None:
        with self.rw_mutex.write():
            self.event_model_updated()

    def clear(self) -> bool:
        self.check_set_config()
        self.driver.clear()
        return True

    def get_status(self, status: dict) -> None:
        if self.driver is not None and hasattr(self.driver, "get_status"):
            status.update({k: str(v) for k, v in self.driver.get_status().items()})
        if self.device is not None:
            import torch
            status["device"] = str(self.device)
            status["hbm_allocated_bytes"] = str(torch.cuda.memory_allocated(self.device))
