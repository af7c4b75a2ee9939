"""Engine configs in the coordinator (reference C10: jubatus/server/common/config.cpp).

``config_tozk`` validates the JSON, takes the ``config_lock`` write lock
(3 tries), refuses while any server of the cluster is running, then writes
``/jubatus/config/<type>/<name>``; ``remove_config_fromzk`` likewise.
Servers hold a *read* lock on config_lock while they run
(server_helper.cpp:117-136).
"""
from __future__ import annotations

import json
import time

from ..utils import logger
from .lock_service import LockService, LockServiceMutex
from .membership import build_actor_path, build_config_lock_path, build_config_path, prepare_jubatus

log = logger.get_logger("config")


class ConfigError(RuntimeError):
    pass


def _try(fn, retry: int) -> bool:
    for i in range(max(1, retry)):
        if fn():
            return True
        time.sleep(0.1 * (i + 1))
    return False


def config_fromzk(ls: LockService, type_: str, name: str) -> str:
    data = ls.read(build_config_path(type_, name))
    if data is None:
        raise ConfigError(f"config is not found: {build_config_path(type_, name)}")
    return data


def config_tozk(ls: LockService, type_: str, name: str, config: str) -> None:
    try:
        json.loads(config)
    except json.JSONDecodeError as e:
        raise ConfigError(f"invalid config json: {e}") from e
    prepare_jubatus(ls, type_, name)
    m = LockServiceMutex(ls, build_config_lock_path(type_, name))
    if not _try(m.try_lock, 3):
        raise ConfigError("any server is running: cannot lock config_lock")
    try:
        if ls.list(build_actor_path(type_, name) + "/nodes"):
            raise ConfigError("any server is running")
        path = build_config_path(type_, name)
        if not (ls.create(path, config) and ls.set(path, config)):
            raise ConfigError(f"failed to write config: {path}")
        log.info("wrote config to %s", path)
    finally:
        m.unlock()


def remove_config_fromzk(ls: LockService, type_: str, name: str) -> None:
    m = LockServiceMutex(ls, build_config_lock_path(type_, name))
    if not _try(m.try_lock, 3):
        raise ConfigError("any server is running: cannot lock config_lock")
    try:
        if ls.list(build_actor_path(type_, name) + "/nodes"):
            raise ConfigError("any server is running")
        path = build_config_path(type_, name)
        if not ls.exists(path):
            raise ConfigError(f"config is not found: {path}")
        ls.remove(path)
    finally:
        m.unlock()


def list_configs(ls: LockService) -> dict[str, list[str]]:
    from .membership import CONFIG_BASE_PATH
    return {t: ls.list(f"{CONFIG_BASE_PATH}/{t}") for t in ls.list(CONFIG_BASE_PATH)}


def get_config_lock(ls: LockService, type_: str, name: str, retry: int = 3) -> LockServiceMutex:
    m = LockServiceMutex(ls, build_config_lock_path(type_, name))
    if not _try(m.try_rlock, retry):
        raise ConfigError("failed to get config lock")
    return m
