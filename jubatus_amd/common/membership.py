"""Coordinator namespace and group membership (reference C8:
jubatus/server/common/membership.{hpp,cpp}).

    /jubatus/supervisors/<ip_port>                 jubavisors (ephemeral)
    /jubatus/jubaproxies/<type>/<ip_port>          proxies (ephemeral)
    /jubatus/actors/<type>/<name>/nodes/<ip_port>  servers (ephemeral)
    /jubatus/actors/<type>/<name>/actives/<ip_port> servers serving requests
    /jubatus/actors/<type>/<name>/{master_lock,config_lock,cht,id_generator,mix}
    /jubatus/config/<type>/<name>                  engine config JSON
"""
from __future__ import annotations

import os
import signal
from typing import Callable

from ..utils import logger
from .lock_service import LockService

log = logger.get_logger("membership")

JUBATUS_BASE_PATH = "/jubatus"
JUBAVISOR_BASE_PATH = "/jubatus/supervisors"
JUBAPROXY_BASE_PATH = "/jubatus/jubaproxies"
ACTOR_BASE_PATH = "/jubatus/actors"
CONFIG_BASE_PATH = "/jubatus/config"


def build_loc_str(ip: str, port: int, i: int = 0) -> str:
    """"127.0.0.1", 9199 -> "127.0.0.1_9199" (membership.cpp:40-47)."""
    s = f"{ip}_{int(port)}"
    return f"{s}_{i}" if i > 0 else s


def build_existence_path(base: str, ip: str, port: int) -> str:
    return f"{base}/{ip}_{int(port)}"


def build_actor_path(type_: str, name: str) -> str:
    return f"{ACTOR_BASE_PATH}/{type_}/{name}"


def build_config_path(type_: str, name: str) -> str:
    return f"{CONFIG_BASE_PATH}/{type_}/{name}"


def build_config_lock_path(type_: str, name: str) -> str:
    return build_actor_path(type_, name) + "/config_lock"


def revert(loc: str) -> tuple[str, int]:
    """"127.0.0.1_9199" -> ("127.0.0.1", 9199)."""
    ip, _, port = loc.partition("_")
    port = port.split("_")[0]
    return ip, int(port) if port.isdigit() else 0


def prepare_jubatus(ls: LockService, type_: str, name: str = "") -> None:
    """Create the base tree (membership.cpp:287-312)."""
    for p in (JUBATUS_BASE_PATH, JUBAVISOR_BASE_PATH, JUBAPROXY_BASE_PATH, ACTOR_BASE_PATH,
              CONFIG_BASE_PATH, f"{ACTOR_BASE_PATH}/{type_}", f"{CONFIG_BASE_PATH}/{type_}",
              f"{JUBAPROXY_BASE_PATH}/{type_}"):
        if not ls.create(p):
            raise RuntimeError(f"failed to prepare coordinator tree: {p}")
    if name:
        base = build_actor_path(type_, name)
        for p in (base, base + "/nodes", base + "/actives", base + "/master_lock",
                  base + "/config_lock", base + "/id_generator", base + "/mix"):
            ls.create(p)


def register_actor(ls: LockService, type_: str, name: str, ip: str, port: int) -> None:
    base = build_actor_path(type_, name)
    ok = ls.create(base) and ls.create(base + "/master_lock", "") and ls.create(base + "/nodes")
    path = build_existence_path(base + "/nodes", ip, port)
    ok = ok and ls.create(path, "", True)
    if not ok:
        raise RuntimeError("Failed to register_actor")
    log.info("actor created: %s", path)


def unregister_actor(ls: LockService, type_: str, name: str, ip: str, port: int) -> None:
    base = build_actor_path(type_, name)
    ls.remove(build_existence_path(base + "/nodes", ip, port))
    ls.remove(build_existence_path(base + "/actives", ip, port))


def register_active(ls: LockService, type_: str, name: str, ip: str, port: int) -> bool:
    base = build_actor_path(type_, name)
    ls.create(base + "/actives")
    path = build_existence_path(base + "/actives", ip, port)
    if ls.exists(path):
        return True
    ok = ls.create(path, "", True)
    if ok:
        log.info("active created: %s", path)
    return ok


def unregister_active(ls: LockService, type_: str, name: str, ip: str, port: int) -> bool:
    path = build_existence_path(build_actor_path(type_, name) + "/actives", ip, port)
    if ls.exists(path):
        return ls.remove(path)
    return True


def watch_delete_actor(ls: LockService, type_: str, name: str, ip: str, port: int,
                       fn: Callable[[str], None]) -> bool:
    """Self-fencing: when our own actor node disappears, stop
    (membership.cpp:170-206, server_helper.cpp:91-94)."""
    path = build_existence_path(build_actor_path(type_, name) + "/nodes", ip, port)
    return ls.bind_delete_watcher(path, fn)


def register_proxy(ls: LockService, type_: str, ip: str, port: int) -> None:
    ls.create(f"{JUBAPROXY_BASE_PATH}/{type_}")
    path = build_existence_path(f"{JUBAPROXY_BASE_PATH}/{type_}", ip, port)
    if not ls.create(path, "", True):
        raise RuntimeError("Failed to register_proxy")


def register_supervisor(ls: LockService, ip: str, port: int) -> None:
    # jubavisor.cpp:70-72 creates the base paths before registering
    for p in (JUBATUS_BASE_PATH, JUBAVISOR_BASE_PATH, ACTOR_BASE_PATH):
        if not ls.exists(p):
            ls.create(p)
    if not ls.create(build_existence_path(JUBAVISOR_BASE_PATH, ip, port), "", True):
        raise RuntimeError("Failed to register_supervisor")


def get_all_nodes(ls: LockService, type_: str, name: str) -> list[tuple[str, int]]:
    return [revert(n) for n in ls.list(build_actor_path(type_, name) + "/nodes")]


def get_all_actives(ls: LockService, type_: str, name: str) -> list[tuple[str, int]]:
    return [revert(n) for n in ls.list(build_actor_path(type_, name) + "/actives")]


def shutdown_server() -> None:
    """reference membership.cpp:257-259: SIGTERM to ourselves."""
    os.kill(os.getpid(), signal.SIGTERM)
