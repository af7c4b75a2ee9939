"""jubactl: cluster control (reference C32, jubatus/server/cmd/jubactl.cpp:56-315).

``-c start|stop``: fan out to every jubavisor registered in the coordinator,
spreading N processes as N/|visors| (+1 on the first N%|visors|); N=0 means
one per visor. ``-c save|load``: call every node of the cluster directly
(id defaults to the cluster name). ``-c status``: list proxies, visors and
nodes. The coordinator location comes from ``-z`` or the ``ZK`` environment
variable.
"""
from __future__ import annotations

import argparse
import os
import sys

from ..common import membership as mb
from ..common.lock_service import CoordinatorClient
from ..common.mprpc import RpcClient
from .jubavisor import argv_to_wire


VISOR_CALL_TIMEOUT = 30.0


def _parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog="jubactl")
    p.add_argument("-c", "--cmd", required=True, choices=("start", "stop", "save", "load", "status"))
    p.add_argument("-s", "--server", required=True, help="server exec name (jubaclassifier, ...)")
    p.add_argument("-n", "--name", required=True)
    p.add_argument("-t", "--type", required=True)
    p.add_argument("-N", "--num", type=int, default=0)
    p.add_argument("-z", "--zookeeper", default="")
    p.add_argument("-i", "--id", default="")
    p.add_argument("-B", "--listen_if", default="")
    p.add_argument("-C", "--thread", type=int, default=2)
    p.add_argument("-T", "--timeout", type=int, default=10)
    p.add_argument("-D", "--datadir", default="/tmp")
    p.add_argument("-L", "--logdir", default="")
    p.add_argument("-G", "--log_config", default="")
    p.add_argument("-X", "--mixer", default="linear_mixer")
    p.add_argument("-S", "--interval_sec", type=int, default=16)
    p.add_argument("-I", "--interval_count", type=int, default=512)
    p.add_argument("-Z", "--zookeeper_timeout", type=int, default=10)
    p.add_argument("-R", "--interconnect_timeout", type=int, default=10)
    p.add_argument("-d", "--debug", action="store_true")
    return p


def split_counts(n: int, nvisors: int) -> list[int]:
    """N/|visors| each, +1 for the first N%|visors| (jubactl.cpp:218-230)"""
    if n == 0:
        n = nvisors
    q, r = divmod(n, nvisors)
    return [q + (1 if i < r else 0) for i in range(nvisors)]


def send2supervisor(ls, a, out=print) -> int:
    name = f"{a.server}/{a.name}"
    argv = {}
    if a.cmd == "start":
        ls.create(mb.build_actor_path(a.type, a.name))
        ls.create(mb.build_actor_path(a.type, a.name) + "/nodes")
        argv = {"port": 0, "bind_address": "", "bind_if": a.listen_if, "timeout": a.timeout,
                "zookeeper_timeout": a.zookeeper_timeout,
                "interconnect_timeout": a.interconnect_timeout, "threadnum": a.thread,
                "program_name": a.type, "type": a.type, "z": a.zookeeper, "name": name,
                "datadir": a.datadir, "logdir": a.logdir, "log_config": a.log_config, "eth": "",
                "interval_sec": a.interval_sec, "interval_count": a.interval_count,
                "mixer": a.mixer, "daemon": False}
    visors = ls.list(mb.JUBAVISOR_BASE_PATH)
    if not visors:
        out(f"no server to {a.cmd} {name}")
        return -1
    rc = 0
    for loc, n in zip(visors, split_counts(a.num, len(visors))):
        host, port = mb.revert(loc)
        out(f"sending {a.cmd} / {name} to {loc}...", end="")
        try:
            # a supervisor's stop waits up to 10 s per child before SIGKILL:
            # the call gets more than that
            with RpcClient(host, port, VISOR_CALL_TIMEOUT) as c:
                r = c.call(a.cmd, name, n, argv_to_wire(argv)) if a.cmd == "start" else c.call(a.cmd, name, n)
        except Exception as e:  # noqa: BLE001
            r = -1
            out(f"failed ({e}).")
            rc = -1
            continue
        out("ok." if r == 0 else "failed.")
        if r != 0:
            rc = r
    return rc


def send2server(ls, a, out=print) -> int:
    mid = a.id or a.name
    nodes = ls.list(mb.build_actor_path(a.type, a.name) + "/nodes")
    if not nodes:
        out(f"no server to {a.cmd} {a.name}")
    rc = 0
    for loc in nodes:
        host, port = mb.revert(loc)
        out(f"sending {a.cmd} / {a.name} to {loc}...", end="")
        try:
            with RpcClient(host, port, 10.0) as c:
                c.call(a.cmd, a.name, mid)
            out("ok.")
        except Exception:  # noqa: BLE001
            out("failed.")
            rc = -1
    return rc


def status(ls, a, out=print) -> None:
    for path, what in ((f"{mb.JUBAPROXY_BASE_PATH}/{a.type}", "jubaproxy"),
                       (mb.JUBAVISOR_BASE_PATH, "jubavisor"),
                       (mb.build_actor_path(a.type, a.name) + "/nodes", a.name)):
        out(f"\033[34mactive {what} members:\033[0m")
        for m in ls.list(path):
            out(m)


def main(argv: list[str] | None = None) -> int:
    a = _parser().parse_args(argv)
    zk = a.zookeeper or os.environ.get("ZK", "")
    if not zk:
        print("can't get ZK location: set 'ZK' environment or specify '-z <somezkaddrs>'")
        return 1
    a.zookeeper = zk
    ls = CoordinatorClient(zk, timeout=10.0)
    try:
        if a.cmd == "status":
            status(ls, a)
            return 0
        if a.cmd in ("start", "stop"):
            return 0 if send2supervisor(ls, a) == 0 else 1
        return 0 if send2server(ls, a) == 0 else 1
    finally:
        ls.close()


def _print(*args, **kw):
    print(*args, **kw, flush=True)


if __name__ == "__main__":
    sys.exit(main())
