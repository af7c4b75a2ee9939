"""jubaconfig: manage engine configs in the coordinator (reference C33,
jubatus/server/cmd/jubaconfig.cpp:63-226).

``-c write -f FILE -t TYPE -n NAME`` (refused while any server of the
cluster runs), ``-c read``, ``-c delete``, ``-c list`` (every
/jubatus/config/<type>/<name>); coordinator from ``-z`` or ``ZK``.
"""
from __future__ import annotations

import argparse
import os
import sys

from ..common import config as zkconfig
from ..common.lock_service import CoordinatorClient


def main(argv: list[str] | None = None, out=print) -> int:
    p = argparse.ArgumentParser(prog="jubaconfig")
    p.add_argument("-c", "--cmd", required=True, choices=("write", "read", "delete", "list"))
    p.add_argument("-f", "--file", default="")
    p.add_argument("-t", "--type", default="")
    p.add_argument("-n", "--name", default="")
    p.add_argument("-z", "--zookeeper", default="")
    p.add_argument("-d", "--debug", action="store_true")
    a = p.parse_args(argv)
    zk = a.zookeeper or os.environ.get("ZK", "")
    if not zk:
        out("can't get ZK location: set 'ZK' environment or specify '-z <somezkaddrs>'")
        return 1
    if a.cmd != "list" and not (a.type and a.name):
        out("type (-t) and name (-n) are required")
        return 1
    ls = CoordinatorClient(zk, timeout=10.0)
    try:
        if a.cmd == "write":
            if not a.file:
                out("config file (-f) is required")
                return 1
            with open(a.file) as f:
                zkconfig.config_tozk(ls, a.type, a.name, f.read())
        elif a.cmd == "read":
            out(zkconfig.config_fromzk(ls, a.type, a.name))
        elif a.cmd == "delete":
            zkconfig.remove_config_fromzk(ls, a.type, a.name)
        else:
            for t, names in sorted(zkconfig.list_configs(ls).items()):
                for n in sorted(names):
                    out(f"config of {t}/{n}:")
                    out(zkconfig.config_fromzk(ls, t, n))
        return 0
    except (zkconfig.ConfigError, OSError) as e:
        out(f"error: {e}")
        return 1
    finally:
        ls.close()


if __name__ == "__main__":
    sys.exit(main())
