"""Shared test helpers: start a standalone engine server in-process."""
import os

from jubatus_amd.framework.server_helper import ServerHelper
from jubatus_amd.framework.server_util import ServerArgv
from jubatus_amd.server import get_serv

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def config_path(rel: str) -> str:
    return os.path.join(ROOT, "config", rel)


def start_standalone(engine, config, tmp_path, extra=()):
    cfg = tmp_path / f"{engine}.json"
    cfg.write_text(open(config).read() if os.path.exists(config) else config)
    a = ServerArgv.parse(["-p", "9199", "-b", "127.0.0.1", "-f", str(cfg), "-d", str(tmp_path),
                          "--cpu", *extra], engine)
    a.port = 0
    h = ServerHelper(get_serv(engine), a, install_signals=False)
    h.start(block=False)
    return h
