"""jubacoordinator: the cluster coordination server (replaces ZooKeeper for
the reference's lock_service usage; see lock_service.py for the data model).

Serves a ZNodeStore over msgpack-RPC (native transport) and expires
sessions whose heartbeat is older than their timeout (ephemeral nodes go
with them - the liveness mechanism of membership, CHT and mixer masters,
SURVEY §5.3).
"""
from __future__ import annotations

import os
import subprocess
import threading

from ..utils import logger
from .lock_service import ZNodeStore
from .mprpc import RpcServer

log = logger.get_logger("coordinator")


class CoordinatorServer:
    def __init__(self, port: int = 2181, bind: str = "0.0.0.0", nthreads: int = 4,
                 store: ZNodeStore | None = None):
        self.store = store or ZNodeStore()
        self.rpc = RpcServer(nthreads=nthreads)
        st = self.store
        self.rpc.add("open_session", st.open_session, 1)
        self.rpc.add("heartbeat", st.heartbeat, 1)
        self.rpc.add("close_session", st.close_session, 1)
        self.rpc.add("create", st.create, 4)
        self.rpc.add("create_seq", lambda sid, p: list(st.create_seq(sid, p)), 2)
        self.rpc.add("set", lambda p, d: list(st.set(p, d)), 2)
        self.rpc.add("remove", st.remove, 1)
        self.rpc.add("exists", st.exists, 1)
        self.rpc.add("list", lambda p: list(st.list(p)), 1)
        self.rpc.add("read", lambda p: list(st.read(p)), 1)
        self.rpc.add("stat_many", st.stat_many, 1)
        self.rpc.add("dump", st.dump, 0)
        self.port = self.rpc.listen(port, bind)
        self._stop = threading.Event()
        self._sweeper = threading.Thread(target=self._sweep, name="coord-sweeper", daemon=True)

    def _sweep(self) -> None:
        while not self._stop.wait(0.1):
            self.store.expire_sessions()

    def start(self) -> "CoordinatorServer":
        self.rpc.start()
        self._sweeper.start()
        log.info("coordinator listening on %d", self.port)
        return self

    def stop(self) -> None:
        self._stop.set()
        self.rpc.stop()

    def join(self) -> None:
        while not self._stop.wait(0.5):
            pass


NATIVE_BIN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                          "native_bin", "jubacoordinator")


def native_available() -> bool:
    return os.access(NATIVE_BIN, os.X_OK)


class NativeCoordinator:
    """The native coordinator (csrc/coord/jubacoordinator.cpp) as a child
    process: same RPC surface as CoordinatorServer, no Python in the server."""

    def __init__(self, port: int = 0, bind: str = "127.0.0.1", nthreads: int = 4,
                 exe: str | None = None, env: dict | None = None, stderr=None):
        if exe is None and not native_available():
            from .. import build_ext
            build_ext.build_tools()
        self.proc = subprocess.Popen([exe or NATIVE_BIN, "-p", str(port), "-b", bind, "-c",
                                      str(nthreads)], stdout=subprocess.PIPE,
                                     stderr=stderr if stderr is not None else subprocess.DEVNULL,
                                     text=True, env=env)
        line = self.proc.stdout.readline()
        if not line.startswith("jubacoordinator ready"):
            self.proc.kill()
            raise RuntimeError(f"native coordinator failed to start: {line!r}")
        self.port = int(line.split()[-1])

    def start(self) -> "NativeCoordinator":
        return self

    def stop(self) -> int:
        if self.proc.poll() is None:
            self.proc.terminate()
            try:
                self.proc.wait(15)
            except subprocess.TimeoutExpired:
                self.proc.kill()
                self.proc.wait()
        return self.proc.returncode


def main(argv: list[str] | None = None) -> int:
    import argparse
    import sys

    from ..utils import signals
    p = argparse.ArgumentParser(prog="jubacoordinator")
    p.add_argument("-p", "--port", type=int, default=2181)
    p.add_argument("-b", "--listen_addr", default="0.0.0.0")
    p.add_argument("-c", "--thread", type=int, default=4)
    a = p.parse_args(sys.argv[1:] if argv is None else argv)
    srv = CoordinatorServer(a.port, a.listen_addr, a.thread).start()
    signals.prepare_signal_handling()
    signals.set_action_on_term(srv.stop)
    srv.join()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
