"""jubavisor: per-host process supervisor (reference C31,
jubatus/server/jubavisor/{jubavisor,process,main}.cpp).

RPC (default port 9198): ``start(server_name, N, server_argv) -> int`` spawns
N server processes of ``juba<engine>/<name>`` on ports taken from a pool
(base+1 .. base+max); ``stop(server_name, N) -> int`` terminates every child
of that name (the reference ignores N too, jubavisor.hpp:80-82). The
supervisor registers an ephemeral ``/jubatus/supervisors/<ip>_<port>`` node;
exited children are reaped and their ports return to the pool (the SIGCHLD
handler of jubavisor.cpp:113-156 - here a reaper thread); losing the
coordinator session stops every child. Children get the reference's flag set
(process.cpp:86-138): -z -n -p -B -c -t -Z -I -d -l -g -s -i -x.

``server_argv`` on the wire is the reference's MSGPACK_DEFINE order
(server_util.hpp:91-94): [port, bind_address, bind_if, timeout,
zookeeper_timeout, interconnect_timeout, threadnum, program_name, type, z,
name, datadir, logdir, log_config, eth, interval_sec, interval_count, mixer,
daemon].
"""
from __future__ import annotations

import argparse
import os
import signal
import subprocess
import sys
import threading

from ..common import membership as mb
from ..common.lock_service import CoordinatorClient
from ..common.mprpc import RpcServer
from ..utils import logger, system

log = logger.get_logger("jubavisor")

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

ARGV_FIELDS = ("port", "bind_address", "bind_if", "timeout", "zookeeper_timeout",
               "interconnect_timeout", "threadnum", "program_name", "type", "z", "name",
               "datadir", "logdir", "log_config", "eth", "interval_sec", "interval_count",
               "mixer", "daemon")


def argv_to_wire(d: dict) -> list:
    return [d.get(k) for k in ARGV_FIELDS]


def argv_from_wire(v) -> dict:
    if isinstance(v, dict):
        return dict(v)
    return {k: (x.decode() if isinstance(x, bytes) else x) for k, x in zip(ARGV_FIELDS, v)}


def count_gpus() -> int:
    """GPUs of this host from the KFD topology (no HIP runtime needed)"""
    n = 0
    for i in range(256):
        try:
            with open(f"/sys/class/kfd/kfd/topology/nodes/{i}/properties") as f:
                props = dict(line.split()[:2] for line in f if len(line.split()) >= 2)
        except OSError:
            break
        if int(props.get("simd_count", "0")) > 0:
            n += 1
    return n


def split_server_name(s: str) -> tuple[str, str]:
    """"jubaclassifier/name" -> ("jubaclassifier", "name") (process.cpp set_names)"""
    if "/" not in s:
        raise ValueError(f"cannot parse {s}")
    server, name = s.split("/", 1)
    if not server.startswith("juba") or not name:
        raise ValueError(f"cannot parse {s}")
    return server, name


def child_command(server: str, name: str, port: int, zk: str, a: dict,
                  listen_addr: str = "", gpu: int = -1) -> list[str]:
    engine = server[len("juba"):]
    cmd = [sys.executable, "-m", "jubatus_amd.cmd.server", engine, "-z", zk, "-n", name,
           "-p", str(port)]
    if gpu >= 0:
        cmd += ["--gpu", str(gpu)]
    if listen_addr:
        cmd += ["-b", listen_addr]
    if a.get("bind_if"):
        cmd += ["-B", str(a["bind_if"])]
    opts = (("-c", "threadnum"), ("-t", "timeout"), ("-Z", "zookeeper_timeout"),
            ("-I", "interconnect_timeout"), ("-d", "datadir"), ("-l", "logdir"),
            ("-g", "log_config"), ("-s", "interval_sec"), ("-i", "interval_count"),
            ("-x", "mixer"))
    for flag, key in opts:
        v = a.get(key)
        if v not in (None, ""):
            cmd += [flag, str(v)]
    return cmd


class Jubavisor:
    def __init__(self, zk: str, port: int, max_children: int = 16, timeout: float = 10.0,
                 listen_addr: str = "", gpus: int = -1):
        self.zk = zk
        # one server process per GPU: children get the least used device
        self.gpu_users = [0] * (gpus if gpus >= 0 else count_gpus())
        self.listen_addr = listen_addr
        self.ls = CoordinatorClient(zk, timeout=timeout)
        self.port_base = port
        self.pool = list(range(port + 1, port + 1 + max_children))
        self.max = max_children
        self.children: dict[str, list[tuple[subprocess.Popen, int, str]]] = {}
        self.lock = threading.Lock()
        self._stop = threading.Event()
        self.ip = listen_addr or system.get_default_v4_address()
        mb.register_supervisor(self.ls, self.ip, port)
        self.ls.push_cleanup(self.stop_all)
        self._reaper = threading.Thread(target=self._reap, daemon=True)
        self._reaper.start()

    def _reap(self) -> None:
        while not self._stop.wait(0.2):
            with self.lock:
                for name, procs in self.children.items():
                    for p in list(procs):
                        if p[0].poll() is not None:
                            log.info("%s with port %d exited pid: %d", p[2], p[1], p[0].pid)
                            self.pool.append(p[1])
                            self._give_gpu(p[3])
                            procs.remove(p)

    def start(self, server_name, n, argv) -> int:
        server_name = server_name.decode() if isinstance(server_name, bytes) else server_name
        try:
            server, name = split_server_name(server_name)
        except ValueError as e:
            log.error("%s", e)
            return -1
        a = argv_from_wire(argv)
        with self.lock:
            procs = self.children.setdefault(name, [])
            if len(procs) > n:
                log.error("%d %s already running at this machine.", len(procs), name)
                return -1
            need = int(n) - len(procs)
            if len(self.pool) < need:
                log.error("cannot spawn more than %d processes.", self.max)
                return -1
            env = dict(os.environ)
            env["PYTHONPATH"] = ROOT + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
            for _ in range(need):
                port = self.pool.pop(0)
                gpu = self._take_gpu()
                cmd = child_command(server, name, port, self.zk, a, self.listen_addr, gpu)
                try:
                    p = subprocess.Popen(cmd, env=env, stdin=subprocess.DEVNULL)
                except OSError as e:
                    log.error("cannot start: %s (%s)", name, e)
                    self.pool.append(port)
                    self._give_gpu(gpu)
                    return -1
                log.info("started %s on port %d (pid %d%s)", server_name, port, p.pid,
                         f", gpu {gpu}" if gpu >= 0 else "")
                procs.append((p, port, server_name, gpu))
        return 0

    def stop(self, server_name, n) -> int:
        server_name = server_name.decode() if isinstance(server_name, bytes) else server_name
        try:
            _, name = split_server_name(server_name)
        except ValueError:
            return -1
        with self.lock:
            procs = self.children.pop(name, [])
        r = 0
        for p, port, _, gpu in procs:
            if not _kill(p):
                r -= 1
            else:
                with self.lock:
                    self.pool.append(port)
                    self._give_gpu(gpu)
        return r

    def _take_gpu(self) -> int:
        if not self.gpu_users:
            return -1
        g = min(range(len(self.gpu_users)), key=lambda i: self.gpu_users[i])
        self.gpu_users[g] += 1
        return g

    def _give_gpu(self, g: int) -> None:
        if 0 <= g < len(self.gpu_users) and self.gpu_users[g] > 0:
            self.gpu_users[g] -= 1

    def stop_all(self) -> None:
        with self.lock:
            allp = [p for procs in self.children.values() for p in procs]
            self.children.clear()
        for p, port, _, _ in allp:
            _kill(p)

    def close(self) -> None:
        self._stop.set()
        self.stop_all()
        self.ls.close()


def _kill(p: subprocess.Popen, timeout: float = 10.0) -> bool:
    if p.poll() is not None:
        return True
    p.send_signal(signal.SIGTERM)
    try:
        p.wait(timeout=timeout)
    except subprocess.TimeoutExpired:
        p.kill()
        p.wait()
    return True


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser(prog="jubavisor")
    ap.add_argument("-p", "--rpc-port", type=int, default=9198)
    ap.add_argument("-z", "--zookeeper", default="localhost:2181")
    ap.add_argument("-m", "--max-children", type=int, default=16)
    ap.add_argument("-l", "--logdir", default="")
    ap.add_argument("-t", "--timeout", type=int, default=10)
    ap.add_argument("-G", "--gpus", type=int, default=-1,
                    help="GPUs handed out one per child (--gpu i); default: the host's count")
    ap.add_argument("-b", "--listen_addr", default="",
                    help="address to register and to bind children to (default: primary IPv4)")
    a = ap.parse_args(argv)
    system.set_program_name("jubavisor")
    v = Jubavisor(a.zookeeper, a.rpc_port, a.max_children, a.timeout, a.listen_addr, a.gpus)
    srv = RpcServer(2)
    srv.add("start", v.start, arity=3)
    srv.add("stop", v.stop, arity=2)
    port = srv.listen(a.rpc_port, a.listen_addr or "0.0.0.0")
    srv.start()
    log.info("jubavisor listening at %s:%d", v.ip, port)
    done = threading.Event()
    for sig in (signal.SIGINT, signal.SIGTERM):
        signal.signal(sig, lambda *_: done.set())
    while not done.wait(0.5):
        pass
    srv.stop()
    v.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
