"""juba<engine>_proxy: stateless request router (reference C25:
jubatus/server/framework/{proxy.hpp,proxy.cpp,proxy_common.cpp}).

Routing per IDL method (idl/specs.py):
  random      one member chosen uniformly from ``actives`` (proxy.hpp:230-247)
  broadcast   every active member, results folded by the aggregator (:249-266)
  cht(n)      the n CHT owners of args[1] (the row/node id) (:268-286)
Defaults: get_config (random), save (broadcast, merge), load (broadcast,
all_and), get_status (broadcast, merge), get_proxy_status (local).

Requests are forwarded *without re-encoding*: the proxy reads only the
cluster name (and the id for cht) from the params bytes and relays them
verbatim. Member lists come from a watch-invalidated cache of the
coordinator (cached_zk). Per-thread session pools keep one connection per
server, expired after ``pool_expire`` seconds idle.
"""
from __future__ import annotations

import os
import random
import threading
import time
from typing import Any

from .. import __version__
from ..common import mprpc
from ..common.cht import CHT
from ..common.membership import build_actor_path, revert
from ..idl import specs
from ..utils import logger, system
from .aggregators import AGGREGATORS
from .server_util import ProxyArgv, get_proxy_identifier

log = logger.get_logger("proxy")


class _Pool(threading.local):
    def __init__(self):
        self.clients: dict[tuple[str, int], list] = {}  # (host, port) -> [client, last_used]


class Proxy:
    def __init__(self, argv: ProxyArgv, coord=None):
        self.argv = argv
        self.type = argv.type
        from ..common.lock_service import CachedLockService, create_lock_service
        raw = coord or create_lock_service("coordinator", argv.z, argv.zookeeper_timeout)
        self.coord = raw if isinstance(raw, CachedLockService) else CachedLockService(raw)
        self.start_time = time.time()
        self.request_counter = 0
        self.forward_counter = 0
        self._lock = threading.Lock()
        self._pool = _Pool()
        self.rpc = mprpc.RpcServer(nthreads=argv.threadnum)
        for m in specs.methods(self.type):
            if m.routing == "internal":
                continue
            self.rpc.add(m.name, self._route(m), raw=True)
        # clients send the cluster name (client.hpp:69-72); it is not needed here
        self.rpc.add("get_proxy_status", lambda *name: self.get_status())

    # ------------------------------------------------------------ members
    def members(self, name: str) -> list[tuple[str, int]]:
        return [revert(x) for x in self.coord.list(build_actor_path(self.type, name) + "/actives")]

    def _client(self, host: str, port: int) -> mprpc.RpcClient:
        now = time.time()
        key = (host, port)
        ent = self._pool.clients.get(key)
        exp = self.argv.session_pool_expire
        if ent is not None and exp and now - ent[1] > exp:
            ent[0].close()
            ent = None
        if ent is None:
            if self.argv.session_pool_size and len(self._pool.clients) >= self.argv.session_pool_size:
                old = min(self._pool.clients, key=lambda k: self._pool.clients[k][1])
                self._pool.clients.pop(old)[0].close()
            ent = [mprpc.RpcClient(host, port, self.argv.interconnect_timeout), now]
            self._pool.clients[key] = ent
        ent[1] = now
        return ent[0]

    def _forward(self, host: str, port: int, method: str, params: bytes) -> Any:
        c = self._client(host, port)
        try:
            return c.call_raw(method, params)
        except (mprpc.RpcIOError, mprpc.RpcTimeoutError):
            self._pool.clients.pop((host, port), None)  # evict broken session
            c.close()
            raise

    # ------------------------------------------------------------ routing
    def _route(self, m: specs.Method):
        agg = AGGREGATORS.get(m.agg, AGGREGATORS["pass"])

        def handler(params: bytes):
            with self._lock:
                self.request_counter += 1
            parts = mprpc.split_params(params)
            if len(parts) != m.arity:
                raise mprpc.ArgumentError(f"{m.name}: expected {m.arity} arguments")
            name = mprpc.unpackb(bytes(parts[0]))
            if not isinstance(name, str):
                raise mprpc.ArgumentError("cluster name must be a string")
            if m.routing == "random":
                targets = self.members(name)
                if not targets:
                    raise RuntimeError(f"no server found in coordinator: {self.type}/{name}")
                targets = [random.choice(targets)]
            elif m.routing == "broadcast":
                targets = self.members(name)
                if not targets:
                    raise RuntimeError(f"no server found in coordinator: {self.type}/{name}")
            else:  # cht
                key = mprpc.unpackb(bytes(parts[1]))
                targets = CHT(self.coord, self.type, name).find(str(key), m.cht_n)
            return self._fanout(m.name, params, targets, agg)
        return handler

    def _fanout(self, method: str, params: bytes, targets, agg) -> Any:
        with self._lock:
            self.forward_counter += len(targets)
        if len(targets) == 1:
            return self._forward(targets[0][0], targets[0][1], method, params)
        results, errors = [], []
        threads = []
        lock = threading.Lock()

        def one(h, p):
            try:
                r = self._forward(h, p, method, params)
                with lock:
                    results.append(r)
            except Exception as e:  # noqa: BLE001
                with lock:
                    errors.append((h, p, e))
        for h, p in targets:
            t = threading.Thread(target=one, args=(h, p))
            t.start()
            threads.append(t)
        for t in threads:
            t.join()
        if errors and not results:
            # prefer a transport error in the reply (proxy.hpp:325-376)
            errors.sort(key=lambda x: 0 if isinstance(x[2], (mprpc.RpcIOError, mprpc.RpcTimeoutError)) else 1)
            h, p, e = errors[0]
            raise RuntimeError(f"{h}:{p}: {e}")
        if errors:
            for h, p, e in errors:
                log.warning("partial failure from %s:%d: %s", h, p, e)
        out = results[0]
        for r in results[1:]:
            out = agg(out, r)
        return out

    # ------------------------------------------------------------ status
    def get_status(self) -> dict:
        with self._lock:
            self.request_counter += 1
        a = self.argv
        now = time.time()
        mt = system.get_machine_status()
        return {get_proxy_identifier(a): {
            "clock_time": str(int(now)), "start_time": str(int(self.start_time)),
            "uptime": str(int(now - self.start_time)),
            "VIRT": str(mt["VIRT"]), "RSS": str(mt["RSS"]), "SHR": str(mt["SHR"]),
            "VERSION": __version__, "PROGNAME": a.program_name, "pid": str(os.getpid()),
            "user": system.get_user_name(), "threadnum": str(a.threadnum),
            "timeout": str(a.timeout), "logdir": a.logdir, "log_config": a.log_config,
            "zookeeper": a.z, "connected_zookeeper": self.coord.get_connected_host_and_port(),
            "zookeeper_timeout": str(a.zookeeper_timeout),
            "interconnect_timeout": str(a.interconnect_timeout),
            "session_pool_expire": str(a.session_pool_expire),
            "session_pool_size": str(a.session_pool_size),
            "request_count": str(self.request_counter),
            "forward_count": str(self.forward_counter),
        }}

    # ------------------------------------------------------------ lifecycle
    def start(self, block: bool = True) -> int:
        port = self.rpc.listen(self.argv.port, self.argv.bind_address)
        if self.argv.port == 0:
            self.argv.port = port
        self.rpc.start()
        from ..common.membership import register_proxy
        register_proxy(self.coord, self.type, self.argv.eth, self.argv.port)
        log.info("%s_proxy listening at %d", self.type, self.argv.port)
        if block:
            from ..utils import signals
            stopped = threading.Event()
            if threading.current_thread() is threading.main_thread():
                signals.prepare_signal_handling()
                signals.set_action_on_term(lambda: (self.stop(), stopped.set()))
            while not stopped.wait(0.5):
                pass
        return 0

    def stop(self) -> None:
        self.rpc.stop()
        try:
            self.coord.close()
        except Exception:  # noqa: BLE001
            pass


def run_proxy(argv_list: list[str], type_: str) -> int:
    from .server_util import ArgvError
    try:
        a = ProxyArgv.parse(argv_list, type_)
    except ArgvError as e:
        return int(e.code or 0)
    return Proxy(a).start(block=True)
