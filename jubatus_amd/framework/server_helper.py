"""Server lifecycle (reference C19: jubatus/server/framework/server_helper.{hpp,cpp}
and run_server, server_util.hpp:135-161).

Construction order (server_helper.hpp:71-117): signals + coordinator
session -> prepare the /jubatus tree -> engine server -> config read-lock ->
``load_file(model_file)`` or ``set_config(get_conf())``. ``start()``: listen
-> RPC workers -> register membership (CHT vnodes when the service has cht
methods, the actor node, self-delete watch) -> TERM action -> mixer start ->
block. ``stop()``: mixer first, then leave the coordinator, then the RPC
server.

RPC methods are registered from the IDL table (idl/specs.py) with the lock
discipline of the generated impls: ``update`` = write lock +
event_model_updated (JWLOCK_), ``analysis`` = read lock (JRLOCK_),
``nolock`` = none (server_helper.hpp:296-303).
"""
from __future__ import annotations

import os
import threading
import time
from typing import Callable

from .. import __version__
from ..common import mprpc
from ..idl import specs
from ..utils import logger, signals, system, trace
from .mixer import create_mixer
from .server_util import ArgvError, ServerArgv, get_conf, get_server_identifier

log = logger.get_logger("server_helper")


class ServerHelper:
    def __init__(self, serv_cls, argv: ServerArgv, use_cht: bool | None = None,
                 coord=None, install_signals: bool = True):
        self.argv = argv
        self.type = argv.type
        self.use_cht = specs.uses_cht(self.type) if use_cht is None else use_cht
        self.start_time = time.time()
        self._stopped = threading.Event()
        self._stop_lock = threading.Lock()
        if install_signals and threading.current_thread() is threading.main_thread():
            signals.prepare_signal_handling()
            signals.set_action_on_hup(logger.reconfigure)
        self.coord = coord
        self.membership = None
        if not argv.is_standalone():
            from ..common import membership
            from ..common.lock_service import create_lock_service
            if self.coord is None:
                self.coord = create_lock_service("coordinator", argv.z, argv.zookeeper_timeout,
                                                 argv.logdir)
            self.membership = membership
            membership.prepare_jubatus(self.coord, self.type, argv.name)
        self.server = serv_cls(argv, self.coord)
        self.server.mixer = create_mixer(argv, self.coord, self.server.rw_mutex, self.type,
                                         self.server.user_data_version())
        self._config_lock = None
        if not argv.is_standalone():
            from ..common import config as zkconfig
            self._config_lock = zkconfig.get_config_lock(self.coord, self.type, argv.name, 3)
        if argv.is_standalone() and argv.modelpath:
            if argv.configpath:
                log.info("both model file and configuration are specified; using configuration "
                         "from model file")
            self.server.load_file(argv.modelpath)
        else:
            from .server_util import parse_config_json
            text = get_conf(argv, self.coord)
            parse_config_json(text, argv.configpath if argv.is_standalone() else "<coordinator>")
            self.server.set_config(text)
        self.rpc = mprpc.RpcServer(nthreads=argv.threadnum)
        self._register()
        if not argv.is_standalone():
            self.server.mixer.register_api(self.rpc)

    # ------------------------------------------------------------ dispatch
    def _wrap(self, m: specs.Method, fn: Callable) -> Callable:
        rw = self.server.rw_mutex
        srv = self.server
        n = m.arity

        def call(*args):
            if len(args) != n:
                raise mprpc.ArgumentError(f"{m.name}: expected {n} arguments")
            args = args[1:]  # cluster name, ignored by servers
            if m.lock == "update":
                with rw.write():
                    srv.event_model_updated()
                    return fn(*args)
            if m.lock == "analysis":
                with rw.read():
                    return fn(*args)
            return fn(*args)
        return call

    def _register(self) -> None:
        common = {"get_config": self.get_config, "save": self.save, "load": self.load,
                  "get_status": self.get_status}
        for m in specs.methods(self.type):
            fn = common.get(m.name) or getattr(self.server, m.name, None)
            if fn is None:
                raise RuntimeError(f"{self.type} server does not implement {m.name}")
            self.rpc.add(m.name, self._wrap(m, fn))
            raw = getattr(self.server, "raw_" + m.name, None)
            if raw is not None:  # zero-copy fast path (e.g. classifier train)
                self.rpc.add(m.name, self._wrap_raw(m, raw), raw=True)
        # arena batching: request bodies copied by the transport into pinned
        # memory, one call per filled slot (classifier train on the GPU)
        arenas = getattr(self.server, "arena_methods", lambda: {})()
        for name, (slots, slot_bytes, fn) in arenas.items():
            self.rpc.set_arena(name, slots, slot_bytes, self._wrap_arena(name, fn))
        # transport-level batching: every queued request of a method, one call
        batched = getattr(self.server, "batched_methods", lambda: {})()
        for m in specs.methods(self.type):
            if m.name in batched:
                self.rpc.add_batch(m.name, self._wrap_batch(m, batched[m.name]))

    def _wrap_raw(self, m: specs.Method, fn: Callable) -> Callable:
        rw = self.server.rw_mutex
        srv = self.server

        def call(params: bytes):
            if m.lock == "update":
                with rw.write():
                    srv.event_model_updated()
                    return fn(params)
            if m.lock == "analysis":
                with rw.read():
                    return fn(params)
            return fn(params)
        return call

    def _wrap_arena(self, name: str, fn: Callable) -> Callable:
        srv = self.server
        rpc = self.rpc

        def call(slot: int, offs, lens):
            try:
                with srv.rw_mutex.write():
                    srv.event_model_updated(len(offs))
                return fn(slot, offs, lens)
            finally:
                rpc.release_slot(slot)
        return call

    def _wrap_batch(self, m: specs.Method, fn: Callable) -> Callable:
        rw = self.server.rw_mutex
        srv = self.server

        def call(params_list: list) -> list:
            if m.lock == "update":
                with rw.write():
                    srv.event_model_updated(len(params_list))
                    return fn(params_list)
            if m.lock == "analysis":
                with rw.read():
                    return fn(params_list)
            return fn(params_list)
        return call

    # -------------------------------------------------------- common RPCs
    def get_config(self) -> str:
        return self.server.get_config()

    def save(self, model_id: str) -> dict[str, str]:
        return self.server.save(model_id)

    def load(self, model_id: str) -> bool:
        return self.server.load(model_id)

    def get_status(self) -> dict[str, dict[str, str]]:
        a = self.argv
        s = self.server
        now = time.time()
        mt = system.get_machine_status()
        data = {
            "clock_time": str(int(now)),
            "start_time": str(int(self.start_time)),
            "uptime": str(int(now - self.start_time)),
            "VIRT": str(mt["VIRT"]), "RSS": str(mt["RSS"]), "SHR": str(mt["SHR"]),
            "timeout": str(a.timeout),
            "threadnum": str(a.threadnum),
            "datadir": a.datadir,
            "is_standalone": "1" if a.is_standalone() else "0",
            "VERSION": __version__,
            "PROGNAME": a.program_name,
            "type": a.type,
            "logdir": a.logdir,
            "log_config": a.log_config,
            "configpath": a.configpath if a.is_standalone() else
            f"/jubatus/config/{a.type}/{a.name}",
            "pid": str(os.getpid()),
            "user": system.get_user_name(),
            "update_count": str(s.update_count),
            "last_saved": str(int(s.last_saved)),
            "last_saved_path": s.last_saved_path,
            "last_loaded": str(int(s.last_loaded)),
            "last_loaded_path": s.last_loaded_path,
        }
        s.get_status(data)
        # the device this server process owns (jubavisor hands out one GPU per
        # child with --gpu; "cpu": host backend)
        gpu = getattr(a, "gpu", None)
        data["gpu"] = "" if gpu is None else str(gpu)
        dev = getattr(s, "device", None)
        data.setdefault("device", str(dev) if dev is not None else "cpu")
        if not a.is_standalone():
            data.update({
                "zk": a.z, "name": a.name,
                "interval_sec": str(a.interval_sec), "interval_count": str(a.interval_count),
                "zookeeper_timeout": str(a.zookeeper_timeout),
                "interconnect_timeout": str(a.interconnect_timeout),
                "connected_zookeeper": self.coord.get_connected_host_and_port() if self.coord else "",
                "use_cht": "1" if self.use_cht else "0",
                "mixer": a.mixer,
            })
            s.mixer.get_status(data)
        data.update(trace.stats())
        return {get_server_identifier(a): data}

    # ----------------------------------------------------------- lifecycle
    def start(self, block: bool = True) -> int:
        a = self.argv
        try:
            port = self.rpc.listen(a.port, a.bind_address)
        except RuntimeError as e:
            log.critical("server failed to start: any process using port %s? (%s)", a.port, e)
            return -1
        if a.port == 0:  # ephemeral port (tests)
            a.port = port
        log.info("start listening at port %d", a.port)
        self.start_time = time.time()
        self.rpc.start()
        if not a.is_standalone():
            self._prepare_for_run()
        log.info("%s RPC server startup", a.program_name)
        if threading.current_thread() is threading.main_thread():
            signals.set_action_on_term(self.stop)
        if a.daemon:
            system.daemonize()
        if not a.is_standalone():
            self.server.mixer.start()
        if block:
            self.join()
        return 0

    def _prepare_for_run(self) -> None:
        a = self.argv
        ident = get_server_identifier(a)
        if self.use_cht:
            from ..common.cht import CHT
            CHT.setup_cht_dir(self.coord, a.type, a.name)
            CHT(self.coord, a.type, a.name).register_node(a.eth, a.port)
        self.membership.register_actor(self.coord, a.type, a.name, a.eth, a.port)
        self.membership.watch_delete_actor(self.coord, a.type, a.name, a.eth, a.port,
                                           lambda path: self.stop())
        log.info("registered group membership as %s", ident)

    def join(self) -> None:
        while not self._stopped.wait(0.2):
            pass

    def stop(self) -> None:
        with self._stop_lock:
            if self._stopped.is_set():
                return
            a = self.argv
            if not a.is_standalone():
                log.info("stopping mixer thread")
                try:
                    self.server.mixer.stop()
                except Exception:  # noqa: BLE001
                    log.exception("mixer stop failed")
                try:
                    self.membership.unregister_actor(self.coord, a.type, a.name, a.eth, a.port)
                except Exception:  # noqa: BLE001
                    pass
            log.info("stopping RPC server")
            self.rpc.stop()
            if self.coord is not None and hasattr(self.coord, "close"):
                try:
                    self.coord.close()
                except Exception:  # noqa: BLE001
                    pass
            self._stopped.set()


def run_server(serv_cls, argv_list: list[str], type_: str, prog: str | None = None) -> int:
    """parse argv -> construct -> start (reference run_server<Impl>)."""
    try:
        a = ServerArgv.parse(argv_list, type_, prog)
    except ArgvError as e:
        return int(e.code or 0)
    try:
        h = ServerHelper(serv_cls, a)
    except ArgvError as e:
        return int(e.code or 1)
    except Exception as e:  # noqa: BLE001
        log.critical("failed to start %s: %s", type_, e)
        return 1
    return h.start(block=True)
