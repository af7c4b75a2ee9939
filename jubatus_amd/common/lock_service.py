"""Coordination service: the ``lock_service`` API and its implementations
(reference C5 lock_service.hpp:34-119, C6 zk.cpp, C7 cached_zk.cpp).

The reference runs on ZooKeeper 3.4. This framework ships its own
coordinator with ZooKeeper's data model and the subset of semantics Jubatus
uses, so a node needs no JVM:

* a tree of nodes with data, a data version and a child version;
* ``create`` needs the parent (non-ephemeral create of an existing node is
  a success, as zk.cpp:158-177); ephemeral nodes are owned by a session and
  removed when it closes or its heartbeat TTL expires;
* ``create_seq``: ephemeral sequential node, name = path + 10-digit counter;
* ``create_id``: bump a node's data version -> (prefix << 32) | version
  (zk.cpp:218-232);
* watches (data/exists, children, delete) are one-shot, delivered by a
  client-side poller that compares node stats.

Implementations:
  ZNodeStore            the tree itself (thread-safe)
  LocalLockService      in-process session on a ZNodeStore (tests, single-node)
  CoordinatorClient     session on a remote ``jubacoordinator`` over msgpack-RPC
  CachedLockService     list()/read() cache invalidated by watches (proxies)
"""
from __future__ import annotations

import itertools
import threading
import time
from dataclasses import dataclass, field
from typing import Callable

from ..utils import logger

log = logger.get_logger("lock_service")

OK, NONODE, NODEEXISTS, NOTEMPTY, NOCHILDREN_FOR_EPHEMERALS, BADARGS, SESSION_EXPIRED = \
    0, -101, -110, -111, -108, -8, -112


def _parent(path: str) -> str:
    p = path.rstrip("/").rsplit("/", 1)[0]
    return p or "/"


def _valid(path: str) -> bool:
    return path.startswith("/") and (path == "/" or not path.endswith("/")) and "//" not in path


@dataclass
class _Node:
    data: str = ""
    owner: int = 0            # ephemeral owner session (0: persistent)
    version: int = 0          # data version
    cversion: int = 0         # child version (also the sequence counter)
    mzxid: int = 0
    pzxid: int = 0
    children: set = field(default_factory=set)


class ZNodeStore:
    """The coordinator's node tree and sessions."""

    def __init__(self):
        self._lock = threading.RLock()
        self._nodes: dict[str, _Node] = {"/": _Node()}
        self._sessions: dict[int, list] = {}   # sid -> [timeout, last_heartbeat]
        self._sid = itertools.count(1)
        self._zxid = 0

    def _tick(self) -> int:
        self._zxid += 1
        return self._zxid

    # ---- sessions
    def open_session(self, timeout: float) -> int:
        with self._lock:
            sid = next(self._sid)
            self._sessions[sid] = [float(timeout), time.monotonic()]
            return sid

    def heartbeat(self, sid: int) -> bool:
        with self._lock:
            s = self._sessions.get(sid)
            if s is None:
                return False
            s[1] = time.monotonic()
            return True

    def close_session(self, sid: int) -> None:
        with self._lock:
            self._sessions.pop(sid, None)
            for p in sorted((p for p, n in self._nodes.items() if n.owner == sid),
                            key=len, reverse=True):
                self._remove(p, force=True)

    def expire_sessions(self) -> list[int]:
        now = time.monotonic()
        with self._lock:
            dead = [sid for sid, (to, hb) in self._sessions.items() if now - hb > to]
            for sid in dead:
                log.info("session %d expired", sid)
                self.close_session(sid)
            return dead

    def session_alive(self, sid: int) -> bool:
        with self._lock:
            return sid in self._sessions

    # ---- nodes
    def create(self, sid: int, path: str, data: str = "", ephemeral: bool = False) -> int:
        with self._lock:
            if not _valid(path) or path == "/":
                return BADARGS
            if ephemeral and sid not in self._sessions:
                return SESSION_EXPIRED
            if path in self._nodes:
                return NODEEXISTS
            par = self._nodes.get(_parent(path))
            if par is None:
                return NONODE
            if par.owner:
                return NOCHILDREN_FOR_EPHEMERALS
            z = self._tick()
            self._nodes[path] = _Node(data=data, owner=sid if ephemeral else 0, mzxid=z, pzxid=z)
            par.children.add(path.rsplit("/", 1)[1])
            par.cversion += 1
            par.pzxid = z
            return OK

    def create_seq(self, sid: int, path: str, data: str = "", ephemeral: bool = True
                   ) -> tuple[int, str]:
        with self._lock:
            par = self._nodes.get(_parent(path))
            if par is None:
                return NONODE, ""
            actual = f"{path}{par.cversion:010d}"
            return self.create(sid, actual, data, ephemeral), actual

    def set(self, path: str, data: str) -> tuple[int, int]:
        with self._lock:
            n = self._nodes.get(path)
            if n is None:
                return NONODE, -1
            n.data = data
            n.version += 1
            n.mzxid = self._tick()
            return OK, n.version

    def _remove(self, path: str, force: bool = False) -> int:
        n = self._nodes.get(path)
        if n is None:
            return NONODE
        if n.children and not force:
            return NOTEMPTY
        for c in list(n.children):
            self._remove(f"{path}/{c}" if path != "/" else f"/{c}", force=True)
        del self._nodes[path]
        par = self._nodes.get(_parent(path))
        if par is not None:
            par.children.discard(path.rsplit("/", 1)[1])
            par.cversion += 1
            par.pzxid = self._tick()
        return OK

    def remove(self, path: str) -> int:
        with self._lock:
            if path == "/":
                return BADARGS
            return self._remove(path)

    def exists(self, path: str) -> bool:
        with self._lock:
            return path in self._nodes

    def list(self, path: str) -> tuple[int, list[str]]:
        with self._lock:
            n = self._nodes.get(path)
            if n is None:
                return NONODE, []
            return OK, sorted(n.children)

    def read(self, path: str) -> tuple[int, str, int]:
        with self._lock:
            n = self._nodes.get(path)
            if n is None:
                return NONODE, "", -1
            return OK, n.data, n.version

    def stat_many(self, paths: list[str]) -> list[list]:
        """[(exists, mzxid, pzxid)] - the watch poller's input."""
        with self._lock:
            out = []
            for p in paths:
                n = self._nodes.get(p)
                out.append([False, 0, 0] if n is None else [True, n.mzxid, n.pzxid])
            return out

    def dump(self) -> dict[str, str]:
        with self._lock:
            return {p: n.data for p, n in self._nodes.items()}


class LockService:
    """The reference's abstract coordination API (lock_service.hpp:34-86)."""

    def __init__(self):
        self._cleanups: list[Callable[[], None]] = []
        self._watches: list[list] = []  # [path, kind, callback, last_stat]
        self._wlock = threading.Lock()
        self._poller: threading.Thread | None = None
        self._stop = threading.Event()
        self.poll_interval = 0.1

    # to implement: _create, _create_seq, _set, _remove, exists, list, read, _stat_many,
    # get_connected_host_and_port, get_hosts, type, close
    def create(self, path: str, payload: str = "", ephemeral: bool = False) -> bool:
        rc = self._create(path, payload, ephemeral)
        if rc == OK or (rc == NODEEXISTS and not ephemeral):
            return True
        if rc != NODEEXISTS:
            log.error("failed to create node: %s (%d)", path, rc)
        return False

    def set(self, path: str, payload: str) -> bool:
        rc, _ = self._set(path, payload)
        return rc == OK

    def remove(self, path: str) -> bool:
        rc = self._remove(path)
        return rc in (OK, NONODE)

    def create_seq(self, path: str) -> str:
        rc, actual = self._create_seq(path)
        if rc != OK:
            log.error("failed to create sequential node: %s (%d)", path, rc)
            return ""
        return actual

    def create_id(self, path: str, prefix: int = 0) -> int:
        rc, version = self._set(path, "dummy")
        if rc != OK:
            raise RuntimeError(f"failed to increment version of node: {path}")
        return (int(prefix) << 32) | version

    def hd_list(self, path: str) -> str:
        """first child in sort order ("" if none)."""
        ch = self.list(path)
        return ch[0] if ch else ""

    def push_cleanup(self, fn: Callable[[], None]) -> None:
        self._cleanups.append(fn)

    def run_cleanup(self) -> None:
        for fn in list(self._cleanups):
            try:
                fn()
            except Exception:  # noqa: BLE001
                log.exception("cleanup failed")

    def reopen_logfile(self) -> None:
        pass

    # ---- watches (one-shot, client-side polling)
    def _watch(self, path: str, kind: str, cb: Callable[[str], None]) -> bool:
        st = self._stat_many([path])[0]
        with self._wlock:
            self._watches.append([path, kind, cb, st])
            if self._poller is None:
                self._poller = threading.Thread(target=self._poll_loop, name="coord-watch",
                                                 daemon=True)
                self._poller.start()
        return True

    def bind_watcher(self, path: str, cb: Callable[[str], None]) -> bool:
        """fires when the node's data changes, or it is created/deleted"""
        return self._watch(path, "data", cb)

    def bind_child_watcher(self, path: str, cb: Callable[[str], None]) -> bool:
        return self._watch(path, "child", cb)

    def bind_delete_watcher(self, path: str, cb: Callable[[str], None]) -> bool:
        return self._watch(path, "delete", cb)

    def _poll_loop(self) -> None:
        while not self._stop.wait(self.poll_interval):
            with self._wlock:
                ws = list(self._watches)
            if not ws:
                continue
            try:
                stats = self._stat_many([w[0] for w in ws])
            except Exception:  # noqa: BLE001 - coordinator unreachable
                continue
            fired = []
            for w, st in zip(ws, stats):
                path, kind, cb, old = w
                hit = False
                if kind == "delete":
                    hit = old[0] and not st[0]
                elif kind == "child":
                    hit = old[0] != st[0] or old[2] != st[2]
                else:
                    hit = old[0] != st[0] or old[1] != st[1]
                if hit:
                    fired.append(w)
            if fired:
                with self._wlock:
                    for w in fired:
                        if w in self._watches:
                            self._watches.remove(w)
                for path, kind, cb, _ in fired:
                    try:
                        cb(path)
                    except Exception:  # noqa: BLE001
                        log.exception("watch callback failed: %s", path)

    def close(self) -> None:
        self._stop.set()


class LocalLockService(LockService):
    """A session on an in-process ZNodeStore (the reference's zk_stub role,
    push_mixer_test_util.hpp:40-127, but with real semantics)."""

    def __init__(self, store: ZNodeStore | None = None, timeout: float = 10.0):
        super().__init__()
        self.store = store or ZNodeStore()
        self.sid = self.store.open_session(timeout)
        self._closed = False

    def _create(self, path, payload, ephemeral):
        return self.store.create(self.sid, path, payload, ephemeral)

    def _create_seq(self, path):
        return self.store.create_seq(self.sid, path)

    def _set(self, path, payload):
        return self.store.set(path, payload)

    def _remove(self, path):
        return self.store.remove(path)

    def exists(self, path: str) -> bool:
        return self.store.exists(path)

    def list(self, path: str) -> list[str]:
        return self.store.list(path)[1]

    def read(self, path: str) -> str | None:
        rc, data, _ = self.store.read(path)
        return data if rc == OK else None

    def _stat_many(self, paths):
        return self.store.stat_many(paths)

    def get_connected_host_and_port(self) -> str:
        return "local"

    def get_hosts(self) -> str:
        return "local"

    def type(self) -> str:
        return "local"

    def close(self) -> None:
        super().close()
        if not self._closed:
            self._closed = True
            self.store.close_session(self.sid)


class CoordinatorClient(LockService):
    """Session on a remote jubacoordinator (``-z host:port[,host:port...]``)."""

    def __init__(self, hosts: str, timeout: float = 10.0, logfile: str = ""):
        super().__init__()
        from .mprpc import RpcClient
        self.hosts = hosts
        self.timeout = float(timeout)
        self._cl = None
        last = None
        deadline = time.monotonic() + self.timeout
        while self._cl is None:
            for hp in hosts.split(","):
                h, _, p = hp.strip().rpartition(":")
                try:
                    c = RpcClient(h or "127.0.0.1", int(p), timeout=self.timeout)
                    self.sid = c.call("open_session", self.timeout)
                    self._cl, self.connected = c, f"{h}:{p}"
                    break
                except Exception as e:  # noqa: BLE001
                    last = e
            if self._cl is None:
                if time.monotonic() > deadline:
                    raise RuntimeError(f"failed to connect to coordinator {hosts}: {last}")
                time.sleep(0.2)
        self._call_lock = threading.Lock()
        self._hb = threading.Thread(target=self._heartbeat, name="coord-heartbeat", daemon=True)
        self._hb.start()

    def _call(self, method, *args):
        with self._call_lock:
            return self._cl.call(method, *args)

    def _heartbeat(self) -> None:
        period = max(0.05, self.timeout / 3.0)
        while not self._stop.wait(period):
            try:
                alive = self._call("heartbeat", self.sid)
            except Exception:  # noqa: BLE001
                alive = None  # unreachable: keep trying until our TTL would expire
            if alive is False:
                log.error("coordinator session expired")
                self.run_cleanup()
                return

    def _create(self, path, payload, ephemeral):
        return self._call("create", self.sid, path, payload, bool(ephemeral))

    def _create_seq(self, path):
        rc, actual = self._call("create_seq", self.sid, path)
        return rc, actual

    def _set(self, path, payload):
        rc, v = self._call("set", path, payload)
        return rc, v

    def _remove(self, path):
        return self._call("remove", path)

    def exists(self, path: str) -> bool:
        return bool(self._call("exists", path))

    def list(self, path: str) -> list[str]:
        rc, ch = self._call("list", path)
        return list(ch) if rc == OK else []

    def read(self, path: str) -> str | None:
        rc, data, _ = self._call("read", path)
        return data if rc == OK else None

    def _stat_many(self, paths):
        return self._call("stat_many", list(paths))

    def get_connected_host_and_port(self) -> str:
        return self.connected

    def get_hosts(self) -> str:
        return self.hosts

    def type(self) -> str:
        return "coordinator"

    def close(self) -> None:
        if self._stop.is_set():
            return
        super().close()
        try:
            self._call("close_session", self.sid)
        except Exception:  # noqa: BLE001
            pass
        self._cl.close()


class CachedLockService(LockService):
    """list()/read() cache for proxies (reference C7 cached_zk.cpp:40-186):
    entries are filled on first use and dropped by a child/data watch."""

    def __init__(self, inner: LockService):
        super().__init__()
        self.inner = inner
        self._lock = threading.Lock()
        self._lists: dict[str, list[str]] = {}
        self._reads: dict[str, str | None] = {}

    def list(self, path: str) -> list[str]:
        with self._lock:
            if path in self._lists:
                return list(self._lists[path])
        ch = self.inner.list(path)
        with self._lock:
            self._lists[path] = list(ch)
        self.inner.bind_child_watcher(path, self._drop_list)
        return ch

    def _drop_list(self, path: str) -> None:
        with self._lock:
            self._lists.pop(path, None)

    def read(self, path: str) -> str | None:
        with self._lock:
            if path in self._reads:
                return self._reads[path]
        v = self.inner.read(path)
        with self._lock:
            self._reads[path] = v
        self.inner.bind_watcher(path, self._drop_read)
        return v

    def _drop_read(self, path: str) -> None:
        with self._lock:
            self._reads.pop(path, None)

    def __getattr__(self, name):  # everything else goes straight through
        return getattr(self.inner, name)

    def create(self, *a, **k):
        return self.inner.create(*a, **k)

    def set(self, *a, **k):
        return self.inner.set(*a, **k)

    def remove(self, *a, **k):
        return self.inner.remove(*a, **k)

    def create_seq(self, *a, **k):
        return self.inner.create_seq(*a, **k)

    def create_id(self, *a, **k):
        return self.inner.create_id(*a, **k)

    def exists(self, path: str) -> bool:
        return self.inner.exists(path)

    def bind_watcher(self, *a):
        return self.inner.bind_watcher(*a)

    def bind_child_watcher(self, *a):
        return self.inner.bind_child_watcher(*a)

    def bind_delete_watcher(self, *a):
        return self.inner.bind_delete_watcher(*a)

    def get_connected_host_and_port(self) -> str:
        return self.inner.get_connected_host_and_port()

    def close(self) -> None:
        self.inner.close()


_local_stores: dict[str, ZNodeStore] = {}


def create_lock_service(kind: str, hosts: str, timeout: float = 10.0, logfile: str = "") -> LockService:
    """kind: "coordinator" (alias "zk") or "cached_coordinator" (alias
    "cached_zk"); ``hosts`` of the form ``local:<name>`` selects an
    in-process store shared by every service of this process."""
    if hosts.startswith("local:"):
        store = _local_stores.setdefault(hosts, ZNodeStore())
        svc: LockService = LocalLockService(store, timeout)
    else:
        svc = CoordinatorClient(hosts, timeout, logfile)
    if kind in ("cached_zk", "cached_coordinator"):
        return CachedLockService(svc)
    if kind not in ("zk", "coordinator"):
        raise ValueError(f"unknown lock service: {kind}")
    return svc


class LockServiceMutex:
    """try-only read/write lock from ephemeral sequential nodes (reference
    zkmutex, zk.cpp:530-631): the lowest ``wlock_`` wins the write lock; a
    reader wins when no ``wlock_`` precedes its ``rlock_``."""

    def __init__(self, ls: LockService, path: str):
        self.ls, self.path = ls, path
        self.seqfile = ""
        self.has_lock = False
        ls.create(path, "")

    def _try(self, prefix: str, ok: Callable[[list[str], str], bool]) -> bool:
        if self.has_lock:
            return True
        seq = self.ls.create_seq(f"{self.path}/{prefix}")
        if not seq:
            return False
        me = seq.rsplit("/", 1)[1]
        ch = self.ls.list(self.path)
        if ok(ch, me):
            self.seqfile, self.has_lock = seq, True
            return True
        self.ls.remove(seq)
        return False

    def try_lock(self) -> bool:
        def ok(ch, me):
            def seqno(n):
                return int(n[-10:])
            return min(ch, key=seqno) == me
        return self._try("wlock_", ok)

    def try_rlock(self) -> bool:
        def ok(ch, me):
            mine = int(me[-10:])
            return not any(c.startswith("wlock_") and int(c[-10:]) < mine for c in ch)
        return self._try("rlock_", ok)

    def unlock(self) -> bool:
        if self.has_lock:
            self.ls.remove(self.seqfile)
            self.has_lock = False
            self.seqfile = ""
        return True

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.unlock()
