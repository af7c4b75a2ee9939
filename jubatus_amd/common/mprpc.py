"""msgpack-RPC: server facade over the native transport, client, multi-client.

Reference: jubatus/server/common/mprpc/ - rpc_server (C1, dispatch and error
mapping rpc_server.cpp:31-54), rpc_mclient (C2, fan-out + reduce
rpc_mclient.hpp:100-312), rpc_result/rpc_error (C3), exception taxonomy
(exception.hpp:32-73).

Wire protocol: request [0, msgid, method, params], response
[1, msgid, error, result], notification [2, method, params]. Strings are
encoded in the old msgpack spec (RAW, ``use_bin_type=False``) like the
reference's msgpack 0.5.9; both specs are accepted on input.

Error values (reference rpc_server.cpp:36-53; numeric values are the
msgpack-rpc library's):
  NO_METHOD_ERROR = 1    unknown method
  ARGUMENT_ERROR  = 2    wrong arity / argument type
  "<message>"            any other exception, as its message string
"""
from __future__ import annotations

import concurrent.futures as cf
import errno
import itertools
import os
import random
import socket
import threading
import time
from dataclasses import dataclass, field
from typing import Any, Callable, Sequence

import msgpack

from .._native import native
from ..utils import fault, trace

NO_METHOD_ERROR = 1
ARGUMENT_ERROR = 2

REQUEST, RESPONSE, NOTIFY = 0, 1, 2


def packb(obj: Any) -> bytes:
    return msgpack.packb(obj, use_bin_type=False)


def unpackb(b: bytes) -> Any:
    return msgpack.unpackb(b, raw=False, unicode_errors="surrogateescape", strict_map_key=False)


# ------------------------------------------------------------------ errors
class RpcError(Exception):
    """Base of every client-side RPC failure (reference exception.hpp)."""

    def __init__(self, msg: str = "", host: str | None = None, port: int | None = None):
        super().__init__(msg)
        self.host, self.port = host, port


class RpcNoClient(RpcError):
    pass


class RpcNoResult(RpcError):
    def __init__(self, msg: str, errors: list["RpcErrorInfo"]):
        super().__init__(msg)
        self.errors = errors


class RpcIOError(RpcError):
    pass


class RpcTimeoutError(RpcError):
    pass


class RpcCallError(RpcError):
    """The server raised: ``error`` is its message."""


class RpcMethodNotFound(RpcError):
    pass


class RpcTypeError(RpcError):
    pass


from .exceptions import ArgumentError  # noqa: E402  (re-export)


def error_from_wire(err: Any, host=None, port=None) -> RpcError:
    if err == NO_METHOD_ERROR:
        return RpcMethodNotFound("method not found", host, port)
    if err == ARGUMENT_ERROR:
        return RpcTypeError("type mismatch", host, port)
    if isinstance(err, bytes):
        err = err.decode("utf-8", "replace")
    return RpcCallError(str(err), host, port)


# ------------------------------------------------------------------ server
@dataclass
class _Method:
    fn: Callable
    arity: int | None
    raw: bool


class RpcServer:
    """Method table + dispatcher in Python, transport in C++
    (csrc/native/jb_rpc.cpp). ``raw`` methods receive the undecoded params
    bytes (the train/classify fast path hands them to the GPU scanner)."""

    def __init__(self, nthreads: int = 2, idle_timeout: float = 0.0, io_threads: int | None = None):
        self._methods: dict[str, _Method] = {}
        self._batch: dict[str, Callable] = {}
        self._srv = native().RpcServer(self._dispatch, nthreads, idle_timeout)
        # epoll IO threads (request framing): one per 4 workers
        self._srv.set_io_threads(io_threads or max(1, nthreads // 4))
        self.port: int | None = None
        self.on_request: Callable[[str], None] | None = None

    def add(self, name: str, fn: Callable, arity: int | None = None, raw: bool = False) -> None:
        self._methods[name] = _Method(fn, arity, raw)

    def add_batch(self, name: str, fn: Callable[[list], list]) -> None:
        """Transport-level batching: every queued request of ``name`` is
        served by ONE call ``fn(list of params bytes) -> list of results``
        (a result may be an Exception: ArgumentError -> ARGUMENT_ERROR,
        others -> message string). Register before start()."""
        self._batch[name] = fn
        self._srv.set_batch(sorted(self._batch), self._dispatch_batch)

    def set_ordered(self, names: list[str]) -> None:
        """Batched methods that write: a batch never takes a request past one
        of another method when either is one of these (pipelined writes of
        different methods apply in arrival order; reads still batch past
        reads). Register before start()."""
        self._srv.set_ordered(sorted(names))

    def set_arena(self, name: str, slots: list[int], slot_bytes: int, fn: Callable) -> None:
        """Arena batching (csrc/native/jb_rpc.cpp): the IO threads copy each
        ``name`` request's body (params [cluster name, body]) into one of the
        pinned ``slots``; ``fn(slot, offs, lens) -> (results int64[n], errors
        dict)`` serves a whole slot; the slot is reused after
        ``release_slot``. Register before start()."""
        self._srv.set_arena_batch(name, list(slots), int(slot_bytes), fn)
        # serve slot k while slot k+1 is submitted
        self._srv.set_batch_threads(int(os.environ.get("JUBATUS_ARENA_THREADS", "2")))

    def release_slot(self, slot: int) -> None:
        self._srv.release_slot(int(slot))

    def batches(self) -> int:
        return self._srv.batches()

    def arena_ns(self) -> tuple[int, int]:
        """nanoseconds the arena batches spent in the handler / sending replies"""
        return tuple(self._srv.arena_ns())

    def _dispatch_batch(self, method: str, params: list, msgids: list) -> list:
        fn = self._batch[method]
        if self.on_request is not None:
            for _ in params:
                try:
                    self.on_request(method)
                except Exception:  # noqa: BLE001
                    pass
        # per-request fault injection (utils/fault.py): drop -> no reply,
        # error -> that request fails; the others are served
        keep, pre = [], {}
        for i in range(len(params)):
            try:
                if fault.on_rpc(method) == "drop":
                    pre[i] = None
                    continue
            except Exception as e:  # noqa: BLE001
                pre[i] = e
                continue
            keep.append(i)
        t0 = time.perf_counter_ns()
        try:
            got = list(fn([params[i] for i in keep])) if keep else []
        except Exception as e:  # noqa: BLE001 - the whole batch failed
            got = [e] * len(keep)
        trace.record("rpc." + method, time.perf_counter_ns() - t0)
        results = [None] * len(params)
        for i, r in zip(keep, got):
            results[i] = r
        out = []
        for i, (mid, r) in enumerate(zip(msgids, results)):
            if i in pre:
                r = pre[i]
                if r is None:
                    out.append(None)
                    continue
            if isinstance(r, ArgumentError):
                out.append(packb([RESPONSE, mid, ARGUMENT_ERROR, None]))
            elif isinstance(r, Exception):
                out.append(packb([RESPONSE, mid, str(r) or type(r).__name__, None]))
            else:
                try:
                    out.append(packb([RESPONSE, mid, None, r]))
                except Exception as e:  # noqa: BLE001
                    out.append(packb([RESPONSE, mid, f"failed to encode result: {e}", None]))
        return out

    def remove(self, name: str) -> None:
        self._methods.pop(name, None)

    def methods(self) -> list[str]:
        return sorted(self._methods)

    def listen(self, port: int, bind: str = "0.0.0.0") -> int:
        self.port = self._srv.listen(bind, port)
        return self.port

    def start(self) -> None:
        self._srv.start()

    def stop(self) -> None:
        self._srv.stop()

    def running(self) -> bool:
        return self._srv.running()

    def served(self) -> int:
        return self._srv.served()

    def _dispatch(self, method: str, params: bytes, msgid: int, notify: bool) -> bytes | None:
        m = self._methods.get(method)
        if self.on_request is not None:
            try:
                self.on_request(method)
            except Exception:
                pass
        err: Any = None
        result: Any = None
        if m is None:
            err = NO_METHOD_ERROR
        else:
            t0 = time.perf_counter_ns()
            try:
                if fault.on_rpc(method) == "drop":
                    return None
                if m.raw:
                    result = m.fn(params)
                else:
                    args = unpackb(params)
                    if not isinstance(args, list):
                        raise ArgumentError("params must be an array")
                    if m.arity is not None and len(args) != m.arity:
                        raise ArgumentError(f"{method}: expected {m.arity} arguments, got {len(args)}")
                    result = m.fn(*args)
            except ArgumentError:
                err = ARGUMENT_ERROR
            except Exception as e:  # application error -> message string
                err = str(e) or type(e).__name__
            trace.record("rpc." + method, time.perf_counter_ns() - t0)
        if notify:
            return None
        try:
            return packb([RESPONSE, msgid, err, result])
        except Exception as e:
            return packb([RESPONSE, msgid, f"failed to encode result: {e}", None])


def name_and_rest(params) -> memoryview:
    """O(1) split of a 2-element params array [name: raw, data]: returns a
    view of ``data`` (unvalidated - the consumer's native scanner validates
    it). Raises ArgumentError unless params is a 2-array led by a raw."""
    mv = memoryview(params).cast("B")
    n = len(mv)
    if n < 2 or mv[0] != 0x92:
        raise ArgumentError("expected a 2-element params array")
    t = mv[1]
    if 0xA0 <= t <= 0xBF:
        pos = 2 + (t & 0x1F)
    elif t in (0xD9, 0xC4) and n >= 3:
        pos = 3 + mv[2]
    elif t in (0xDA, 0xC5) and n >= 4:
        pos = 4 + ((mv[2] << 8) | mv[3])
    elif t in (0xDB, 0xC6) and n >= 6:
        pos = 6 + ((mv[2] << 24) | (mv[3] << 16) | (mv[4] << 8) | mv[5])
    else:
        raise ArgumentError("cluster name must be a string")
    if pos >= n:
        raise ArgumentError("truncated params")
    return mv[pos:]


def split_params(params: bytes) -> list[memoryview]:
    """Top-level elements of a params array as zero-copy views."""
    mv = memoryview(params)
    nat = native()
    b0 = params[0]
    if 0x90 <= b0 <= 0x9F:
        n, pos = b0 & 0x0F, 1
    elif b0 == 0xDC:
        n, pos = int.from_bytes(params[1:3], "big"), 3
    elif b0 == 0xDD:
        n, pos = int.from_bytes(params[1:5], "big"), 5
    else:
        raise ArgumentError("params must be an array")
    out = []
    for _ in range(n):
        ln = nat.msgpack_frame(mv[pos:])
        if ln <= 0:
            raise ArgumentError("malformed params")
        out.append(mv[pos:pos + ln])
        pos += ln
    return out


# ------------------------------------------------------------------ client
class RpcClient:
    """Synchronous msgpack-RPC client with a persistent connection."""

    def __init__(self, host: str, port: int, timeout: float = 10.0):
        self.host, self.port, self.timeout = host, int(port), float(timeout)
        self._sock: socket.socket | None = None
        self._unpacker = None
        self._ids = itertools.count(1)
        self._lock = threading.Lock()

    def _connect(self) -> None:
        try:
            s = socket.create_connection((self.host, self.port), timeout=self.timeout)
        except socket.timeout as e:
            raise RpcTimeoutError(f"connect timeout {self.host}:{self.port}", self.host, self.port) from e
        except OSError as e:
            raise RpcIOError(f"connect failed {self.host}:{self.port}: {e}", self.host, self.port) from e
        s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self._sock = s
        self._unpacker = msgpack.Unpacker(raw=False, unicode_errors="surrogateescape",
                                          strict_map_key=False, max_buffer_size=1 << 31)

    def close(self) -> None:
        with self._lock:
            if self._sock is not None:
                try:
                    self._sock.close()
                finally:
                    self._sock = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def call(self, method: str, *args: Any) -> Any:
        return self.call_raw(method, packb(list(args)))

    def call_raw(self, method: str, params: bytes) -> Any:
        """params: an already-encoded msgpack array."""
        with self._lock:
            if self._sock is None:
                self._connect()
            msgid = next(self._ids) & 0xFFFFFFFF
            head = packb([REQUEST, msgid, method])
            # splice: [0, msgid, method] header of a 4-array + encoded params
            req = bytes([0x94]) + head[1:] + params
            try:
                self._sock.sendall(req)
                deadline = time.monotonic() + self.timeout
                while True:
                    for msg in self._unpacker:
                        if (isinstance(msg, list) and len(msg) == 4 and msg[0] == RESPONSE
                                and msg[1] == msgid):
                            if msg[2] is not None:
                                raise error_from_wire(msg[2], self.host, self.port)
                            return msg[3]
                    left = deadline - time.monotonic()
                    if left <= 0:
                        raise socket.timeout()
                    self._sock.settimeout(left)
                    chunk = self._sock.recv(1 << 20)
                    if not chunk:
                        raise ConnectionResetError("connection closed by peer")
                    self._unpacker.feed(chunk)
            except socket.timeout as e:
                self._drop()
                raise RpcTimeoutError(f"timeout calling {method} on {self.host}:{self.port}",
                                      self.host, self.port) from e
            except RpcError:
                raise
            except OSError as e:
                self._drop()
                raise RpcIOError(f"io error calling {method} on {self.host}:{self.port}: {e}",
                                 self.host, self.port) from e

    def notify(self, method: str, *args: Any) -> None:
        with self._lock:
            if self._sock is None:
                self._connect()
            self._sock.sendall(packb([NOTIFY, method, list(args)]))

    def _drop(self) -> None:
        try:
            if self._sock is not None:
                self._sock.close()
        finally:
            self._sock = None


# ------------------------------------------------------------ multi-client
@dataclass
class RpcErrorInfo:
    host: str
    port: int
    error: Exception

    def __str__(self) -> str:
        return f"{self.host}:{self.port}: {type(self.error).__name__}: {self.error}"


@dataclass
class RpcResult:
    value: Any = None
    errors: list[RpcErrorInfo] = field(default_factory=list)
    responses: list[Any] = field(default_factory=list)

    def has_error(self) -> bool:
        return bool(self.errors)


class RpcMClient:
    """Fan one call out to many hosts and fold the results (reference
    rpc_mclient.hpp:136-199): raises RpcNoClient without hosts and
    RpcNoResult when every host failed; partial failures are reported in
    ``RpcResult.errors``."""

    _pool = cf.ThreadPoolExecutor(max_workers=32, thread_name_prefix="mclient")

    def __init__(self, hosts: Sequence[tuple[str, int]], timeout: float = 10.0):
        self.hosts = [(h, int(p)) for h, p in hosts]
        self.timeout = timeout

    def call(self, method: str, *args: Any, reducer: Callable[[Any, Any], Any] | None = None
             ) -> RpcResult:
        if not self.hosts:
            raise RpcNoClient("no client")
        params = packb(list(args))

        def one(hp):
            with RpcClient(hp[0], hp[1], self.timeout) as c:
                return c.call_raw(method, params)
        futs = [(hp, self._pool.submit(one, hp)) for hp in self.hosts]
        res = RpcResult()
        first = True
        for hp, f in futs:
            try:
                v = f.result()
            except Exception as e:  # noqa: BLE001 - collected per host
                res.errors.append(RpcErrorInfo(hp[0], hp[1], e))
                continue
            res.responses.append(v)
            if reducer is None:
                if first:
                    res.value = v
            else:
                res.value = v if first else reducer(res.value, v)
            first = False
        if first:
            raise RpcNoResult("no result: " + "; ".join(map(str, res.errors)), res.errors)
        return res


def choose(hosts: Sequence[Any]) -> Any:
    return random.choice(list(hosts))


def wait_server(host: str, port: int, timeout: float = 10.0) -> bool:
    """Poll until a TCP server accepts (reference test helper, rpc_client_test.cpp:57-75)."""
    deadline = time.monotonic() + timeout
    delay = 0.01
    while time.monotonic() < deadline:
        try:
            with socket.create_connection((host, port), timeout=1.0):
                return True
        except OSError as e:
            if e.errno not in (errno.ECONNREFUSED, errno.ECONNRESET, None) and \
                    not isinstance(e, socket.timeout):
                pass
            time.sleep(delay)
            delay = min(delay * 2, 0.2)
    return False
