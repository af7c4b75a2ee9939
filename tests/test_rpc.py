"""msgpack-RPC transport, client and multi-client (reference test strategy:
jubatus/server/common/mprpc/rpc_client_test.cpp - many in-process servers on
a port range, reducers, a 4 MiB payload, unknown methods, refused and
never-answering peers)."""
import socket
import threading

import msgpack
import pytest

from jubatus_amd.common import mprpc


@pytest.fixture
def servers():
    srvs = []
    for i in range(5):
        s = mprpc.RpcServer(nthreads=2)
        s.add("add", lambda a, b: a + b, arity=2)
        s.add("concat", lambda a, b: a + b, arity=2)
        s.add("ident", lambda v: v, arity=1)
        s.add("whoami", (lambda i: (lambda: i))(i), arity=0)
        s.add("boom", lambda: (_ for _ in ()).throw(RuntimeError("kaboom")), arity=0)
        s.add("rawlen", lambda params: len(params), raw=True)
        port = s.listen(0, "127.0.0.1")
        s.start()
        srvs.append((s, port))
    yield srvs
    for s, _ in srvs:
        s.stop()


def test_call_and_types(servers):
    _, port = servers[0]
    with mprpc.RpcClient("127.0.0.1", port) as c:
        assert c.call("add", 1, 2) == 3
        assert c.call("concat", "ab", "cd") == "abcd"
        assert c.call("ident", {"k": [1, 2.5, None, True]}) == {"k": [1, 2.5, None, True]}
        assert c.call("whoami") == 0
        assert c.call("rawlen", 1, 2) == len(msgpack.packb([1, 2]))


def test_errors(servers):
    _, port = servers[0]
    with mprpc.RpcClient("127.0.0.1", port) as c:
        with pytest.raises(mprpc.RpcMethodNotFound):
            c.call("nope")
        with pytest.raises(mprpc.RpcTypeError):
            c.call("add", 1)
        with pytest.raises(mprpc.RpcCallError, match="kaboom"):
            c.call("boom")
        assert c.call("add", 5, 6) == 11  # connection still usable


def test_wire_error_codes(servers):
    # raw protocol check: NO_METHOD_ERROR == 1, ARGUMENT_ERROR == 2
    _, port = servers[0]
    with socket.create_connection(("127.0.0.1", port)) as s:
        s.sendall(msgpack.packb([0, 7, "nope", []]) + msgpack.packb([0, 8, "add", [1]]))
        up = msgpack.Unpacker(raw=False)
        got = []
        while len(got) < 2:
            up.feed(s.recv(4096))
            got.extend(up)
    assert sorted(got) == [[1, 7, 1, None], [1, 8, 2, None]]


def test_old_spec_raw_strings(servers):
    _, port = servers[0]
    with socket.create_connection(("127.0.0.1", port)) as s:
        s.sendall(msgpack.packb([0, 1, "concat", ["x", "y"]], use_bin_type=False))
        resp = msgpack.unpackb(s.recv(4096), raw=True)
    assert resp == [1, 1, None, b"xy"]
    # the server answers with old-spec RAW (0xa2 fixraw), never str8/bin
    assert b"\xa2xy" in msgpack.packb([1, 1, None, "xy"], use_bin_type=False)


def test_mclient_reduce_and_big_payload(servers):
    hosts = [("127.0.0.1", p) for _, p in servers]
    mc = mprpc.RpcMClient(hosts)
    r = mc.call("whoami", reducer=lambda a, b: a + b)
    assert r.value == 0 + 1 + 2 + 3 + 4 and not r.errors
    r = mc.call("add", 1, 1, reducer=lambda a, b: a and b == 2)
    assert r.value
    big = list(range(1 << 20))  # ~4 MiB, reference rpc_client_test.cpp:384-394
    r = mc.call("ident", big, reducer=lambda a, b: a if a == b else None)
    assert r.value == big


def test_mclient_errors(servers):
    with pytest.raises(mprpc.RpcNoClient):
        mprpc.RpcMClient([]).call("whoami")
    hosts = [("127.0.0.1", p) for _, p in servers]
    with pytest.raises(mprpc.RpcNoResult) as ei:
        mprpc.RpcMClient(hosts).call("nope")
    assert all(isinstance(e.error, mprpc.RpcMethodNotFound) for e in ei.value.errors)
    # one refused peer -> partial result with an io error
    dead = socket.socket()
    dead.bind(("127.0.0.1", 0))
    dport = dead.getsockname()[1]
    dead.close()
    r = mprpc.RpcMClient(hosts[:2] + [("127.0.0.1", dport)]).call("whoami", reducer=max)
    assert r.value == 1 and len(r.errors) == 1
    assert isinstance(r.errors[0].error, mprpc.RpcIOError)


def test_timeout_on_silent_server():
    # a socket that accepts and never answers (rpc_client_test.cpp:177-266)
    ls = socket.socket()
    ls.bind(("127.0.0.1", 0))
    ls.listen(8)
    port = ls.getsockname()[1]
    conns = []
    t = threading.Thread(target=lambda: conns.append(ls.accept()), daemon=True)
    t.start()
    try:
        with pytest.raises(mprpc.RpcTimeoutError):
            mprpc.RpcClient("127.0.0.1", port, timeout=0.5).call("x")
    finally:
        ls.close()


def test_concurrent_clients(servers):
    _, port = servers[1]
    out = []

    def work(k):
        with mprpc.RpcClient("127.0.0.1", port) as c:
            out.append(sum(c.call("add", k, i) for i in range(50)))
    ts = [threading.Thread(target=work, args=(k,)) for k in range(8)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert sorted(out) == sorted(50 * k + sum(range(50)) for k in range(8))


def test_split_params():
    b = msgpack.packb(["name", [[1, 2], "x"], 3.5])
    parts = mprpc.split_params(b)
    assert [msgpack.unpackb(bytes(p)) for p in parts] == ["name", [[1, 2], "x"], 3.5]


def test_transport_batching_merges_concurrent_requests():
    """RpcServer.add_batch: queued requests of a method are served by one
    call; per-request results / ArgumentError / exceptions are routed back"""
    import threading
    import time as _t

    from jubatus_amd.common.mprpc import ArgumentError, RpcCallError, RpcClient, RpcServer, RpcTypeError

    sizes = []

    def batch(params_list):
        sizes.append(len(params_list))
        _t.sleep(0.005)
        out = []
        for p in params_list:
            (x,) = msgpack.unpackb(p)
            out.append(ArgumentError("neg") if x < 0 else (RuntimeError("boom") if x == 13 else x * 2))
        return out

    srv = RpcServer(nthreads=2)
    srv.add("double", lambda x: x * 2, 1)        # per-request path is shadowed by the batch
    srv.add_batch("double", batch)
    port = srv.listen(0, "127.0.0.1")
    srv.start()
    try:
        res, errs = {}, {}

        def client(i):
            c = RpcClient("127.0.0.1", port, 10)
            for j in range(10):
                x = i * 100 + j
                try:
                    res[x] = c.call("double", x)
                except Exception as e:  # noqa: BLE001
                    errs[x] = e
            c.close()
        ts = [threading.Thread(target=client, args=(i,)) for i in range(12)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert not errs and res == {x: 2 * x for x in res} and len(res) == 120
        assert sum(sizes) == 120 and srv.batches() < 120
        c = RpcClient("127.0.0.1", port, 10)
        with pytest.raises(RpcTypeError):
            c.call("double", -1)
        with pytest.raises(RpcCallError):
            c.call("double", 13)
        c.close()
    finally:
        srv.stop()


def test_batches_keep_arrival_order_around_writes():
    """csrc/native/jb_rpc.cpp set_ordered: pipelined requests of batched
    methods on one connection - a batch of a write never takes a request
    past one of another method, no batch takes a request past a write;
    reads may still batch past other reads"""
    import time as _t

    from jubatus_amd.common.mprpc import RpcServer

    seen = []
    lock = threading.Lock()

    def mk(name):
        def fn(params_list):
            with lock:
                seen.extend((name, msgpack.unpackb(p)[0]) for p in params_list)
            _t.sleep(0.002)          # (requests pile up behind the batch)
            return [0] * len(params_list)
        return fn

    srv = RpcServer(nthreads=2)
    for m in ("w1", "w2", "r1", "r2"):
        srv.add_batch(m, mk(m))
    srv.set_ordered(["w1", "w2"])
    port = srv.listen(0, "127.0.0.1")
    srv.start()
    try:
        rng = __import__("random").Random(3)
        calls = [(rng.choice(["w1", "w2", "r1", "r2", "w1"]), i) for i in range(400)]
        s = socket.create_connection(("127.0.0.1", port))
        s.sendall(b"".join(msgpack.packb([0, i, m, [i]]) for m, i in calls))
        up = msgpack.Unpacker(raw=False)
        got = set()
        while len(got) < len(calls):
            chunk = s.recv(1 << 16)
            assert chunk
            up.feed(chunk)
            for msg in up:
                got.add(msg[1])
        s.close()
        assert len(seen) == len(calls)
        pos = {i: n for n, (_, i) in enumerate(seen)}
        writes = [i for m, i in calls if m.startswith("w")]
        # every write keeps its place against every other request
        for _, i in calls:
            for w in writes:
                if i != w:
                    assert (pos[i] < pos[w]) == (i < w), (i, w)
    finally:
        srv.stop()


@pytest.mark.parametrize("name", ["", "c", "x" * 40, "y" * 300])
def test_name_and_rest(name):
    from jubatus_amd.common.mprpc import ArgumentError, name_and_rest
    body = msgpack.packb([name, [[1, 2], "abc"]], use_bin_type=False)
    assert msgpack.unpackb(bytes(name_and_rest(body))) == [[1, 2], "abc"]
    for bad in (msgpack.packb([name]), msgpack.packb([1, 2]), msgpack.packb([name, 1, 2]), b""):
        with pytest.raises(ArgumentError):
            name_and_rest(bad)
