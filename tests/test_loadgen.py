"""jubaloadgen (csrc/tools/jubaloadgen.cpp) against a recording msgpack-RPC
peer: the replay mode sends the params file as is; the fresh mode (-r)
redraws the first numeric value of every sample it sends (v + N(0, 1/4)) and
leaves every other byte alone, so a served stream does not repeat."""
import json
import os
import socket
import subprocess
import threading

import msgpack
import numpy as np
import pytest

from tests.helpers import ROOT

EXE = os.path.join(ROOT, "jubatus_amd", "native_bin", "jubaloadgen")
pytestmark = pytest.mark.skipif(not os.access(EXE, os.X_OK), reason="jubaloadgen not built")


def _params(tmp_path, n_req=4, per_req=32):
    rng = np.random.default_rng(0)
    reqs = []
    with open(tmp_path / "p.bin", "wb") as f:
        for _ in range(n_req):
            body = []
            for _ in range(per_req):
                y = int(rng.integers(2))
                body.append([f"l{y}", [[["w", "a" if y else "b"], ["t", f"t{int(rng.integers(100, 999))}"]],
                                       [["x", float(y)], ["z", 0.5]], []]])
            reqs.append(["", body])
            f.write(msgpack.packb(["", body], use_bin_type=False))
    return str(tmp_path / "p.bin"), reqs


class Recorder:
    """accepts connections, answers every request with true, keeps the params"""

    def __init__(self):
        self.sock = socket.socket()
        self.sock.bind(("127.0.0.1", 0))
        self.sock.listen(8)
        self.port = self.sock.getsockname()[1]
        self.got = []
        self.lock = threading.Lock()
        threading.Thread(target=self._accept, daemon=True).start()

    def _accept(self):
        while True:
            try:
                c, _ = self.sock.accept()
            except OSError:
                return
            threading.Thread(target=self._serve, args=(c,), daemon=True).start()

    def _serve(self, c):
        up = msgpack.Unpacker(raw=False)
        with c:
            while True:
                data = c.recv(65536)
                if not data:
                    return
                up.feed(data)
                for msg in up:
                    _, msgid, _, params = msg
                    with self.lock:
                        self.got.append(params)
                    c.sendall(msgpack.packb([1, msgid, None, True]))

    def close(self):
        self.sock.close()


def _run(port, pfile, *extra):
    r = subprocess.run([EXE, "-p", str(port), "-m", "train", "-f", pfile, "-c", "2", "-d", "2", *extra],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_loadgen_replay_and_fresh_values(tmp_path):
    pfile, reqs = _params(tmp_path)
    rec = Recorder()
    try:
        out = _run(rec.port, pfile, "-o", "1")
        assert out["requests"] == 4 and out["fresh_values"] is False
        assert sorted(map(repr, rec.got)) == sorted(map(repr, reqs))
        rec.got.clear()
        out = _run(rec.port, pfile, "-t", "0.3", "-r", "7")
        assert out["fresh_values"] is True and out["requests"] >= 8
        with rec.lock:
            got = list(rec.got)
        deltas, tokens = [], set()
        for g in got:
            # the source: same labels and first string values (the templates)
            src = next(r for r in reqs if all(a[0] == b[0] and a[1][0][0] == b[1][0][0]
                                              for a, b in zip(g[1], r[1])))
            for a, b in zip(g[1], src[1]):
                assert a[1][0][0] == b[1][0][0] and a[1][1][1] == b[1][1][1]  # untouched
                ta, tb = a[1][0][1][1], b[1][0][1][1]
                assert ta[0] == "t" and len(ta) == len(tb) and ta[1:].isdigit()   # redrawn digits
                tokens.add(ta)
                assert a[1][1][0][0] == "x"
                deltas.append(a[1][1][0][1] - b[1][1][0][1])
        d = np.asarray(deltas)
        assert np.all(d != 0.0)
        assert 0.4 < d.std() < 0.6 and abs(d.mean()) < 0.1, (d.mean(), d.std())   # N(0, 1/4) around v
        assert len(tokens) > 900          # 3-digit tokens: (nearly) all 1000 drawn
    finally:
        rec.close()


def test_loadgen_fresh_rejects_params_without_float_values(tmp_path):
    p = tmp_path / "q.bin"
    p.write_bytes(msgpack.packb(["", [["l0", [[["w", "a"]], [], []]]]], use_bin_type=False))
    r = subprocess.run([EXE, "-p", "1", "-m", "train", "-f", str(p), "-r", "1"], capture_output=True,
                       text=True, timeout=30)
    assert r.returncode == 1 and "float64" in r.stderr
