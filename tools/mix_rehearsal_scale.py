"""Row-diff MIX at scale on the CPU: N jb_mix_rehearsal -R ranks (the row
engines' MIX code, csrc/server/jb_row_mix.hpp) join one cluster through the
native coordinator, each writes R rows of its own, then one MIX folds the
union into every rank. Reports, per rank, the MIX's bytes and seconds (the
mixer's status keys - the reference's MIX log line, linear_mixer.cpp:538-543),
the rows applied and the per-row apply cost.

Usage: python tools/mix_rehearsal_scale.py [--ranks 8] [--rows 100000] [--out FILE]
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
BIN = os.path.join(ROOT, "jubatus_amd", "native_bin", "jb_mix_rehearsal")


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--rows", type=int, default=100_000)
    ap.add_argument("--mixer", default="linear_mixer")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    from jubatus_amd.common.coordinator import NativeCoordinator
    from jubatus_amd.common.mprpc import RpcClient, wait_server
    coord = NativeCoordinator(0, "127.0.0.1")
    procs, clients = [], []
    name = "scale"
    try:
        for i in range(a.ranks):
            port = free_port()
            log = open(os.path.join(tempfile.gettempdir(), f"rowmix_scale_{port}.log"), "wb")
            procs.append(subprocess.Popen([BIN, "-R", "-x", a.mixer, "-z", f"127.0.0.1:{coord.port}", "-n", name,
                                           "-p", str(port), "-I", "600", "-i", "0", "-s", "0", "-Z", "10"],
                                          stdout=subprocess.DEVNULL, stderr=log))
            assert wait_server("127.0.0.1", port, 30)
            clients.append(RpcClient("127.0.0.1", port, 900.0))

        def status(c):
            (_, st), = c.call("get_status", name).items()
            return {(k.decode() if isinstance(k, bytes) else k): (v.decode() if isinstance(v, bytes) else v)
                    for k, v in st.items()}
        deadline = time.time() + 60
        while time.time() < deadline:
            if all(status(c).get(f"{a.mixer}.group_size") == str(a.ranks) for c in clients):
                break
            time.sleep(0.2)
        t = time.perf_counter()
        for i, c in enumerate(clients):       # disjoint key spaces of 10^12 ids: ~R fresh rows each
            c.call("put", name, 7919 * (i + 1), a.rows, 10**12)
        fill_s = time.perf_counter() - t
        t = time.perf_counter()
        ok = clients[0].call("do_mix", name)
        mix_wall = time.perf_counter() - t
        sts = [status(c) for c in clients]
        per_rank = []
        for i, st in enumerate(sts):
            sec = float(st.get(f"{a.mixer}.last_mix_sec", "nan"))
            applied = int(st.get("mix.last_rows_applied", "0"))
            per_rank.append({"rank": i, "num_rows": int(st.get("num_rows", "0")),
                             "mix_bytes": int(st.get(f"{a.mixer}.last_mix_bytes", "0")),
                             "mix_sec": sec, "rows_applied": applied,
                             "apply_us_per_row": round(sec * 1e6 / applied, 3) if applied else None})
        rec = {"ranks": a.ranks, "rows_per_rank": a.rows, "mixer": a.mixer, "do_mix": bool(ok),
               "fill_s": round(fill_s, 2), "mix_wall_s": round(mix_wall, 3),
               "host": "CPU rehearsal (native control plane, no GPU)", "per_rank": per_rank}
        print(json.dumps(rec), flush=True)
        if a.out:
            with open(a.out, "w") as f:
                json.dump(rec, f, indent=1)
    finally:
        for c in clients:
            c.close()
        for p in procs:
            p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
        coord.stop()


if __name__ == "__main__":
    main()
