"""MIX of the row engines (recommender, nearest_neighbor, anomaly) over
tensor collectives - no pickled objects.

Reference: linear_mixer's get_diff / mix / put_diff over msgpack-RPC
(jubatus/server/framework/mixer/linear_mixer.cpp:422-544); the row stores
behind it (jubatus_core EXTERNAL) ship every row changed since the last MIX
with its version, and the newest version wins (anomaly_serv.cpp:178-211 for
LOF). Here one MIX is:

1. every rank packs its diff into ONE byte tensor: a msgpack section (row
   ids, versions, datums for decode_row, removals), the rows' hashed feature
   vectors as CSR (int64 row_ptr, int32 idx, float32 val), the LSH
   signature words + norms taken straight from the HBM table (so receivers
   never re-hash or re-sign), and the sparse document-frequency diff;
2. sizes are all-gathered, then the padded buffers (RCCL over xGMI on GPUs:
   the buffer lives in HBM; gloo on hosts);
3. every rank folds the diffs in rank order - newest version wins, ties go
   to the higher rank (mix_diff's order) - and applies the winners it does
   not already hold: datum + fv into the host row store, signatures scattered
   into the HBM table (index_copy_), inverted-index rows appended to the
   device pool from the shipped CSR.

``pair_mix`` runs the same exchange between two ranks (push_mixer's
symmetric pull/push, push_mixer.cpp:354-388) over send / recv.
"""
from __future__ import annotations

import time
from typing import Any

import msgpack
import numpy as np
import torch
import torch.distributed as dist

_HDR = 8           # int64 header words: blob, n, nnz, bits words, norms, df entries, words, flags


def _align(n: int) -> int:
    return (n + 7) // 8 * 8


def _comm_device(group) -> torch.device:
    if str(dist.get_backend(group)) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


class _Local:
    """one rank's diff, packed"""

    def __init__(self, eng: Any, dev: torch.device):
        rows = eng.rows
        ids = sorted(r for r in rows.dirty if r in rows.slot_of)
        slots = np.asarray([rows.slot_of[r] for r in ids], dtype=np.int64)
        vers = [int(rows.version.get(r, 0)) for r in ids]
        datums = [[dict(x) for x in rows.datum[s]] for s in slots.tolist()]
        removed = [[r, int(rows.version.get(r, 0))] for r in sorted(rows.removed)]
        fvs = [rows.fv[s] for s in slots.tolist()]
        lens = np.fromiter((len(f[0]) for f in fvs), dtype=np.int64, count=len(fvs))
        rp = np.zeros(len(fvs) + 1, dtype=np.int64)
        np.cumsum(lens, out=rp[1:])
        idx = np.fromiter((i for f in fvs for i in f[0]), dtype=np.int32, count=int(rp[-1]))
        val = np.fromiter((v for f in fvs for v in f[1]), dtype=np.float32, count=int(rp[-1]))
        sig = eng.index.export_signatures(slots) if hasattr(eng.index, "export_signatures") else None
        w = eng.conv.weights
        wd = w.get_diff() if eng.conv.uses_global_weight else {"docs": 0, "len": 0, "idx": [], "df": []}
        blob = np.frombuffer(msgpack.packb({"ids": ids, "ver": vers, "datum": datums,
                                            "removed": removed, "w": [wd["docs"], wd["len"]]},
                                           use_bin_type=True), dtype=np.uint8)
        widx = np.asarray(wd["idx"], dtype=np.int64)
        wcnt = np.asarray(wd["df"], dtype=np.int64)
        words = 0
        pieces: list[torch.Tensor] = []

        def add(t: torch.Tensor) -> None:
            if t.numel() == 0:
                return
            b = t.contiguous().view(-1).view(torch.uint8).to(dev)
            pieces.append(b)
            pad = _align(b.numel()) - b.numel()
            if pad:
                pieces.append(torch.zeros(pad, dtype=torch.uint8, device=dev))

        add(torch.from_numpy(blob.copy()))
        add(torch.from_numpy(rp))
        add(torch.from_numpy(idx))
        add(torch.from_numpy(val))
        nbits = nnorm = 0
        if sig is not None:
            bits, norms = sig
            words = int(bits.shape[1]) if bits.ndim == 2 else 0
            add(torch.as_tensor(bits).view(torch.int64) if isinstance(bits, torch.Tensor)
                else torch.from_numpy(np.ascontiguousarray(bits).view(np.int64)))
            add(torch.as_tensor(norms))
            nbits, nnorm = int(bits.shape[0]) * words, int(norms.shape[0])
        add(torch.from_numpy(widx))
        add(torch.from_numpy(wcnt))
        self.data = torch.cat(pieces) if pieces else torch.zeros(0, dtype=torch.uint8, device=dev)
        self.hdr = torch.tensor([blob.size, len(ids), int(rp[-1]), nbits, nnorm, widx.size, words,
                                 self.data.numel()], dtype=torch.int64, device=dev)
        self.n = len(ids)


def _unpack(hdr: list[int], buf: torch.Tensor) -> dict:
    """sections of one rank's buffer (host parts on the host, signature rows
    where the buffer lives)"""
    blob_n, n, nnz, nbits, nnorm, nw, words, _ = hdr
    off = 0

    def take(nbytes: int) -> torch.Tensor:
        nonlocal off
        t = buf[off:off + nbytes]
        off += _align(nbytes)
        return t
    host = buf.device.type == "cpu"
    b = take(blob_n)
    meta = msgpack.unpackb((b if host else b.cpu()).numpy().tobytes(), raw=False,
                           strict_map_key=False)
    rp = take(8 * (n + 1)).cpu().view(torch.int64).numpy()
    idx = take(4 * nnz).cpu().view(torch.int32).numpy()
    val = take(4 * nnz).cpu().view(torch.float32).numpy()
    bits = norms = None
    if nbits or nnorm or words:
        bits = take(8 * nbits).view(torch.int64).view(n, words) if words else None
        norms = take(4 * nnorm).view(torch.float32)
    widx = take(8 * nw).cpu().view(torch.int64).numpy()
    wcnt = take(8 * nw).cpu().view(torch.int64).numpy()
    return {"meta": meta, "rp": rp, "idx": idx, "val": val, "bits": bits, "norms": norms,
            "widx": widx, "wcnt": wcnt}


def _gather_all(loc: _Local, group) -> list[tuple[list[int], torch.Tensor]]:
    n = dist.get_world_size(group)
    hdrs = [torch.empty_like(loc.hdr) for _ in range(n)]
    dist.all_gather(hdrs, loc.hdr, group=group)
    hdrs = [h.cpu().tolist() for h in hdrs]
    mx = max(max(h[7] for h in hdrs), 8)
    data = loc.data
    if data.numel() < mx:
        data = torch.cat([data, torch.zeros(mx - data.numel(), dtype=torch.uint8, device=data.device)])
    bufs = [torch.empty(mx, dtype=torch.uint8, device=data.device) for _ in range(n)]
    dist.all_gather(bufs, data, group=group)
    return [(h, b[:h[7]]) for h, b in zip(hdrs, bufs)]


def _exchange_pair(loc: _Local, peer: int, group) -> list[tuple[list[int], torch.Tensor]]:
    me = dist.get_rank(group)
    theirs_h = torch.empty_like(loc.hdr)
    if me < peer:
        dist.send(loc.hdr, peer, group=group)
        dist.recv(theirs_h, peer, group=group)
    else:
        dist.recv(theirs_h, peer, group=group)
        dist.send(loc.hdr, peer, group=group)
    th = theirs_h.cpu().tolist()
    buf = torch.empty(max(th[7], 1), dtype=torch.uint8, device=loc.data.device)
    mine = loc.data if loc.data.numel() else torch.zeros(1, dtype=torch.uint8, device=buf.device)
    if me < peer:
        dist.send(mine, peer, group=group)
        dist.recv(buf, peer, group=group)
    else:
        dist.recv(buf, peer, group=group)
        dist.send(mine, peer, group=group)
    pairs = [(loc.hdr.cpu().tolist(), loc.data), (th, buf[:th[7]])]
    return pairs if me < peer else pairs[::-1]


def _apply(eng: Any, parts: list[dict]) -> int:
    """fold the diffs in order (newest version wins, later part on ties) and
    apply what this rank does not hold yet; -> rows written"""
    rows = eng.rows
    win: dict[str, tuple[int, int, int]] = {}          # rid -> (version, part, i)
    gone: dict[str, int] = {}
    for p, d in enumerate(parts):
        m = d["meta"]
        for i, (rid, v) in enumerate(zip(m["ids"], m["ver"])):
            cur = win.get(rid)
            if cur is None or v >= cur[0]:
                win[rid] = (int(v), p, i)
        for rid, v in m["removed"]:
            gone[rid] = max(int(v), gone.get(rid, -1))
    todo = [(rid, v, p, i) for rid, (v, p, i) in win.items()
            if rows.version.get(rid, -1) < v or rid not in rows.slot_of]
    by_part: dict[int, list] = {}
    for t in todo:
        by_part.setdefault(t[2], []).append(t)
    written = 0
    for p, items in sorted(by_part.items()):
        d = parts[p]
        sel = np.asarray([i for _, _, _, i in items], dtype=np.int64)
        rp = d["rp"]
        lens = rp[sel + 1] - rp[sel]
        rp2 = np.zeros(sel.size + 1, dtype=np.int64)
        np.cumsum(lens, out=rp2[1:])
        gat = (np.repeat(rp[sel] - rp2[:-1], lens) + np.arange(int(rp2[-1]), dtype=np.int64)
               if rp2[-1] else np.zeros(0, np.int64))
        idx, val = d["idx"][gat], d["val"][gat]
        put = [(rid, tuple(dict(x) for x in d["meta"]["datum"][i])) for rid, _, _, i in items]
        slots = rows.put_many(put, rp2, idx, val, bump=False)
        for rid, v, _, _ in items:
            rows.version[rid] = v
        if d["bits"] is not None and hasattr(eng.index, "import_signatures"):
            eng.index.import_signatures(slots, d["bits"][torch.as_tensor(sel, device=d["bits"].device)],
                                        d["norms"][torch.as_tensor(sel, device=d["norms"].device)])
        else:
            eng.index.set_rows_csr(slots, rp2, idx, val)
        eng._rows_changed(slots)
        written += len(items)
        for rid, _, _, _ in items:                 # unlearner bookkeeping, as a local write
            for victim in eng.unlearner.touch(rid):
                if victim != rid:
                    eng._remove(victim)
    for rid, v in gone.items():
        if rows.version.get(rid, -1) <= v:
            eng._remove(rid, record=False)
            rows.version[rid] = v
    if eng.conv.uses_global_weight:
        docs = sum(d["meta"]["w"][0] for d in parts)
        ln = sum(d["meta"]["w"][1] for d in parts)
        acc: dict[int, int] = {}
        for d in parts:
            for i, c in zip(d["widx"].tolist(), d["wcnt"].tolist()):
                acc[i] = acc.get(i, 0) + c
        ks = sorted(acc)
        eng.conv.weights.put_diff({"docs": docs, "len": ln, "idx": ks, "df": [acc[k] for k in ks]})
    rows.dirty.clear()
    rows.removed.clear()
    return written


def row_mix(eng: Any, group=None, peer: int | None = None) -> dict:
    """one MIX of a row engine over the process group (all ranks) or with
    one peer; -> stats (bytes sent by this rank, rows applied, seconds)"""
    t0 = time.perf_counter()
    with eng._lock:
        dev = _comm_device(group)
        loc = _Local(eng, dev)
        got = _gather_all(loc, group) if peer is None else _exchange_pair(loc, peer, group)
        parts = [_unpack(h, b) for h, b in got]
        n = _apply(eng, parts)
    return {"bytes": int(loc.data.numel()), "rows_sent": loc.n, "rows_applied": n,
            "seconds": time.perf_counter() - t0}
