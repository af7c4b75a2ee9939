"""Sparse / chunked-dense table MIX (parallel/table_mix.py) on 2 gloo ranks:
the result equals the dense cluster mean, bytes scale with the touched rows,
and updates made while the collective runs are kept (overlap semantics of
linear_mixer.cpp:547-564 get_diff / :613-662 put_diff)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

H, C = 4096, 8


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, mode, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from jubatus_amd.parallel.table_mix import TableMix
    try:
        g = torch.Generator().manual_seed(7)
        base_w = torch.randn(H, C, generator=g)
        base_p = torch.rand(H, C, generator=g) + 1.0
        W, P = base_w.clone(), base_p.clone()
        touched = torch.zeros(H, dtype=torch.uint8)
        # rank r updates its own rows plus a shared band
        rr = torch.randperm(H, generator=torch.Generator().manual_seed(100 + rank))[:200]
        rows = torch.cat([rr, torch.arange(10, 30)])
        W[rows] += (rank + 1) * 0.5
        P[rows] += rank + 1.0
        touched[rows] = 1
        # every rank's tables, for the dense reference mean
        allw = [torch.empty_like(W) for _ in range(world)]
        allp = [torch.empty_like(P) for _ in range(world)]
        dist.all_gather(allw, W)
        dist.all_gather(allp, P)
        ref_w = torch.stack(allw).mean(0)
        ref_p = torch.stack(allp).mean(0)
        if mode == "full_union":
            # dense_frac 1.0 and one rank without a touched map: that rank
            # goes dense at once, the other sees a full union and must follow
            job = TableMix([W, P], touched if rank == 0 else None, None, dense_frac=1.0).begin()
            while not job.ready():
                pass
            nbytes = job.end()
            q.put((rank, job.stats(), nbytes, float((W - ref_w).abs().max()),
                   float((P - ref_p).abs().max()), int(touched.sum())))
            return
        if mode in ("sparse", "sparse_bf16"):
            job = TableMix([W, P], touched, None, wire_dtype="bf16" if mode == "sparse_bf16" else "fp32").begin()
        else:      # dense, chunked into 16 KiB pieces
            job = TableMix([W, P], None, None, chunk_bytes=16 << 10).begin()
            assert job.chunk_rows < H
        # an update made while the collective is in flight survives the MIX
        # (dense: in the first chunk, whose snapshot begin() took)
        late = (3000 if mode.startswith("sparse") else 5) + rank
        W[late, 0] += 100.0
        while not job.ready():
            pass
        nbytes = job.end()
        ref_w[late, 0] += 100.0
        st = job.stats()
        q.put((rank, st, nbytes, float((W - ref_w).abs().max()), float((P - ref_p).abs().max()),
               int(touched.sum())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["sparse", "dense", "full_union", "sparse_bf16"])
def test_table_mix_equals_dense_mean(mode):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for rank, st, nbytes, ew, ep, left in res:
        if mode == "sparse_bf16":
            # bf16 on the wire: the mean is rounded once (|values| < ~8 here:
            # 2^-8 relative -> < 0.05), half the bytes; the late update stays exact
            assert ew < 0.05 and ep < 0.05, (rank, ew, ep)
            assert st["wire"] == "bf16" and nbytes == st["rows"] * 2 * C * 2 + H
            continue
        assert ew < 1e-5 and ep < 1e-5, (rank, ew, ep)
        if mode == "sparse":
            assert st["mode"] == "sparse"
            assert 200 <= st["rows"] <= 420                 # the union, not the table
            assert nbytes == st["rows"] * 2 * C * 4 + H      # rows + the union bitmap (uint8[H])
            assert left == 0                                 # touched map cleared
        else:
            assert st["mode"] == "dense" and nbytes == H * 2 * C * 4 + H
