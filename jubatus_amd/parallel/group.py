"""Cluster process group over RCCL (GPU) or gloo (host), formed through the
coordinator.

The reference mixes over msgpack-RPC among whatever servers are registered
under ``<actor>/nodes`` (linear_mixer.cpp:126-137). Collectives need a fixed
rank set, so membership changes become *group epochs*:

  <actor>/mix_epoch = {"epoch": e, "members": [ident...], "addr": a, "port": p}

* the leader (smallest live ident) publishes a new epoch whenever the live
  ``nodes/`` set differs from the current epoch's members, with a fresh
  rendezvous port on its host;
* every member polls the epoch each mixer tick; when a new epoch lists it,
  it tears down the old group and joins the new one
  (``init_process_group(tcp://addr:port, rank=index)``);
* a member missing from the epoch waits (it is obsolete until it joins);
* an epoch that lists a member whose node is gone is not joined (the leader
  publishes its successor once the dead member's session expires), and an
  epoch whose group failed is re-joined only after a back-off, so a
  survivor does not burn rendezvous timeouts waiting for a dead rank.

One group per server process (= per GPU). The group carries the mixer's
trigger agreement (a 2-int all-reduce) and the MIX collectives.

Watchdog (reference: server-to-server calls are bounded by
``--interconnect_timeout``, server_util.cpp:190-194, and a MIX skips peers
that failed, linear_mixer.cpp:455-489): once formed, the group's operation
timeout is the interconnect timeout, every collective the mixer waits for
is polled against that deadline, and a collective that misses it aborts the
communicator (``abort``: RCCL comm abort, then teardown) and marks the epoch
failed, so the survivors re-form a group without the stuck member instead of
hanging. RCCL's own watchdog runs in "clean up the communicator only" mode
(TORCH_NCCL_ASYNC_ERROR_HANDLING=2): a timed-out collective raises in the
waiting thread and the server process stays up.
"""
from __future__ import annotations

import json
import os
import socket
import time
from datetime import timedelta

# a timed-out RCCL collective must not take the server process down
os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "2")


class CollectiveTimeout(RuntimeError):
    pass

from ..common import membership as mb
from ..utils import logger

log = logger.get_logger("group")


def _free_port(host: str) -> int:
    s = socket.socket()
    try:
        s.bind((host if host not in ("", "0.0.0.0") else "", 0))
        return s.getsockname()[1]
    finally:
        s.close()


class ProcessGroupManager:
    def __init__(self, coord, type_: str, name: str, ident: str, eth: str, backend: str,
                 device=None, timeout: float = 30.0, op_timeout: float | None = None):
        self.coord, self.type, self.name = coord, type_, name
        self.ident, self.eth = ident, eth
        self.backend = backend
        self.device = device
        self.timeout = timeout                    # rendezvous
        self.op_timeout = op_timeout or timeout   # every collective (interconnect_timeout)
        self.aborts = 0
        self.epoch = -1
        self.members: list[str] = []
        self.rank = -1
        self.world = 0
        self.failed: dict[int, float] = {}   # epoch -> time its group failed
        self.retry_after = timeout
        self.path = mb.build_actor_path(type_, name) + "/mix_epoch"
        coord.create(self.path, "")

    # ------------------------------------------------------------ epochs
    def _read_epoch(self) -> dict | None:
        data = self.coord.read(self.path)
        if not data:
            return None
        try:
            return json.loads(data)
        except json.JSONDecodeError:
            return None

    def _live(self) -> list[str]:
        return sorted(self.coord.list(mb.build_actor_path(self.type, self.name) + "/nodes"))

    def maybe_publish(self) -> None:
        live = self._live()
        if not live or live[0] != self.ident:
            return  # not the leader
        cur = self._read_epoch()
        if cur is not None and cur.get("members") == live:
            return
        e = (cur or {}).get("epoch", 0) + 1
        host = self.eth if self.eth not in ("", "0.0.0.0", "localhost") else "127.0.0.1"
        new = {"epoch": e, "members": live, "addr": host, "port": _free_port(host)}
        self.coord.set(self.path, json.dumps(new))
        log.info("published mix group epoch %d: %s", e, live)

    def ensure(self) -> bool:
        """(Re)join the current epoch's group; True when a new group was formed."""
        self.maybe_publish()
        cur = self._read_epoch()
        if cur is None or cur["epoch"] == self.epoch:
            return False
        if self.ident not in cur["members"]:
            return False
        t = self.failed.get(cur["epoch"])
        if t is not None and time.time() - t < self.retry_after:
            return False
        if any(m not in self._live() for m in cur["members"]):
            return False  # a member is gone: wait for the next epoch
        self._destroy()
        rank = cur["members"].index(self.ident)
        world = len(cur["members"])
        if world > 1:
            import torch.distributed as dist
            kw = {}
            if self.backend == "nccl" and self.device is not None:
                kw["device_id"] = self.device
            try:
                dist.init_process_group(self.backend, init_method=f"tcp://{cur['addr']}:{cur['port']}",
                                        rank=rank, world_size=world,
                                        timeout=timedelta(seconds=self.timeout), **kw)
            except Exception as e:  # noqa: BLE001 - a member died during rendezvous
                log.warning("failed to join mix group epoch %d: %s", cur["epoch"], e)
                try:
                    if dist.is_initialized():
                        dist.destroy_process_group()
                except Exception:  # noqa: BLE001
                    pass
                time.sleep(0.2)
                return False
            try:
                from torch.distributed import distributed_c10d as c10d
                c10d._set_pg_timeout(timedelta(seconds=self.op_timeout), None)
            except Exception:  # noqa: BLE001 - older torch: the rendezvous timeout stays
                pass
        self.epoch, self.members, self.rank, self.world = cur["epoch"], cur["members"], rank, world
        log.info("joined mix group epoch %d as rank %d/%d", self.epoch, rank, world)
        return True

    # ---------------------------------------------------------- watchdog
    def wait(self, done, what: str = "collective", timeout: float | None = None) -> None:
        """poll ``done()`` (a work's is_completed, a job's ready) until it is
        true; past the interconnect timeout abort the group and raise"""
        deadline = time.time() + (timeout if timeout is not None else self.op_timeout)
        spin = 0
        while not done():
            if time.time() > deadline:
                self.abort(f"{what} exceeded the interconnect timeout ({self.op_timeout:g} s)")
                raise CollectiveTimeout(what)
            spin += 1
            time.sleep(0 if spin < 100 else 0.001)

    def abort(self, why: str) -> None:
        """abort the communicator of a stuck collective and leave the epoch"""
        self.aborts += 1
        log.warning("aborting mix group epoch %d: %s", self.epoch, why)
        try:
            import torch.distributed as dist
            from torch.distributed import distributed_c10d as c10d
            if dist.is_initialized() and hasattr(c10d, "_abort_process_group"):
                c10d._abort_process_group()
        except Exception as e:  # noqa: BLE001
            log.warning("communicator abort failed: %s", e)
        self.close()

    def _destroy(self) -> None:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            try:
                dist.destroy_process_group()
            except Exception:  # noqa: BLE001
                pass
        self.rank, self.world = -1, 0

    def close(self) -> None:
        """tear down after a failed collective; the epoch is not re-joined
        before ``retry_after`` seconds unless a new one is published"""
        if self.epoch >= 0:
            self.failed[self.epoch] = time.time()
        self._destroy()
        self.epoch = -1

    # ------------------------------------------------------------ helpers
    def tensor_device(self):
        import torch
        if self.backend == "nccl":
            return self.device if self.device is not None else torch.device("cuda", torch.cuda.current_device())
        return torch.device("cpu")

    def allreduce_max_ints(self, vals: list[int]) -> list[int]:
        if self.world <= 1:
            return list(vals)
        import torch
        import torch.distributed as dist
        t = torch.tensor(vals, dtype=torch.int64, device=self.tensor_device())
        w = dist.all_reduce(t, op=dist.ReduceOp.MAX, async_op=True)
        self.wait(w.is_completed, "trigger all-reduce")
        w.wait()
        return [int(x) for x in t.cpu().tolist()]
