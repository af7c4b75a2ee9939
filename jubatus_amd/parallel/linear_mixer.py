"""linear_mixer: periodic cluster-wide model averaging as a collective
(reference C23: jubatus/server/framework/mixer/linear_mixer.{hpp,cpp}).

Reference: a stabilizer thread wakes every 0.5 s; when ``counter >=
interval_count`` or ``now - ticktime > interval_sec`` (and counter > 0) the
node that wins the ZK master_lock gathers get_diff from every node, folds
and scatters put_diff over msgpack-RPC (linear_mixer.cpp:358-544).

MI355X design: every server is one rank of a process group (parallel/group.py,
RCCL over xGMI on GPUs, gloo on hosts). Each tick all ranks agree on the
trigger with one 2-int all-reduce(MAX) - "some rank wants to mix" /
"do_mix was called somewhere" - so the whole cluster runs the same MIX
collective, which for dense models is a bucketed all-reduce mean of the HBM
tables. No master lock, no TCP model traffic, no serialised fold.

Obsolete protocol (linear_mixer.cpp:394-410,582-611): a node joining a group
is obsolete; when a group forms, the lowest-rank up-to-date member broadcasts
its model to the group before the next MIX, then everyone registers as
active (proxies route only to actives).

RPC: ``do_mix(name) -> bool`` forces a MIX at the next tick and waits for it.
Status keys: linear_mixer.count / ticktime / is_obsolete / is_running
(linear_mixer.cpp:346-356) plus mix latency/bytes.
"""
from __future__ import annotations

import threading
import time

from ..common import membership as mb
from ..framework.mixer import Mixer
from ..utils import fault, logger, trace
from .group import ProcessGroupManager
from .mixable import broadcast_model, linear_mix

log = logger.get_logger("linear_mixer")

TICK = 0.5


class CollectiveMixer(Mixer):
    """Shared machinery of the linear and push mixers."""

    kind = "linear_mixer"

    def __init__(self, argv, coord, rw_mutex, server_type: str, protocol_version: int = 1,
                 backend: str | None = None):
        self.argv = argv
        self.coord = coord
        self.rw = rw_mutex
        self.type = server_type
        self.protocol_version = protocol_version
        self.backend = backend
        self.driver = None
        self.counter = 0
        self.ticktime = time.time()
        self.mix_count = 0
        self.is_obsolete = True
        self.running = False
        self.last_mix = {"bytes": 0, "seconds": 0.0}
        self._lock = threading.Condition()
        self._force = False
        self._stop = threading.Event()
        self._thread: threading.Thread | None = None
        self.group: ProcessGroupManager | None = None
        self.ident = mb.build_loc_str(argv.eth, argv.port)

    # ------------------------------------------------------------ API
    def register_api(self, rpc) -> None:
        rpc.add("do_mix", lambda name: self.do_mix(), 1)

    def set_driver(self, driver) -> None:
        self.driver = driver

    def type(self) -> str:  # noqa: A003 - reference name
        return self.kind

    def _device(self):
        return getattr(self.driver, "device", None)

    def start(self) -> None:
        dev = self._device()
        backend = self.backend or ("nccl" if dev is not None else "gloo")
        self.group = ProcessGroupManager(self.coord, self.type, self.argv.name, self.ident,
                                         self.argv.eth, backend, dev,
                                         timeout=max(5.0, 3.0 * self.argv.interconnect_timeout),
                                         op_timeout=max(1.0, float(self.argv.interconnect_timeout)))
        self.running = True
        self._thread = threading.Thread(target=self._loop, name=self.kind, daemon=True)
        self._thread.start()

    def stop(self) -> None:
        self._stop.set()
        with self._lock:
            self._lock.notify_all()
        if self._thread is not None:
            self._thread.join(timeout=0.5)
            if self._thread.is_alive() and self.group is not None and self.group.epoch >= 0:
                # a collective in flight would hold the shutdown for the whole
                # interconnect timeout: abort it (the watchdog's abort; the
                # peers then leave the epoch too)
                self.group.abort("server stopping")
            self._thread.join(timeout=2.0)
            if self._thread.is_alive():
                # still inside a group rendezvous (its timeout is several
                # interconnect timeouts): the thread is a daemon, the server
                # goes on stopping without it
                log.warning("mixer thread still in a collective or rendezvous: not waiting for it")
        self.running = False
        if self.group is not None:
            self.group.close()

    def updated(self, n: int = 1) -> None:
        with self._lock:
            self.counter += n
            if 0 < self.argv.interval_count <= self.counter:
                self._lock.notify_all()

    def do_mix(self) -> bool:
        with self._lock:
            target = self.mix_count + 1
            self._force = True
            self._lock.notify_all()
            deadline = time.time() + max(30.0, 4 * self.argv.interconnect_timeout)
            while self.mix_count < target and time.time() < deadline and not self._stop.is_set():
                self._lock.wait(0.1)
            return self.mix_count >= target

    def get_status(self, status: dict) -> None:
        k = self.kind
        status[f"{k}.count"] = str(self.counter)
        status[f"{k}.ticktime"] = str(int(self.ticktime))
        status[f"{k}.is_obsolete"] = "1" if self.is_obsolete else "0"
        status[f"{k}.is_running"] = "1" if self.running else "0"
        status[f"{k}.mix_count"] = str(self.mix_count)
        status[f"{k}.last_mix_bytes"] = str(self.last_mix["bytes"])
        status[f"{k}.last_mix_sec"] = f"{self.last_mix['seconds']:.6f}"
        status[f"{k}.overlapped"] = str(self.last_mix.get("overlap", 0))
        if self.group is not None:
            status[f"{k}.watchdog_aborts"] = str(self.group.aborts)
            status[f"{k}.group_epoch"] = str(self.group.epoch)
            status[f"{k}.group_rank"] = str(self.group.rank)
            status[f"{k}.group_size"] = str(self.group.world)
            status[f"{k}.backend"] = self.group.backend

    # ------------------------------------------------------------ loop
    def _want(self) -> bool:
        a = self.argv
        if self.counter <= 0:
            return False
        if 0 < a.interval_count <= self.counter:
            return True
        return 0 < a.interval_sec < time.time() - self.ticktime

    def _register_active(self) -> None:
        mb.register_active(self.coord, self.type, self.argv.name, self.argv.eth, self.argv.port)

    def _loop(self) -> None:
        while not self._stop.is_set():
            with self._lock:
                self._lock.wait(TICK)
            if self._stop.is_set():
                break
            try:
                self._tick()
            except Exception as e:  # noqa: BLE001 - a member died or stalled mid-collective
                log.warning("mix tick failed (%s); re-forming the group", e)
                if self.group is not None and self.group.epoch >= 0:
                    self.group.abort(f"collective failed: {e}")
                time.sleep(TICK)

    def _tick(self) -> None:
        g = self.group
        formed = g.ensure()
        if g.world == 0:
            return  # not (yet) part of an epoch
        if g.world == 1:
            # alone in the cluster: nothing to mix, serve requests
            if self.is_obsolete:
                self.is_obsolete = False
                self._register_active()
            with self._lock:
                if self._force or self._want():
                    self._mixed({"bytes": 0, "seconds": 0.0})
            return
        if formed:
            fault.on_mix("handover")
            with trace.span("mix.handover"):
                self._hand_over()
        with self._lock:
            want = 1 if self._want() else 0
            force = 1 if self._force else 0
            count = self.mix_count
        # the MIX count is agreed too (the push mixers' pairing of a round
        # follows it; members' own counts differ after solo ticks, a late join
        # or a MIX that failed on one side): every member mixes round max(counts)
        flags = g.allreduce_max_ints([want, force, self.protocol_version, -self.protocol_version, count])
        if flags[2] != -flags[3]:
            log.critical("mix protocol version mismatch in the cluster: shutting down")
            mb.shutdown_server()
            return
        if flags[0] or flags[1]:
            self.round_no = int(flags[4])
            st = self.mix_once()
            with self._lock:
                self.mix_count = self.round_no      # every member leaves at the same count
                self._mixed(st)
            log.info("mixed with %d servers in %.6f secs, %d bytes", g.world, st["seconds"],
                     st["bytes"])

    def _mixed(self, st: dict) -> None:
        self.counter = 0
        self.ticktime = time.time()
        self.mix_count += 1
        self._force = False
        self.last_mix = st
        self._lock.notify_all()

    def _hand_over(self) -> None:
        """New group: if a member is obsolete (newly joined), it receives the
        model of the lowest-rank up-to-date member (linear_mixer.cpp:394-410,
        582-611); up-to-date members keep theirs - a group re-formed after a
        failure does not overwrite anyone's training."""
        g = self.group
        big = 1 << 30
        r = g.allreduce_max_ints([-(big if self.is_obsolete else g.rank),
                                  1 if self.is_obsolete else 0])
        src, any_obsolete = -r[0], r[1]
        if any_obsolete and src < big:
            with self.rw.write():
                broadcast_model(self.driver, src, apply=self.is_obsolete)
            if self.is_obsolete:
                log.info("model fetched from rank %d", src)
        self.is_obsolete = False
        self._register_active()

    def mix_once(self) -> dict:
        """One MIX. Drivers with an overlapped MIX (mix_begin / mix_ready /
        mix_end: the linear classifier's sparse all-reduce) hold the model
        write lock only to snapshot and to fold; the collective itself runs
        while train/classify continue, polled by the group watchdog. Other
        drivers mix synchronously under the write lock (the reference holds
        it for put_diff, linear_mixer.cpp:613-662)."""
        fault.on_mix("allreduce")
        d = self.driver
        with trace.span("mix.linear"):
            if hasattr(d, "mix_begin"):
                t0 = time.perf_counter()
                with self.rw.write():
                    h = d.mix_begin()
                self.group.wait(lambda: d.mix_ready(h), "MIX all-reduce")
                with self.rw.write():
                    nbytes = d.mix_end(h)
                return {"bytes": int(nbytes or 0), "seconds": time.perf_counter() - t0,
                        "overlap": 1}
            with self.rw.write():
                return linear_mix(d)


class LinearMixer(CollectiveMixer):
    kind = "linear_mixer"
