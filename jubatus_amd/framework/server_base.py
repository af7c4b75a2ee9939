"""server_base (reference C18: jubatus/server/framework/server_base.{hpp,cpp}).

Holds the argv, the model read/write lock, ``update_count`` and the
last-saved/loaded bookkeeping; implements save(id)/load(id)/load_file(path)
over the model container (save_load.py) and ``event_model_updated`` (which
drives the mixer's update counter).
"""
from __future__ import annotations

import fcntl
import os
import threading
import time
from contextlib import contextmanager
from typing import Any

from ..utils import logger
from . import save_load
from .server_util import ServerArgv, get_server_identifier

log = logger.get_logger("server_base")


class RWLock:
    """Writer-preferring read/write lock (model rw_mutex, reference
    server_base.hpp:105 and the JRLOCK_/JWLOCK_ macros)."""

    def __init__(self):
        self._cond = threading.Condition(threading.Lock())
        self._readers = 0
        self._writer = False
        self._waiting_writers = 0
        self._owner: int | None = None
        self._depth = 0

    @contextmanager
    def read(self):
        me = threading.get_ident()
        if self._owner == me:  # a writer may read
            yield
            return
        with self._cond:
            while self._writer or self._waiting_writers:
                self._cond.wait()
            self._readers += 1
        try:
            yield
        finally:
            with self._cond:
                self._readers -= 1
                if self._readers == 0:
                    self._cond.notify_all()

    @contextmanager
    def write(self):
        me = threading.get_ident()
        if self._owner == me:  # reentrant writer
            self._depth += 1
            try:
                yield
            finally:
                self._depth -= 1
            return
        with self._cond:
            self._waiting_writers += 1
            while self._writer or self._readers:
                self._cond.wait()
            self._waiting_writers -= 1
            self._writer = True
            self._owner = me
        try:
            yield
        finally:
            with self._cond:
                self._writer = False
                self._owner = None
                self._cond.notify_all()


class ServerBase:
    """Base of every engine server (the ``*_serv`` classes)."""

    type_name = ""

    def __init__(self, argv: ServerArgv, coord=None):
        self._argv = argv
        self.coord = coord
        self.update_count = 0
        self.rw_mutex = RWLock()
        self._status_lock = threading.Lock()
        self.last_saved = 0.0
        self.last_saved_path = ""
        self.last_loaded = 0.0
        self.last_loaded_path = ""
        self.mixer = None

    # ---- to override
    def get_driver(self):
        raise NotImplementedError

    def set_config(self, config: str) -> None:
        raise NotImplementedError

    def get_config(self) -> str:
        raise NotImplementedError

    def get_status(self, status: dict[str, str]) -> None:
        pass

    def user_data_version(self) -> int:
        return 1

    def get_mixer(self):
        return self.mixer

    # ---- common
    def argv(self) -> ServerArgv:
        return self._argv

    def clear(self) -> bool:
        self.get_driver().clear()
        return True

    def event_model_updated(self, n: int = 1) -> None:
        """n updates (a batch of update RPCs counts each of them)"""
        self.update_count += n
        if self.mixer is not None:
            self.mixer.updated(n)

    def _local_path(self, model_id: str) -> str:
        a = self._argv
        return os.path.join(a.datadir, f"{a.eth}_{a.port}_{a.type}_{model_id}.jubatus")

    def save(self, model_id: str) -> dict[str, str]:
        if model_id == "":
            raise RuntimeError("empty id is not allowed")
        path = self._local_path(model_id)
        log.info("starting save to %s", path)
        try:
            f = open(path, "wb")
        except OSError as e:
            raise RuntimeError(f"cannot open output file: {path}: {e.strerror}") from e
        try:
            try:
                fcntl.flock(f.fileno(), fcntl.LOCK_EX | fcntl.LOCK_NB)
            except OSError as e:
                raise RuntimeError("cannot get the lock of file; any RPC is saving to same file?"
                                   f": {path}") from e
            try:
                drv = self.get_driver()
                save_load.save_server(f, self._argv.type, model_id, self.get_config(),
                                      self.user_data_version(), drv.pack())
                f.close()
            except Exception as e:
                f.close()
                try:
                    os.remove(path)
                except OSError:
                    log.warning("failed to cleanup dirty model file: %s", path)
                raise RuntimeError(f"cannot write output file: {path}: {e}") from e
        finally:
            if not f.closed:
                f.close()
        with self._status_lock:
            self.last_saved = time.time()
            self.last_saved_path = path
        log.info("saved to %s", path)
        return {get_server_identifier(self._argv): path}

    def _load_file_impl(self, path: str, overwrite_config: bool) -> None:
        log.info("starting load from %s", path)
        try:
            f = open(path, "rb")
        except OSError as e:
            raise RuntimeError(f"cannot open input file: {path}: {e.strerror}") from e
        with f:
            current = None
            try:
                current = self.get_config()
            except Exception:
                current = None
            config, payload = save_load.load_server(f, self._argv.type, current,
                                                    self.user_data_version(), overwrite_config)
        if overwrite_config and (current is None or not save_load.compare_config(config, current)):
            self.set_config(config)
        self.get_driver().unpack(payload)
        with self._status_lock:
            self.last_loaded = time.time()
            self.last_loaded_path = path
        log.info("loaded from %s", path)

    def load(self, model_id: str) -> bool:
        if model_id == "":
            raise RuntimeError("empty id is not allowed")
        self._load_file_impl(self._local_path(model_id), overwrite_config=False)
        return True

    def load_file(self, path: str) -> None:
        self._load_file_impl(path, overwrite_config=True)

    def driver_pack(self) -> Any:
        return self.get_driver().pack()
