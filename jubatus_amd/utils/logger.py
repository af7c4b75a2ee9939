"""Logger (reference C16: jubatus/server/common/logger/logger.{hpp,cpp}).

Console pattern ``%d %X{tid} %-5p [%F:%L] %m%n`` (logger.cpp:105-110): time,
thread id, level, file:line, message. With ``-g <config>`` (a log
configuration file, JSON or the reference's log4cxx XML with a file appender
pattern) logs go to a file whose name may use ${JUBATUS_PROCESS},
${JUBATUS_HOST}, ${JUBATUS_PORT}, ${JUBATUS_PID} (log4cxx.xml:12-18). SIGHUP
reloads the configuration (server_util.cpp:68-92).

Levels: FATAL (logs then aborts the process), ERROR, WARN, INFO, DEBUG, TRACE.
"""
from __future__ import annotations

import logging
import os
import re
import sys
import threading

TRACE = 5
logging.addLevelName(TRACE, "TRACE")
logging.addLevelName(logging.WARNING, "WARN")
logging.addLevelName(logging.CRITICAL, "FATAL")

_ROOT = "jubatus"
_params = {"JUBATUS_PROCESS": "jubatus", "JUBATUS_HOST": "localhost", "JUBATUS_PORT": "0",
           "JUBATUS_PID": str(os.getpid())}
_config_path = ""
_lock = threading.Lock()


class _Formatter(logging.Formatter):
    def format(self, record: logging.LogRecord) -> str:
        ts = self.formatTime(record, "%Y-%m-%d %H:%M:%S")
        ts = f"{ts},{int(record.msecs):03d}"
        return (f"{ts} {threading.get_native_id() if record.thread == threading.get_ident() else record.thread}"
                f" {record.levelname:<5} [{os.path.basename(record.pathname)}:{record.lineno}] "
                f"{record.getMessage()}")


def get_logger(name: str | None = None) -> logging.Logger:
    return logging.getLogger(_ROOT if not name else f"{_ROOT}.{name}")


def setup_parameters(progname: str, host: str, port: int) -> None:
    """Reference logger::setup_parameters: values usable in file names."""
    _params.update({"JUBATUS_PROCESS": os.path.basename(progname), "JUBATUS_HOST": host,
                    "JUBATUS_PORT": str(port), "JUBATUS_PID": str(os.getpid())})
    for k, v in _params.items():
        os.environ[k] = v


def _expand(path: str) -> str:
    return re.sub(r"\$\{(\w+)\}", lambda m: _params.get(m.group(1), os.environ.get(m.group(1), "")), path)


def _file_from_config(path: str) -> tuple[str | None, int]:
    """Pick the log file and level out of a JSON or log4cxx-XML config."""
    with open(path, encoding="utf-8") as f:
        text = f.read()
    level = logging.INFO
    m = re.search(r'<level\s+value="(\w+)"', text) or re.search(r'"level"\s*:\s*"(\w+)"', text)
    if m:
        level = {"TRACE": TRACE, "DEBUG": logging.DEBUG, "INFO": logging.INFO, "WARN": logging.WARNING,
                 "ERROR": logging.ERROR, "FATAL": logging.CRITICAL}.get(m.group(1).upper(), logging.INFO)
    m = re.search(r'<param\s+name="File"\s+value="([^"]+)"', text) or \
        re.search(r'"file"\s*:\s*"([^"]+)"', text)
    return (_expand(m.group(1)) if m else None), level


def configure_logger(log_config: str = "", level: int | None = None) -> None:
    global _config_path
    with _lock:
        _config_path = log_config
        root = logging.getLogger(_ROOT)
        for h in list(root.handlers):
            root.removeHandler(h)
            h.close()
        target, lvl = (None, logging.INFO)
        if log_config:
            target, lvl = _file_from_config(log_config)
        if level is not None:
            lvl = level
        if target:
            os.makedirs(os.path.dirname(os.path.abspath(target)), exist_ok=True)
            h: logging.Handler = logging.FileHandler(target)
        else:
            h = logging.StreamHandler(sys.stderr)
        h.setFormatter(_Formatter())
        root.addHandler(h)
        root.setLevel(lvl)
        root.propagate = False


def reconfigure() -> None:
    """SIGHUP action: reload the configuration / reopen the log file."""
    configure_logger(_config_path)


def fatal(msg: str, *args) -> None:
    """LOG(FATAL): log then abort (reference logger.hpp: FATAL aborts)."""
    get_logger().critical(msg, *args, stacklevel=2)
    logging.shutdown()
    os._exit(1)


if not logging.getLogger(_ROOT).handlers:
    configure_logger()
