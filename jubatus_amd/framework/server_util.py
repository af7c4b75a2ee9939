"""Server / proxy command-line arguments and helpers (reference C20:
jubatus/server/framework/server_util.{hpp,cpp}).

Flags and defaults are identical to the reference (server_util.cpp:151-198,
401-425). MI355X additions: ``--gpu`` selects the HIP device (default: the
LOCAL_RANK env, else 0 when a GPU is present) and ``--cpu`` forces the host
backend.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from dataclasses import dataclass, field

from .. import __version__
from ..utils import logger, system

log = logger.get_logger("server_util")


class ArgvError(SystemExit):
    pass


def _range(lo: int, hi: int | None = None):
    def f(v: str) -> int:
        x = int(v)
        if x < lo or (hi is not None and x > hi):
            raise argparse.ArgumentTypeError(f"{v} out of range")
        return x
    return f


def _parser(prog: str, proxy: bool) -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog=prog, add_help=True)
    p.add_argument("-p", "--rpc-port", type=_range(1, 65535), default=9199, help="port number")
    p.add_argument("-b", "--listen_addr", default="", help="bind IP address")
    p.add_argument("-B", "--listen_if", default="", help="bind network interfance")
    p.add_argument("-c", "--thread", type=_range(1), default=4 if proxy else 2,
                   help="concurrency = thread number")
    p.add_argument("-t", "--timeout", type=_range(0), default=10, help="time out (sec)")
    p.add_argument("-Z", "--zookeeper_timeout", type=int, default=10,
                   help="coordinator (zookeeper) time out (sec)")
    p.add_argument("-I", "--interconnect_timeout", type=int, default=10,
                   help="interconnect time out between servers (sec)")
    p.add_argument("-D", "--daemon", action="store_true", help="launch in daemon mode (ignores SIGHUP)")
    p.add_argument("-l", "--logdir", default="", help="directory to output coordinator logs")
    p.add_argument("-g", "--log_config", default="", help="log configuration file")
    p.add_argument("-v", "--version", action="store_true", help="version")
    if proxy:
        p.add_argument("-z", "--zookeeper", default="localhost:2181", help="coordinator location")
        p.add_argument("-E", "--pool_expire", type=_range(0), default=60, help="session-pool expire time (sec)")
        p.add_argument("-S", "--pool_size", type=_range(0), default=0, help="session-pool maximum size")
    else:
        p.add_argument("-d", "--datadir", default="/tmp", help="directory to save and load models")
        p.add_argument("-f", "--configpath", default="",
                       help="config option need to specify json file when standalone mode")
        p.add_argument("-m", "--model_file", default="", help="model data to load at startup")
        p.add_argument("-z", "--zookeeper", default="", help="coordinator (zookeeper) location")
        p.add_argument("-n", "--name", default="", help="learning machine instance name")
        p.add_argument("-x", "--mixer", default="linear_mixer", help="mixer strategy")
        p.add_argument("-s", "--interval_sec", type=_range(0), default=16, help="mix interval by seconds")
        p.add_argument("-i", "--interval_count", type=_range(0), default=512,
                       help="mix interval by update count")
        p.add_argument("--gpu", type=int, default=None, help="HIP device index (MI355X)")
        p.add_argument("--cpu", action="store_true", help="run on the host backend (no GPU)")
    return p


def _address(bind_address: str, bind_if: str) -> tuple[str, str]:
    if bind_address:
        return bind_address, bind_address
    if bind_if:
        ip = system.get_ip(bind_if)
        return ip, ip
    return "0.0.0.0", system.get_default_v4_address()


@dataclass
class ServerArgv:
    type: str = ""
    port: int = 9199
    bind_address: str = "0.0.0.0"
    bind_if: str = ""
    threadnum: int = 2
    timeout: int = 10
    program_name: str = ""
    datadir: str = "/tmp"
    logdir: str = ""
    log_config: str = ""
    configpath: str = ""
    modelpath: str = ""
    daemon: bool = False
    z: str = ""
    name: str = ""
    mixer: str = "linear_mixer"
    # reference quirk: the default-constructed argv uses 5 / 1024, while the CLI
    # defaults are 16 / 512 (server_util.cpp:327-341 vs :184-189)
    interval_sec: int = 5
    interval_count: int = 1024
    zookeeper_timeout: int = 10
    interconnect_timeout: int = 10
    eth: str = "localhost"
    gpu: int | None = None
    cpu: bool = False
    extra: dict = field(default_factory=dict)

    def is_standalone(self) -> bool:
        return self.z == ""

    @classmethod
    def parse(cls, argv: list[str], type_: str, prog: str | None = None) -> "ServerArgv":
        prog = prog or f"juba{type_}"
        system.set_program_name(prog)
        p = _parser(prog, proxy=False)
        try:
            a = p.parse_args(argv)
        except SystemExit as e:
            raise ArgvError(e.code if e.code else 0)
        if a.version:
            print(f"jubatus-{__version__} (mi355x)")
            raise ArgvError(0)
        bind, eth = _address(a.listen_addr, a.listen_if)
        r = cls(type=type_, port=a.rpc_port, bind_address=bind, bind_if=a.listen_if,
                threadnum=a.thread, timeout=a.timeout, program_name=prog, datadir=a.datadir,
                logdir=a.logdir, log_config=a.log_config, configpath=a.configpath,
                modelpath=a.model_file, daemon=a.daemon, z=a.zookeeper, name=a.name,
                mixer=a.mixer, interval_sec=a.interval_sec, interval_count=a.interval_count,
                zookeeper_timeout=a.zookeeper_timeout,
                interconnect_timeout=a.interconnect_timeout, eth=eth, gpu=a.gpu, cpu=a.cpu)
        if r.log_config:
            r.log_config = system.real_path(r.log_config)
        logger.setup_parameters(prog, eth, r.port)
        logger.configure_logger(r.log_config)

        def die(msg: str) -> None:
            sys.stderr.write(msg + "\n" + p.format_usage())
            raise ArgvError(1)
        if not r.is_standalone() and not r.name:
            die("can't start multinode mode without name specified")
        if r.is_standalone() and not r.configpath and not r.modelpath:
            die("config path or model file must be specified for standalone mode")
        if r.configpath:
            r.configpath = system.real_path(r.configpath)
        if r.modelpath:
            r.modelpath = system.real_path(r.modelpath)
        if not r.is_standalone() and r.zookeeper_timeout < 1:
            die("can't start with zookeeper_timeout less than 1")
        if not r.is_standalone() and r.interconnect_timeout < 1:
            die("can't start with interconnect_timeout less than 1")
        if r.datadir:
            r.datadir = system.real_path(r.datadir)
            if not system.is_writable(r.datadir):
                die(f"can't use datadir: {r.datadir}")
        if r.logdir:
            r.logdir = system.real_path(r.logdir)
            if not system.is_writable(r.logdir):
                die("can't write to the coordinator log directory")
        r.boot_message()
        return r

    def boot_message(self) -> None:
        lines = [f"starting {self.program_name} {__version__} RPC server at {self.eth}:{self.port}",
                 f"    pid                  : {os.getpid()}",
                 f"    user                 : {system.get_user_name()}",
                 f"    mode                 : {'standalone mode' if self.is_standalone() else 'multinode mode'}",
                 f"    timeout              : {self.timeout}",
                 f"    thread               : {self.threadnum}",
                 f"    datadir              : {self.datadir}",
                 f"    logdir               : {self.logdir}",
                 f"    log config           : {self.log_config}",
                 f"    zookeeper            : {self.z}",
                 f"    name                 : {self.name}",
                 f"    interval sec         : {self.interval_sec if self.interval_sec > 0 else 'disabled'}",
                 f"    interval count       : {self.interval_count if self.interval_count > 0 else 'disabled'}",
                 f"    zookeeper timeout    : {self.zookeeper_timeout}",
                 f"    interconnect timeout : {self.interconnect_timeout}"]
        log.info("\n".join(lines))


@dataclass
class ProxyArgv:
    type: str = ""
    port: int = 9199
    bind_address: str = "0.0.0.0"
    bind_if: str = ""
    threadnum: int = 4
    timeout: int = 10
    zookeeper_timeout: int = 10
    interconnect_timeout: int = 10
    program_name: str = ""
    z: str = "localhost:2181"
    session_pool_expire: int = 60
    session_pool_size: int = 0
    logdir: str = ""
    log_config: str = ""
    eth: str = ""
    daemon: bool = False

    @classmethod
    def parse(cls, argv: list[str], type_: str, prog: str | None = None) -> "ProxyArgv":
        prog = prog or f"juba{type_}_proxy"
        system.set_program_name(prog)
        p = _parser(prog, proxy=True)
        try:
            a = p.parse_args(argv)
        except SystemExit as e:
            raise ArgvError(e.code if e.code else 0)
        if a.version:
            print(f"jubatus-{__version__} (mi355x)")
            raise ArgvError(0)
        bind, eth = _address(a.listen_addr, a.listen_if)
        r = cls(type=type_, port=a.rpc_port, bind_address=bind, bind_if=a.listen_if,
                threadnum=a.thread, timeout=a.timeout, zookeeper_timeout=a.zookeeper_timeout,
                interconnect_timeout=a.interconnect_timeout, program_name=prog, z=a.zookeeper,
                session_pool_expire=a.pool_expire, session_pool_size=a.pool_size,
                logdir=a.logdir, log_config=a.log_config, eth=eth, daemon=a.daemon)
        logger.setup_parameters(prog, eth, r.port)
        logger.configure_logger(r.log_config)
        if r.zookeeper_timeout < 1 or r.interconnect_timeout < 1:
            sys.stderr.write("can't start with a timeout less than 1\n" + p.format_usage())
            raise ArgvError(1)
        if r.logdir and not system.is_writable(r.logdir):
            sys.stderr.write("can't create log file\n")
            raise ArgvError(1)
        log.info(f"starting {prog} {__version__} RPC server at {eth}:{r.port}")
        return r


def get_server_identifier(a) -> str:
    """'<eth>_<port>' (reference server_util.cpp:390-396)."""
    return f"{a.eth}_{a.port}"


get_proxy_identifier = get_server_identifier


def get_conf(a: ServerArgv, coord=None) -> str:
    """Config JSON text from the local file (standalone) or the coordinator
    (reference server_util.cpp:100-117, common/config.cpp:39-48)."""
    if a.is_standalone():
        with open(a.configpath, encoding="utf-8") as f:
            return f.read()
    from ..common import config as zkconfig
    return zkconfig.config_fromzk(coord, a.type, a.name)


def parse_config_json(text: str, where: str) -> dict:
    try:
        obj = json.loads(text)
    except json.JSONDecodeError as e:
        # reference: JSON syntax error -> log and exit(1) (server_helper.hpp:100-113)
        log.error(f"syntax error in configuration: {where}:{e.lineno}:{e.colno} {e.msg}")
        raise ArgvError(1)
    if not isinstance(obj, dict):
        raise ValueError("configuration must be a JSON object")
    return obj
