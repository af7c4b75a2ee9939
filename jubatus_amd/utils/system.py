"""OS helpers (reference C13: jubatus/server/common/{system,network,filesystem}.cpp).

get_program_name (/proc/self/exe equivalent: the running entry point),
get_user_name, get_machine_status (VIRT/RSS/SHR KiB from /proc/self/statm),
daemonize, get_default_v4_address (first non-loopback IPv4), get_ip(nic),
is_writable, base_name, real_path, loadavg/memory for get_loads.
"""
from __future__ import annotations

import fcntl
import getpass
import os
import socket
import struct
import sys

_PAGE_KB = os.sysconf("SC_PAGE_SIZE") // 1024
_progname: str | None = None


def set_program_name(name: str) -> None:
    global _progname
    _progname = name


def get_program_name() -> str:
    if _progname:
        return _progname
    return os.path.basename(sys.argv[0]) if sys.argv and sys.argv[0] else "jubatus"


def get_user_name() -> str:
    try:
        return getpass.getuser()
    except Exception:  # no passwd entry (containers)
        return str(os.getuid())


def get_machine_status() -> dict[str, int]:
    """{'VIRT','RSS','SHR'} in KiB (reference system.cpp:165-185)."""
    try:
        with open("/proc/self/statm") as f:
            size, resident, share = (int(x) for x in f.read().split()[:3])
    except OSError:
        size = resident = share = 0
    return {"VIRT": size * _PAGE_KB, "RSS": resident * _PAGE_KB, "SHR": share * _PAGE_KB}


def get_loads() -> dict[str, str]:
    out = {"loadavg": "0", "total_memory": "0", "free_memory": "0"}
    try:
        out["loadavg"] = str(os.getloadavg()[0])
        with open("/proc/meminfo") as f:
            mi = {l.split(":")[0]: int(l.split()[1]) for l in f if ":" in l}
        out["total_memory"] = str(mi.get("MemTotal", 0) * 1024)
        out["free_memory"] = str(mi.get("MemFree", 0) * 1024)
    except Exception:
        pass
    return out


def daemonize() -> None:
    """Ignore SIGHUP (the reference's daemon mode: server_util.cpp
    daemonize_process keeps the process in the foreground)."""
    import signal
    signal.signal(signal.SIGHUP, signal.SIG_IGN)


def _ifaces() -> list[tuple[str, str]]:
    out = []
    try:
        names = os.listdir("/sys/class/net")
    except OSError:
        names = []
    s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    try:
        for n in sorted(names):
            try:
                r = fcntl.ioctl(s.fileno(), 0x8915, struct.pack("256s", n.encode()[:15]))  # SIOCGIFADDR
                out.append((n, socket.inet_ntoa(r[20:24])))
            except OSError:
                continue
    finally:
        s.close()
    return out


def get_ip(nic: str) -> str:
    for n, ip in _ifaces():
        if n == nic:
            return ip
    raise RuntimeError(f"failed to get IP address of interface {nic}")


def get_default_v4_address() -> str:
    for _, ip in _ifaces():
        if not ip.startswith("127."):
            return ip
    return "127.0.0.1"


def is_writable(path: str) -> bool:
    return os.path.isdir(path) and os.access(path, os.W_OK | os.X_OK)


def base_name(path: str) -> str:
    return os.path.basename(path.rstrip("/")) if path not in ("", "/") else path


def real_path(path: str) -> str:
    return os.path.realpath(path)
