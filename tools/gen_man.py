"""Generate the man pages (man/*.1, man/*.8) from the tools' own --help.

Reference: man/en/*.{1,8} (jenerator.1, jubaconfig.8, jubaconv.1, jubactl.8,
jubadump.1, jubatus_proxy.8, jubatus_server.8, jubavisor.8), written by
hand there; here each page is rendered from the option parser it documents,
so a page can never list a flag the tool does not have (tests/test_tools.py
checks that the committed pages are current).

Usage: python tools/gen_man.py [--check]
"""
from __future__ import annotations

import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PAGES = [
    ("jubatus_server", 8, ["bin/jubaclustering", "--help"],
     "engine server (jubaclassifier, jubaregression, jubarecommender, jubanearest_neighbor, "
     "jubaanomaly, jubaclustering, jubaburst, jubabandit, jubastat, jubagraph, jubaweight)",
     "Serves one engine over msgpack-RPC. Each server process drives one GPU (--gpu, or "
     "LOCAL_RANK, or the least-used device assigned by jubavisor); models live in HBM and are "
     "mixed with the other members of the cluster over RCCL. Without --zookeeper the server "
     "runs standalone. jubaclassifier, jubaregression, jubarecommender, jubanearest_neighbor, "
     "jubaanomaly, jubaclustering, jubastat, jubabandit, jubaburst, jubagraph and jubaweight "
     "are native binaries (no "
     "Python) for standalone configurations whose converter runs on the native hashers; they "
     "hand every other setup to this server with the same flags."),
    ("jubatus_proxy", 8, ["bin/jubaclassifier_proxy", "--help"],
     "engine proxy (juba*_proxy)",
     "Native proxy in front of a cluster of engine servers: routes every request to one, "
     "several or all members (random, consistent hash, broadcast) and aggregates the answers."),
    ("jubavisor", 8, ["bin/jubavisor", "--help"],
     "process supervisor",
     "Starts and stops engine servers on request of jubactl, one GPU per child process."),
    ("jubactl", 8, ["bin/jubactl", "--help"],
     "cluster control",
     "Starts, stops, saves, loads and inspects the servers of a named cluster through the "
     "jubavisors registered in the coordinator."),
    ("jubaconfig", 8, ["bin/jubaconfig", "--help"],
     "configuration store client",
     "Writes, reads, deletes and lists engine configurations in the coordinator."),
    ("jubaconv", 1, ["bin/jubaconv", "--help"],
     "converter test tool",
     "Runs the feature converter of a configuration on JSON or datum input and prints the "
     "datum or the feature vector."),
    ("jubadump", 1, ["bin/jubadump", "--help"],
     "model file dumper",
     "Prints the contents of a saved model file (header, system data and model) as JSON."),
    ("jenerator", 1, [sys.executable, "-m", "jubatus_amd.idl.jenerator", "--help"],
     "IDL compiler",
     "Generates client libraries, server skeletons, proxy tables and documentation from the "
     "engine IDL files."),
]


def _esc(s: str) -> str:
    return s.replace("\\", "\\\\").replace("-", "\\-")


def render(name: str, sec: int, cmd: list[str], short: str, desc: str) -> str:
    # the Python server's help (the launchers' native binaries take the same flags)
    env = dict(os.environ, PYTHONPATH=ROOT, COLUMNS="100", JUBATUS_NATIVE_SERVER="0", JUBATUS_PY_TOOLS="1")
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    help_text = (out.stdout or out.stderr).rstrip()
    lines = [f'.TH {name.upper()} {sec} "" "jubatus_amd" "jubatus_amd manual"',
             ".SH NAME", f"{_esc(name)} \\- {_esc(short)}",
             ".SH SYNOPSIS", ".nf"]
    usage, rest = [], []
    in_usage = True
    for ln in help_text.splitlines():
        if in_usage and (ln.startswith("usage:") or (usage and ln.startswith(" "))):
            usage.append(ln)
            continue
        in_usage = False
        rest.append(ln)
    lines += [_esc(u.replace("usage: ", "", 1)) for u in usage] + [".fi", ".SH DESCRIPTION",
                                                                   _esc(desc), ".SH OPTIONS", ".nf"]
    lines += [_esc(r) for r in rest if r.strip()]
    lines += [".fi", ".SH SEE ALSO",
              ", ".join(f"\\fB{_esc(n)}\\fR({s})" for n, s, *_ in PAGES if n != name)]
    return "\n".join(lines) + "\n"


def flags_of(text: str) -> set[str]:
    return set(re.findall(r"(?<![\w-])(--?[A-Za-z][\w-]*)", text))


def main() -> int:
    check = "--check" in sys.argv
    mandir = os.path.join(ROOT, "man")
    os.makedirs(mandir, exist_ok=True)
    stale = []
    for name, sec, cmd, short, desc in PAGES:
        page = render(name, sec, cmd, short, desc)
        path = os.path.join(mandir, f"{name}.{sec}")
        if check:
            cur = open(path).read() if os.path.exists(path) else ""
            if cur != page:
                stale.append(path)
        else:
            with open(path, "w") as f:
                f.write(page)
    if stale:
        print("stale man pages (run tools/gen_man.py):", *stale, sep="\n  ")
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
