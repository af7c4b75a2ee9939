"""In-tree build of the native components.

* ``jubatus_amd/_jubatus_native*.so`` - host C++17 runtime (pybind11):
  request scanner, label table, hashing, CRC32, MD5, msgpack codec, RPC core.
* ``jubatus_amd/libjubatus_hip.so`` - every HIP kernel, compiled for gfx950
  only (``hipcc --offload-arch=gfx950``), exported through a C ABI and
  loaded with ctypes (jubatus_amd/ops/hip.py).
* ``jubatus_amd/plugins/libjubatus_{sample_plugins,ux_splitter}.so`` -
  fv_converter plug-ins (C ABI csrc/plugins/jb_plugin.h) in the in-tree
  plug-in directory.
* ``jubatus_amd/native_bin/{jubacoordinator,jubaproxy}`` - the Python-free
  coordination server (csrc/coord) and request router (csrc/proxy).
* ``jubatus_amd/native_bin/jubaclassifier`` - the Python-free classifier
  server (csrc/server), linked against ``libjubatus_hip.so``.

All are built in-tree so they travel with the repository snapshot to the
GPU box. Incremental: a target is rebuilt only if a source is newer.

Usage: ``python -m jubatus_amd.build_ext [--force] [-j N]``
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
BUILD = os.path.join(PKG, "csrc", "build")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

NATIVE_SO = os.path.join(PKG, "_jubatus_native" + sysconfig.get_config_var("EXT_SUFFIX"))
HIP_SO = os.path.join(PKG, "libjubatus_hip.so")


def _newer(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        sys.stderr.write(" ".join(cmd) + "\n" + r.stdout)
        raise RuntimeError(f"build failed: {cmd[0]} (exit {r.returncode})")


def _compile_all(jobs: list[tuple[str, list[str]]], nproc: int) -> None:
    with cf.ThreadPoolExecutor(max_workers=max(1, nproc)) as ex:
        futs = [ex.submit(_run, cmd) for _, cmd in jobs]
        for f in futs:
            f.result()


def build_native(force: bool = False, nproc: int = 8) -> str:
    import pybind11

    srcs = sorted(glob.glob(os.path.join(CSRC, "native", "*.cpp")))
    hdrs = sorted(glob.glob(os.path.join(CSRC, "native", "*.hpp")))
    if not force and not _newer(NATIVE_SO, srcs + hdrs):
        return NATIVE_SO
    os.makedirs(BUILD, exist_ok=True)
    inc = [f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}",
           f"-I{os.path.join(CSRC, 'native')}"]
    flags = ["-O3", "-std=c++17", "-fPIC", "-pthread", "-fvisibility=hidden", "-Wall",
             "-Wno-unused-function"]
    objs, jobs = [], []
    for s in srcs:
        o = os.path.join(BUILD, "native_" + os.path.basename(s) + ".o")
        objs.append(o)
        if force or _newer(o, [s] + hdrs):
            jobs.append((o, ["g++", *flags, *inc, "-c", s, "-o", o]))
    _compile_all(jobs, nproc)
    _run(["g++", "-shared", "-pthread", "-o", NATIVE_SO, *objs, "-ldl"])
    return NATIVE_SO


def build_hip(force: bool = False, nproc: int = 8) -> str:
    srcs = sorted(glob.glob(os.path.join(CSRC, "hip", "*.hip")))
    hdrs = sorted(glob.glob(os.path.join(CSRC, "hip", "*.hpp")))
    if not force and not _newer(HIP_SO, srcs + hdrs):
        return HIP_SO
    os.makedirs(BUILD, exist_ok=True)
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=fast",
             f"-I{os.path.join(CSRC, 'hip')}"]
    objs, jobs = [], []
    for s in srcs:
        o = os.path.join(BUILD, "hip_" + os.path.basename(s) + ".o")
        objs.append(o)
        if force or _newer(o, [s] + hdrs):
            jobs.append((o, [HIPCC, *flags, "-c", s, "-o", o]))
    _compile_all(jobs, nproc)
    _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", HIP_SO, *objs])
    return HIP_SO


PLUGIN_DIR = os.path.join(PKG, "plugins")
PLUGIN_SO = os.path.join(PLUGIN_DIR, "libjubatus_sample_plugins.so")
# one shared object per plug-in source
PLUGINS = {"sample_plugins.cpp": "libjubatus_sample_plugins.so",
           "ux_splitter.cpp": "libjubatus_ux_splitter.so",
           "mecab_splitter.cpp": "libjubatus_mecab_splitter.so"}


def build_plugins(force: bool = False) -> str:
    hdrs = sorted(glob.glob(os.path.join(CSRC, "plugins", "*.h")))
    os.makedirs(PLUGIN_DIR, exist_ok=True)
    for src, lib in PLUGINS.items():
        s = os.path.join(CSRC, "plugins", src)
        target = os.path.join(PLUGIN_DIR, lib)
        if force or _newer(target, [s] + hdrs):
            _run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall",
                  f"-I{os.path.join(CSRC, 'plugins')}", "-o", target, s, "-ldl"])
    return PLUGIN_DIR


NATIVE_BIN = os.path.join(PKG, "native_bin")
# native executables: name -> (sources, extra include dirs)
TOOLS = {
    "jubacoordinator": (["coord/jubacoordinator.cpp", "native/jb_rpc.cpp"],
                        ["coord", "native", "../client_cpp/include"]),
    "jubaproxy": (["proxy/jubaproxy.cpp", "native/jb_rpc.cpp"],
                  ["proxy", "native", "../client_cpp/include"]),
    "jubavisor": (["visor/jubavisor.cpp", "native/jb_rpc.cpp"],
                  ["visor", "native", "../client_cpp/include"]),
    "jubaloadgen": (["tools/jubaloadgen.cpp", "native/jb_rpc.cpp"], ["native"]),
    # operator tools (csrc/cmd): cluster control and configs in the coordinator
    "jubactl": (["cmd/jubactl.cpp", "native/jb_rpc.cpp"], ["cmd", "native", "../client_cpp/include"]),
    "jubaconfig": (["cmd/jubaconfig.cpp", "native/jb_rpc.cpp"],
                   ["cmd", "native", "server", "../client_cpp/include"]),
    # host-only rehearsal of the native distributed model plane (jb_mix_group.hpp)
    "jb_mix_rehearsal": (["tools/jb_mix_rehearsal.cpp", "native/jb_rpc.cpp"],
                         ["native", "server", "../client_cpp/include"]),
}


def build_tools(force: bool = False, nproc: int = 8, sanitize: str | None = None) -> str:
    """Python-free native executables (coordinator, proxy, jubavisor, load generator). ``sanitize``
    ("address", "thread", "undefined") builds instrumented copies into
    native_bin/<sanitizer>/ (the reference's --fsanitize build option,
    wscript:55-57,143-146; host code only)."""
    out = os.path.join(NATIVE_BIN, sanitize) if sanitize else NATIVE_BIN
    os.makedirs(out, exist_ok=True)
    opt = ["-O1", "-g", "-fno-omit-frame-pointer", f"-fsanitize={sanitize}"] if sanitize else ["-O2"]
    jobs = []
    for name, (srcs, incs) in TOOLS.items():
        target = os.path.join(out, name)
        paths = [os.path.join(CSRC, x) for x in srcs]
        deps = paths + [h for d in incs for h in glob.glob(os.path.join(CSRC, d, "**", "*.h*"),
                                                            recursive=True)]
        if force or _newer(target, deps):
            jobs.append((target, ["g++", *opt, "-std=c++17", "-pthread", "-Wall",
                                  *[f"-I{os.path.join(CSRC, d)}" for d in incs], *paths,
                                  "-o", target]))
    _compile_all(jobs, nproc)
    return out


# native engine servers (csrc/server): host C++ over the HIP runtime and the
# kernel library (linked against libjubatus_hip.so, found via $ORIGIN/..)
SERVERS = {
    "jubaclassifier": (["server/jubaclassifier.cpp", "native/jb_rpc.cpp"],
                       ["server", "native", "hip"]),   # + RCCL (distributed mode)
    "jubaregression": (["server/jubaregression.cpp", "native/jb_rpc.cpp"],
                       ["server", "native", "hip"]),
    # row engines over the LSH / inverted-index kernels (jb_row_server.hpp)
    "jubarecommender": (["server/jubarecommender.cpp", "native/jb_rpc.cpp"],
                        ["server", "native", "hip"]),
    "jubanearest_neighbor": (["server/jubanearest_neighbor.cpp", "native/jb_rpc.cpp"],
                             ["server", "native", "hip"]),
    "jubaanomaly": (["server/jubaanomaly.cpp", "native/jb_rpc.cpp"], ["server", "native", "hip"]),
    # host engines: no GPU, no HIP libraries
    "jubastat": (["server/jubastat.cpp", "native/jb_rpc.cpp"], ["server", "native", "hip"]),
    "jubabandit": (["server/jubabandit.cpp", "native/jb_rpc.cpp"], ["server", "native", "hip"]),
    "jubaburst": (["server/jubaburst.cpp", "native/jb_rpc.cpp"], ["server", "native", "hip"]),
    "jubagraph": (["server/jubagraph.cpp", "native/jb_rpc.cpp"], ["server", "native", "hip"]),
    "jubaweight": (["server/jubaweight.cpp", "native/jb_rpc.cpp"], ["server", "native", "hip"]),
    # coresets + k-means++ / Lloyd / GMM EM in csrc/hip/clustering.hip
    "jubaclustering": (["server/jubaclustering.cpp", "native/jb_rpc.cpp"], ["server", "native", "hip"]),
    # jubaconv (operator tool) over the native wide converter: host code only
    "jubaconv": (["cmd/jubaconv.cpp", "native/jb_rpc.cpp"], ["cmd", "server", "native", "hip"]),
    # check of the RCCL data plane of the native MIX on one GPU (not a server)
    "jb_rccl_check": (["tools/jb_rccl_check.cpp", "native/jb_rpc.cpp"], ["server", "native", "hip"]),
}
HOST_SERVERS = {"jubastat", "jubabandit", "jubaburst", "jubagraph", "jubaweight", "jubaconv"}
# servers with a native distributed mode (the model plane over RCCL)
RCCL_SERVERS = {"jubaclassifier", "jubaregression", "jb_rccl_check", "jubarecommender",
                "jubanearest_neighbor", "jubaanomaly", "jubaclustering"}


def build_servers(force: bool = False, nproc: int = 8) -> str:
    """Python-free engine servers (they exec the Python server for the
    configurations they do not serve natively)."""
    os.makedirs(NATIVE_BIN, exist_ok=True)
    jobs = []
    for name, (srcs, incs) in SERVERS.items():
        target = os.path.join(NATIVE_BIN, name)
        paths = [os.path.join(CSRC, x) for x in srcs]
        incs = incs + ["../client_cpp/include"]
        deps = paths + [HIP_SO] + [h for d in incs for h in glob.glob(os.path.join(CSRC, d, "*.h*"))]
        libs = [] if name in HOST_SERVERS else [
            f"-L{PKG}", "-ljubatus_hip", "-L/opt/rocm/lib", "-lamdhip64",
            "-Wl,-rpath,$ORIGIN/..", "-Wl,-rpath,/opt/rocm/lib"]
        if name in RCCL_SERVERS:
            libs.append("-lrccl")
        if force or _newer(target, deps):
            jobs.append((target, ["g++", "-O2", "-std=c++17", "-pthread", "-Wall",
                                  "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
                                  *[f"-I{os.path.join(CSRC, d)}" for d in incs], *paths, *libs,
                                  "-o", target]))
    _compile_all(jobs, nproc)
    return NATIVE_BIN


def build_all(force: bool = False, nproc: int | None = None) -> tuple[str, ...]:
    nproc = nproc or min(8, os.cpu_count() or 4)
    return (build_native(force, nproc), build_hip(force, nproc), build_plugins(force),
            build_tools(force, nproc), build_servers(force, nproc))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=None)
    ap.add_argument("--sanitize", choices=("address", "thread", "undefined"), default=None,
                    help="also build sanitizer-instrumented native executables")
    a = ap.parse_args()
    if a.sanitize:
        print(build_tools(a.force, a.j or 8, a.sanitize))
    for p in build_all(a.force, a.j):
        print(p)


if __name__ == "__main__":
    main()
