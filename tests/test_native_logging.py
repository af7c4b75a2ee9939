"""Native server logging flags (csrc/native/jb_log.hpp, reference C16 and
server_util.cpp:68-92,236-242,379-388, server_helper.cpp:34-44): -g names a
log configuration whose file appender the server writes to, SIGHUP reloads
it (a rotated file is reopened), -D ignores SIGHUP, and an unusable -l / -g
stops the server at startup. Runs the host-engine server jubastat on the CPU."""
import json
import os
import signal
import socket
import subprocess
import time

from helpers import ROOT
from jubatus_amd.common.mprpc import RpcClient, RpcIOError, RpcTimeoutError

NATIVE_BIN = os.path.join(ROOT, "jubatus_amd", "native_bin")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _start(tmp_path, *extra):
    port = _free_port()
    cfg = tmp_path / "stat.json"
    cfg.write_text(json.dumps({"window_size": 16}))
    p = subprocess.Popen([os.path.join(NATIVE_BIN, "jubastat"), "-p", str(port), "-b", "127.0.0.1",
                          "-f", str(cfg), "-d", str(tmp_path), *extra],
                         stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    deadline = time.time() + 30
    while True:
        try:
            with RpcClient("127.0.0.1", port, 5.0) as c:
                c.call("get_config", "")
            return p, port
        except (OSError, RpcIOError, RpcTimeoutError):
            assert p.poll() is None and time.time() < deadline, p.stdout.read()
            time.sleep(0.1)


def _wait_for(path, text, timeout=10.0):
    deadline = time.time() + timeout
    while time.time() < deadline:
        if os.path.exists(path) and text in open(path).read():
            return True
        time.sleep(0.05)
    return False


def test_log_config_file_and_hup_reopen(tmp_path):
    logcfg = tmp_path / "log.json"
    logcfg.write_text(json.dumps({"file": str(tmp_path / "${JUBATUS_PROCESS}.${JUBATUS_PORT}.log"),
                                  "level": "INFO"}))
    p, port = _start(tmp_path, "-g", str(logcfg))
    try:
        log = tmp_path / f"jubastat.{port}.log"
        assert _wait_for(log, "start listening"), p.stdout.read1() if p.stdout else ""
        # the file appender took the lines: nothing on stderr after configure
        rotated = tmp_path / "rotated.log"
        os.rename(log, rotated)
        p.send_signal(signal.SIGHUP)
        assert _wait_for(log, "log configuration reloaded"), "HUP did not reopen the log file"
        assert "reloading log configuration" in rotated.read_text()
        assert p.poll() is None
        with RpcClient("127.0.0.1", port, 5.0) as c:
            c.call("save", "", "m1")
        assert _wait_for(log, "saved to")
        assert "saved to" not in rotated.read_text()
    finally:
        p.terminate()
        p.wait(timeout=30)


def test_log4cxx_xml_config_and_level(tmp_path):
    logcfg = tmp_path / "log4cxx.xml"
    target = tmp_path / "xml_${JUBATUS_PORT}.log"
    logcfg.write_text(f"""<?xml version="1.0" encoding="UTF-8" ?>
<log4j:configuration xmlns:log4j="http://jakarta.apache.org/log4j/">
  <appender name="file" class="org.apache.log4j.FileAppender">
    <param name="File" value="{target}" />
  </appender>
  <root><level value="WARN" /><appender-ref ref="file" /></root>
</log4j:configuration>
""")
    p, port = _start(tmp_path, "-g", str(logcfg))
    try:
        log = tmp_path / f"xml_{port}.log"
        deadline = time.time() + 5
        while not log.exists() and time.time() < deadline:
            time.sleep(0.05)
        assert log.exists()
        time.sleep(0.3)
        assert "start listening" not in log.read_text()     # INFO is below WARN
    finally:
        p.terminate()
        p.wait(timeout=30)


def test_daemon_mode_ignores_hup(tmp_path):
    logcfg = tmp_path / "log.json"
    logcfg.write_text(json.dumps({"file": str(tmp_path / "d.log")}))
    p, port = _start(tmp_path, "-D", "-g", str(logcfg))
    try:
        log = tmp_path / "d.log"
        assert _wait_for(log, "set daemon mode (SIGHUP is now ignored)")
        p.send_signal(signal.SIGHUP)
        time.sleep(0.5)
        assert p.poll() is None                               # still serving
        with RpcClient("127.0.0.1", port, 5.0) as c:
            assert c.call("get_config", "")
        assert "reloading log configuration" not in log.read_text()
    finally:
        p.terminate()
        p.wait(timeout=30)


def test_hup_without_config_keeps_running(tmp_path):
    p, port = _start(tmp_path)
    try:
        p.send_signal(signal.SIGHUP)       # the default action would end the process
        time.sleep(0.3)
        assert p.poll() is None
    finally:
        p.terminate()
        p.wait(timeout=30)


def test_unusable_logdir_or_config_stops_startup(tmp_path):
    port = _free_port()
    cfg = tmp_path / "stat.json"
    cfg.write_text(json.dumps({"window_size": 16}))
    exe = os.path.join(NATIVE_BIN, "jubastat")
    r = subprocess.run([exe, "-p", str(port), "-f", str(cfg), "-l", str(tmp_path / "missing")],
                       capture_output=True, text=True, timeout=30)
    assert r.returncode == 1 and "logdir" in r.stderr
    bad = tmp_path / "log.json"
    bad.write_text(json.dumps({"file": str(tmp_path / "nodir" / "x.log")}))
    r = subprocess.run([exe, "-p", str(port), "-f", str(cfg), "-g", str(bad)],
                       capture_output=True, text=True, timeout=30)
    assert r.returncode == 1 and "failed to configure logger" in r.stderr
