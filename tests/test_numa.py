"""NUMA binding helper (jubatus_amd/utils/numa.py): cpulist parsing and the
off/unknown paths, which must leave the affinity untouched."""
import os

import pytest

from jubatus_amd.utils import numa


def test_cpulist_parse():
    assert numa._cpulist("0-3,8,10-11\n") == {0, 1, 2, 3, 8, 10, 11}
    assert numa._cpulist("") == set()


def test_node_cpus_missing_sysfs(tmp_path):
    assert numa.node_cpus(0, sysfs=str(tmp_path)) == set()
    (tmp_path / "node0").mkdir()
    (tmp_path / "node0" / "cpulist").write_text("0-1\n")
    assert numa.node_cpus(0, sysfs=str(tmp_path)) == {0, 1}


@pytest.mark.skipif(not hasattr(os, "sched_getaffinity"), reason="no affinity API")
def test_bind_off_keeps_affinity(monkeypatch):
    before = os.sched_getaffinity(0)
    monkeypatch.setenv("JB_NUMA_BIND", "off")
    assert numa.bind_to_device(0) == {}
    assert os.sched_getaffinity(0) == before


@pytest.mark.skipif(not hasattr(os, "sched_getaffinity"), reason="no affinity API")
def test_bind_explicit_node_without_cpus(monkeypatch):
    # a node with no CPUs in our mask: nothing is bound
    before = os.sched_getaffinity(0)
    monkeypatch.setenv("JB_NUMA_BIND", "4095")
    assert numa.bind_to_device(0) == {}
    assert os.sched_getaffinity(0) == before
