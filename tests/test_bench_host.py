"""bench.py's host facts for the CPU baseline (no GPU): the usable CPUs are the affinity
set bounded by a cgroup v2 CPU quota (the reference's cpu_count()-sized pool as the host
runs it, VA:21 / VA:462)."""
import builtins
import io
import os

import bench


def _with_cpu_max(monkeypatch, text):
    real_open = builtins.open

    def fake_open(path, *a, **k):
        if path == "/sys/fs/cgroup/cpu.max":
            if text is None:
                raise FileNotFoundError(path)
            return io.StringIO(text)
        return real_open(path, *a, **k)

    monkeypatch.setattr(builtins, "open", fake_open)


def test_host_cpus_quota_bounds_affinity(monkeypatch):
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: set(range(256)))
    monkeypatch.setattr(os, "cpu_count", lambda: 256)
    _with_cpu_max(monkeypatch, "1600000 100000\n")
    assert bench.host_cpus() == (16, 256, 256, 16.0)
    _with_cpu_max(monkeypatch, "150000 100000\n")  # 1.5 CPUs -> 2 processes
    assert bench.host_cpus()[0] == 2


def test_host_cpus_without_quota(monkeypatch):
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: set(range(12)))
    monkeypatch.setattr(os, "cpu_count", lambda: 64)
    _with_cpu_max(monkeypatch, "max 100000\n")
    assert bench.host_cpus() == (12, 64, 12, None)
    _with_cpu_max(monkeypatch, None)
    assert bench.host_cpus() == (12, 64, 12, None)
