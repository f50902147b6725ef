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


def test_rank_envs_are_torchrun_like():
    """bench.py --gpus N without torchrun starts N rank processes with torchrun's variables."""
    envs = bench.rank_envs(3, {"PATH": "/bin", "HSA_ENABLE_IPC_MODE_LEGACY": "0"}, 29555)
    assert [e["RANK"] for e in envs] == ["0", "1", "2"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2"]
    for e in envs:
        assert e["WORLD_SIZE"] == "3" and e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "29555"
        assert e["PATH"] == "/bin" and e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_check_devices_refuses_missing_gpus():
    import pytest

    bench.check_devices(8, 8, False)
    bench.check_devices(2, 1, True)  # the one-device gloo rehearsal
    with pytest.raises(SystemExit, match="only 1 device"):
        bench.check_devices(8, 1, False)
    with pytest.raises(SystemExit):
        bench.check_devices(2, 0, False)


def test_bench_gpus_without_devices_exits_nonzero():
    """The whole command: --gpus 2 on a host with no GPU refuses before doing any work."""
    import subprocess
    import sys

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "KCMC_BENCH_ONE_DEVICE")}
    r = subprocess.run([sys.executable, bench.__file__, "--gpus", "2", "--steps", "1", "--warmup", "0"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "device(s) visible" in r.stderr
    assert '"n_gpus"' not in r.stdout


def test_spawn_ranks_children_and_exit_code(tmp_path):
    """spawn_ranks starts one child per rank with its own RANK and returns a failing rank's code."""
    import sys

    script = tmp_path / "child.py"
    script.write_text("import os, sys\n"
                      "open(os.path.join(os.path.dirname(__file__), 'r' + os.environ['RANK']), 'w').write("
                      "os.environ['WORLD_SIZE'] + ' ' + os.environ['LOCAL_RANK'])\n"
                      "sys.exit(3 if os.environ['RANK'] == '1' and len(sys.argv) > 1 else 0)\n")
    real = bench.__file__
    try:
        bench.__file__ = str(script)
        assert bench.spawn_ranks(2, []) == 0
        assert (tmp_path / "r0").read_text() == "2 0" and (tmp_path / "r1").read_text() == "2 1"
        assert bench.spawn_ranks(2, ["fail"]) == 3
    finally:
        bench.__file__ = real
