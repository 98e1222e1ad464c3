"""NUMA-local binding of a GPU rank (parallel/affinity.py) against a fake sysfs."""
import os

import numpy as np

from twitter_stream_ml_amd.parallel.affinity import bind_local_numa, gpu_numa_node, parse_cpulist


def _sysfs(tmp_path, bdf="0000:05:00.0", node="1", cpulist="4-7,12"):
    dev = tmp_path / "bus" / "pci" / "devices" / bdf
    dev.mkdir(parents=True)
    (dev / "numa_node").write_text(node + "\n")
    nd = tmp_path / "devices" / "system" / "node" / f"node{node}"
    nd.mkdir(parents=True)
    (nd / "cpulist").write_text(cpulist + "\n")
    return str(tmp_path)


def test_parse_cpulist():
    assert parse_cpulist("0-3,8,10-11\n") == {0, 1, 2, 3, 8, 10, 11}
    assert parse_cpulist("") == set()


def test_gpu_numa_node(tmp_path):
    root = _sysfs(tmp_path)
    assert gpu_numa_node("0000:05:00.0", root) == 1
    assert gpu_numa_node("0000:06:00.0", root) is None


def test_bind_intersects_with_current_affinity(tmp_path, monkeypatch):
    monkeypatch.delenv("TWTML_NUMA_BIND", raising=False)
    root = _sysfs(tmp_path)
    calls = []
    got = bind_local_numa(3, pci_bus_id=lambda d: "0000:05:00.0", sysfs=root,
                          setaffinity=lambda pid, cpus: calls.append(set(cpus)),
                          getaffinity=lambda pid: set(range(0, 10)))
    assert got == {4, 5, 6, 7} and calls == [{4, 5, 6, 7}]


def test_bind_is_best_effort(tmp_path, monkeypatch):
    monkeypatch.delenv("TWTML_NUMA_BIND", raising=False)
    root = _sysfs(tmp_path, node="-1")
    never = lambda pid, cpus: (_ for _ in ()).throw(AssertionError("must not bind"))  # noqa: E731
    cur = lambda pid: {0, 1}  # noqa: E731
    assert bind_local_numa(0, lambda d: "0000:05:00.0", root, never, cur) is None    # no NUMA info
    root2 = _sysfs(tmp_path / "b", cpulist="4-7")
    assert bind_local_numa(0, lambda d: "0000:05:00.0", root2, never, cur) is None   # cpuset excludes node
    def boom(d):
        raise RuntimeError("no device")
    assert bind_local_numa(0, boom, root2, never, cur) is None
    monkeypatch.setenv("TWTML_NUMA_BIND", "0")
    root3 = _sysfs(tmp_path / "c", cpulist="0")
    assert bind_local_numa(0, lambda d: "0000:05:00.0", root3, never, lambda pid: {0, 1}) is None


def test_real_process_affinity_untouched_without_gpu():
    before = os.sched_getaffinity(0)
    bind_local_numa(0, pci_bus_id=lambda d: "ffff:ff:ff.f")   # nonexistent device path
    assert os.sched_getaffinity(0) == before


def test_share_host_threads_divides_the_node(monkeypatch, tmp_path):
    """8 ranks on 2 NUMA nodes (4 GPUs each): a rank gets its node's CPUs / 4."""
    from functools import partial
    from twitter_stream_ml_amd.parallel import affinity
    share_host_threads = partial(affinity.share_host_threads, cgroup=str(tmp_path))   # no quota
    monkeypatch.delenv("TWTML_HOST_THREADS", raising=False)
    nodes = {d: 0 if d < 4 else 1 for d in range(8)}
    monkeypatch.setattr("twitter_stream_ml_amd.parallel.affinity.gpu_numa_node",
                        lambda bdf, sysfs: nodes[int(bdf)])
    n = share_host_threads(5, 5, 8, 8, pci_bus_id=str, getaffinity=lambda pid: set(range(64)))
    assert n == 16 and os.environ["TWTML_HOST_THREADS"] == "16"
    # every rank on one GPU (the gloo rehearsal): the 8 ranks share the node
    monkeypatch.delenv("TWTML_HOST_THREADS")
    assert share_host_threads(0, 3, 8, 1, pci_bus_id=str, getaffinity=lambda pid: set(range(64))) == 8
    # an explicit setting wins
    assert share_host_threads(0, 3, 8, 1, pci_bus_id=str, getaffinity=lambda pid: set(range(64))) == 8
    monkeypatch.setenv("TWTML_HOST_THREADS", "3")
    assert share_host_threads(0, 0, 8, 8, pci_bus_id=str, getaffinity=lambda pid: set(range(64))) == 3


def test_native_generator_uses_host_threads(monkeypatch):
    """The synthetic generator honours TWTML_HOST_THREADS (sized from the
    affinity mask otherwise, never the machine's CPU count)."""
    from twitter_stream_ml_amd.sources.synthetic import SynthConfig, generate_batch
    monkeypatch.setenv("TWTML_HOST_THREADS", "1")
    a = generate_batch(SynthConfig.profile("bench", seed=3), 0, 20000, batch_time_ms=0)
    monkeypatch.setenv("TWTML_HOST_THREADS", "5")
    b = generate_batch(SynthConfig.profile("bench", seed=3), 0, 20000, batch_time_ms=0)
    np.testing.assert_array_equal(a.text, b.text)   # thread count never changes the data


def test_cgroup_quota_caps_host_threads(monkeypatch, tmp_path):
    """A 256-CPU affinity mask in a 16-CPU cgroup (the MI355X boxes): 16
    threads for one rank, 2 each for 8 ranks; v1 files too; no limit -> 0."""
    from twitter_stream_ml_amd.parallel.affinity import cgroup_cpu_limit, share_host_threads
    (tmp_path / "cpu.max").write_text("1600000 100000\n")
    assert cgroup_cpu_limit(str(tmp_path)) == 16
    wide = lambda pid: set(range(256))   # noqa: E731
    monkeypatch.delenv("TWTML_HOST_THREADS", raising=False)
    assert share_host_threads(0, 0, 1, 1, pci_bus_id=str, getaffinity=wide, cgroup=str(tmp_path)) == 16
    monkeypatch.delenv("TWTML_HOST_THREADS")
    assert share_host_threads(0, 3, 8, 1, pci_bus_id=str, getaffinity=wide, cgroup=str(tmp_path)) == 2
    (tmp_path / "cpu.max").write_text("max 100000\n")
    assert cgroup_cpu_limit(str(tmp_path)) == 0
    v1 = tmp_path / "v1"
    (v1 / "cpu").mkdir(parents=True)
    (v1 / "cpu" / "cpu.cfs_quota_us").write_text("250000\n")
    (v1 / "cpu" / "cpu.cfs_period_us").write_text("100000\n")
    assert cgroup_cpu_limit(str(v1)) == 3
    assert cgroup_cpu_limit(str(tmp_path / "none")) == 0
