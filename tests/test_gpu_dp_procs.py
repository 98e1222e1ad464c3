"""Cross-process data parallelism on one MI355X (SURVEY §2.4 DP, §2.5 CS2).

N ranks (2, 3 and 4) are N processes sharing GPU 0; each owns an engine whose collectives
go through the host-staged torch.distributed gloo communicator
(``parallel/dist.make_comm(..., "gloo")`` -> ``csrc/hip/comm.cpp`` HostComm).
This is the engine DP path a one-GPU-per-rank RCCL job runs -- per-rank shards,
per-rank kept counts / sampling offsets, the active-id all-gather union, the
tiered slot-count all-reduce (on a second, prep communicator while the
previous batch's per-iteration gradient all-reduces run), stats and
early-exit agreement -- across real process boundaries; only the transport
differs (RCCL refuses two ranks on one device).  DP over shards must equal a
single engine on the concatenated batch, and the replicas must be
bit-identical.  The last test drives the real launcher:
``torch.distributed.run ... bench.py --gpus 2 --comm gloo``.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
NOW = 1_700_000_000_000
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# (profile, F, hash, rows per batch, batches, expect tiered)
LR_CASES = [("twitter", 1 << 20, "java", 6000, 3, False),
            ("wide", 1 << 20, "java", 20000, 2, True),
            ("wide", 100_000_000, "murmur3", 20000, 2, True)]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _lr_cfg(F, hash, rows):
    from twitter_stream_ml_amd.ops.lr_engine import LRDeviceConfig
    return LRDeviceConfig(num_text_features=F, hash=hash, max_rows=rows, max_units=rows * 300,
                          num_iterations=20)


def _km_cfg():
    from twitter_stream_ml_amd.ops.kmeans_engine import KMDeviceConfig
    return KMDeviceConfig(k=6, text_dims=4, seed=2, max_rows=8192, max_units=8192 * 300)


def _batches(profile, rows, n, seed):
    from twitter_stream_ml_amd.sources.synthetic import SynthConfig, generate_batch
    synth = SynthConfig.profile(profile, seed=seed)
    return [generate_batch(synth, t * rows, rows, batch_time_ms=NOW + t * 5000) for t in range(n)]


def _worker(rank, world, port, out_dir):
    # every rank adds the parts of a floating-point all-reduce in a different
    # order (csrc/hip/comm.cpp): the engines' collectives are int64 sums, so
    # DP must still equal one engine bit for bit
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), TWTML_HOSTCOMM_ORDER="rotate")
    import torch  # noqa: F401  (binds the HIP runtime before the engine loads)
    from twitter_stream_ml_amd.ops.kmeans_engine import DeviceKMeans
    from twitter_stream_ml_amd.ops.lr_engine import DeviceLinearRegression
    from twitter_stream_ml_amd.parallel import dist as D
    D.init_distributed(backend="gloo")
    comm = D.make_comm(0, "gloo")
    out = {}
    for ci, (profile, F, hash, rows, nb, _) in enumerate(LR_CASES):
        eng = DeviceLinearRegression(_lr_cfg(F, hash, rows), device=0, comm=comm)
        meta = []
        shards = [full.shard(rank, world) for full in _batches(profile, rows, nb, seed=40 + ci)]
        for sh in shards[:eng.raw_slots - 1]:   # queued ahead: exercises the prepare-ahead path
            eng.prefetch(sh)
        for sh in shards:
            r = eng.train_batch(sh, want_pred=False)
            assert r["stats_spill"] == 0   # every moment went through the exact int64 path
            meta.append([r["iterations"], r["n_kept_global"], r["n_unique"], int(r["tiered"])]
                        + list(r["stats"]))
        out[f"lr{ci}_w"] = eng.get_weights()
        out[f"lr{ci}_meta"] = np.array(meta, np.float64)
        del eng
    km = DeviceKMeans(_km_cfg(), device=0, comm=comm)
    for t, full in enumerate(_batches("twitter", 4000, 3, seed=8)):
        r = km.update_raw(full.shard(rank, world))
        c, w = km.get_state()
        out[f"km{t}_c"], out[f"km{t}_w"] = c, w
        out[f"km{t}_n"] = np.array([r["n"], r["n_local"]])
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), **out)
    D.barrier()
    D.shutdown()


@pytest.fixture(scope="module", params=[2, 3, 4], ids=["world2", "world3", "world4"])
def dp_runs(request, tmp_path_factory, hip_module):
    """2 ranks, and 3 (odd world: uneven shards, all-gather parts of unequal
    fill, fixed-order reductions over an odd number of partials)."""
    import torch.multiprocessing as mp
    world = request.param
    out = tmp_path_factory.mktemp(f"dp_procs{world}")
    mp.start_processes(_worker, args=(world, _free_port(), str(out)), nprocs=world, join=True,
                       start_method="spawn")
    return world, [dict(np.load(out / f"r{r}.npz")) for r in range(world)]


@pytest.mark.parametrize("ci", range(len(LR_CASES)))
def test_lr_dp_processes_equal_single_engine(dp_runs, ci):
    from twitter_stream_ml_amd.ops.lr_engine import DeviceLinearRegression
    world, ranks = dp_runs
    profile, F, hash, rows, nb, tiered = LR_CASES[ci]
    single = DeviceLinearRegression(_lr_cfg(F, hash, rows), device=0)
    for t, full in enumerate(_batches(profile, rows, nb, seed=40 + ci)):
        r1 = single.train_batch(full, want_pred=False)
        assert bool(r1["tiered"]) == tiered
        for d in ranks:
            it, kept, nu, tr = d[f"lr{ci}_meta"][t][:4]
            stats = d[f"lr{ci}_meta"][t][4:]
            assert (int(it), int(kept), int(nu), bool(tr)) == (r1["iterations"], r1["n_kept"],
                                                                r1["n_unique"], tiered)
            # exact GD arithmetic (int32 / int64 fixed point, csrc/hip/sgd.hip) and
            # int64 batch moments (k_batch_stats): the prequential stats and the
            # weights of DP over any sharding and any summation order are the
            # single engine's, bit for bit
            np.testing.assert_array_equal(stats, np.asarray(r1["stats"]))
    w1 = single.get_weights()
    for d in ranks:
        np.testing.assert_array_equal(d[f"lr{ci}_w"], w1)


def test_kmeans_dp_processes(dp_runs):
    """Exact integer scaler moments and cluster sums: DP k-means over 2-4
    processes equals the single engine on every cluster, bit for bit."""
    from twitter_stream_ml_amd.ops.kmeans_engine import DeviceKMeans
    world, ranks = dp_runs
    single = DeviceKMeans(_km_cfg(), device=0)
    for t, full in enumerate(_batches("twitter", 4000, 3, seed=8)):
        r1 = single.update_raw(full)
        assert sum(int(d[f"km{t}_n"][1]) for d in ranks) == r1["n"]
        c1, w1 = single.get_state()
        for d in ranks:
            assert int(d[f"km{t}_n"][0]) == r1["n"]
            np.testing.assert_array_equal(d[f"km{t}_c"], c1)
            np.testing.assert_array_equal(d[f"km{t}_w"], w1)


def _torchrun_bench(nproc, extra, env_extra=None, timeout=300):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="4", **(env_extra or {}))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "bench.py"),
           "--gpus", str(nproc), "--comm", "gloo"] + extra
    return subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)


@pytest.mark.parametrize("nproc", [2, 4])
def test_torchrun_bench_gloo(hip_module, nproc):
    """The driver's launcher on one GPU: N ranks, engine DP through gloo.
    The JSON carries what a first real multi-GPU run needs to be diagnosed
    (VERDICT r4 #2): per-iteration all-reduce time and bytes, the RCCL
    version and NCCL_/RCCL_ environment, and the end-of-run replica check."""
    p = _torchrun_bench(nproc, ["--batch", "100000", "--steps", "3", "--warmup", "1", "--pool", "2"])
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == nproc and d["config"]["parallelism"] == f"dp{nproc}-gloo"
    assert d["config"]["global_batch"] == 100000 * nproc and d["value"] > 0
    assert d["replicas_identical"] is True
    assert d["grad_allreduce_per_step"] > 1 and d["grad_allreduce_us_per_iter"] > 0
    # one packed int64 buffer per GD iteration (near columns + tail + far
    # slots), averaged over the window's batches
    assert d["allreduce_bytes_per_iter"] > 8 * 64
    # the DP cost model's check: all-reduce time per step ~ per-iteration time x all-reduces per step
    assert d["comm_ms_per_step"] > 0
    assert abs(d["comm_ms_per_step"] * 1e3 - d["grad_allreduce_us_per_iter"] * d["grad_allreduce_per_step"]) \
        <= 0.5 * d["comm_ms_per_step"] * 1e3 + 1.0
    assert isinstance(d["rccl_version"], str) and d["rccl_version"]
    assert isinstance(d["comm_env"], dict) and d["comm_env"].get("HSA_ENABLE_IPC_MODE_LEGACY") == "0"
    print(f"dp{nproc}: {d['grad_allreduce_us_per_iter']} us / {d['allreduce_bytes_per_iter']} B per all-reduce")


def test_torchrun_bench_hang_exits_nonzero(hip_module):
    """A rank that hangs (TWTML_BENCH_HANG=1:2: rank 1 never processes its
    second step) leaves rank 0 blocked in a collective; the bench watchdog
    dumps the stacks, aborts the communicator and exits non-zero on every
    rank well inside the driver's timeout."""
    import time
    t = time.monotonic()
    p = _torchrun_bench(2, ["--batch", "50000", "--steps", "3", "--warmup", "1", "--pool", "2",
                            "--timeout", "40"], env_extra={"TWTML_BENCH_HANG": "1:2"}, timeout=240)
    took = time.monotonic() - t
    assert p.returncode != 0, p.stdout[-2000:]
    assert "watchdog: run not finished" in p.stderr, p.stderr[-4000:]
    assert "Python stacks" in p.stderr and "counters" in p.stderr
    print(f"hung run exited {p.returncode} after {took:.1f} s")
    assert took < 200


def test_torchrun_bench_global_prep_failure_ends_the_group(hip_module):
    """a failure in the DP global prep (after the packet
    all-gather) raises on that rank only; its peers wait in the batch's
    first gradient all-reduce.  The group still ends promptly and non-zero:
    the failing rank exits, the launcher tears the others down, and the
    bench watchdog bounds whatever is left."""
    import time
    t = time.monotonic()
    p = _torchrun_bench(2, ["--batch", "50000", "--steps", "3", "--warmup", "1", "--pool", "2",
                            "--timeout", "60"], env_extra={"TWTML_INJECT_GLOBAL_PREP_FAIL": "1:2"}, timeout=240)
    took = time.monotonic() - t
    assert p.returncode != 0, p.stdout[-2000:]
    assert "injected global prep failure" in p.stderr, p.stderr[-4000:]
    print(f"global prep failure: group exited {p.returncode} after {took:.1f} s")
    assert took < 200
