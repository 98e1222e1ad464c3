"""Multi-process data parallelism on CPU (gloo, world_size 2, 3 and 8 -- the driver's node size).

Mirrors what one process per GPU does on an MI355X node (SURVEY §2.4 DP row):
every rank owns a shard of each micro-batch, the per-iteration gradient (and
counts/statistics) are all-reduced, and the replicated model must equal the
single-process model trained on the concatenated batch.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir, fraction):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from twitter_stream_ml_amd.models.kmeans import CpuKMeans, kmeans_features
    from twitter_stream_ml_amd.models.linear_regression import CpuLinearRegression, CpuLRConfig
    from twitter_stream_ml_amd.parallel import dist as D
    from twitter_stream_ml_amd.sources.synthetic import SynthConfig, generate_batch
    info = D.init_distributed(backend="gloo")
    red = D.allreduce_fn()
    cfg = CpuLRConfig(num_text_features=1 << 12, num_iterations=15, fraction=fraction)
    lr = CpuLinearRegression(cfg, allreduce=red, rank=info.rank, world=info.world)
    km = CpuKMeans(5, 2, allreduce=red, seed=3)
    synth = SynthConfig.profile("twitter", seed=17)
    res = []
    for t in range(3):
        full = generate_batch(synth, t * 1500, 1500, batch_time_ms=1_700_000_000_000)
        shard = full.shard(info.rank, info.world)
        r = lr.train_batch(shard)
        X, _ = kmeans_features(shard)
        km.update_batch(X)
        res.append((r["iterations"], r["n_kept_global"], r["stats"]))
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), w=lr.get_weights(), c=km.state.centers,
             cw=km.state.weights, meta=np.array([x[0] for x in res] + [x[1] for x in res]),
             stats=np.array([x[2] for x in res]))
    D.barrier()
    D.shutdown()


@pytest.mark.parametrize("world,fraction", [(2, 1.0), (3, 0.7), (8, 1.0)])
def test_cpu_dp_equals_single_process(tmp_path, world, fraction):
    port = _free_port()
    mp.start_processes(_worker, args=(world, port, str(tmp_path), fraction), nprocs=world,
                       join=True, start_method="spawn")
    from twitter_stream_ml_amd.models.kmeans import CpuKMeans, kmeans_features
    from twitter_stream_ml_amd.models.linear_regression import CpuLinearRegression, CpuLRConfig
    from twitter_stream_ml_amd.sources.synthetic import SynthConfig, generate_batch
    lr = CpuLinearRegression(CpuLRConfig(num_text_features=1 << 12, num_iterations=15,
                                         fraction=fraction))
    km = CpuKMeans(5, 2, seed=3)
    synth = SynthConfig.profile("twitter", seed=17)
    iters, kept, stats = [], [], []
    for t in range(3):
        full = generate_batch(synth, t * 1500, 1500, batch_time_ms=1_700_000_000_000)
        r = lr.train_batch(full)
        km.update_batch(kmeans_features(full)[0])
        iters.append(r["iterations"]); kept.append(r["n_kept_global"]); stats.append(r["stats"])
    for rank in range(world):
        d = np.load(tmp_path / f"r{rank}.npz")
        np.testing.assert_array_equal(d["meta"], np.array(iters + kept))
        np.testing.assert_allclose(d["stats"], np.array(stats), rtol=1e-12)
        np.testing.assert_allclose(d["w"], lr.get_weights(), rtol=1e-9, atol=1e-15)
        np.testing.assert_allclose(d["c"], km.state.centers, rtol=1e-9, atol=1e-12)
        np.testing.assert_allclose(d["cw"], km.state.weights, rtol=1e-12)


def _sum_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from twitter_stream_ml_amd.parallel import dist as D
    D.init_distributed(backend="gloo")
    red = D.allreduce_fn()
    rng = np.random.default_rng(100 + rank)
    # magnitudes spread over 30 decades: the fp64 sum depends on the order
    v = rng.standard_normal(4096) * 10.0 ** rng.integers(-15, 15, 4096)
    np.save(os.path.join(out_dir, f"in{rank}.npy"), v)
    np.save(os.path.join(out_dir, f"out{rank}.npy"), red(v))
    D.barrier()
    D.shutdown()


@pytest.mark.parametrize("world", [3, 4])
def test_allreduce_fn_bit_identical_in_rank_order(tmp_path, world):
    """> 2 ranks: every rank gets the same bits -- the parts added in rank
    order -- so replicas (and their convergence verdicts) cannot diverge."""
    mp.start_processes(_sum_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    ins = [np.load(tmp_path / f"in{r}.npy") for r in range(world)]
    outs = [np.load(tmp_path / f"out{r}.npy") for r in range(world)]
    ref = ins[0].copy()
    for x in ins[1:]:
        ref += x
    for o in outs:
        np.testing.assert_array_equal(o, ref)


def _plot_worker(rank, world, port, lgn_url, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      TWTML_METRICS=os.path.join(out_dir, f"m{rank}.jsonl"))
    from twitter_stream_ml_amd.apps import linear_regression as app
    rc = app.main(["--master", "local[1]", "--lightning", lgn_url, "--twtweb", "http://127.0.0.1:9",
                   "--seconds", "0", "--batchSize", "1200", "--sourceRate", "0", "--numBatches", "3",
                   "-f", "1000", "--plotPoints", "50"])
    assert rc == 0


def test_dp_driver_plot_samples_reach_rank0(tmp_path):
    """2 gloo ranks run the LR driver with a (fake) Lightning plot: each rank
    samples plotPoints / world (pred, real) pairs, the plot shipper threads
    gather them to rank 0 over their own gloo group, and rank 0's session
    appends one 4-series update per batch with every rank's points."""
    import json
    from fakes import FakeLightning
    lgn = FakeLightning().start()
    try:
        mp.start_processes(_plot_worker, args=(2, _free_port(), lgn.url, str(tmp_path)), nprocs=2,
                           join=True, start_method="spawn")
        appends = lgn.appends()
    finally:
        lgn.stop()
    assert len(appends) == 3
    for a in appends:
        series = a["data"]["series"]
        assert len(series) == 4 and len(series[0]) == len(series[1]) == 50   # 25 per rank
        assert all(100 <= v <= 1000 for v in series[0])                      # real: kept retweet counts
    recs = [json.loads(l) for l in open(tmp_path / "m0.jsonl") if '"summary"' not in l]
    assert len(recs) == 3 and all("step_ms" in r for r in recs)


class _RecSession:
    """append_plot recorder standing in for rank 0's SessionStats."""

    def __init__(self):
        self.plots = []

    def append_plot(self, batch, real_sd, pred_sd, real, pred):
        self.plots.append((int(batch), np.array(real), np.array(pred)))


def _stall_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import json
    import time
    from twitter_stream_ml_amd.parallel import dist as D
    from twitter_stream_ml_amd.report import plot_shipper as P
    D.init_distributed(backend="gloo")
    real_gather = D.gather_parts
    calls = [0]

    def slow_gather(arr, group=None):   # the last rank's gathers stall for the first batches
        calls[0] += 1
        if rank == world - 1 and calls[0] <= 6:
            time.sleep(0.25)
        return real_gather(arr, group)

    D.gather_parts = slow_gather
    sess = _RecSession() if rank == 0 else None
    sh = P.PlotShipper(sess, rank, world, maxsize=4)
    n = 60
    worst = 0.0
    for b in range(n):   # the "training thread": one submit per batch, never held up
        real = np.full(3, 1000.0 * rank + b)   # encodes (rank, batch)
        t = time.perf_counter()
        sh.submit((b, b + 1, 0, 0, 0), real, -real)
        worst = max(worst, time.perf_counter() - t)
        time.sleep(0.002)
    sh.close(timeout=60)
    out = {"worst_submit_s": worst, "dropped": sh.dropped, "shipped": sh.shipped, "stopped": sh.stopped}
    if rank == 0:
        out.update(skipped=sh.skipped, plots=[(b, r.tolist()) for b, r, _ in sess.plots])
    with open(os.path.join(out_dir, f"s{rank}.json"), "w") as fh:
        json.dump(out, fh)
    D.barrier()
    D.shutdown()


def test_plot_shipper_backpressure_never_blocks_training(tmp_path):
    """A stalled gather on one rank: submit() returns at
    once on every rank, samples beyond the backlog are dropped, every rank
    still gathers every batch in order (paired), and rank 0 plots only
    batches for which it holds every rank's sample of that same batch."""
    import json
    world = 2
    mp.start_processes(_stall_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    outs = [json.load(open(tmp_path / f"s{r}.json")) for r in range(world)]
    for o in outs:
        assert o["worst_submit_s"] < 0.05, o
        assert not o["stopped"] and o["shipped"] == 60
    assert outs[world - 1]["dropped"] > 0 or outs[0]["dropped"] > 0   # the stall did fill a backlog
    plots, skipped = outs[0]["plots"], outs[0]["skipped"]
    assert len(plots) + skipped == 60 and skipped > 0
    for batch, real in plots:
        b = batch - 1
        assert real == [float(b)] * 3 + [1000.0 + b] * 3   # rank 0's then rank 1's sample of batch b
