"""Failure detection, fault injection and exact resume.

Two gloo ranks run the LR driver on size-sealed batches with a checkpoint
every batch.  A fault kills rank 1 right before batch 4; the surviving rank
fails out of its collective, the job dies.  Restarting with ``--resume auto``
continues each rank's stream from its recorded position, and the final model
equals the uninterrupted run (up to the tweet-age feature, which -- as in the
reference -- is measured against the wall-clock batch time).
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from twitter_stream_ml_amd.checkpoint import load_linear_regression, load_progress


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, argv, fault, ck_async="1"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), TWTML_CHECKPOINT_ASYNC=ck_async)
    if fault:
        os.environ["TWTML_FAULT"] = fault
    else:
        os.environ.pop("TWTML_FAULT", None)
    from twitter_stream_ml_amd.apps import linear_regression as app
    rc = app.main(argv)
    from twitter_stream_ml_amd.parallel import dist as D
    D.shutdown()
    if rc:
        raise SystemExit(rc)


def _run(world, argv, fault=None, ck_async="1"):
    mp.start_processes(_rank_main, args=(world, _free_port(), argv, fault, ck_async), nprocs=world,
                       join=True, start_method="spawn")


def _argv(ck, batches=6):
    return ["--master", "local[1]", "--lightning", "http://127.0.0.1:9",
            "--twtweb", "http://127.0.0.1:9", "--seconds", "0", "--batchSize", "400",
            "--sourceRate", "0", "--numBatches", str(batches), "-f", "4096", "-i", "10",
            "--checkpoint", str(ck), "--checkpointInterval", "1", "--checkReplicas", "1"]


@pytest.mark.parametrize("ck_async", ["0", "1"], ids=["sync", "async"])
def test_kill_rank_then_resume_equals_uninterrupted(tmp_path, ck_async):
    """Synchronous checkpoints leave batch 3 (the last batch every rank
    finished) on disk.  Asynchronous ones skip a checkpoint that comes due
    while the previous write is in flight, so the model on disk is from some
    batch 1..3, or there is none yet -- resume must continue exactly from
    whichever it is."""
    world = 2
    ref = tmp_path / "ref"
    _run(world, _argv(ref), ck_async=ck_async)
    w_ref, _ = load_linear_regression(str(ref))
    assert load_progress(str(ref))["batches"] == 6

    ck = tmp_path / "ck"
    with pytest.raises(Exception):
        _run(world, _argv(ck), fault="rank=1,batch=4,kind=exit", ck_async=ck_async)
    prog = load_progress(str(ck))
    if ck_async == "0":
        assert prog["batches"] == 3                 # last batch every rank finished
    else:
        # the first write may still be in flight when the job dies: then no
        # checkpoint is durable yet and --resume auto starts from scratch
        assert prog is None or 1 <= prog["batches"] <= 3
    if prog is not None:
        w3, _ = load_linear_regression(str(ck))
        assert not np.array_equal(w3, w_ref)

    _run(world, _argv(ck) + ["--resume", "auto"], ck_async=ck_async)   # restart: continue
    w, _ = load_linear_regression(str(ck))
    assert load_progress(str(ck)) == load_progress(str(ref))
    np.testing.assert_array_equal(w[:-1], w_ref[:-1])        # text + 3 count features
    np.testing.assert_allclose(w[-1], w_ref[-1], rtol=1e-6)  # age x 1e-14 (wall clock)


def test_fault_hook_and_watchdog_unit():
    from twitter_stream_ml_amd.utils.faults import FaultInjected, Watchdog, maybe_inject
    maybe_inject(0, 3, "rank=1,batch=3,kind=raise")          # other rank: no-op
    maybe_inject(1, 2, "rank=1,batch=3,kind=raise")          # other batch: no-op
    with pytest.raises(FaultInjected):
        maybe_inject(1, 3, "rank=1,batch=3,kind=raise")
    fired = []
    wd = Watchdog(0.2, lambda: fired.append(1))
    with wd:
        import time
        time.sleep(0.6)
    wd.close()
    assert fired == [1] and wd.fired
    wd2 = Watchdog(5.0, lambda: fired.append(2))
    with wd2:
        pass
    wd2.close()
    assert fired == [1]


def test_replica_digest_detects_divergence():
    from twitter_stream_ml_amd.parallel.dist import replica_digest
    a = np.arange(10.0)
    b = a.copy()
    assert replica_digest(a) == replica_digest(b)
    b[3] = np.nextafter(b[3], 10)
    assert replica_digest(a) != replica_digest(b)


def test_kmeans_resume_auto_equals_uninterrupted(tmp_path):
    from twitter_stream_ml_amd.apps import kmeans as km_app
    from twitter_stream_ml_amd.checkpoint import load_kmeans
    base = ["--master", "local[1]", "--seconds", "0", "--batchSize", "300", "--sourceRate", "0",
            "--k", "4", "--textDims", "3", "--checkpointInterval", "1"]
    ref = tmp_path / "ref"
    assert km_app.main(base + ["--numBatches", "5", "--checkpoint", str(ref)]) == 0
    ck = tmp_path / "ck"
    assert km_app.main(base + ["--numBatches", "2", "--checkpoint", str(ck)]) == 0
    assert load_progress(str(ck))["batches"] == 2
    assert km_app.main(base + ["--numBatches", "5", "--checkpoint", str(ck), "--resume", "auto"]) == 0
    c_ref, w_ref = load_kmeans(str(ref))
    c, w = load_kmeans(str(ck))
    np.testing.assert_array_equal(c, c_ref)
    np.testing.assert_array_equal(w, w_ref)
    assert load_progress(str(ck)) == load_progress(str(ref))
