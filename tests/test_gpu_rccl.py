"""The real RCCL communicator (``RcclComm``) on one MI355X.

The multi-GPU path (``parallel/dist.py:make_rccl_comm`` -> ``csrc/hip/comm.cpp``)
only runs with several GPUs, and RCCL refuses two ranks on one device, so the
DP orchestration itself is covered by ``test_gpu_dp_loopback.py``.  Here a
world-1 communicator goes through the same ``ncclGetUniqueId`` ->
``ncclCommInitRank`` -> ``ncclAllReduce`` calls on a real stream, and engines
built with it train exactly like engines without one.
"""
import numpy as np
import pytest

from twitter_stream_ml_amd.sources.synthetic import SynthConfig, generate_batch

pytestmark = pytest.mark.gpu
NOW = 1_700_000_000_000


def _comm(h):
    return h.Comm(h.rccl_unique_id(), 0, 1, 0)


def test_rccl_world1_allreduce_identity(hip_module):
    import torch
    h = hip_module
    assert len(h.rccl_unique_id()) == 128
    assert int(h.rccl_version()) > 0
    comm = _comm(h)
    assert (comm.rank, comm.world) == (0, 1)
    x = torch.arange(1, 4097, dtype=torch.float64, device="cuda:0") * 0.25
    ref = x.clone()
    torch.cuda.synchronize()
    comm.allreduce_f64(x.data_ptr(), x.numel())
    torch.testing.assert_close(x, ref, rtol=0, atol=0)
    comm.check()


def test_engines_with_rccl_comm_match_no_comm(hip_module):
    from twitter_stream_ml_amd.ops.kmeans_engine import DeviceKMeans, KMDeviceConfig
    from twitter_stream_ml_amd.ops.lr_engine import DeviceLinearRegression, LRDeviceConfig
    h = hip_module
    synth = SynthConfig.profile("twitter", seed=5, unicode_fraction=0.1)
    batches = [generate_batch(synth, t * 2000, 2000, batch_time_ms=NOW + t) for t in range(2)]

    cfg = LRDeviceConfig(num_text_features=1 << 20, max_rows=4096, max_units=4096 * 300,
                         num_iterations=10)
    a = DeviceLinearRegression(cfg, device=0, comm=_comm(h))
    b = DeviceLinearRegression(cfg, device=0)
    for bt in batches:
        ra, rb = a.train_batch(bt, want_pred=False), b.train_batch(bt, want_pred=False)
        assert ra["iterations"] == rb["iterations"]
    # the cold-tail gradient flush uses fp64 atomics, so two runs agree to
    # rounding, not bitwise (same tolerance as test_gpu_dp_loopback.py)
    wb = b.get_weights()
    np.testing.assert_allclose(a.get_weights(), wb, rtol=1e-4, atol=1e-6 * max(np.abs(wb).max(), 1e-12))

    kcfg = KMDeviceConfig(k=64, text_dims=14, half_life=5.0, max_rows=4096,
                          max_units=4096 * 300, seed=3)
    ka = DeviceKMeans(kcfg, device=0, comm=_comm(h))
    kb = DeviceKMeans(kcfg, device=0)
    for bt in batches:
        ka.update_raw(bt, want_pred=False)
        kb.update_raw(bt, want_pred=False)
    (ca, wa), (cb, wb) = ka.get_state(), kb.get_state()
    np.testing.assert_allclose(ca, cb, rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(wa, wb, rtol=1e-12)
