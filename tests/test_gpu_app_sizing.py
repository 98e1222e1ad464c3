"""LR app engine capacity: TWTML_BATCH_ROWS (rows, or 'hbm' sizing)."""
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cap", ["300000", "hbm"])
def test_app_batch_rows_override(hip_module, monkeypatch, cap):
    from twitter_stream_ml_amd.apps.linear_regression import build_engine
    from twitter_stream_ml_amd.config.arguments import ConfArguments
    monkeypatch.setenv("TWTML_BATCH_ROWS", cap)
    conf = ConfArguments().parse(["--master", "rocm[1]", "--numTextFeatures", "1000"])
    eng = build_engine(conf, rank=0, world=1)
    rows = eng.cfg.max_rows
    if cap == "hbm":
        assert rows >= 4_000_000   # 0.8 x ~288 GB holds millions of tweet rows
    else:
        assert rows == 300000
    del eng
    import gc
    gc.collect()   # the engine wrapper holds reference cycles: free its HBM now


def test_engine_frees_device_memory_on_del(hip_module):
    """No reference cycle in the engine wrappers: dropping the last reference
    releases the engine's HBM at once (no wait for the cyclic GC)."""
    import torch
    from twitter_stream_ml_amd.ops.kmeans_engine import DeviceKMeans, KMDeviceConfig
    from twitter_stream_ml_amd.ops.lr_engine import DeviceLinearRegression, LRDeviceConfig
    free0 = torch.cuda.mem_get_info(0)[0]
    lr = DeviceLinearRegression(LRDeviceConfig(num_text_features=100_000_000, hash="murmur3",
                                               max_rows=200_000, max_units=200_000 * 300), device=0)
    km = DeviceKMeans(KMDeviceConfig(k=64, text_dims=14, max_rows=200_000, max_units=200_000 * 300), device=0)
    free1 = torch.cuda.mem_get_info(0)[0]
    assert free0 - free1 > 1 << 30            # the F = 1e8 weights and maps alone are > 1 GB
    del lr, km
    free2 = torch.cuda.mem_get_info(0)[0]
    assert free0 - free2 < 256 << 20, (free0, free1, free2)


def test_hbm_sized_engine_trains_tiered_batch(hip_module, monkeypatch):
    """The HBM sizing counts what the first tiered batch allocates (the
    entry-sized far lists and CSC of both prepared buffers, ``lazy_bytes``):
    an hbm-sized engine trains a tiered batch without running out of memory
    and keeps headroom for the active-set buffers."""
    import gc

    import torch
    from twitter_stream_ml_amd.apps.linear_regression import build_engine
    from twitter_stream_ml_amd.config.arguments import ConfArguments
    from twitter_stream_ml_amd.sources.synthetic import SynthConfig, generate_batch
    monkeypatch.setenv("TWTML_BATCH_ROWS", "hbm")
    monkeypatch.setenv("TWTML_FORCE_TIERED", "1")
    conf = ConfArguments().parse(["--master", "rocm[1]", "--numTextFeatures", "1000000"])
    eng = build_engine(conf, rank=0, world=1)
    assert eng._eng.lazy_bytes > 0
    r = eng.train_batch(generate_batch(SynthConfig.profile("wide", seed=3), 0, 50_000,
                                       batch_time_ms=1_700_000_000_000))
    assert r["tiered"] and not r["diverged"] and r["iterations"] > 0
    torch.cuda.synchronize()
    free, total = torch.cuda.mem_get_info(0)
    assert free > 0.05 * total, (free, total)   # 0.8 of free memory was the target
    del eng
    gc.collect()
