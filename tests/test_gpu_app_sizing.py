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
