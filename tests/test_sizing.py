"""HBM micro-batch sizing (ops/sizing.py) against a fake allocator."""
import pytest

from twitter_stream_ml_amd.ops import sizing


class _Alloc:
    def __init__(self):
        self.total = 0


def _fake(monkeypatch, fixed, per_row):
    a = _Alloc()
    monkeypatch.setattr(sizing, "_allocated", lambda: a.total)

    def make(rows):
        a.total += fixed + per_row * rows
        return object()
    return make


def test_footprint_model_recovers_affine_cost(monkeypatch):
    make = _fake(monkeypatch, fixed=1_300_000_000, per_row=31_000)
    fixed, per_row = sizing.footprint_model(make, probe=(65536, 262144))
    assert fixed == pytest.approx(1.3e9)
    assert per_row == pytest.approx(31_000)


def test_hbm_max_rows_fits_budget(monkeypatch):
    make = _fake(monkeypatch, fixed=2_000_000_000, per_row=30_000)
    free = 288 * 2**30
    rows = sizing.hbm_max_rows(make, free, fraction=0.8)
    assert rows % 65536 == 0
    assert 2e9 + 30_000 * rows <= 0.8 * free < 2e9 + 30_000 * (rows + 65536)


def test_hbm_max_rows_rejects_flat_footprint(monkeypatch):
    make = _fake(monkeypatch, fixed=10, per_row=0)
    with pytest.raises(RuntimeError):
        sizing.hbm_max_rows(make, 1 << 30)
