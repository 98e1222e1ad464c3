"""Host-side native runtime (C++): synthetic source, Unicode lowering, CPU featurizer."""
import numpy as np
import pytest
import scipy.sparse as sp
from hypothesis import given, settings, strategies as st

from twitter_stream_ml_amd.ops._native import host
from twitter_stream_ml_amd.oracle import featurize_batch
from twitter_stream_ml_amd.records import RawBatch, units_to_str, utf16_units
from twitter_stream_ml_amd.sources.synthetic import SynthConfig, generate_batch


def test_generator_is_deterministic_and_sliceable():
    cfg = SynthConfig(seed=3, unicode_fraction=0.3, special_fraction=0.05)
    a = generate_batch(cfg, 0, 500)
    b = generate_batch(cfg, 0, 500, nthreads=1)
    np.testing.assert_array_equal(a.text, b.text)
    np.testing.assert_array_equal(a.scalars, b.scalars)
    c = RawBatch.concat([generate_batch(cfg, 0, 200), generate_batch(cfg, 200, 300)])
    np.testing.assert_array_equal(a.text, c.text)
    np.testing.assert_array_equal(a.offsets, c.offsets)
    d = generate_batch(SynthConfig(seed=4), 0, 500)
    assert not np.array_equal(a.scalars, d.scalars)


def test_generator_schema_ranges():
    b = generate_batch(SynthConfig.profile("bench", seed=1), 0, 2000)
    lens = np.diff(b.offsets)
    assert lens.min() >= 1 and lens.max() <= 280
    assert np.all(b.is_retweet == 1)
    rc = b.scalars[0]
    assert rc.min() >= 0 and rc.max() <= 1200
    frac_kept = ((rc >= 100) & (rc <= 1000)).mean()
    assert frac_kept > 0.8
    t = generate_batch(SynthConfig.profile("twitter", seed=1), 0, 4000)
    assert 0.5 < t.is_retweet.mean() < 0.7
    # surrogate pairs are never split at the truncation point
    for i in range(200):
        s = t.text[t.offsets[i]:t.offsets[i + 1]]
        assert not (0xD800 <= int(s[-1]) <= 0xDBFF)


@settings(max_examples=300, deadline=None)
@given(st.text(alphabet=st.characters(blacklist_categories=("Cs",)), max_size=30))
def test_full_lowering_matches_python(s):
    got = units_to_str(host().lower_row(utf16_units(s)))
    assert got == s.lower()


@pytest.mark.parametrize("s", ["İstanbul", "ΟΔΟΣ ΣΟΦΙΑ", "Σ", "aΣ", "aΣb", "ΛΟΓΟΣ.", "A'Σ",
                               "𐐀𐐁𐐂 Σ", "𞤀𞤁", "ΜΑΣ ΤΟΥΣ", "x\ud83d", "\ude00y"])
def test_special_rows(s):
    u = utf16_units(s)
    expect = units_to_str(u).lower() if "\ud83d" not in s and "\ude00" not in s else None
    got = units_to_str(host().lower_row(u))
    if expect is not None:
        assert got == expect


@pytest.mark.parametrize("F,hash", [(1000, "java"), (1 << 20, "java"), (1 << 20, "murmur3"),
                                    (7, "murmur3")])
def test_cpu_featurizer_matches_oracle(F, hash):
    cfg = SynthConfig(seed=8, special_fraction=0.05, unicode_fraction=0.3)
    raw = generate_batch(cfg, 0, 1500)
    fb = featurize_batch(raw, F, 100, 1000, hash=hash)
    indptr, idx = host().featurize_rows(raw.text, raw.offsets, fb.rows, F, hash, 0)
    X = sp.csr_matrix((np.ones(idx.shape[0]), idx, indptr), shape=(fb.n, F))
    X.sum_duplicates()
    assert abs(fb.X[:, :F] - X).max() == 0


def test_prelower_rewrites_only_special_rows():
    raw = RawBatch.from_statuses([])
    texts = ["İi abc", "plain", "ΟΔΟΣ"]
    from twitter_stream_ml_amd.records import Status
    raw = RawBatch.from_statuses([Status(text=t) for t in texts])
    h = host()
    assert h.count_special_rows(raw.text, raw.offsets) == 2
    text, offsets, changed = h.prelower_special_rows(raw.text, raw.offsets)
    assert changed == 2
    out = [units_to_str(text[offsets[i]:offsets[i + 1]]) for i in range(3)]
    assert out == ["i̇i abc", "plain", "οδος"]
