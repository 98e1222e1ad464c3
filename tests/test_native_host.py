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


def _wire_roundtrip(raw, nthreads=0):
    h = host()
    out = np.zeros(h.wire_bound(raw.total_units, raw.n), np.uint8)
    woff = np.zeros(raw.n + 1, np.int64)
    flags = np.zeros(raw.n, np.uint8)
    nb = h.wire_pack(raw.text, raw.offsets, raw.is_retweet, out, woff, flags, nthreads)
    assert woff[raw.n] == nb
    text, offsets, is_rt = h.wire_unpack(out[:nb], woff, flags)
    np.testing.assert_array_equal(text, raw.text)
    np.testing.assert_array_equal(offsets, raw.offsets)
    np.testing.assert_array_equal(is_rt, raw.is_retweet)
    lens = np.diff(raw.offsets)
    wide = (flags & 2) != 0
    cesu = (flags & 4) != 0
    assert not np.any(wide & cesu)
    narrow = ~(wide | cesu)
    nbytes = np.diff(woff)
    np.testing.assert_array_equal(nbytes[wide], 2 * lens[wide])
    np.testing.assert_array_equal(nbytes[narrow], lens[narrow])
    assert np.all(nbytes[cesu] < 2 * lens[cesu])           # cesu only when smaller than UTF-16
    for r in range(min(raw.n, 300)):
        u = raw.text[raw.offsets[r]:raw.offsets[r + 1]]
        assert bool(narrow[r]) == (not (u.size and u.max() >= 256))   # narrow <=> every unit < 256
        if not narrow[r]:   # cesu size: 1 / 2 / 3 bytes per unit
            c = int(np.where(u < 0x80, 1, np.where(u < 0x800, 2, 3)).sum())
            assert cesu[r] == (c < 2 * u.size)
            if cesu[r]:
                assert nbytes[r] == c
    return nb


@pytest.mark.parametrize("n,threads", [(0, 0), (1, 0), (777, 1), (70_000, 0), (70_000, 5)])
def test_wire_pack_roundtrip(n, threads):
    raw = generate_batch(SynthConfig(seed=9, unicode_fraction=0.4, special_fraction=0.05), 0, n)
    nb = _wire_roundtrip(raw, threads)
    assert nb <= 2 * raw.total_units


def test_wire_cesu_rows_exact_for_any_units():
    """cesu rows round-trip every UTF-16 unit sequence: lone / swapped
    surrogates, U+07FF/U+0800 boundaries, emoji pairs, NUL."""
    from twitter_stream_ml_amd.records.batch import RawBatch
    rows = [[0x41, 0xD800, 0x42, 0x43, 0x44, 0x45, 0x46], [0xDC00, 0xD800, 0x61, 0x62, 0x63, 0x64],
            [0x7F, 0x80, 0x7FF, 0x800, 0x61, 0x62, 0x63, 0x64, 0x65, 0x66],
            [0xD83D, 0xDE00, 0x61, 0x62, 0x63, 0x64, 0x65], [0x0, 0x100, 0x61, 0x62, 0x63],
            [0x4E2D, 0x6587], [0x61] * 3 + [0xFFFF]]
    units = [np.array(r, np.uint16) for r in rows]
    off = np.zeros(len(rows) + 1, np.int64)
    off[1:] = np.cumsum([u.size for u in units])
    raw = RawBatch(np.concatenate(units), off, np.ones(len(rows), bool),
                   np.zeros((5, len(rows)), np.int64), 0)
    _wire_roundtrip(raw, 1)


@settings(max_examples=50, deadline=None)
@given(st.lists(st.text(max_size=12), min_size=1, max_size=20))
def test_wire_pack_arbitrary_text(texts):
    units = [utf16_units(t) for t in texts]
    offsets = np.concatenate([[0], np.cumsum([len(u) for u in units])]).astype(np.int64)
    text = np.concatenate(units).astype(np.uint16) if offsets[-1] else np.zeros(0, np.uint16)
    raw = RawBatch(text, offsets, np.arange(len(texts)) % 2, np.zeros((5, len(texts)), np.int64), 0)
    _wire_roundtrip(raw)
