"""GPU numerics of the streaming-LR engine against the fp64 oracle.

K1-K3 (filter, lower-case, bigram hash, numeric features) are compared entry
for entry with ``oracle.featurize_batch``; K4-K7 (prequential predictions and
stats, GD iterations, convergence) against ``oracle.run_minibatch_sgd`` over
several warm-started batches.
"""
import numpy as np
import pytest

from twitter_stream_ml_amd.oracle import (featurize_batch, round_half_up_array,
                                          run_minibatch_sgd)
from twitter_stream_ml_amd.sources.synthetic import SynthConfig, generate_batch

pytestmark = pytest.mark.gpu

NOW = 1_700_000_000_000


def _engine(F, hash="java", **kw):
    from twitter_stream_ml_amd.ops.lr_engine import DeviceLinearRegression, LRDeviceConfig
    kw = {"max_rows": 8192, "max_units": 8192 * 300, **kw}
    cfg = LRDeviceConfig(num_text_features=F, hash=hash, **kw)
    return DeviceLinearRegression(cfg, device=0)


def _rows_from_debug(dbg):
    """Per kept row (kept order) -> sorted multiset of hashed feature ids.

    SELL-16x4 layout: chunk c = 16 rows, row r owns lanes 4r..4r+3.
    """
    nk = int(dbg["counters"][0])
    idx, clen8, cbase, perm = dbg["idx"], dbg["clen8"], dbg["cbase"], dbg["perm"]
    rows = [None] * nk
    for c in range(clen8.shape[0]):
        g0, L8 = int(cbase[c]), int(clen8[c])
        block = idx[g0 * 512:(g0 + L8) * 512].reshape(L8, 64, 8)
        for r in range(16):
            k = int(perm[c * 16 + r])
            if k < 0:
                continue
            v = block[:, 4 * r:4 * r + 4, :].reshape(-1)
            rows[k] = np.sort(v[v >= 0])
    return rows


def _with_long_row(raw, k=3, n_units=9000):
    """Row k becomes 9000 Cyrillic units (18000 wire bytes >= 16 KiB)."""
    from twitter_stream_ml_amd.records.batch import RawBatch, utf16_units
    texts = ["\u0436" * n_units if i == k else raw.text_of(i) for i in range(raw.n)]
    units = [utf16_units(t) for t in texts]
    off = np.zeros(raw.n + 1, np.int64)
    off[1:] = np.cumsum([u.shape[0] for u in units])
    return RawBatch(np.concatenate(units), off, raw.is_retweet, raw.scalars, raw.batch_time_ms)


@pytest.mark.parametrize("F,hash,wide,longrow,ingest", [
    (1000, "java", False, False, "wire"), (1 << 20, "java", False, False, "wire"),
    (1 << 20, "murmur3", False, False, "wire"), (1000, "java", True, False, "wire"),
    (1 << 20, "java", False, True, "wire"),
    (1 << 20, "java", False, False, "utf16"), (1 << 20, "murmur3", True, True, "utf16"),
    (1 << 20, "java", False, False, "utf8"), (1 << 20, "murmur3", True, True, "utf8")])
def test_featurize_matches_oracle(hip_module, F, hash, wide, longrow, ingest):
    """Featurize == oracle; also covers the wire encodings: wide (int64)
    scalar columns and the plain-offsets fallback of a >= 16 KiB row, and
    raw UTF-16 ingest (Latin-1 rows narrowed on the device) and raw UTF-8
    ingest (non-ASCII rows decoded, 4-byte sequences included).  Special rows
    (5 %) are fully lower-cased on the device (rows.hip), not on the host."""
    cfg = SynthConfig.profile("twitter", seed=11, special_fraction=0.05, unicode_fraction=0.3)
    raw = generate_batch(cfg, 0, 3000, batch_time_ms=NOW)
    if wide:   # followers / createdAt ranges beyond 32 bits: those columns ship as int64
        raw.scalars[1, 5] = (1 << 40) + 7
        raw.scalars[4, 9] = 0
    if longrow:
        raw = _with_long_row(raw)
        raw.scalars[0, 3] = 500   # keep it: it passes the [100, 1000] filter
        raw.is_retweet[3] = True
    eng = _engine(F, hash, lazy_idx=False, ingest=ingest)   # every hashed id kept for inspection
    res = eng.train_batch(raw, want_pred=True)
    assert res["rows_lowered"] > 0
    if ingest == "utf16":
        assert res["rows_narrowed"] > 0.5 * raw.n
    hb = eng._staging[0]
    sw = hb._hb.scalar_wire
    assert sw["rows"] == raw.n
    assert sw["wide_mask"] == (0b10010 if wide else 0), sw
    # bits per value: the column's range (bit-packed), or 64 (raw int64)
    sc = raw.scalars.astype(np.int64)
    for c, w in enumerate(sw["widths"]):
        span = int(sc[c].max()) - int(sc[c].min())
        assert w == (64 if span >= 1 << 32 else max(1, span.bit_length())), (c, w, span)
    assert hb.rows_packed == (not longrow)
    dbg = eng._eng.debug_prepared()
    fb = featurize_batch(raw, F, 100, 1000, now_ms=NOW, hash=hash)
    assert int(dbg["counters"][0]) == fb.n
    rows = _rows_from_debug(dbg)
    Xt = fb.X[:, :F].tocsr()
    for k in range(fb.n):
        s, e = Xt.indptr[k], Xt.indptr[k + 1]
        want = np.repeat(Xt.indices[s:e], Xt.data[s:e].astype(np.int64))
        np.testing.assert_array_equal(rows[k], np.sort(want), err_msg=f"row {k}")
    # active set = union of touched ids
    touched = np.unique(Xt.indices)
    np.testing.assert_array_equal(np.sort(dbg["uniq"]), touched)
    # labels / numeric features (fp32 of the fp64 oracle values)
    nk = fb.n
    y = np.zeros(nk, np.float32)
    num = np.zeros((nk, 4), np.float32)
    perm = dbg["perm"]
    R = perm.shape[0]
    for pos in range(R):
        k = int(perm[pos])
        if k >= 0:
            y[k] = dbg["y"][pos]
            num[k] = dbg["num"][np.arange(4) * R + pos]
    np.testing.assert_array_equal(y, fb.y.astype(np.float32))
    want_num = fb.X[:, F:F + 4].toarray()
    np.testing.assert_allclose(num, want_num, rtol=2e-7, atol=0)


_SPECIAL_TEXTS = [
    "\u0130stanbul", "ŞEHİR", "KIZ İ", "İ", "ΟΔΟΣ", "ΣΟΦΙΑ", "ΛΟΓΟΣ.", "ΣΑΣ", "Σ", "ΑΣ'", "ΑΣ'Β", "ΑΣ\u0308",
    "α Σ β", "ΑΣ \U00010400", "\U00010400ΣΑ", "\U00010400\U00010401\U00010402 mixed", "\U0001E900\U0001E901",
    "ΜΑΣ ΤΟΥΣ", "plain ascii then İ", "x\ud801", "\udc00Σ\ud801\udc00", "ab\ud801\ud801\udc00Σ",
    "caf\u00e9 İ ok", "\U0001F600 emoji Σ",
]


@pytest.mark.parametrize("ingest", ["wire", "utf16", "utf8"])
def test_device_special_lowering(hip_module, ingest):
    """Rows whose lower-casing is not one unit per unit (U+0130 -> 2 units,
    Final_Sigma context incl. case-ignorables and astral neighbours, astral
    cased letters, lone surrogates), as narrow / cesu / wide wire rows or raw
    UTF-16: device featurize == oracle (Java toLowerCase semantics)."""
    from twitter_stream_ml_amd.records.batch import RawBatch, utf16_units
    base = generate_batch(SynthConfig.profile("twitter", seed=3), 0, 400, batch_time_ms=NOW)
    texts = [base.text_of(i) for i in range(base.n)]
    for j, s in enumerate(_SPECIAL_TEXTS):
        texts[7 * j] = s
    units = [utf16_units(s) for s in texts]
    off = np.zeros(len(texts) + 1, np.int64)
    off[1:] = np.cumsum([u.shape[0] for u in units])
    is_rt = np.ones(len(texts), np.uint8)
    sc = base.scalars.copy()
    sc[0, :] = 500   # every row passes the filter
    raw = RawBatch(np.concatenate(units), off, is_rt, sc, NOW)
    eng = _engine(1 << 20, "murmur3", lazy_idx=False, ingest=ingest)
    res = eng.train_batch(raw, want_pred=True)
    assert res["rows_lowered"] >= 18, res["rows_lowered"]
    dbg = eng._eng.debug_prepared()
    fb = featurize_batch(raw, 1 << 20, 100, 1000, now_ms=NOW, hash="murmur3")
    assert int(dbg["counters"][0]) == fb.n == raw.n
    rows = _rows_from_debug(dbg)
    Xt = fb.X[:, :1 << 20].tocsr()
    for k in range(fb.n):
        s, e = Xt.indptr[k], Xt.indptr[k + 1]
        want = np.repeat(Xt.indices[s:e], Xt.data[s:e].astype(np.int64))
        np.testing.assert_array_equal(rows[k], np.sort(want), err_msg=f"row {k}: {texts[k]!r}")


def test_utf8_cesu_surrogate_pairs_are_lowered(hip_module):
    """a receiver that writes astral letters as a surrogate pair of
    3-byte sequences (CESU-8, Java's modified UTF-8: ED A0 81 ED B0 80 for
    U+10400) must get them lower-cased like 4-byte UTF-8 does.  The decoder
    flags such rows as special candidates (ED A0), so the flagged-rows-only
    normaliser (the default) lowers them: device == oracle."""
    from twitter_stream_ml_amd.records.batch import RawBatch, Utf8Text, utf16_units
    base = generate_batch(SynthConfig.profile("twitter", seed=5), 0, 300, batch_time_ms=NOW)
    texts = [base.text_of(i) for i in range(base.n)]
    for j, s in enumerate(["\U00010400bc", "x \U00010401\U00010402 y", "\U0001E900 adlam", "ok \U00010427",
                           "\U0001F600 emoji only", "\U00010C80 hungarian"]):
        texts[11 * j + 1] = s

    def cesu(s):
        out = bytearray()
        for ch in s:
            c = ord(ch)
            if c > 0xFFFF:
                c -= 0x10000
                out += chr(0xD800 + (c >> 10)).encode("utf-8", "surrogatepass")
                out += chr(0xDC00 + (c & 0x3FF)).encode("utf-8", "surrogatepass")
            else:
                out += ch.encode("utf-8", "surrogatepass")
        return bytes(out)

    units = [utf16_units(s) for s in texts]
    off = np.zeros(len(texts) + 1, np.int64)
    off[1:] = np.cumsum([u.shape[0] for u in units])
    enc = [cesu(s) for s in texts]
    boff = np.zeros(len(texts) + 1, np.int64)
    boff[1:] = np.cumsum([len(b) for b in enc])
    u8 = Utf8Text(np.frombuffer(b"".join(enc), np.uint8).copy(), boff)
    sc = base.scalars.copy()
    sc[0, :] = 500
    raw = RawBatch(np.concatenate(units), off, np.ones(len(texts), np.uint8), sc, NOW, utf8=u8)
    eng = _engine(1 << 20, "murmur3", lazy_idx=False, ingest="utf8")
    res = eng.train_batch(raw, want_pred=True)
    assert res["rows_lowered"] >= 1, res["rows_lowered"]
    dbg = eng._eng.debug_prepared()
    fb = featurize_batch(raw, 1 << 20, 100, 1000, now_ms=NOW, hash="murmur3")
    rows = _rows_from_debug(dbg)
    Xt = fb.X[:, :1 << 20].tocsr()
    for k in range(fb.n):
        s, e = Xt.indptr[k], Xt.indptr[k + 1]
        want = np.repeat(Xt.indices[s:e], Xt.data[s:e].astype(np.int64))
        np.testing.assert_array_equal(rows[k], np.sort(want), err_msg=f"row {k}: {texts[k]!r}")


@pytest.mark.parametrize("profile,F,hash", [("twitter", 1 << 20, "java"), ("wide", 1 << 20, "java"),
                                            ("wide", 100_000_000, "murmur3")])
def test_utf8_ingest_trains_like_wire(hip_module, profile, F, hash):
    """UTF-8 ingest (the receiver's bytes, decoded on the device) gives the
    same featurization and row classes, hence the same training as the
    host-packed wire format, batch after batch -- bit for bit, since the GD
    arithmetic is exact fixed point (row order and layout do not matter)."""
    cfg = SynthConfig.profile(profile, seed=19, special_fraction=0.02)
    engs = {k: _engine(F, hash, ingest=k, max_rows=20000, max_units=20000 * 300) for k in ("wire", "utf8")}
    for t in range(3):
        raw = generate_batch(cfg, t * 20000, 20000, batch_time_ms=NOW + t * 5000)
        res = {k: e.train_batch(raw, want_pred=True) for k, e in engs.items()}
        a, b = res["wire"], res["utf8"]
        for key in ("n_kept", "n_unique", "iterations", "tiered", "rows_lowered"):
            assert a[key] == b[key], (key, a[key], b[key])
        assert list(b["stats"]) == list(a["stats"])   # exact fixed-point GD: layout-independent
        np.testing.assert_array_equal(np.asarray(a["pred"]), np.asarray(b["pred"]))
    wa, wb = engs["wire"].get_weights(), engs["utf8"].get_weights()
    np.testing.assert_array_equal(wb, wa)


@pytest.mark.parametrize("F,dedup,hybrid", [(1000, False, True), (1 << 20, False, True),
                                             (1000, True, False), (1000, False, False)])
def test_sgd_matches_oracle_over_batches(hip_module, F, dedup, hybrid):
    cfg = SynthConfig.profile("twitter", seed=5, unicode_fraction=0.1)
    eng = _engine(F, step_size=0.005, num_iterations=50, dedup=dedup, hybrid=hybrid)
    w = np.zeros(F + 4)
    for t in range(4):
        raw = generate_batch(cfg, t * 2500, 2500, batch_time_ms=NOW + t * 5000)
        fb = featurize_batch(raw, F, 100, 1000)
        pred_o = round_half_up_array(fb.X @ w)
        res = eng.train_batch(raw, want_pred=True)
        assert res["n_kept"] == fb.n
        # prequential predictions (output op #1) with the pre-training weights
        pred_g = np.asarray(res["pred"], np.float64)
        mism = np.abs(pred_g - pred_o) > 0
        assert mism.mean() < 0.01, mism.mean()
        assert np.all(np.abs(pred_g - pred_o) <= 1.0 + 1e-3 * np.abs(pred_o))
        n, sy, sy2, sp, sp2, se2 = res["stats"]
        assert int(n) == fb.n
        np.testing.assert_allclose(sy, fb.y.sum(), rtol=1e-12)
        np.testing.assert_allclose(se2 / n, np.mean((fb.y - pred_o) ** 2), rtol=2e-3)
        # training: the oracle continues from its own weights (no re-seeding),
        # so errors would accumulate over the warm-started batches
        r = run_minibatch_sgd(fb.X, fb.y, w, 0.005, 50)
        w = r.weights
        wg = eng.get_weights()
        scale = max(np.abs(w).max(), 1e-12)
        assert abs(res["iterations"] - r.iterations) <= 1, (res["iterations"], r.iterations)
        # one iteration more or less moves w by one step below the tolerance (1e-3 |w|)
        tol = 1e-6 if res["iterations"] == r.iterations else 3e-3
        assert np.linalg.norm(wg - w) <= tol * max(np.linalg.norm(w), 1e-30), (t, np.linalg.norm(wg - w))
        np.testing.assert_allclose(wg, w, rtol=2e-3, atol=2e-4 * scale)


def test_fraction_sampling_matches_oracle(hip_module):
    F = 1000
    cfg = SynthConfig.profile("twitter", seed=9)
    eng = _engine(F, fraction=0.5, num_iterations=10)
    raw = generate_batch(cfg, 0, 3000, batch_time_ms=NOW)
    fb = featurize_batch(raw, F, 100, 1000)
    res = eng.train_batch(raw)
    r = run_minibatch_sgd(fb.X, fb.y, np.zeros(F + 4), 0.005, 10, mini_batch_fraction=0.5)
    assert res["iterations"] == r.iterations
    wg = eng.get_weights()
    np.testing.assert_allclose(wg, r.weights, rtol=2e-3, atol=2e-4 * np.abs(r.weights).max())


def test_empty_and_filtered_out_batch(hip_module):
    F = 1000
    eng = _engine(F)
    cfg = SynthConfig.profile("twitter", seed=1, retweet_fraction=0.0)
    raw = generate_batch(cfg, 0, 500, batch_time_ms=NOW)
    res = eng.train_batch(raw)
    assert res["n_kept"] == 0 and res["iterations"] == 0
    assert np.all(eng.get_weights() == 0)


def test_merged_counts_match_hashingtf(hip_module):
    """Per-row duplicate merging: (slot, count) entries == HashingTF term counts."""
    F = 1000
    cfg = SynthConfig.profile("twitter", seed=12, unicode_fraction=0.2)
    raw = generate_batch(cfg, 0, 3000, batch_time_ms=NOW)
    eng = _engine(F, "java", dedup=True)
    eng.train_batch(raw, want_pred=False)
    dbg = eng._eng.debug_prepared()
    mg = eng._eng.debug_merged()
    assert mg["clen8d"].shape[0] > 0, "merging should be active for a small active set"
    assert np.all(mg["clen8d"] <= dbg["clen8"])
    uniq = np.sort(dbg["uniq"])
    nU = uniq.shape[0]
    fb = featurize_batch(raw, F, 100, 1000, now_ms=NOW)
    Xt = fb.X[:, :F].tocsr()
    perm, cbase = dbg["perm"], dbg["cbase"]
    slot, cnt = mg["slot"], mg["cnt"]
    for c in range(mg["clen8d"].shape[0]):
        g0, L8 = int(cbase[c]), int(mg["clen8d"][c])
        blk_s = slot[g0 * 512:(g0 + L8) * 512].reshape(L8, 64, 8)
        blk_c = cnt[g0 * 512:(g0 + L8) * 512].reshape(L8, 64, 8)
        for r in range(16):
            k = int(perm[c * 16 + r])
            if k < 0:
                continue
            s = blk_s[:, 4 * r:4 * r + 4, :].reshape(-1)
            n = blk_c[:, 4 * r:4 * r + 4, :].reshape(-1)
            real = (s >= 4) & (s < 4 + nU) & (n > 0)
            ids = uniq[s[real] - 4]
            assert np.unique(ids).shape[0] == ids.shape[0], f"row {k} not merged"
            got = dict(zip(ids.tolist(), n[real].tolist()))
            a, b = Xt.indptr[k], Xt.indptr[k + 1]
            want = dict(zip(Xt.indices[a:b].tolist(), Xt.data[a:b].astype(int).tolist()))
            assert got == want, f"row {k}"


def _with_repeats(raw, every=7, text="ha" * 40):
    """Replace every `every`-th text so some bigrams repeat > 15 times in a row."""
    from twitter_stream_ml_amd.records.batch import RawBatch, utf16_units
    texts = [text if i % every == 0 else raw.text_of(i) for i in range(raw.n)]
    units = [utf16_units(t) for t in texts]
    off = np.zeros(raw.n + 1, np.int64)
    off[1:] = np.cumsum([u.shape[0] for u in units])
    return RawBatch(np.concatenate(units), off, raw.is_retweet, raw.scalars, raw.batch_time_ms)


@pytest.mark.parametrize("F,hash,repeats,lazy", [(1000, "java", False, True), (1000, "java", True, True),
                                                 (1 << 20, "java", False, True),
                                                 (1 << 20, "java", True, False),
                                                 (1 << 20, "murmur3", False, True)])
def test_hybrid_layout_matches_hashingtf(hip_module, F, hash, repeats, lazy):
    """Hybrid layout: 4-bit hot counts + cold SELL entries == HashingTF term counts
    (lazy: fast chunks' ids re-derived from the text by the remap)."""
    cfg = SynthConfig.profile("twitter", seed=14, unicode_fraction=0.2)
    raw = generate_batch(cfg, 0, 4000, batch_time_ms=NOW)
    if repeats:
        raw = _with_repeats(raw)
    eng = _engine(F, hash, hybrid=True, lazy_idx=lazy)
    eng.train_batch(raw, want_pred=False)
    dbg = eng._eng.debug_prepared()
    hy = eng._eng.debug_hybrid()
    assert hy["clen8c"].shape[0] > 0, "hybrid layout should be active for a small active set"
    uniq = np.sort(dbg["uniq"])
    nU = uniq.shape[0]
    hot_slot = hy["hot_slot"]
    real_hot = (hot_slot >= 4) & (hot_slot < 4 + nU)
    assert real_hot.sum() == min(128, nU)
    assert np.unique(hot_slot[real_hot]).shape[0] == real_hot.sum()
    fb = featurize_batch(raw, F, 100, 1000, now_ms=NOW, hash=hash)
    Xt = fb.X[:, :F].tocsr()
    perm, cbase, clen8 = dbg["perm"], dbg["cbase"], dbg["clen8"]
    dense = hy["hot_dense"].reshape(-1, 64, 4)
    cslot = hy["cslot"]
    big = 0
    for c in range(hy["clen8c"].shape[0]):
        L4c = int(hy["clen8c"][c])            # cold 4-entry groups per lane
        assert 0 <= L4c <= 2 * int(clen8[c])
        g0 = int(cbase[c])
        blk = cslot[g0 * 512:g0 * 512 + L4c * 256].reshape(L4c, 64, 4)
        for r in range(16):
            k = int(perm[c * 16 + r])
            if k < 0:
                continue
            got = {}
            for t in range(4):
                words = dense[c, 4 * r + t]
                for i in range(32):
                    n = (int(words[i // 8]) >> (4 * (i % 8))) & 15
                    if n:
                        fid = int(uniq[hot_slot[32 * t + i] - 4])
                        got[fid] = got.get(fid, 0) + n
            sl = blk[:, 4 * r:4 * r + 4, :].reshape(-1)
            sl = sl[(sl >= 4) & (sl < 4 + nU)]
            for fid in uniq[sl - 4].tolist():
                got[fid] = got.get(fid, 0) + 1
            a, b = Xt.indptr[k], Xt.indptr[k + 1]
            want = dict(zip(Xt.indices[a:b].tolist(), Xt.data[a:b].astype(int).tolist()))
            big += sum(1 for v in want.values() if v > 15)
            assert got == want, f"row {k}"
    if repeats:
        assert big > 0, "test data should exercise the > 15 count overflow"
    # the hybrid iteration trains like the plain one
    plain = _engine(F, hash, hybrid=False)
    plain.train_batch(raw, want_pred=False)
    wh, wp = eng.get_weights(), plain.get_weights()
    np.testing.assert_array_equal(wh, wp)   # exact fixed-point GD: layout-independent


def test_wide_murmur3_hybrid_matches_plain_remap(hip_module):
    """F = 1e8 murmur3: the hybrid remap (LDS id cache for wide ids,
    hot_split.hip:id_code) trains the same model as the plain k_remap path."""
    from twitter_stream_ml_amd.ops.lr_engine import DeviceLinearRegression, LRDeviceConfig
    from twitter_stream_ml_amd.sources.synthetic import SynthConfig, generate_batch
    synth = SynthConfig.profile("twitter", seed=21, unicode_fraction=0.2)
    batches = [generate_batch(synth, t * 20000, 20000, batch_time_ms=1_700_000_000_000 + t) for t in range(2)]
    kw = dict(num_text_features=100_000_000, hash="murmur3", max_rows=32768, max_units=32768 * 300,
              num_iterations=10)
    a = DeviceLinearRegression(LRDeviceConfig(hybrid=True, **kw), device=0)
    b = DeviceLinearRegression(LRDeviceConfig(hybrid=False, **kw), device=0)
    for bt in batches:
        ra, rb = a.train_batch(bt, want_pred=False), b.train_batch(bt, want_pred=False)
        assert ra["n_kept"] == rb["n_kept"] and ra["iterations"] == rb["iterations"]
        assert list(ra["loss_history"]) == list(rb["loss_history"])
    np.testing.assert_array_equal(a.get_weights(), b.get_weights())


def test_utf8_truncated_sequences_stay_in_their_row(hip_module):
    """Malformed UTF-8 from a receiver (a 4-byte lead with its continuation
    bytes missing at a row end, stray continuation bytes) garbles only its
    own row: every other row featurizes exactly as the oracle."""
    from twitter_stream_ml_amd.ops.lr_engine import Utf8Text, encode_utf8
    cfg = SynthConfig.profile("twitter", seed=23, unicode_fraction=0.3)
    raw = generate_batch(cfg, 0, 800, batch_time_ms=NOW)
    raw.is_retweet[:] = 1
    raw.scalars[0, :] = 500
    u8 = encode_utf8(raw)
    bad = set(range(5, raw.n, 37))
    parts, off = [], [0]
    for i in range(raw.n):
        b = bytes(u8.data[u8.offsets[i]:u8.offsets[i + 1]])
        if i in bad:
            b = b + (b"\xf0" if i % 2 else b"\x80\xf0\x9f")   # truncated lead / stray continuation
        parts.append(b)
        off.append(off[-1] + len(b))
    bad_u8 = Utf8Text(np.frombuffer(b"".join(parts), np.uint8).copy(), np.asarray(off, np.int64))
    eng = _engine(1 << 20, lazy_idx=False, ingest="utf8")
    hb = eng.staging(0).load_utf8(raw, bad_u8, copy_text=True)
    eng.submit(hb, 0)
    eng.process(0, NOW)
    dbg = eng._eng.debug_prepared()
    fb = featurize_batch(raw, 1 << 20, 100, 1000, now_ms=NOW)
    assert int(dbg["counters"][0]) == fb.n == raw.n
    rows = _rows_from_debug(dbg)
    Xt = fb.X[:, :1 << 20].tocsr()
    for k in range(fb.n):
        if k in bad:
            continue
        s, e = Xt.indptr[k], Xt.indptr[k + 1]
        want = np.repeat(Xt.indices[s:e], Xt.data[s:e].astype(np.int64))
        np.testing.assert_array_equal(rows[k], np.sort(want), err_msg=f"row {k}")


def test_long_run_parity_wide(hip_module):
    """the fixed-point GD departs from MLlib's fp64 update
    (weights quantised relative to max |w|, residuals to a bound); over a
    long stream the drift must stay bounded.  60 warm-started batches of the
    realistic multi-script vocabulary, the fp64 oracle continuing from its own
    weights (never re-seeded): early-stop iteration counts agree (a one-step
    difference only where the oracle's own convergence margin is tiny), the
    prequential MSE per batch agrees, and the weight drift stays small."""
    F = 1 << 20
    cfg = SynthConfig.profile("wide", seed=21)
    eng = _engine(F, step_size=0.005, num_iterations=50)
    w = np.zeros(F + 4)
    same = 0
    worst_mse = worst_w = 0.0
    T = 60
    for t in range(T):
        raw = generate_batch(cfg, t * 2000, 2000, batch_time_ms=NOW + t * 5000)
        fb = featurize_batch(raw, F, 100, 1000)
        pred_o = round_half_up_array(fb.X @ w)
        res = eng.train_batch(raw, want_pred=False)
        assert res["n_kept"] == fb.n
        n, sy, sy2, sp, sp2, se2 = res["stats"]
        mse_o = float(np.mean((fb.y - pred_o) ** 2))
        worst_mse = max(worst_mse, abs(se2 / n - mse_o) / max(mse_o, 1e-30))
        r = run_minibatch_sgd(fb.X, fb.y, w, 0.005, 50)
        w = r.weights
        assert abs(res["iterations"] - r.iterations) <= 1, (t, res["iterations"], r.iterations)
        same += res["iterations"] == r.iterations
        wg = eng.get_weights()
        worst_w = max(worst_w, np.linalg.norm(wg - w) / max(np.linalg.norm(w), 1e-30))
    print(f"long run: iterations equal in {same}/{T} batches, worst mse rel {worst_mse:.2e}, "
          f"worst |dw|/|w| {worst_w:.2e}")
    assert same >= 0.9 * T
    assert worst_mse < 1e-3
    assert worst_w < 1e-3
