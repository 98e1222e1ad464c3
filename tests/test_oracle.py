"""fp64 oracle semantics (U1-U11) pinned against hand computations.

The reference has no tests for any of this (SURVEY §4 "Not tested at all");
these pin the MLlib 1.6.1 semantics the HIP kernels are then checked against.
"""
import math

import numpy as np
import pytest
import scipy.sparse as sp
from hypothesis import given, settings, strategies as st

from twitter_stream_ml_amd.models.hashing_tf import (HashingTF, bigram_hashes, java_string_hash,
                                                     murmur3_spark_hash, non_negative_mod,
                                                     text_units)
from twitter_stream_ml_amd.models.mllib_helper import MllibHelper
from twitter_stream_ml_amd.oracle import (KMeansState, StatCounter, decay_factor_from_half_life,
                                          featurize_batch, find_closest, kmeans_update,
                                          round_half_up, round_half_up_array, run_minibatch_sgd,
                                          sgd_uniform, standard_scaler_fit,
                                          standard_scaler_transform)
from twitter_stream_ml_amd.records import RawBatch, Status, User


# ---- Utils.round ------------------------------------------------------------
@pytest.mark.parametrize("x,want", [(2.5, 3.0), (-2.5, -3.0), (2.4999, 2.0), (0.5, 1.0),
                                    (-0.5, -1.0), (0.49999999999999994, 0.0), (7.0, 7.0),
                                    (-1e15 - 0.5, -1e15 - 1.0)])
def test_round_half_up(x, want):
    assert round_half_up(x) == want
    assert round_half_up_array(np.array([x]))[0] == want


def test_round_non_finite_throws():
    for v in (float("nan"), float("inf")):
        with pytest.raises(ValueError):
            round_half_up(v)


# ---- StatCounter ------------------------------------------------------------
def test_stat_counter_population_stdev_and_merge():
    v = np.array([1.0, 2.0, 4.0, 7.0])
    s = StatCounter.of(v)
    assert s.stdev() == pytest.approx(np.std(v))           # population, like RDD.stdev
    assert s.sampleStdev() == pytest.approx(np.std(v, ddof=1))
    m = StatCounter.of(v[:1]).merge(StatCounter.of(v[1:]))
    assert (m.n, m.mean(), m.stdev()) == pytest.approx((4, v.mean(), np.std(v)))


# ---- HashingTF / bigrams --------------------------------------------------------
def test_java_hash_of_bigrams():
    assert java_string_hash(text_units("ab")) == 31 * 97 + 98
    assert java_string_hash(text_units("hello world")) == "hello world".__hash__() * 0 + 1794106052
    assert list(bigram_hashes(text_units("abc"))) == [31 * 97 + 98, 31 * 98 + 99]
    assert list(bigram_hashes(text_units("x"))) == [ord("x")]      # 1-char text -> 1 term
    assert bigram_hashes(text_units("")).shape == (0,)


def test_non_negative_mod():
    assert non_negative_mod(-7, 5) == 3
    assert non_negative_mod(7, 5) == 2
    assert non_negative_mod(-(2 ** 31), 1000) == 352


def test_hashing_tf_transform_counts_and_sorted():
    tf = HashingTF(1000)
    v = tf.transform([(97, 98), (97, 98), (98, 99)])
    assert list(v.indices) == sorted([3105 % 1000, (31 * 98 + 99) % 1000])
    assert dict(zip(v.indices, v.values))[105] == 2.0


def test_surrogate_pairs_split_into_code_units():
    units = text_units("a😀")          # U+1F600 = D83D DE00
    assert list(units) == [97, 0xD83D, 0xDE00]
    assert list(bigram_hashes(units)) == [31 * 97 + 0xD83D, 31 * 0xD83D + 0xDE00]


def test_murmur3_matches_standard_murmur_on_aligned_input():
    from sklearn.utils import murmurhash3_32
    for s in ["abcd", "éé", "日本語!", "12345678"]:
        b = s.encode("utf-8")
        if len(b) % 4 == 0:
            assert murmur3_spark_hash(b, 42) == murmurhash3_32(b, seed=42, positive=False)


@settings(max_examples=200, deadline=None)
@given(st.text(min_size=0, max_size=40))
def test_bigram_index_properties(s):
    tf = HashingTF(997)
    idx = tf.bigram_indices(text_units(s))
    assert np.all((idx >= 0) & (idx < 997))
    u = text_units(s)
    assert idx.shape[0] == (u.shape[0] - 1 if u.shape[0] >= 2 else u.shape[0])


# ---- MllibHelper.featurize / filtrate ----------------------------------------------
def _status(text, rc, fol=5, fav=6, fri=7, created=1000, retweet=True):
    orig = Status(text=text, retweetCount=rc, createdAt=created, user=User(fol, fav, fri))
    return Status(text="RT " + text, retweetedStatus=orig) if retweet else orig


def test_featurize_matches_mllib_helper():
    MllibHelper.configure(1000)
    s = _status("AB", 150)
    lp = MllibHelper.featurize(s, now_ms=2000)
    assert lp.label == 150.0
    assert list(lp.features.indices) == [105, 1000, 1001, 1002, 1003]
    np.testing.assert_allclose(lp.features.values, [1.0, 5e-12, 6e-12, 7e-12, 1000 * 1e-14])
    MllibHelper.numRetweetBegin, MllibHelper.numRetweetEnd = 100, 1000
    assert MllibHelper.filtrate(s)
    assert not MllibHelper.filtrate(_status("x", 99))
    assert MllibHelper.filtrate(_status("x", 1000))
    assert not MllibHelper.filtrate(_status("x", 500, retweet=False))
    # columnar oracle agrees with the row-wise helper
    raw = RawBatch.from_statuses([s, _status("x", 99), _status("İΣ abc", 200)], batch_time_ms=2000)
    fb = featurize_batch(raw, 1000, 100, 1000)
    assert fb.n == 2 and list(fb.rows) == [0, 2]
    np.testing.assert_allclose(fb.X[0].toarray()[0], lp.features.toArray())
    lp2 = MllibHelper.featurize(_status("İΣ abc", 200), now_ms=2000)
    np.testing.assert_allclose(fb.X[1].toarray()[0], lp2.features.toArray())


# ---- GradientDescent --------------------------------------------------------------
def test_sgd_one_iteration_by_hand():
    X = sp.csr_matrix(np.array([[1.0, 0.0], [0.0, 1.0]]))
    y = np.array([1.0, 2.0])
    r = run_minibatch_sgd(X, y, np.zeros(2), step_size=1.0, num_iterations=1)
    np.testing.assert_allclose(r.weights, [0.5, 1.0])   # w -= 1/sqrt(1) * g/m
    assert r.iterations == 1 and not r.converged
    r2 = run_minibatch_sgd(X, y, np.zeros(2), step_size=1.0, num_iterations=2)
    # iteration 2: g = X^T(Xw - y) = [-0.5, -1], step 1/sqrt(2)
    np.testing.assert_allclose(r2.weights, [0.5 + 0.25 / math.sqrt(2), 1.0 + 0.5 / math.sqrt(2)])
    assert r2.loss_history[0] == pytest.approx((1 + 4) / 2 / 2)


def test_sgd_convergence_and_empty_batch():
    X = sp.csr_matrix(np.ones((4, 1)))
    y = np.full(4, 3.0)
    r = run_minibatch_sgd(X, y, np.array([3.0]), 0.1, 50)   # already optimal -> dw = 0
    assert r.converged and r.iterations == 2                 # needs two updates to test
    e = run_minibatch_sgd(sp.csr_matrix((0, 3)), np.zeros(0), np.array([1.0, 2, 3]), 0.1, 50)
    np.testing.assert_array_equal(e.weights, [1, 2, 3])
    assert e.iterations == 0
    with pytest.raises(ValueError):
        run_minibatch_sgd(X, y, np.zeros(1), 0.1, 5, mini_batch_fraction=1.23)


def test_sgd_sampling_is_seeded_per_iteration():
    u1 = sgd_uniform(43, np.arange(1000, dtype=np.uint64))
    u2 = sgd_uniform(44, np.arange(1000, dtype=np.uint64))
    assert 0.4 < (u1 < 0.5).mean() < 0.6 and not np.array_equal(u1, u2)
    np.testing.assert_array_equal(u1, sgd_uniform(43, np.arange(1000, dtype=np.uint64)))


def test_sgd_dp_allreduce_equals_single():
    rng = np.random.default_rng(0)
    X = sp.random(200, 30, density=0.2, random_state=1, format="csr")
    y = rng.normal(size=200)
    full = run_minibatch_sgd(X, y, np.zeros(30), 0.05, 20, mini_batch_fraction=0.6)
    # two "ranks" in lock-step on threads; allreduce sums their vectors
    import threading
    barrier = threading.Barrier(2)
    slots = [None, None]
    out = [None, None]

    def make_ar(k):
        def ar(v):
            slots[k] = v.copy()
            barrier.wait()
            s = slots[0] + slots[1]
            barrier.wait()
            return s
        return ar

    def rank(k, lo, hi):
        out[k] = run_minibatch_sgd(X[lo:hi], y[lo:hi], np.zeros(30), 0.05, 20,
                                   mini_batch_fraction=0.6, allreduce=make_ar(k), row_offset=lo)

    th = [threading.Thread(target=rank, args=(0, 0, 120)), threading.Thread(target=rank, args=(1, 120, 200))]
    [t.start() for t in th]
    [t.join() for t in th]
    for k in range(2):
        np.testing.assert_allclose(out[k].weights, full.weights, rtol=1e-12, atol=1e-14)
        assert out[k].iterations == full.iterations


# ---- StandardScaler / KMeans --------------------------------------------------------
def test_standard_scaler_sample_std_and_zero_std():
    X = np.array([[1.0, 5.0], [3.0, 5.0], [5.0, 5.0]])
    std = standard_scaler_fit(X)
    np.testing.assert_allclose(std, [2.0, 0.0])
    np.testing.assert_allclose(standard_scaler_transform(X, std), [[0.5, 0], [1.5, 0], [2.5, 0]])
    assert np.all(standard_scaler_fit(X[:1]) == 0)


def test_kmeans_update_by_hand():
    a = decay_factor_from_half_life(5)
    assert a == pytest.approx(0.8705505632961241)
    st0 = KMeansState(np.array([[0.0, 0.0], [10.0, 10.0]]), np.array([1.0, 1.0]))
    X = np.array([[1.0, 0.0], [0.0, 1.0], [9.0, 9.0]])
    s1, labels = kmeans_update(st0, X, 0.5)
    assert list(labels) == [0, 0, 1]
    # cluster 0: w = 1*0.5 + 2 = 2.5, lambda = 2/2.5; c = 0.2*0 + (0.8/2)*[1,1]
    np.testing.assert_allclose(s1.weights, [2.5, 1.5])
    np.testing.assert_allclose(s1.centers[0], [0.4, 0.4])
    np.testing.assert_allclose(s1.centers[1], (1 - 1 / 1.5) * 10 + (1 / 1.5) * 9)


def test_kmeans_dying_cluster_split_and_ties():
    st0 = KMeansState(np.array([[0.0], [0.0], [5.0]]), np.zeros(3))
    s1, labels = kmeans_update(st0, np.array([[0.1], [0.2]]), 1.0)
    assert list(labels) == [0, 0]           # tie between 0 and 1 -> first index
    # weights [2, 0, 0]: smallest (index 1) is dying -> split the largest (0)
    assert s1.weights[0] == s1.weights[1] == 1.0
    assert s1.centers[0, 0] > s1.centers[1, 0]
    assert s1.centers[0, 0] - s1.centers[1, 0] == pytest.approx(2e-14 * 1.0, rel=1e-3)
    assert list(find_closest(np.array([[0.0], [0.0]]), np.array([[1.0]]))) == [0]


def test_active_column_oracle_equals_full_width():
    """run_minibatch_sgd_active (touched columns + constant rest norm) takes
    the same iterates as the full-width MLlib loop, warm-started from a
    model with weight outside the batch's columns; and the native featurizer
    equals the Python one."""
    from twitter_stream_ml_amd.oracle import (featurize_batch, featurize_batch_native,
                                              run_minibatch_sgd, run_minibatch_sgd_active)
    from twitter_stream_ml_amd.sources.synthetic import SynthConfig, generate_batch
    cfg = SynthConfig.profile("wide", seed=4, special_fraction=0.02)
    F = 1 << 16
    raw = generate_batch(cfg, 0, 1500, batch_time_ms=1_700_000_000_000)
    fb = featurize_batch(raw, F, 100, 1000, hash="murmur3")
    fn = featurize_batch_native(raw, F, 100, 1000, hash="murmur3")
    assert abs(fb.X - fn.X).max() == 0 and np.array_equal(fb.y, fn.y)
    rng = np.random.default_rng(1)
    w0 = rng.standard_normal(F + 4) * 1e-3   # mass outside the touched columns too
    for tol in (1e-3, 1e-4):
        a = run_minibatch_sgd(fb.X, fb.y, w0, 0.005, 50, convergence_tol=tol)
        b = run_minibatch_sgd_active(fb.X, fb.y, w0, 0.005, 50, convergence_tol=tol)
        assert a.iterations == b.iterations and a.converged == b.converged
        np.testing.assert_allclose(b.weights, a.weights, rtol=1e-10, atol=1e-13)
        np.testing.assert_allclose(b.loss_history, a.loss_history, rtol=1e-10)
