"""Streaming linear regression: MLlib API + the CPU engine.

* :class:`LinearRegressionModel` — ``weights`` (fp64) + ``intercept`` (always 0
  here, ``LinearRegressionWithSGD`` adds none), ``predict``, MLlib-layout
  ``save``/``load`` (checkpoint/saveable.py).
* :class:`StreamingLinearRegressionWithSGD` — the MLlib builder
  (``setNumIterations``/``setStepSize``/``setMiniBatchFraction``/
  ``setInitialWeights``, ``LinearRegression.scala:28-32``), ``latestModel``,
  ``trainOn`` (warm start from the previous batch's weights, skip empty
  batches, [upstream] ``StreamingLinearAlgorithm.trainOn``), ``predictOn``.
  ``trainOn`` accepts a LabeledPoint DStream (generic MLlib path) or, with an
  engine attached, the raw tweet stream (fused filter/featurize/train).
* :class:`CpuLinearRegression` — the ``local[N]`` engine with the same batch
  contract as the MI355X engine (``ops/lr_engine.DeviceLinearRegression``):
  ``train_batch(raw) -> result dict``.  Featurization is the native C++
  featurizer, the math is the fp64 oracle (scipy sparse), and data
  parallelism is an all-reduce callable (gloo).
"""
from __future__ import annotations

import logging
from dataclasses import dataclass
from typing import Callable, Dict, Optional, Sequence, Union

import numpy as np
import scipy.sparse as sp

from ..oracle.mllib import CONVERGENCE_TOL, round_half_up_array, run_minibatch_sgd
from ..records.batch import CREATED_AT, FAVOURITES, FOLLOWERS, FRIENDS, RETWEET_COUNT, RawBatch
from .mllib_helper import NUMBER_SCALES
from .vectors import DenseVector, LabeledPoint, SparseVector, Vector, Vectors

__all__ = ["LinearRegressionModel", "StreamingLinearRegressionWithSGD", "CpuLinearRegression",
           "featurize_columnar", "stats_from_predictions"]

log = logging.getLogger("org.apache.spark.mllib.regression.StreamingLinearRegressionWithSGD")


class LinearRegressionModel:
    def __init__(self, weights, intercept: float = 0.0):
        self.weights = np.asarray(weights.toArray() if isinstance(weights, Vector) else weights,
                                  dtype=np.float64).copy()
        self.intercept = float(intercept)

    @property
    def numFeatures(self) -> int:
        return int(self.weights.shape[0])

    def predict(self, x):
        from ..runtime.rdd import RDD
        if isinstance(x, RDD):
            return x.map(self.predict)
        if isinstance(x, Vector):
            return float(x.dot(DenseVector(self.weights))) + self.intercept
        if sp.issparse(x):
            return np.asarray(x @ self.weights).reshape(-1) + self.intercept
        arr = np.asarray(x, dtype=np.float64)
        return arr @ self.weights + self.intercept

    def save(self, path: str, progress: Optional[dict] = None) -> None:
        from ..checkpoint.saveable import save_linear_regression
        save_linear_regression(path, self.weights, self.intercept, progress)

    @staticmethod
    def save_sparse(path: str, weights, intercept: float = 0.0, progress: Optional[dict] = None) -> None:
        """Save weights given as ``checkpoint.SparseWeights`` (non-zeros only)."""
        from ..checkpoint.saveable import save_linear_regression
        save_linear_regression(path, weights, intercept, progress)

    @classmethod
    def load(cls, path: str) -> "LinearRegressionModel":
        from ..checkpoint.saveable import load_linear_regression
        w, b = load_linear_regression(path)
        return cls(w, b)


# ---------------------------------------------------------------------------
def featurize_columnar(raw: RawBatch, num_text_features: int, begin: int, end: int,
                       now_ms: Optional[int] = None, hash: str = "java", apply_filter: bool = True):
    """Native-featurizer version of ``oracle.featurize_batch`` (same CSR)."""
    from ..ops._native import host
    F = int(num_text_features)
    now = raw.batch_time_ms if now_ms is None else int(now_ms)
    rc = raw.scalars[RETWEET_COUNT]
    mask = (raw.is_retweet != 0) & (rc >= begin) & (rc <= end) if apply_filter else np.ones(raw.n, bool)
    rows = np.nonzero(mask)[0].astype(np.int64)
    n = rows.shape[0]
    if n == 0:
        return sp.csr_matrix((0, F + 4)), np.zeros(0), rows
    raw.ensure_text()   # a replayed batch may carry only its UTF-8 bytes
    indptr, idx = host().featurize_rows(raw.text, raw.offsets, rows, F, hash, 0)
    lens = np.diff(indptr)
    row_of = np.repeat(np.arange(n, dtype=np.int64), lens)
    sc = raw.scalars[:, rows].astype(np.float64)
    nums = np.stack([sc[FOLLOWERS] * NUMBER_SCALES[0], sc[FAVOURITES] * NUMBER_SCALES[1],
                     sc[FRIENDS] * NUMBER_SCALES[2],
                     (now - raw.scalars[CREATED_AT, rows]).astype(np.float64) * NUMBER_SCALES[3]],
                    axis=1)
    r = np.concatenate([row_of, np.repeat(np.arange(n, dtype=np.int64), 4)])
    c = np.concatenate([idx, np.tile(np.arange(F, F + 4, dtype=np.int64), n)])
    v = np.concatenate([np.ones(idx.shape[0]), nums.reshape(-1)])
    X = sp.csr_matrix((v, (r, c)), shape=(n, F + 4))
    X.sum_duplicates()
    return X, rc[rows].astype(np.float64), rows


def stats_from_predictions(y: np.ndarray, pred: np.ndarray) -> list:
    """The 6 moments the engines report: n, sum y, sum y^2, sum p, sum p^2, sum (y-p)^2."""
    e = y - pred
    return [float(y.shape[0]), float(y.sum()), float(y @ y), float(pred.sum()), float(pred @ pred),
            float(e @ e)]


@dataclass
class CpuLRConfig:
    num_text_features: int = 1000
    hash: str = "java"
    step_size: float = 0.005
    num_iterations: int = 50
    fraction: float = 1.0
    tol: float = CONVERGENCE_TOL
    begin: int = 100
    end: int = 1000


class CpuLinearRegression:
    """fp64 CPU engine with the DeviceLinearRegression batch contract."""

    def __init__(self, cfg: CpuLRConfig, allreduce: Optional[Callable[[np.ndarray], np.ndarray]] = None,
                 rank: int = 0, world: int = 1):
        self.cfg = cfg
        self.allreduce = allreduce
        self.rank, self.world = rank, world
        self.w = np.zeros(cfg.num_text_features + 4)

    @property
    def num_weights(self) -> int:
        return int(self.w.shape[0])

    def get_weights(self) -> np.ndarray:
        return self.w.copy()

    def set_weights(self, w) -> None:
        w = np.asarray(w, dtype=np.float64)
        if w.shape != self.w.shape:
            raise ValueError(f"expected {self.w.shape[0]} weights, got {w.shape}")
        self.w = w.copy()

    def train_batch(self, raw: RawBatch, want_pred: bool = True, plot_points: int = 0,
                    slot: int = 0) -> Dict[str, object]:
        c = self.cfg
        X, y, rows = featurize_columnar(raw, c.num_text_features, c.begin, c.end, hash=c.hash)
        red = self.allreduce
        # per-rank kept counts -> global count and this rank's sampling offset
        counts = np.zeros(self.world)
        counts[self.rank] = y.shape[0]
        if red is not None:
            counts = red(counts)
        n_glob = int(round(counts.sum()))
        row_offset = int(round(counts[:self.rank].sum()))
        pred = round_half_up_array(X @ self.w) if y.shape[0] else np.zeros(0)
        stats = np.array(stats_from_predictions(y, pred))
        if red is not None:
            stats = red(stats)
        res: Dict[str, object] = {"n_raw": raw.n, "n_kept": int(y.shape[0]),
                                  "n_kept_global": n_glob, "iterations": 0, "converged": False,
                                  "loss_history": [], "stats": stats.tolist(),
                                  "pred": None, "real": None,
                                  "n_unique": int(np.unique(X.indices).shape[0]) if X.nnz else 0,
                                  "prep_ms": 0.0, "train_ms": 0.0, "diverged": False}
        if want_pred:   # the plot's series: all kept rows, or plot_points evenly spaced ones
            P = y.shape[0] if plot_points <= 0 else min(int(plot_points), y.shape[0])
            idx = (np.arange(P, dtype=np.int64) * max(y.shape[0] - 1, 0)) // max(P - 1, 1)
            res["pred"], res["real"] = pred[idx].astype(np.float32), y[idx].astype(np.float32)
        if n_glob == 0:
            return res
        r = run_minibatch_sgd(X, y, self.w, c.step_size, c.num_iterations, c.fraction, c.tol,
                              allreduce=red, row_offset=row_offset)
        self.w = r.weights
        res.update(iterations=r.iterations, converged=r.converged, loss_history=r.loss_history)
        return res

    def synchronize(self) -> None:
        pass


# ---------------------------------------------------------------------------
class StreamingLinearRegressionWithSGD:
    """``StreamingLinearRegressionWithSGD`` (MLlib 1.6 builder API)."""

    def __init__(self, stepSize: float = 0.1, numIterations: int = 50,
                 miniBatchFraction: float = 1.0, engine=None):
        self.stepSize = float(stepSize)
        self.numIterations = int(numIterations)
        self.miniBatchFraction = float(miniBatchFraction)
        self.convergenceTol = CONVERGENCE_TOL
        self.model: Optional[LinearRegressionModel] = None
        self.engine = engine          # CpuLinearRegression | DeviceLinearRegression (raw path)
        self.allreduce = None
        self.last_result: Optional[Dict[str, object]] = None

    # builder ------------------------------------------------------------
    def setStepSize(self, v: float) -> "StreamingLinearRegressionWithSGD":
        self.stepSize = float(v)
        return self

    def setNumIterations(self, v: int) -> "StreamingLinearRegressionWithSGD":
        self.numIterations = int(v)
        return self

    def setMiniBatchFraction(self, v: float) -> "StreamingLinearRegressionWithSGD":
        self.miniBatchFraction = float(v)
        return self

    def setConvergenceTol(self, v: float) -> "StreamingLinearRegressionWithSGD":
        self.convergenceTol = float(v)
        return self

    def setInitialWeights(self, w) -> "StreamingLinearRegressionWithSGD":
        self.model = LinearRegressionModel(w, 0.0)
        if self.engine is not None:
            self.engine.set_weights(self.model.weights)
        return self

    def setEngine(self, engine) -> "StreamingLinearRegressionWithSGD":
        self.engine = engine
        if self.model is not None:
            engine.set_weights(self.model.weights)
        return self

    def latestModel(self) -> LinearRegressionModel:
        if self.model is None:
            raise ValueError("Model must be initialized before starting training.")
        if self.engine is not None:
            self.model = LinearRegressionModel(self.engine.get_weights(), 0.0)
        return self.model

    # training -------------------------------------------------------------
    def train_rdd(self, rdd) -> None:
        """One ``algorithm.run(rdd, model.weights)`` on a LabeledPoint RDD."""
        if self.model is None:
            raise ValueError("Model must be initialized before starting training.")
        pts = rdd.collect()
        if not pts:
            return
        n = self.model.numFeatures
        rows, cols, vals = [], [], []
        y = np.empty(len(pts))
        for i, lp in enumerate(pts):
            f = lp.features
            if isinstance(f, SparseVector):
                rows.append(np.full(f.indices.shape[0], i)); cols.append(f.indices); vals.append(f.values)
            else:
                a = f.toArray(); nz = np.nonzero(a)[0]
                rows.append(np.full(nz.shape[0], i)); cols.append(nz); vals.append(a[nz])
            y[i] = lp.label
        X = sp.csr_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))),
                          shape=(len(pts), n))
        r = run_minibatch_sgd(X, y, self.model.weights, self.stepSize, self.numIterations,
                              self.miniBatchFraction, self.convergenceTol, allreduce=self.allreduce)
        self.model = LinearRegressionModel(r.weights, 0.0)
        log.info("Model updated")
        shown = ",".join(repr(float(v)) for v in r.weights[:100])
        log.info("Current model: weights, [%s%s", shown, "..." if r.weights.shape[0] > 100 else "]")

    def trainOn(self, stream) -> None:
        if self.model is None:
            raise ValueError("Model must be initialized before starting training.")

        def op(rdd):
            if self.engine is not None and getattr(rdd, "raw", None) is not None and \
                    isinstance(rdd.raw, RawBatch) and not rdd.isEmpty():
                self.last_result = self.engine.train_batch(rdd.raw, want_pred=False)
            elif not rdd.isEmpty():
                self.train_rdd(rdd)
        stream.foreachRDD(op)

    def predictOn(self, stream):
        return stream.map(lambda lp: self.latestModel().predict(lp.features if isinstance(lp, LabeledPoint) else lp))

    def predictOnValues(self, stream):
        return stream.map(lambda kv: (kv[0], self.latestModel().predict(kv[1])))
