"""Streaming k-means and the standard scaler: MLlib API + CPU engine (C2, U8-U10).

* :class:`StreamingKMeans` — builder (``setK``, ``setDecayFactor``,
  ``setHalfLife(h, "batches"|"points")``, ``setRandomCenters(dim, weight,
  seed)``, ``setInitialCenters``), ``latestModel``, ``trainOn``,
  ``predictOn`` (``KMeans.scala:69-73``).
* :class:`StreamingKMeansModel` — ``update(data, decayFactor, timeUnit)``,
  ``predict``, ``clusterCenters`` / ``clusterWeights``, checkpoint save/load.
* :class:`StandardScaler` / :class:`StandardScalerModel` —
  ``StandardScaler(withMean=false, withStd=true).fit(rdd).transform(rdd)``
  re-fitted every batch (``KMeans.scala:103``).
* :func:`kmeans_features` — the KMeans job's featurization of a raw batch:
  retweets only (``KMeans.scala:77-80``), ``[retweetCount, followersCount]``
  of the original (``:19-29``), optionally followed by ``text_dims`` hashed
  bigram counts (engine extension for the k=1024 configuration).
* :class:`CpuKMeans` — the ``local[N]`` engine with the batch contract of the
  MI355X k-means engine (``ops/kmeans_engine.py``).
"""
from __future__ import annotations

import math
from typing import Callable, Dict, Optional

import numpy as np

from ..oracle.mllib import (KMeansState, decay_factor_from_half_life, find_closest, kmeans_update,
                            standard_scaler_fit, standard_scaler_transform)
from ..records.batch import FOLLOWERS, RETWEET_COUNT, RawBatch
from .vectors import DenseVector, Vector

__all__ = ["StreamingKMeans", "StreamingKMeansModel", "StandardScaler", "StandardScalerModel",
           "kmeans_features", "CpuKMeans"]

BATCHES = "batches"
POINTS = "points"


def kmeans_features(raw: RawBatch, text_dims: int = 0, hash: str = "java"):
    """Dense (n_retweets, 2 + text_dims) fp64 features and the kept row ids."""
    rows = np.nonzero(raw.is_retweet != 0)[0].astype(np.int64)
    n = rows.shape[0]
    X = np.zeros((n, 2 + text_dims))
    X[:, 0] = raw.scalars[RETWEET_COUNT, rows]
    X[:, 1] = raw.scalars[FOLLOWERS, rows]
    if text_dims > 0 and n:
        from ..ops._native import host
        raw.ensure_text()   # a replayed batch may carry only its UTF-8 bytes
        indptr, idx = host().featurize_rows(raw.text, raw.offsets, rows, text_dims, hash, 0)
        r = np.repeat(np.arange(n), np.diff(indptr))
        np.add.at(X, (r, 2 + idx), 1.0)
    return X, rows


class StandardScalerModel:
    def __init__(self, std: np.ndarray, mean: Optional[np.ndarray] = None,
                 withStd: bool = True, withMean: bool = False):
        self.std = np.asarray(std, np.float64)
        self.mean = mean
        self.withStd, self.withMean = withStd, withMean

    def transform(self, data):
        from ..runtime.rdd import RDD
        if isinstance(data, RDD):
            return data.map(lambda v: DenseVector(self.transform(v.toArray() if isinstance(v, Vector) else v)))
        X = np.asarray(data, np.float64)
        if self.withMean and self.mean is not None:
            X = X - self.mean
        return standard_scaler_transform(X, self.std) if self.withStd else X


class StandardScaler:
    def __init__(self, withMean: bool = False, withStd: bool = True):
        self.withMean, self.withStd = withMean, withStd

    def fit(self, data, allreduce=None) -> StandardScalerModel:
        from ..runtime.rdd import RDD
        if isinstance(data, RDD):
            X = np.stack([v.toArray() if isinstance(v, Vector) else np.asarray(v) for v in data.collect()])
        else:
            X = np.asarray(data, np.float64)
        std = standard_scaler_fit(X, allreduce)
        mean = X.mean(axis=0) if self.withMean and X.shape[0] else None
        return StandardScalerModel(std, mean, self.withStd, self.withMean)


class StreamingKMeansModel:
    def __init__(self, clusterCenters: np.ndarray, clusterWeights: np.ndarray):
        self.state = KMeansState(np.asarray(clusterCenters, np.float64).copy(),
                                 np.asarray(clusterWeights, np.float64).copy())

    @property
    def clusterCenters(self) -> np.ndarray:
        return self.state.centers

    @property
    def clusterWeights(self) -> np.ndarray:
        return self.state.weights

    @property
    def k(self) -> int:
        return int(self.state.centers.shape[0])

    def predict(self, x):
        from ..runtime.rdd import RDD
        if isinstance(x, RDD):
            return x.map(self.predict)
        if isinstance(x, Vector):
            return int(find_closest(self.state.centers, x.toArray()[None, :])[0])
        X = np.asarray(x, np.float64)
        if X.ndim == 1:
            return int(find_closest(self.state.centers, X[None, :])[0])
        return find_closest(self.state.centers, X)

    def update(self, data, decayFactor: float, timeUnit: str = BATCHES, allreduce=None):
        from ..runtime.rdd import RDD
        if isinstance(data, RDD):
            pts = data.collect()
            X = np.stack([p.toArray() if isinstance(p, Vector) else np.asarray(p) for p in pts]) \
                if pts else np.zeros((0, self.state.centers.shape[1]))
        else:
            X = np.asarray(data, np.float64)
        self.state, labels = kmeans_update(self.state, X, decayFactor, timeUnit, allreduce)
        return self

    def save(self, path: str, progress: Optional[dict] = None) -> None:
        from ..checkpoint.saveable import save_kmeans
        save_kmeans(path, self.state.centers, self.state.weights, progress)

    @classmethod
    def load(cls, path: str) -> "StreamingKMeansModel":
        from ..checkpoint.saveable import load_kmeans
        c, w = load_kmeans(path)
        return cls(c, w if w is not None else np.ones(c.shape[0]))


class StreamingKMeans:
    def __init__(self, k: int = 2, decayFactor: float = 1.0, timeUnit: str = BATCHES):
        self.k = int(k)
        self.decayFactor = float(decayFactor)
        self.timeUnit = timeUnit
        self.model: Optional[StreamingKMeansModel] = None
        self.allreduce = None

    def setK(self, k: int) -> "StreamingKMeans":
        self.k = int(k)
        return self

    def setDecayFactor(self, a: float) -> "StreamingKMeans":
        self.decayFactor = float(a)
        return self

    def setHalfLife(self, halfLife: float, timeUnit: str) -> "StreamingKMeans":
        if timeUnit not in (BATCHES, POINTS):
            raise ValueError(f"Invalid time unit for decay: {timeUnit}")
        self.decayFactor = decay_factor_from_half_life(halfLife)
        self.timeUnit = timeUnit
        return self

    def setRandomCenters(self, dim: int, weight: float, seed: Optional[int] = None) -> "StreamingKMeans":
        seed = int(np.random.SeedSequence().entropy % (1 << 63)) if seed is None else int(seed)
        st = KMeansState.random(self.k, dim, weight, seed)
        self.model = StreamingKMeansModel(st.centers, st.weights)
        return self

    def setInitialCenters(self, centers, weights) -> "StreamingKMeans":
        self.model = StreamingKMeansModel(np.asarray(centers), np.asarray(weights))
        self.k = self.model.k
        return self

    def latestModel(self) -> StreamingKMeansModel:
        if self.model is None:
            raise ValueError("Initial cluster centers must be set before starting predictions")
        return self.model

    def trainOn(self, stream) -> None:
        def op(rdd):
            self.latestModel().update(rdd, self.decayFactor, self.timeUnit, self.allreduce)
        stream.foreachRDD(op)

    def predictOn(self, stream):
        return stream.map(lambda v: self.latestModel().predict(v))

    def predictOnValues(self, stream):
        return stream.map(lambda kv: (kv[0], self.latestModel().predict(kv[1])))


class CpuKMeans:
    """fp64 engine: per batch scaler fit + transform, then the streaming update."""

    def __init__(self, k: int, dim: int, half_life: float = 5.0, time_unit: str = BATCHES,
                 init_weight: float = 0.0, seed: int = 42, scale: bool = True,
                 allreduce: Optional[Callable[[np.ndarray], np.ndarray]] = None):
        st = KMeansState.random(k, dim, init_weight, seed)
        self.state = st
        self.decay = decay_factor_from_half_life(half_life)
        self.time_unit = time_unit
        self.scale = scale
        self.allreduce = allreduce

    def set_state(self, centers, weights) -> None:
        self.state = KMeansState(np.asarray(centers, np.float64).copy(), np.asarray(weights, np.float64).copy())

    def get_state(self):
        return self.state.centers.copy(), self.state.weights.copy()

    def update_batch(self, X: np.ndarray) -> Dict[str, object]:
        n_local = np.array([float(X.shape[0])])
        n = self.allreduce(n_local)[0] if self.allreduce else n_local[0]
        if n == 0:
            return {"n": 0, "labels": np.zeros(0, np.int64), "std": None}
        std = standard_scaler_fit(X, self.allreduce) if self.scale else np.ones(X.shape[1])
        Xs = standard_scaler_transform(X, std) if self.scale else X
        self.state, labels = kmeans_update(self.state, Xs, self.decay, self.time_unit, self.allreduce)
        # KMeans.scala:113 predicts with the *updated* model
        pred = find_closest(self.state.centers, Xs) if Xs.shape[0] else np.zeros(0, np.int64)
        return {"n": int(n), "labels": labels, "pred": pred, "std": std, "scaled": Xs}
