"""fp64 golden oracle of the MLlib 1.6.1 semantics the reference executes.

Every function here is the CPU ("plumbing", ``--master local[N]``) engine and
the reference the HIP kernels are tested against (SURVEY §4 "Implications",
§7.2 step 3).  Upstream semantics implemented:

* U5  ``GradientDescent.runMiniBatchSGD`` — full-batch (or Bernoulli-sampled)
  gradient per iteration, ``w -= (stepSize/sqrt(i)) * g/m``, convergence
  ``||w_i - w_{i-1}|| < tol * max(||w_i||, 1)`` checked once two updates
  exist, early return of the initial weights on an empty batch.
* U6  ``LeastSquaresGradient`` — ``diff = x.w - y``, ``g += diff*x``,
  ``loss += diff^2/2``.
* U7  ``SimpleUpdater`` — no regularisation.
* U8/U9 ``StreamingKMeansModel.update`` / ``findClosest`` — decay, weighted
  centroid update, dying-cluster split; first index wins ties.
* U10 ``StandardScaler(withMean=false, withStd=true)`` — sample variance.
* U11 ``StatCounter`` — population ``stdev``, ``mean``.
* ``Utils.round`` (``spark/.../Utils.scala:3-7``) — HALF_UP on the decimal
  value, i.e. half away from zero; non-finite input throws.

Data-parallel execution (SURVEY §2.4 DP row): every reduction takes an
optional ``allreduce`` callable summing a float64 vector across ranks, so the
same code runs single-process or sharded over ``torch.distributed`` (gloo on
CPU).  ``row_offset`` gives each rank's global row ids so Bernoulli sampling
is identical to the single-process run on the concatenated batch.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np
import scipy.sparse as sp

__all__ = [
    "round_half_up", "round_half_up_array", "StatCounter", "sgd_uniform",
    "SGDResult", "run_minibatch_sgd", "run_minibatch_sgd_active", "least_squares_gradient", "KMeansState",
    "find_closest", "kmeans_update", "standard_scaler_fit", "standard_scaler_transform",
    "decay_factor_from_half_life", "CONVERGENCE_TOL",
]

CONVERGENCE_TOL = 1e-3
AllReduce = Optional[Callable[[np.ndarray], np.ndarray]]


# ---------------------------------------------------------------------------
# Utils.round
# ---------------------------------------------------------------------------
def round_half_up(x: float) -> float:
    """``BigDecimal(x).setScale(0, HALF_UP).toDouble`` — half away from zero."""
    if not math.isfinite(x):
        raise ValueError(f"Utils.round: cannot round {x}")  # NumberFormatException
    t = math.trunc(x)
    frac = abs(x - t)          # exact in binary floating point
    if frac >= 0.5:
        t += 1 if x > 0 else -1
    return float(t)


def round_half_up_array(x: np.ndarray) -> np.ndarray:
    x = np.asarray(x, dtype=np.float64)
    if not np.all(np.isfinite(x)):
        raise ValueError("Utils.round: non-finite prediction")
    t = np.trunc(x)
    return t + np.where(np.abs(x - t) >= 0.5, np.sign(x), 0.0)


# ---------------------------------------------------------------------------
# StatCounter (population stdev) with a mergeable moment form
# ---------------------------------------------------------------------------
@dataclass
class StatCounter:
    n: int = 0
    mu: float = 0.0
    m2: float = 0.0

    @classmethod
    def of(cls, values: np.ndarray) -> "StatCounter":
        v = np.asarray(values, dtype=np.float64)
        if v.size == 0:
            return cls()
        mu = float(v.mean())
        return cls(int(v.size), mu, float(((v - mu) ** 2).sum()))

    def merge(self, o: "StatCounter") -> "StatCounter":
        if o.n == 0:
            return StatCounter(self.n, self.mu, self.m2)
        if self.n == 0:
            return StatCounter(o.n, o.mu, o.m2)
        n = self.n + o.n
        d = o.mu - self.mu
        return StatCounter(n, self.mu + d * o.n / n, self.m2 + o.m2 + d * d * self.n * o.n / n)

    @property
    def count(self) -> int:
        return self.n

    def mean(self) -> float:
        return self.mu if self.n else float("nan")

    def variance(self) -> float:
        return self.m2 / self.n if self.n else float("nan")

    def stdev(self) -> float:
        return math.sqrt(self.variance())

    def sampleStdev(self) -> float:
        return math.sqrt(self.m2 / (self.n - 1)) if self.n > 1 else float("nan")


# ---------------------------------------------------------------------------
# Bernoulli sampling used for miniBatchFraction < 1
# ---------------------------------------------------------------------------
_M64 = (1 << 64) - 1


def _splitmix64(x: np.ndarray) -> np.ndarray:
    x = (x + np.uint64(0x9E3779B97F4A7C15)) & np.uint64(_M64)
    x = ((x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & np.uint64(_M64)
    x = ((x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & np.uint64(_M64)
    return x ^ (x >> np.uint64(31))


def sgd_uniform(seed: int, global_rows: np.ndarray) -> np.ndarray:
    """Counter-based U[0,1) per (seed, global row id); the HIP kernel computes
    the identical bits (``csrc/hip/common.h: sample_uniform``).

    Spark samples with ``XORShiftRandom(seed + partitionIndex)``; that stream
    depends on the partition layout, so exact parity is unpinned — the
    sampling *distribution* (Bernoulli(fraction), seed 42+i) is kept.
    """
    with np.errstate(over="ignore"):
        key = (np.asarray(global_rows, dtype=np.uint64)
               ^ (np.uint64(seed & _M64) * np.uint64(0xD1B54A32D192ED03)))
        bits = _splitmix64(key)
    return (bits >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))


# ---------------------------------------------------------------------------
# GradientDescent.runMiniBatchSGD with LeastSquaresGradient + SimpleUpdater
# ---------------------------------------------------------------------------
def least_squares_gradient(X: sp.csr_matrix, y: np.ndarray, w: np.ndarray,
                           mask: Optional[np.ndarray] = None) -> Tuple[np.ndarray, float, int]:
    """Sum of LeastSquaresGradient over (sampled) rows: (g, loss, m)."""
    if mask is not None:
        X = X[mask]
        y = y[mask]
    diff = X @ w - y
    g = X.T @ diff
    return np.asarray(g, dtype=np.float64).reshape(-1), float(0.5 * diff @ diff), int(y.shape[0])


@dataclass
class SGDResult:
    weights: np.ndarray
    loss_history: List[float] = field(default_factory=list)
    iterations: int = 0           # iterations executed (i at exit - 1)
    converged: bool = False
    num_examples: int = 0


def run_minibatch_sgd(X: sp.csr_matrix, y: np.ndarray, w0: np.ndarray, step_size: float,
                      num_iterations: int, mini_batch_fraction: float = 1.0,
                      convergence_tol: float = CONVERGENCE_TOL, allreduce: AllReduce = None,
                      row_offset: int = 0) -> SGDResult:
    """``GradientDescent.runMiniBatchSGD`` [upstream mllib/optimization].

    ``X``/``y`` are this rank's rows; with ``allreduce`` the gradient, loss,
    sample count and the example count are summed across ranks.
    """
    if mini_batch_fraction > 1.0 + 1e-12 or mini_batch_fraction <= 0:
        raise ValueError(f"miniBatchFraction must be in (0, 1], got {mini_batch_fraction}")
    red = allreduce if allreduce is not None else (lambda v: v)
    n_local = int(y.shape[0])
    num_examples = int(round(red(np.array([float(n_local)]))[0]))
    w = np.array(w0, dtype=np.float64, copy=True)
    res = SGDResult(w, num_examples=num_examples)
    if num_examples == 0:
        return res                                # "returning initial weights"
    prev: Optional[np.ndarray] = None
    cur: Optional[np.ndarray] = None
    converged = False
    i = 1
    rows = np.arange(row_offset, row_offset + n_local, dtype=np.uint64)
    while not converged and i <= num_iterations:
        mask = None
        if mini_batch_fraction < 1.0:
            mask = sgd_uniform(42 + i, rows) < mini_batch_fraction
        g, loss, m = least_squares_gradient(X, y, w, mask)
        packed = red(np.concatenate([g, [loss, float(m)]]))
        g, loss, m = packed[:-2], packed[-2], int(round(packed[-1]))
        if m > 0:
            res.loss_history.append(loss / m)
            w = w - (step_size / math.sqrt(i)) * (g / m)
            prev, cur = cur, w
            if prev is not None and cur is not None:
                diff = float(np.linalg.norm(prev - cur))
                converged = diff < convergence_tol * max(float(np.linalg.norm(cur)), 1.0)
        i += 1
    res.weights = w
    res.iterations = i - 1
    res.converged = converged
    return res


def run_minibatch_sgd_active(X: sp.csr_matrix, y: np.ndarray, w0: np.ndarray, step_size: float,
                             num_iterations: int, convergence_tol: float = CONVERGENCE_TOL) -> SGDResult:
    """:func:`run_minibatch_sgd` (miniBatchFraction 1, one rank) on the
    columns the batch touches.  Untouched columns have a zero gradient, so
    their weights never move; ``||w||`` adds their constant norm.  Same
    iterates as the full-width loop (up to fp64 summation order), at a cost
    independent of the feature width -- the oracle for F = 1e8 batches."""
    cols = np.unique(X.indices)
    Xc = X[:, cols].tocsr()
    w = np.array(w0, dtype=np.float64, copy=True)
    wc = w[cols].copy()
    rest2 = max(float(np.dot(w, w)) - float(np.dot(wc, wc)), 0.0)
    res = SGDResult(w, num_examples=int(y.shape[0]))
    if y.shape[0] == 0:
        return res
    prev = None
    converged = False
    i = 1
    while not converged and i <= num_iterations:
        diff = Xc @ wc - y
        g = np.asarray(Xc.T @ diff, dtype=np.float64).reshape(-1)
        m = int(y.shape[0])
        res.loss_history.append(float(0.5 * diff @ diff) / m)
        new = wc - (step_size / math.sqrt(i)) * (g / m)
        if prev is not None or i > 1:
            d = float(np.linalg.norm(new - wc))
            converged = d < convergence_tol * max(math.sqrt(float(new @ new) + rest2), 1.0)
        prev, wc = wc, new
        i += 1
    w[cols] = wc
    res.weights = w
    res.iterations = i - 1
    res.converged = converged
    return res


# ---------------------------------------------------------------------------
# StandardScaler(withMean = false, withStd = true)
# ---------------------------------------------------------------------------
def standard_scaler_fit(X: np.ndarray, allreduce: AllReduce = None) -> np.ndarray:
    """Column std with the n-1 denominator (``MultivariateOnlineSummarizer``).

    Two-pass and DP-safe: global mean first, then the centred sum of squares.
    Returns ``std`` (0 where n < 2).
    """
    red = allreduce if allreduce is not None else (lambda v: v)
    X = np.asarray(X, dtype=np.float64)
    d = X.shape[1]
    s = red(np.concatenate([[float(X.shape[0])], X.sum(axis=0)]))
    n = s[0]
    if n < 2:
        return np.zeros(d)
    mean = s[1:] / n
    m2 = red(((X - mean) ** 2).sum(axis=0))
    return np.sqrt(m2 / (n - 1.0))


def standard_scaler_transform(X: np.ndarray, std: np.ndarray) -> np.ndarray:
    factor = np.where(std != 0.0, 1.0 / np.where(std != 0.0, std, 1.0), 0.0)
    return np.asarray(X, dtype=np.float64) * factor


# ---------------------------------------------------------------------------
# StreamingKMeans
# ---------------------------------------------------------------------------
def decay_factor_from_half_life(half_life: float) -> float:
    """``setHalfLife(h, "batches")``: ``exp(ln(0.5)/h)`` (0.8706 for h=5)."""
    return math.exp(math.log(0.5) / half_life)


@dataclass
class KMeansState:
    centers: np.ndarray   # (k, d) fp64
    weights: np.ndarray   # (k,)  fp64

    @classmethod
    def random(cls, k: int, dim: int, weight: float, seed: int) -> "KMeansState":
        rng = np.random.default_rng(seed)
        return cls(rng.standard_normal((k, dim)), np.full(k, float(weight)))

    def copy(self) -> "KMeansState":
        return KMeansState(self.centers.copy(), self.weights.copy())


def find_closest(centers: np.ndarray, X: np.ndarray) -> np.ndarray:
    """argmin_k ||x - c_k||^2, first index on ties (``KMeans.findClosest``)."""
    X = np.asarray(X, dtype=np.float64)
    d2 = ((X[:, None, :] - centers[None, :, :]) ** 2).sum(axis=2) if X.shape[0] * centers.shape[0] \
        <= 4_000_000 else (np.sum(X * X, 1)[:, None] - 2 * X @ centers.T + np.sum(centers ** 2, 1)[None])
    return np.argmin(d2, axis=1).astype(np.int64)


def kmeans_update(state: KMeansState, X: np.ndarray, decay: float, time_unit: str = "batches",
                  allreduce: AllReduce = None) -> Tuple[KMeansState, np.ndarray]:
    """``StreamingKMeansModel.update(data, decayFactor, timeUnit)``.

    Returns the new state and the labels assigned (with the *old* centres).
    """
    red = allreduce if allreduce is not None else (lambda v: v)
    k, d = state.centers.shape
    X = np.asarray(X, dtype=np.float64)
    labels = find_closest(state.centers, X) if X.shape[0] else np.zeros(0, np.int64)
    sums = np.zeros((k, d))
    np.add.at(sums, labels, X)
    counts = np.bincount(labels, minlength=k).astype(np.float64)
    packed = red(np.concatenate([sums.reshape(-1), counts]))
    sums = packed[:k * d].reshape(k, d)
    counts = packed[k * d:]
    if time_unit == "batches":
        discount = decay
    elif time_unit == "points":
        discount = decay ** counts.sum()
    else:
        raise ValueError(f"unknown time unit {time_unit}")
    centers = state.centers.copy()
    weights = state.weights * discount
    for label in range(k):
        cnt = counts[label]
        if cnt <= 0:
            continue  # only clusters present in pointStats are updated
        updated = weights[label] + cnt
        lam = cnt / max(updated, 1e-16)
        weights[label] = updated
        centers[label] = (1.0 - lam) * centers[label] + (lam / cnt) * sums[label]
    largest = int(np.argmax(weights))
    smallest = int(np.argmin(weights))
    max_w, min_w = weights[largest], weights[smallest]
    if min_w < 1e-8 * max_w:
        w = (max_w + min_w) / 2.0
        weights[largest] = w
        weights[smallest] = w
        x = centers[largest].copy()
        p = 1e-14 * np.maximum(np.abs(x), 1.0)
        centers[largest] = x + p
        centers[smallest] = x - p
    return KMeansState(centers, weights), labels
