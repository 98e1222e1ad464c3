"""Micro-batch dataset: the slice of Spark's ``RDD`` API the jobs use.

The reference calls ``count``, ``isEmpty``, ``map``, ``filter``, ``take``,
``collect``/``toArray``, ``stdev``, ``mean`` and ``first`` on each batch RDD
(``LinearRegression.scala:54-77``; ``KMeans.scala:101-113``).  A
micro-batch lives in one process here (the data-parallel split is one process
per GPU, not partitions), so an :class:`RDD` is a lazily transformed Python
sequence with Spark's action semantics (``stdev`` is the *population* stdev).
``raw`` carries the columnar :class:`RawBatch` the batch came from, so native
operators can bypass the per-record Python path.
"""
from __future__ import annotations

import math
from typing import Any, Callable, Generic, Iterable, Iterator, List, Optional, Sequence, TypeVar

import numpy as np

T = TypeVar("T")
U = TypeVar("U")

__all__ = ["RDD"]


class RDD(Generic[T]):
    def __init__(self, data: Iterable[T] | Callable[[], Iterable[T]], raw=None, num_slices: int = 1):
        self._src = data
        self._cache: Optional[List[T]] = None
        self.raw = raw
        self.num_slices = max(1, int(num_slices))

    # ---- evaluation ----------------------------------------------------
    def _iter(self) -> Iterator[T]:
        if self._cache is not None:
            return iter(self._cache)
        src = self._src() if callable(self._src) else self._src
        return iter(src)

    def _list(self) -> List[T]:
        if self._cache is not None:
            return self._cache
        return list(self._iter())

    def cache(self) -> "RDD[T]":
        if self._cache is None:
            self._cache = list(self._iter())
        return self

    persist = cache

    # ---- transformations (lazy) --------------------------------------------
    def map(self, f: Callable[[T], U]) -> "RDD[U]":
        return RDD(lambda: (f(x) for x in self._iter()), self.raw, self.num_slices)

    def filter(self, f: Callable[[T], bool]) -> "RDD[T]":
        return RDD(lambda: (x for x in self._iter() if f(x)), None, self.num_slices)

    def flatMap(self, f: Callable[[T], Iterable[U]]) -> "RDD[U]":
        return RDD(lambda: (y for x in self._iter() for y in f(x)), None, self.num_slices)

    def zip(self, other: "RDD[U]") -> "RDD[tuple]":
        return RDD(lambda: zip(self._iter(), other._iter()), None, self.num_slices)

    def sample(self, with_replacement: bool, fraction: float, seed: int = 0) -> "RDD[T]":
        if with_replacement:
            raise NotImplementedError("sampling with replacement")
        rng = np.random.default_rng(seed)
        return RDD(lambda: (x for x in self._iter() if rng.random() < fraction), None,
                   self.num_slices)

    # ---- actions ---------------------------------------------------------
    def collect(self) -> List[T]:
        return self._list()

    def toArray(self) -> np.ndarray:
        return np.asarray(self._list())

    def count(self) -> int:
        if self._cache is not None:
            return len(self._cache)
        return sum(1 for _ in self._iter())

    def isEmpty(self) -> bool:
        for _ in self._iter():
            return False
        return True

    def first(self) -> T:
        for x in self._iter():
            return x
        raise ValueError("empty collection")

    def take(self, n: int) -> List[T]:
        out = []
        for x in self._iter():
            if len(out) >= n:
                break
            out.append(x)
        return out

    def reduce(self, f: Callable[[T, T], T]) -> T:
        it = self._iter()
        try:
            acc = next(it)
        except StopIteration:
            raise ValueError("empty collection") from None
        for x in it:
            acc = f(acc, x)
        return acc

    def foreach(self, f: Callable[[T], Any]) -> None:
        for x in self._iter():
            f(x)

    def sum(self) -> float:
        return float(np.sum(np.asarray(self._list(), dtype=np.float64)))

    def mean(self) -> float:
        v = np.asarray(self._list(), dtype=np.float64)
        return float(v.mean()) if v.size else float("nan")

    def stdev(self) -> float:
        """Population standard deviation (``DoubleRDDFunctions.stdev``)."""
        v = np.asarray(self._list(), dtype=np.float64)
        return float(v.std()) if v.size else float("nan")

    def sampleStdev(self) -> float:
        v = np.asarray(self._list(), dtype=np.float64)
        return float(v.std(ddof=1)) if v.size > 1 else float("nan")

    def __len__(self) -> int:
        return self.count()

    def __repr__(self) -> str:  # pragma: no cover
        return f"RDD(cached={self._cache is not None})"
