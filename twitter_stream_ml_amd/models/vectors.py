"""``mllib.linalg`` / ``mllib.regression.LabeledPoint`` equivalents (fp64).

Semantics the reference relies on: ``Vectors.sparse(size,
indices, values)`` with ascending indices, ``Vectors.dense``,
``Vectors.zeros(n)``; everything fp64.  ``dot`` follows MLlib's BLAS.dot
(sparse·dense iterates the sparse side).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Iterable, Sequence, Union

import numpy as np

__all__ = ["Vector", "DenseVector", "SparseVector", "Vectors", "LabeledPoint"]


class Vector:
    size: int

    def toArray(self) -> np.ndarray:  # pragma: no cover - abstract
        raise NotImplementedError

    def dot(self, other: "Vector") -> float:
        return vec_dot(self, other)

    def __len__(self) -> int:
        return self.size


class DenseVector(Vector):
    __slots__ = ("values",)

    def __init__(self, values: Iterable[float]):
        self.values = np.asarray(values, dtype=np.float64).reshape(-1)

    @property
    def size(self) -> int:
        return int(self.values.shape[0])

    def toArray(self) -> np.ndarray:
        return self.values

    def __getitem__(self, i: int) -> float:
        return float(self.values[i])

    apply = __getitem__

    def __eq__(self, other: object) -> bool:
        return isinstance(other, Vector) and np.array_equal(self.toArray(), other.toArray())

    def __repr__(self) -> str:
        return "[" + ",".join(repr(float(v)) for v in self.values) + "]"


class SparseVector(Vector):
    __slots__ = ("_size", "indices", "values")

    def __init__(self, size: int, indices: Iterable[int], values: Iterable[float]):
        self._size = int(size)
        self.indices = np.asarray(indices, dtype=np.int64).reshape(-1)
        self.values = np.asarray(values, dtype=np.float64).reshape(-1)
        if self.indices.shape != self.values.shape:
            raise ValueError("indices and values must have the same length")
        if self.indices.shape[0] and (np.any(np.diff(self.indices) <= 0)
                                      or self.indices[0] < 0 or self.indices[-1] >= self._size):
            raise ValueError("sparse indices must be strictly increasing and within size")

    @property
    def size(self) -> int:
        return self._size

    def toArray(self) -> np.ndarray:
        out = np.zeros(self._size, np.float64)
        out[self.indices] = self.values
        return out

    def __getitem__(self, i: int) -> float:
        j = np.searchsorted(self.indices, i)
        if j < self.indices.shape[0] and self.indices[j] == i:
            return float(self.values[j])
        return 0.0

    apply = __getitem__

    def __eq__(self, other: object) -> bool:
        return isinstance(other, Vector) and self.size == other.size and np.array_equal(
            self.toArray(), other.toArray())

    def __repr__(self) -> str:
        return f"({self._size},{list(self.indices)},{list(self.values)})"


def vec_dot(a: Vector, b: Vector) -> float:
    if a.size != b.size:
        raise ValueError(f"dot: size mismatch {a.size} vs {b.size}")
    if isinstance(a, SparseVector) and isinstance(b, SparseVector):
        common, ia, ib = np.intersect1d(a.indices, b.indices, assume_unique=True,
                                        return_indices=True)
        return float(np.dot(a.values[ia], b.values[ib]))
    if isinstance(a, SparseVector):
        return float(np.dot(a.values, b.toArray()[a.indices]))
    if isinstance(b, SparseVector):
        return float(np.dot(b.values, a.toArray()[b.indices]))
    return float(np.dot(a.toArray(), b.toArray()))


class Vectors:
    @staticmethod
    def dense(*values: Union[float, Sequence[float], np.ndarray]) -> DenseVector:
        if len(values) == 1 and not np.isscalar(values[0]):
            return DenseVector(values[0])
        return DenseVector(values)

    @staticmethod
    def sparse(size: int, indices: Iterable[int], values: Iterable[float]) -> SparseVector:
        return SparseVector(size, indices, values)

    @staticmethod
    def zeros(n: int) -> DenseVector:
        return DenseVector(np.zeros(int(n), np.float64))


@dataclass
class LabeledPoint:
    label: float
    features: Vector

    def __repr__(self) -> str:
        return f"({self.label},{self.features!r})"
