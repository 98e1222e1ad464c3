"""Columnar fp64 featurization of a :class:`RawBatch` (K1+K2+K3 oracle).

Produces exactly what ``stream.filter(MllibHelper.filtrate).map(
MllibHelper.featurize)`` produces for the batch (``LinearRegression.scala:
44-47``), as one CSR matrix of shape ``(n_kept, F + 4)`` plus labels, so the
CPU engine can run the SGD with sparse BLAS and the HIP kernels can be
checked entry-for-entry.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np
import scipy.sparse as sp

from ..models.hashing_tf import HashingTF, java_lower, text_units
from ..models.mllib_helper import NUMBER_SCALES
from ..records.batch import (CREATED_AT, FAVOURITES, FOLLOWERS, FRIENDS, RETWEET_COUNT,
                             RawBatch, units_to_str)

__all__ = ["FeaturizedBatch", "filter_mask", "featurize_batch", "featurize_batch_native", "lowered_units"]


@dataclass
class FeaturizedBatch:
    X: sp.csr_matrix          # (n_kept, F + 4) fp64, duplicates summed, sorted indices
    y: np.ndarray             # (n_kept,) fp64 labels (original retweet counts)
    rows: np.ndarray          # (n_kept,) row ids in the raw batch
    num_text_features: int

    @property
    def n(self) -> int:
        return int(self.y.shape[0])


def filter_mask(raw: RawBatch, begin: int, end: int) -> np.ndarray:
    rc = raw.scalars[RETWEET_COUNT]
    return (raw.is_retweet != 0) & (rc >= begin) & (rc <= end)


def lowered_units(raw: RawBatch, i: int) -> np.ndarray:
    raw.ensure_text()
    return text_units(java_lower(units_to_str(raw.text[raw.offsets[i]:raw.offsets[i + 1]])))


def featurize_batch(raw: RawBatch, num_text_features: int, begin: int, end: int,
                    now_ms: Optional[int] = None, hash: str = "java",
                    apply_filter: bool = True) -> FeaturizedBatch:
    F = int(num_text_features)
    now = raw.batch_time_ms if now_ms is None else int(now_ms)
    mask = filter_mask(raw, begin, end) if apply_filter else np.ones(raw.n, bool)
    rows = np.nonzero(mask)[0].astype(np.int64)
    tf = HashingTF(F, hash)
    indptr = np.zeros(rows.shape[0] + 1, np.int64)
    idx_parts = []
    val_parts = []
    for j, r in enumerate(rows):
        idx = tf.bigram_indices(lowered_units(raw, int(r)))
        uniq, counts = np.unique(idx, return_counts=True)
        sc = raw.scalars[:, r]
        nums = np.array([sc[FOLLOWERS] * NUMBER_SCALES[0], sc[FAVOURITES] * NUMBER_SCALES[1],
                         sc[FRIENDS] * NUMBER_SCALES[2],
                         (now - int(sc[CREATED_AT])) * NUMBER_SCALES[3]], np.float64)
        idx_parts.append(np.concatenate([uniq, np.arange(F, F + 4)]))
        val_parts.append(np.concatenate([counts.astype(np.float64), nums]))
        indptr[j + 1] = indptr[j] + idx_parts[-1].shape[0]
    indices = np.concatenate(idx_parts) if idx_parts else np.zeros(0, np.int64)
    values = np.concatenate(val_parts) if val_parts else np.zeros(0, np.float64)
    X = sp.csr_matrix((values, indices, indptr), shape=(rows.shape[0], F + 4))
    y = raw.scalars[RETWEET_COUNT, rows].astype(np.float64)
    return FeaturizedBatch(X, y, rows, F)


def featurize_batch_native(raw: RawBatch, num_text_features: int, begin: int, end: int,
                           now_ms: Optional[int] = None, hash: str = "java",
                           apply_filter: bool = True) -> FeaturizedBatch:
    """Same result as :func:`featurize_batch`, with the bigram hashing done by
    the host C++ featurizer (``csrc/host/featurize_cpu.cpp``: full case
    mapping of special rows, Java / murmur3 hashing; checked against the
    Python path in ``tests/test_oracle.py``) -- for oracle runs over
    bench-sized batches (10^5-10^6 rows)."""
    from ..ops._native import host
    F = int(num_text_features)
    now = raw.batch_time_ms if now_ms is None else int(now_ms)
    mask = filter_mask(raw, begin, end) if apply_filter else np.ones(raw.n, bool)
    rows = np.nonzero(mask)[0].astype(np.int64)
    raw.ensure_text()   # a replayed batch may carry only its UTF-8 bytes
    indptr, indices = host().featurize_rows(raw.text, raw.offsets, rows, F, hash)
    n = rows.shape[0]
    T = sp.csr_matrix((np.ones(indices.shape[0]), indices, indptr), shape=(n, F))
    T.sum_duplicates()   # term counts, sorted indices
    sc = raw.scalars[:, rows]
    nums = np.stack([sc[FOLLOWERS] * NUMBER_SCALES[0], sc[FAVOURITES] * NUMBER_SCALES[1],
                     sc[FRIENDS] * NUMBER_SCALES[2], (now - sc[CREATED_AT]) * NUMBER_SCALES[3]],
                    axis=1).astype(np.float64)
    X = sp.hstack([T, sp.csr_matrix(nums)], format="csr")
    y = raw.scalars[RETWEET_COUNT, rows].astype(np.float64)
    return FeaturizedBatch(X, y, rows, F)
