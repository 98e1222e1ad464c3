"""HashingTF over character bigrams (K1 on the CPU side).

Reference semantics: ``MllibHelper.featurizeText`` lower-cases the original
tweet text, takes ``text.sliding(2)`` and feeds the bigrams to a Spark-1.6
``HashingTF`` (``MllibHelper.scala:42-56``).  In Spark 1.6
``HashingTF.indexOf(term) = Utils.nonNegativeMod(term.##, numFeatures)`` and
``transform`` sums 1.0 per term occurrence into a sparse vector with sorted
indices [upstream ``mllib/feature/HashingTF.scala``].

For a 2-code-unit Java string ``##`` is ``String.hashCode = 31*c0 + c1``
(UTF-16 code units), so a bigram hash is always in ``[0, 2_097_120]`` and never
overflows.  ``"x".sliding(2)`` yields the single 1-char term (hash ``c0``); the
empty string yields no term.

``hash="murmur3"`` selects Spark 2.x's ``HashingTF`` hash instead
(``Murmur3_x86_32.hashUnsafeBytes`` of the UTF-8 bytes, seed 42), useful for
very wide feature spaces where Java-hash bigrams would only ever reach the
first ~2.1M indices (long-context row).

Lower-casing: Java ``String.toLowerCase`` is approximated by Python's
``str.lower`` — both implement full case mapping (U+0130 -> "i̇") and the
Final_Sigma context.  Known divergences (parity unpinned): Java 7 uses Unicode
6.0 tables and bounds the Final_Sigma scan with a word ``BreakIterator``.
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Sequence, Tuple

import numpy as np

from .vectors import SparseVector

__all__ = ["HashingTF", "java_lower", "java_string_hash", "non_negative_mod",
           "bigram_hashes", "bigram_terms", "murmur3_spark_hash", "text_units"]


def java_lower(text: str) -> str:
    return text.lower()


def text_units(text: str) -> np.ndarray:
    return np.frombuffer(text.encode("utf-16-le", "surrogatepass"), dtype="<u2")


def java_string_hash(units: Sequence[int]) -> int:
    """``java.lang.String.hashCode`` of a code-unit sequence (signed 32-bit)."""
    h = 0
    for u in units:
        h = (31 * h + int(u)) & 0xFFFFFFFF
    return h - (1 << 32) if h >= (1 << 31) else h


def non_negative_mod(x: int, mod: int) -> int:
    """``org.apache.spark.util.Utils.nonNegativeMod`` (Java ``%`` then fix)."""
    raw = int(np.fmod(x, mod)) if x < 0 else x % mod
    return raw + mod if raw < 0 else raw


def bigram_hashes(units: np.ndarray) -> np.ndarray:
    """Java hashCodes of ``text.sliding(2)`` terms, vectorised (int64)."""
    u = np.asarray(units, dtype=np.int64)
    if u.shape[0] >= 2:
        return 31 * u[:-1] + u[1:]
    return u.copy()  # 1 unit -> single 1-char term; 0 units -> no terms


def bigram_terms(units: np.ndarray) -> List[Tuple[int, ...]]:
    u = [int(x) for x in units]
    if len(u) >= 2:
        return [(u[i], u[i + 1]) for i in range(len(u) - 1)]
    return [tuple(u)] if u else []


# -- Spark 2.x murmur3 ------------------------------------------------------
_C1, _C2 = 0xCC9E2D51, 0x1B873593
_M32 = 0xFFFFFFFF


def _rotl(x: int, r: int) -> int:
    return ((x << r) | (x >> (32 - r))) & _M32


def _mix_k1(k1: int) -> int:
    k1 = (k1 * _C1) & _M32
    k1 = _rotl(k1, 15)
    return (k1 * _C2) & _M32


def _mix_h1(h1: int, k1: int) -> int:
    h1 ^= k1
    h1 = _rotl(h1, 13)
    return (h1 * 5 + 0xE6546B64) & _M32


def _fmix(h1: int, length: int) -> int:
    h1 ^= length
    h1 ^= h1 >> 16
    h1 = (h1 * 0x85EBCA6B) & _M32
    h1 ^= h1 >> 13
    h1 = (h1 * 0xC2B2AE35) & _M32
    h1 ^= h1 >> 16
    return h1


def murmur3_spark_hash(data: bytes, seed: int = 42) -> int:
    """``Murmur3_x86_32.hashUnsafeBytes`` (Spark's non-standard tail handling).

    Whole 4-byte little-endian words are mixed normally; each trailing byte is
    then mixed as a full (sign-extended) int, as Spark < 2.3 compatibility
    requires.  Returns a signed 32-bit int.
    """
    h1 = seed & _M32
    n = len(data)
    aligned = n - n % 4
    for i in range(0, aligned, 4):
        k = int.from_bytes(data[i:i + 4], "little")
        h1 = _mix_h1(h1, _mix_k1(k))
    for i in range(aligned, n):
        b = data[i]
        b = b - 256 if b >= 128 else b
        h1 = _mix_h1(h1, _mix_k1(b & _M32))
    h = _fmix(h1, n)
    return h - (1 << 32) if h >= (1 << 31) else h


def _term_utf8(term_units: Tuple[int, ...]) -> bytes:
    s = np.asarray(term_units, dtype="<u2").tobytes().decode("utf-16-le", "surrogatepass")
    # Java's UTF-8 encoder writes '?' for an unpaired surrogate.
    return s.encode("utf-8", "replace")


class HashingTF:
    """``org.apache.spark.mllib.feature.HashingTF`` (Spark 1.6 / 2.x hash)."""

    def __init__(self, numFeatures: int = 1 << 20, hash: str = "java"):
        if numFeatures <= 0:
            raise ValueError("numFeatures must be positive")
        if hash not in ("java", "murmur3"):
            raise ValueError(f"unknown hash {hash!r}")
        self.numFeatures = int(numFeatures)
        self.hash = hash

    def indexOf(self, term) -> int:
        """Index of a term: a ``str`` or a tuple of UTF-16 code units."""
        units = tuple(text_units(term)) if isinstance(term, str) else tuple(term)
        if self.hash == "java":
            h = java_string_hash(units)
        else:
            h = murmur3_spark_hash(_term_utf8(units))
        return non_negative_mod(h, self.numFeatures)

    def transform(self, terms: Iterable) -> SparseVector:
        tf: Dict[int, float] = {}
        for t in terms:
            i = self.indexOf(t)
            tf[i] = tf.get(i, 0.0) + 1.0
        idx = np.array(sorted(tf), dtype=np.int64)
        return SparseVector(self.numFeatures, idx, np.array([tf[i] for i in idx], np.float64))

    def bigram_indices(self, units: np.ndarray) -> np.ndarray:
        """Hash index of every bigram occurrence (duplicates kept), int64."""
        if self.hash == "java":
            return bigram_hashes(units) % self.numFeatures  # hashes are >= 0
        return np.array([self.indexOf(t) for t in bigram_terms(units)], dtype=np.int64)

    def transform_text(self, lowered_text: str) -> SparseVector:
        """``transform(text.sliding(2).toSeq)`` for an already lower-cased text."""
        idx = self.bigram_indices(text_units(lowered_text))
        uniq, counts = np.unique(idx, return_counts=True)
        return SparseVector(self.numFeatures, uniq, counts.astype(np.float64))
