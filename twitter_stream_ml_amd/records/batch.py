"""Columnar micro-batch of raw tweets (host side).

A :class:`RawBatch` is what a receiver seals every interval: struct-of-arrays
scalars plus the *original* tweet texts as one ragged UTF-16 buffer with CSR
offsets.  It is the unit that crosses PCIe to the GPU (SURVEY §7.1
``records/``; U14/U15).  Text is stored as UTF-16 **code units** because Java
strings are UTF-16 and the reference's bigrams are ``String.sliding(2)`` over
code units.

Scalar rows (``scalars[k]``), all of the *retweeted* (original) status, as the
reference reads them through ``getRetweetedStatus`` (``MllibHelper.scala:43,59,
81,85``):

====  ======================  ==========================================
row   name                    source
====  ======================  ==========================================
0     retweet_count           ``getRetweetCount`` (label, filter)
1     followers               ``getUser.getFollowersCount``
2     favourites              ``getUser.getFavouritesCount``
3     friends                 ``getUser.getFriendsCount``
4     created_at_ms           ``getCreatedAt.getTime``
====  ======================  ==========================================

``is_retweet`` is separate (uint8).  For non-retweets the scalar/text columns
hold the tweet's own fields; every consumer filters on ``is_retweet`` first.

A receiver may also hand over the text as it holds it -- UTF-8 bytes
(:class:`Utf8Text`, the form the network delivers) -- in ``utf8``; the device
engines then DMA those bytes and decode on the GPU.  Such a batch may leave
``text`` empty (``offsets`` still count UTF-16 units); :meth:`ensure_text`
decodes it on demand for host consumers.
"""
from __future__ import annotations

from dataclasses import dataclass, replace
from typing import Iterable, List, Optional, Sequence

import numpy as np

from .schema import Status, User

__all__ = ["RawBatch", "Utf8Text", "SCALAR_FIELDS", "RETWEET_COUNT", "FOLLOWERS", "FAVOURITES",
           "FRIENDS", "CREATED_AT", "utf16_units", "units_to_str"]

RETWEET_COUNT, FOLLOWERS, FAVOURITES, FRIENDS, CREATED_AT = range(5)
SCALAR_FIELDS = ("retweet_count", "followers", "favourites", "friends", "created_at_ms")


def utf16_units(s: str) -> np.ndarray:
    """Java ``String`` code units of ``s`` (surrogate pairs for astral chars)."""
    return np.frombuffer(s.encode("utf-16-le", "surrogatepass"), dtype="<u2")


def units_to_str(units: np.ndarray) -> str:
    return np.asarray(units, dtype="<u2").tobytes().decode("utf-16-le", "surrogatepass")


@dataclass
class Utf8Text:
    """A batch's tweet text as UTF-8 bytes + byte offsets [n+1]: the form a
    network receiver holds (the Twitter stream delivers UTF-8 JSON).
    ``pinned``: the bytes are page-locked (``register_host``), so the engines
    DMA them without a staging copy."""
    data: np.ndarray      # uint8 [bytes]
    offsets: np.ndarray   # int64 [n + 1]
    pinned: bool = False

    @property
    def nbytes(self) -> int:
        return int(self.offsets[-1]) if self.offsets.shape[0] else 0


@dataclass
class RawBatch:
    text: np.ndarray          # uint16 [total_units] (may be empty when utf8 holds the text)
    offsets: np.ndarray       # int64  [n+1], UTF-16 units
    is_retweet: np.ndarray    # uint8  [n]
    scalars: np.ndarray       # int64  [5, n]
    batch_time_ms: int = 0    # seal time ("now" for featurizeNumbers)
    utf8: Optional[Utf8Text] = None   # the receiver's UTF-8 bytes of the same text
    # int64 [2, 5]: per-column min / max of ``scalars``, recorded by the
    # receiver while it sealed the batch (:meth:`with_scalar_range`); the host
    # staging encodes the wire columns from it in one pass and checks every
    # value against it (a wrong range costs a second pass, never correctness)
    scalar_range: Optional[np.ndarray] = None

    def __post_init__(self) -> None:
        self.text = np.ascontiguousarray(self.text, dtype=np.uint16)
        self.offsets = np.ascontiguousarray(self.offsets, dtype=np.int64)
        self.is_retweet = np.ascontiguousarray(self.is_retweet, dtype=np.uint8)
        self.scalars = np.ascontiguousarray(self.scalars, dtype=np.int64)
        n = self.n
        if self.offsets.shape != (n + 1,) or self.scalars.shape != (5, n):
            raise ValueError(f"inconsistent RawBatch shapes: n={n} offsets={self.offsets.shape} "
                             f"scalars={self.scalars.shape}")
        if self.utf8 is not None and self.utf8.offsets.shape != (n + 1,):
            raise ValueError("UTF-8 offsets do not match the batch")
        text_dropped = self.utf8 is not None and self.text.shape[0] == 0
        if n and (self.offsets[0] != 0 or (self.offsets[-1] != self.text.shape[0] and not text_dropped)):
            raise ValueError("offsets must start at 0 and end at len(text)")

    # ------------------------------------------------------------------
    @property
    def n(self) -> int:
        return int(self.is_retweet.shape[0])

    def __len__(self) -> int:
        return self.n

    @property
    def total_units(self) -> int:
        return int(self.offsets[-1]) if self.offsets.shape[0] else 0

    def ensure_text(self) -> "RawBatch":
        """Decode the UTF-16 text from ``utf8`` if the receiver dropped it."""
        if self.text.shape[0] != self.total_units and self.utf8 is not None:
            raw = bytes(self.utf8.data[:self.utf8.nbytes])
            self.text = utf16_units(raw.decode("utf-8", "surrogatepass"))
        return self

    def with_time(self, batch_time_ms: int) -> "RawBatch":
        """Shallow copy (arrays shared) with another seal time."""
        return replace(self, batch_time_ms=int(batch_time_ms))

    def with_scalar_range(self) -> "RawBatch":
        """Record the per-column scalar bounds (what a receiver tracks while it
        parses the records it seals into this batch)."""
        if self.n:
            self.scalar_range = np.stack([self.scalars.min(axis=1), self.scalars.max(axis=1)]).astype(np.int64)
        return self

    @property
    def nbytes(self) -> int:
        return (self.text.nbytes + self.offsets.nbytes + self.is_retweet.nbytes
                + self.scalars.nbytes)

    def column(self, k: int) -> np.ndarray:
        return self.scalars[k]

    def text_of(self, i: int) -> str:
        self.ensure_text()
        return units_to_str(self.text[self.offsets[i]:self.offsets[i + 1]])

    # ------------------------------------------------------------------
    @classmethod
    def empty(cls, batch_time_ms: int = 0) -> "RawBatch":
        return cls(np.zeros(0, np.uint16), np.zeros(1, np.int64), np.zeros(0, np.uint8),
                   np.zeros((5, 0), np.int64), batch_time_ms)

    @classmethod
    def from_statuses(cls, statuses: Sequence[Status], batch_time_ms: int = 0) -> "RawBatch":
        n = len(statuses)
        chunks: List[np.ndarray] = []
        offsets = np.zeros(n + 1, np.int64)
        is_rt = np.zeros(n, np.uint8)
        sc = np.zeros((5, n), np.int64)
        for i, st in enumerate(statuses):
            src = st.retweetedStatus if st.retweetedStatus is not None else st
            is_rt[i] = 1 if st.retweetedStatus is not None else 0
            u = utf16_units(src.text)
            chunks.append(u)
            offsets[i + 1] = offsets[i] + u.shape[0]
            sc[RETWEET_COUNT, i] = src.retweetCount
            sc[FOLLOWERS, i] = src.user.followersCount
            sc[FAVOURITES, i] = src.user.favouritesCount
            sc[FRIENDS, i] = src.user.friendsCount
            sc[CREATED_AT, i] = src.createdAt
        text = np.concatenate(chunks) if chunks else np.zeros(0, np.uint16)
        return cls(text, offsets, is_rt, sc, batch_time_ms)

    def to_statuses(self) -> List[Status]:
        out: List[Status] = []
        for i in range(self.n):
            orig = Status(
                text=self.text_of(i),
                retweetCount=int(self.scalars[RETWEET_COUNT, i]),
                createdAt=int(self.scalars[CREATED_AT, i]),
                user=User(int(self.scalars[FOLLOWERS, i]), int(self.scalars[FAVOURITES, i]),
                          int(self.scalars[FRIENDS, i])),
            )
            if self.is_retweet[i]:
                out.append(Status(text="RT " + orig.text, retweetCount=orig.retweetCount,
                                  createdAt=orig.createdAt, retweetedStatus=orig))
            else:
                out.append(orig)
        return out

    def take(self, rows: Iterable[int]) -> "RawBatch":
        self.ensure_text()
        rows = np.asarray(list(rows), dtype=np.int64)
        lens = self.offsets[rows + 1] - self.offsets[rows]
        offsets = np.zeros(rows.shape[0] + 1, np.int64)
        np.cumsum(lens, out=offsets[1:])
        text = (np.concatenate([self.text[self.offsets[r]:self.offsets[r + 1]] for r in rows])
                if rows.shape[0] else np.zeros(0, np.uint16))
        return RawBatch(text, offsets, self.is_retweet[rows], self.scalars[:, rows],
                        self.batch_time_ms)

    def slice(self, start: int, stop: int) -> "RawBatch":
        self.ensure_text()
        start = max(0, start)
        stop = min(self.n, stop)
        t0, t1 = int(self.offsets[start]), int(self.offsets[stop])
        return RawBatch(self.text[t0:t1], self.offsets[start:stop + 1] - t0,
                        self.is_retweet[start:stop], self.scalars[:, start:stop],
                        self.batch_time_ms)

    def shard(self, rank: int, world: int) -> "RawBatch":
        """Contiguous shard ``rank`` of ``world`` (DP split of one micro-batch)."""
        per = (self.n + world - 1) // world
        return self.slice(rank * per, (rank + 1) * per)

    @staticmethod
    def concat(batches: Sequence["RawBatch"], batch_time_ms: Optional[int] = None) -> "RawBatch":
        if not batches:
            return RawBatch.empty(batch_time_ms or 0)
        if len(batches) == 1:   # a receiver that delivers whole batches: no copy
            b = batches[0]
            return b.with_time(b.batch_time_ms if batch_time_ms is None else batch_time_ms)
        text = np.concatenate([b.ensure_text().text for b in batches])
        lens = np.concatenate([np.diff(b.offsets) for b in batches])
        offsets = np.zeros(lens.shape[0] + 1, np.int64)
        np.cumsum(lens, out=offsets[1:])
        return RawBatch(text, offsets, np.concatenate([b.is_retweet for b in batches]),
                        np.concatenate([b.scalars for b in batches], axis=1),
                        batches[0].batch_time_ms if batch_time_ms is None else batch_time_ms)
