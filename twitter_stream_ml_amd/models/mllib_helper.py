"""Feature engineering of the LR job (``MllibHelper.scala:11-95``; K1-K3 on CPU).

* :meth:`MllibHelper.filtrate` — ``isRetweet && begin <= rtCount <= end``
  (``:84-95``).
* :meth:`MllibHelper.featurizeText` — lower-case the *original* tweet's text,
  character bigrams, HashingTF (``:42-56``).  The NFD accent strip at
  ``:49-51`` is computed but unused by the reference, so it is not done here.
* :meth:`MllibHelper.featurizeNumbers` — followers, favourites, friends
  ×1e-12 and ``(now - createdAt)`` ms ×1e-14 (``:58-71``).  ``now`` is the
  batch seal time passed in explicitly (the reference calls
  ``System.currentTimeMillis`` per record, which is not reproducible).
* :meth:`MllibHelper.featurize` — sparse vector of size ``F + 4``, label =
  original retweet count (``:73-82``).

``reset`` honours ``numTextFeatures`` (the reference shadows its fields with
locals at ``:27-29`` so ``-f`` never takes effect; ``--legacyNumTextFeatures``
reproduces that).
"""
from __future__ import annotations

import numpy as np

from ..records.schema import Status
from .hashing_tf import HashingTF, java_lower
from .vectors import LabeledPoint, SparseVector

__all__ = ["MllibHelper", "NUM_NUMBER_FEATURES", "NUMBER_SCALES"]

NUM_NUMBER_FEATURES = 4
# multipliers of followers, favourites, friends, age-ms (MllibHelper.scala:64-67)
NUMBER_SCALES = (1e-12, 1e-12, 1e-12, 1e-14)


class MllibHelper:
    numNumberFeatures = NUM_NUMBER_FEATURES
    numRetweetBegin = 100
    numRetweetEnd = 1000
    numTextFeatures = 1000
    hashText = HashingTF(1000)
    numFeatures = numTextFeatures + numNumberFeatures
    numberFeatureIndices = np.arange(numTextFeatures, numFeatures, dtype=np.int64)

    @classmethod
    def reset(cls, conf) -> None:
        cls.numRetweetBegin = int(conf.numRetweetBegin)
        cls.numRetweetEnd = int(conf.numRetweetEnd)
        cls.numTextFeatures = int(conf.numTextFeatures)
        width = int(getattr(conf, "effectiveNumTextFeatures", 1000))
        cls.configure(width, getattr(conf, "hash", "java"))

    @classmethod
    def configure(cls, num_text_features: int, hash: str = "java") -> None:
        cls.hashText = HashingTF(num_text_features, hash)
        cls.numFeatures = num_text_features + cls.numNumberFeatures
        cls.numberFeatureIndices = np.arange(num_text_features, cls.numFeatures, dtype=np.int64)

    @classmethod
    def featurizeText(cls, status: Status) -> SparseVector:
        text = java_lower(status.getRetweetedStatus().getText())
        return cls.hashText.transform_text(text)

    @classmethod
    def featurizeNumbers(cls, status: Status, now_ms: int) -> np.ndarray:
        orig = status.getRetweetedStatus()
        user = orig.getUser()
        time_left = int(now_ms) - int(orig.getCreatedAt())
        return np.array([user.getFollowersCount() * NUMBER_SCALES[0],
                         user.getFavouritesCount() * NUMBER_SCALES[1],
                         user.getFriendsCount() * NUMBER_SCALES[2],
                         time_left * NUMBER_SCALES[3]], dtype=np.float64)

    @classmethod
    def featurize(cls, status: Status, now_ms: int) -> LabeledPoint:
        text = cls.featurizeText(status)
        nums = cls.featurizeNumbers(status, now_ms)
        feats = SparseVector(cls.numFeatures,
                             np.concatenate([text.indices, cls.numberFeatureIndices]),
                             np.concatenate([text.values, nums]))
        return LabeledPoint(float(status.getRetweetedStatus().getRetweetCount()), feats)

    @staticmethod
    def retweetInterval(status: Status, start: int, end: int) -> bool:
        n = status.getRetweetedStatus().getRetweetCount()
        return start <= n <= end

    @classmethod
    def filtrate(cls, status: Status) -> bool:
        return status.isRetweet() and cls.retweetInterval(status, cls.numRetweetBegin,
                                                         cls.numRetweetEnd)
