"""Python face of the MI355X streaming k-means engine (``csrc/hip/kmeans_engine.cpp``).

Per micro-batch, on one GPU (``KMeans.scala:77-115``):

1. filter ``isRetweet`` and build dense features ``[retweetCount, followers,
   hashed bigram counts...]`` straight from the raw UTF-16 batch;
2. ``StandardScaler(withMean=false, withStd=true)`` fitted on the batch
   (two-pass, sample std, all-reduced across ranks);
3. assignment to the *current* centres on the matrix cores (``-2 x·c +
   |c|^2``, argmin): split-bf16 ``mfma_f32_32x32x16_bf16`` x3 for d >= 16,
   ``mfma_f32_32x32x2f32`` below, near ties re-decided in fp64; per-cluster
   sums by a counting sort over labels, all-reduced;
4. the decayed centre/weight update with the dying-cluster split on device;
5. optional prediction with the *updated* model (``:113``).

The engine matches :class:`~twitter_stream_ml_amd.models.kmeans.CpuKMeans`
(same random initial centres for the same seed) up to fp32 distance rounding.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional

import weakref

import numpy as np

from ..oracle.mllib import KMeansState, decay_factor_from_half_life
from ..records.batch import RawBatch
from ._native import hip
from .ingest import SlotPipeline
from .lr_engine import HostBatchView, Utf8Text, raw_slots_entry


def no_text(raw: RawBatch) -> Utf8Text:
    """Zero-length rows: what a 2-feature k-means (text_dims 0, the
    reference's [retweetCount, followers]) needs of a batch's text -- only
    the row words (retweet flags) and the two scalar columns cross PCIe."""
    return Utf8Text(np.empty(0, np.uint8), np.zeros(raw.n + 1, np.int64))

__all__ = ["KMDeviceConfig", "DeviceKMeans"]


@dataclass
class KMDeviceConfig:
    k: int = 3
    text_dims: int = 0
    half_life: float = 5.0
    time_unit: str = "batches"
    init_weight: float = 0.0
    scale: bool = True
    mfma: bool = True
    # matrix-core precision of the distances: "bf16x3" (split bf16 operands,
    # 3 MFMAs, ~1e-5 relative; used when d pads to >= 16) or "fp32"
    precision: str = "bf16x3"
    max_rows: int = 1 << 16
    max_units: int = (1 << 16) * 281
    seed: int = 42
    # host staging of the text (text_dims > 0): "utf8" ships the receiver's
    # UTF-8 bytes (DMA'd in place when page-locked; the device decodes),
    # "wire" runs the host packer
    ingest: str = "utf8"
    # take the DP path (scaler / cluster-sum all-reduces) even with a
    # world-1 communicator: RCCL carries the collectives on one GPU
    force_dp: bool = False
    raw_slots: int = 0   # device raw-batch slots (0: TWTML_RAW_SLOTS or the engine default; lr_engine)

    def as_dict(self) -> Dict[str, object]:
        if self.time_unit not in ("batches", "points"):
            raise ValueError(f"Invalid time unit for decay: {self.time_unit}")
        return {
            "k": int(self.k),
            "text_dims": int(self.text_dims),
            "decay": float(decay_factor_from_half_life(self.half_life)),
            "points_unit": int(self.time_unit == "points"),
            "scale": int(bool(self.scale)),
            "mfma": 0 if not self.mfma else (1 if self.precision == "bf16x3" else 2),
            "max_rows": int(self.max_rows),
            "max_units": int(self.max_units),
            "force_dp": int(bool(self.force_dp)),
            **raw_slots_entry(self.raw_slots),
        }


class DeviceKMeans:
    """StreamingKMeans state + fused batch pipeline on one GPU."""

    def __init__(self, cfg: KMDeviceConfig, device: int = 0, comm=None):
        self.cfg = cfg
        self.device = int(device)
        self.dim = 2 + int(cfg.text_dims)
        self.comm = comm
        self._eng = hip().KMEngine(self.device, cfg.as_dict(), comm)
        st = KMeansState.random(cfg.k, self.dim, cfg.init_weight, cfg.seed)
        self.set_state(st.centers, st.weights)
        self._staging: List[HostBatchView] = []
        self.raw_slots = int(self._eng.raw_slots)
        me = weakref.proxy(self)   # no reference cycle (see DeviceLinearRegression)
        self._pipe = SlotPipeline(self.raw_slots, lambda s, raw: me._stage(s, raw),
                                  lambda hb, slot: me.submit(hb, slot), lambda: me.synchronize(),
                                  discard=lambda slot: me._eng.discard(int(slot)))

    def _stage(self, slot: int, raw: RawBatch) -> HostBatchView:
        hb = self.staging(slot)
        if self.cfg.text_dims == 0:
            return hb.load_utf8(raw, no_text(raw), copy_text=True)
        return hb.load(raw, self.cfg.ingest)

    # ---- model state (latestModel.clusterCenters / clusterWeights) -------
    def get_state(self):
        c, w = self._eng.get_state()
        return np.asarray(c), np.asarray(w)

    def set_state(self, centers, weights) -> None:
        c = np.ascontiguousarray(centers, dtype=np.float64)
        w = np.ascontiguousarray(weights, dtype=np.float64)
        if c.shape != (self.cfg.k, self.dim) or w.shape != (self.cfg.k,):
            raise ValueError(f"expected centers ({self.cfg.k}, {self.dim}) and weights "
                             f"({self.cfg.k},), got {c.shape} / {w.shape}")
        self._eng.set_state(c, w)

    @property
    def state(self) -> KMeansState:
        c, w = self.get_state()
        return KMeansState(c, w)

    # ---- pipeline ---------------------------------------------------------
    def staging(self, i: int = 0) -> HostBatchView:
        while len(self._staging) <= i:
            hb = HostBatchView(self.cfg.max_rows, self.cfg.max_units)
            hb._hb.scalar_cols = 2   # the features read retweetCount and followersCount only
            self._staging.append(hb)
        return self._staging[i]

    def submit(self, hb: HostBatchView, slot: int) -> None:
        self._eng.submit(hb._hb, int(hb.n), int(hb.bytes), int(slot), int(hb.ext_text))

    def process(self, slot: int, want_pred: bool = True) -> Dict[str, object]:
        r = self._eng.process(int(slot), bool(want_pred))
        if r["std"] is not None and len(r["std"]):
            r["std"] = np.asarray(r["std"])
        else:
            r["std"] = None
        if want_pred and r["pred"] is None:
            r["pred"] = np.zeros(0, np.int32)
        return r

    def prefetch(self, raw: RawBatch) -> bool:
        """Stage + async H2D of a queued future batch (overlaps the current one)."""
        return self._pipe.prefetch(raw)

    def update_raw(self, raw: RawBatch, want_pred: bool = True) -> Dict[str, object]:
        """One micro-batch: uses its prefetched slot, else stages + H2D now."""
        return self.process(self._pipe.take(raw), want_pred)

    @property
    def h2d_bytes(self) -> int:
        """Host-to-device bytes submitted so far (every copy of every batch)."""
        return int(self._eng.h2d_bytes)

    def synchronize(self) -> None:
        self._eng.synchronize()
