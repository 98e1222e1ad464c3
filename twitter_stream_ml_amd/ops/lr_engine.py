"""Python face of the MI355X streaming-LR engine (``csrc/hip/engine.cpp``).

The engine executes, per micro-batch and entirely on the GPU, what the
reference runs as ~60 Spark jobs: filter (K3), featurize
(K1+K2), prequential predict + stats (K4+K7, output op #1 of
``LinearRegression.scala:53-81``) and ``numIterations`` steps of
``GradientDescent`` (K5+K6, output op #2 ``model.trainOn`` at ``:86``).

Host-side contract: raw batches live in pinned :class:`HostBatch` buffers in
the wire format (narrow/wide ``text`` bytes, byte ``offsets``, per-row
``flags``, packed ``[5][n]`` scalars; ``csrc/host/wire.h``).  Rows whose
lower-casing is not per-UTF-16-unit (U+0130, U+03A3, astral cased letters)
are rewritten on the host first (:func:`prelower`); everything else is
lowered on the device.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np

from ..records.batch import RETWEET_COUNT, RawBatch
from ._native import hip, host
from .ingest import SlotPipeline

__all__ = ["LRDeviceConfig", "DeviceLinearRegression", "prelower", "HostBatchView"]


def prelower(raw: RawBatch) -> RawBatch:
    """Host pre-pass: full-case-map the rare rows the GPU cannot lower per unit."""
    h = host()
    if h.count_special_rows(raw.text, raw.offsets) == 0:
        return raw
    text, offsets, _ = h.prelower_special_rows(raw.text, raw.offsets)
    return RawBatch(text, offsets, raw.is_retweet, raw.scalars, raw.batch_time_ms)


@dataclass
class LRDeviceConfig:
    num_text_features: int = 1000
    hash: str = "java"
    step_size: float = 0.005
    num_iterations: int = 50
    fraction: float = 1.0
    tol: float = 1e-3
    begin: int = 100
    end: int = 1000
    require_retweet: bool = True
    range_filter: bool = True
    max_rows: int = 1 << 16
    max_units: int = (1 << 16) * 281
    sgd_grid: int = 0
    ablate: int = 0          # perf diagnostics only (1: no scatter, 2: no gather/scatter)
    # merge a row's repeated bigrams into term counts before the GD loop.
    # Measured on MI355X (1M-tweet batches, 35 iterations): -7% per iteration
    # but the merge pass costs more than it saves, so it is off by default.
    dedup: bool = False
    # dense 4-bit counts for the batch's 128 hottest bigrams (csrc/hip/hot_split.hip)
    hybrid: bool = True
    # hybrid layout only: the featurizer materialises hashed ids just for the
    # chunks the hot-slot histogram samples; the remap re-derives the rest
    # from the raw text (csrc/hip/narrow_text.h).  False keeps every id
    # (debug_prepared() inspection).
    lazy_idx: bool = True

    def as_dict(self) -> Dict[str, object]:
        return {
            "num_text_features": int(self.num_text_features),
            "hash_kind": 0 if self.hash == "java" else 1,
            "step_size": float(self.step_size),
            "num_iterations": int(self.num_iterations),
            "fraction": float(self.fraction),
            "tol": float(self.tol),
            "begin": int(self.begin),
            "end": int(self.end),
            "require_retweet": int(bool(self.require_retweet)),
            "range_filter": int(bool(self.range_filter)),
            "max_rows": int(self.max_rows),
            "max_units": int(self.max_units),
            "sgd_grid": int(self.sgd_grid),
            "ablate": int(self.ablate),
            "dedup": int(bool(self.dedup)),
            "hybrid": int(bool(self.hybrid)),
            "lazy_idx": int(bool(self.lazy_idx)),
        }


class HostBatchView:
    """Pinned host staging buffer in the wire format, with numpy views.

    ``load`` pre-lowers the special rows, then packs the UTF-16 batch into
    narrow (Latin-1, 1 byte/unit) / wide (UTF-16LE) rows with the native
    multi-threaded packer (``csrc/host/wire.cpp``): typical tweet text
    crosses PCIe at half the UTF-16 size.  The five int64 scalar columns
    ship as u32 offsets from a per-batch base when their range fits (exact),
    and a row's byte offset + flags as one u16 (length | flags << 14) that
    the device scans back into offsets (rows of >= 16 KiB: plain offsets).
    """

    def __init__(self, max_rows: int, max_units: int):
        self.max_units = int(max_units)
        self._hb = hip().HostBatch(int(max_rows), int(host().wire_bound(self.max_units, int(max_rows))))
        self.text = self._hb.text
        self.offsets = self._hb.offsets
        self.flags = self._hb.flags
        self.scalars_flat = self._hb.scalars_flat
        self.n = 0
        self.units = 0
        self.bytes = 0
        self.batch_time_ms = 0
        self.rows_packed = False

    @property
    def max_rows(self) -> int:
        return self._hb.max_rows

    def scalars(self) -> np.ndarray:
        return self.scalars_flat[:5 * self.n].reshape(5, self.n)

    def load(self, raw: RawBatch) -> "HostBatchView":
        raw = prelower(raw)
        n, u = raw.n, raw.total_units
        if n > self.max_rows or u > self.max_units:
            raise ValueError(f"batch ({n} rows, {u} units) exceeds staging capacity "
                             f"({self.max_rows}, {self.max_units})")
        self.bytes = int(host().wire_pack(raw.text, raw.offsets, raw.is_retweet, self.text,
                                          self.offsets, self.flags))
        self.scalars_flat[:5 * n] = raw.scalars.reshape(-1)
        self._hb.pack_scalars(n)   # u32 + per-batch base where a column's range fits
        self.rows_packed = bool(self._hb.pack_rows(n))   # offsets + flags as 2 B per row
        self.n, self.units, self.batch_time_ms = n, u, raw.batch_time_ms
        return self

    def as_raw(self) -> RawBatch:
        text, offsets, is_rt = host().wire_unpack(self.text[:self.bytes], self.offsets[:self.n + 1],
                                                  self.flags[:self.n])
        return RawBatch(text, offsets, is_rt, self.scalars().copy(), self.batch_time_ms)


class DeviceLinearRegression:
    """StreamingLinearRegressionWithSGD state + pipeline on one GPU."""

    def __init__(self, cfg: LRDeviceConfig, device: int = 0, comm=None):
        self.cfg = cfg
        self.device = int(device)
        self.comm = comm
        self._eng = hip().LREngine(self.device, cfg.as_dict(), comm)
        self._staging: List[HostBatchView] = []
        self.raw_slots = int(hip().RAW_SLOTS)
        self._pipe = SlotPipeline(self.raw_slots, lambda s, raw: self.staging(s).load(raw),
                                  self.submit, self.synchronize)

    # ---- weights (MLlib setInitialWeights / latestModel.weights) ---------
    @property
    def num_weights(self) -> int:
        return int(self._eng.num_weights)

    def get_weights(self) -> np.ndarray:
        return np.asarray(self._eng.get_weights())

    def set_weights(self, w: np.ndarray) -> None:
        w = np.ascontiguousarray(w, dtype=np.float64)
        if w.shape != (self.num_weights,):
            raise ValueError(f"expected {self.num_weights} weights, got {w.shape}")
        self._eng.set_weights(w)

    # ---- staging / pipeline ----------------------------------------------
    def staging(self, i: int = 0) -> HostBatchView:
        while len(self._staging) <= i:
            self._staging.append(HostBatchView(self.cfg.max_rows, self.cfg.max_units))
        return self._staging[i]

    def submit(self, hb: HostBatchView, slot: int) -> None:
        self._eng.submit(hb._hb, int(hb.n), int(hb.bytes), int(slot))

    def process(self, slot: int, now_ms: int, want_pred: bool = False) -> Dict[str, object]:
        return self._eng.process(int(slot), int(now_ms), bool(want_pred))

    def prefetch(self, raw: RawBatch) -> bool:
        """Stage + async H2D of a queued future batch (overlaps the current one)."""
        return self._pipe.prefetch(raw)

    def train_batch(self, raw: RawBatch, want_pred: bool = True) -> Dict[str, object]:
        """Train on one micro-batch: uses its prefetched slot, else stages + H2D now."""
        return self.process(self._pipe.take(raw), raw.batch_time_ms, want_pred)

    def synchronize(self) -> None:
        self._eng.synchronize()


def batch_report(res: Dict[str, object]) -> Dict[str, float]:
    """Population stdevs / MSE from the fused stats (``LinearRegression.scala:59-65``)."""
    n, sy, sy2, sp, sp2, se2 = res["stats"]
    if n <= 0:
        return {"count": 0, "mse": float("nan"), "realStdev": float("nan"),
                "predStdev": float("nan")}
    my, mp = sy / n, sp / n
    return {
        "count": int(round(n)),
        "mse": se2 / n,
        "realStdev": float(np.sqrt(max(sy2 / n - my * my, 0.0))),
        "predStdev": float(np.sqrt(max(sp2 / n - mp * mp, 0.0))),
    }
