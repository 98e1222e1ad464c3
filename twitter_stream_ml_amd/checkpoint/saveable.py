"""Model checkpoints in the MLlib ``Saveable`` layout (SURVEY §5 checkpoint row).

The reference never saves its model (it lives in driver memory only).  The
engine writes what MLlib 1.6's ``model.save(sc, path)`` would, so a Spark user
can ``LinearRegressionModel.load(sc, path)`` it [upstream
``GLMRegressionModel.SaveLoadV1_0``, ``KMeansModel.SaveLoadV1_0``]:

* ``<path>/metadata/part-00000`` — one JSON line, e.g.
  ``{"class":"org.apache.spark.mllib.regression.LinearRegressionModel",
  "version":"1.0","numFeatures":N}`` (+ ``_SUCCESS``);
* ``<path>/data/part-00000.parquet`` — one row ``{weights: VectorUDT,
  intercept: double}`` for LR, rows ``{id: int, point: VectorUDT}`` for
  k-means (+ ``_SUCCESS``).  ``VectorUDT`` is
  ``struct<type: tinyint, size: int, indices: array<int>, values:
  array<double>>`` with ``type = 1`` (dense; size/indices null) or ``0``
  (sparse).

Streaming k-means also needs the cluster weights, which ``KMeansModel`` does
not store; they go to ``<path>/streaming/weights.json`` (extension, ignored
by Spark).  Writes are atomic (temporary directory + rename).
"""
from __future__ import annotations

import json
import os
import shutil
import tempfile
from typing import Dict, Optional, Tuple

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq

__all__ = ["save_linear_regression", "load_linear_regression", "save_kmeans", "load_kmeans",
           "LR_CLASS", "KMEANS_CLASS", "vector_udt_type"]

LR_CLASS = "org.apache.spark.mllib.regression.LinearRegressionModel"
KMEANS_CLASS = "org.apache.spark.mllib.clustering.KMeansModel"


def vector_udt_type() -> pa.DataType:
    return pa.struct([
        pa.field("type", pa.int8(), nullable=False),
        pa.field("size", pa.int32(), nullable=True),
        pa.field("indices", pa.list_(pa.field("element", pa.int32(), nullable=False)), nullable=True),
        pa.field("values", pa.list_(pa.field("element", pa.float64(), nullable=False)), nullable=True),
    ])


def _dense(v: np.ndarray) -> dict:
    return {"type": 1, "size": None, "indices": None, "values": np.asarray(v, np.float64).tolist()}


def _from_udt(d: dict) -> np.ndarray:
    if d["type"] == 1:
        return np.asarray(d["values"], dtype=np.float64)
    out = np.zeros(int(d["size"]), np.float64)
    out[np.asarray(d["indices"], np.int64)] = np.asarray(d["values"], np.float64)
    return out


def _write_dir(path: str, metadata: dict, table: pa.Table,
               streaming: Optional[Dict[str, dict]] = None) -> None:
    """Write a Saveable directory atomically (tmp dir + rename).

    ``streaming`` holds extension JSON files (cluster weights, stream
    progress) under ``<path>/streaming/`` -- MLlib loaders ignore them.
    """
    parent = os.path.dirname(os.path.abspath(path)) or "."
    os.makedirs(parent, exist_ok=True)
    tmp = tempfile.mkdtemp(prefix=".twtml-ckpt-", dir=parent)
    try:
        os.makedirs(os.path.join(tmp, "metadata"))
        os.makedirs(os.path.join(tmp, "data"))
        with open(os.path.join(tmp, "metadata", "part-00000"), "w") as fh:
            fh.write(json.dumps(metadata, separators=(",", ":")) + "\n")
        open(os.path.join(tmp, "metadata", "_SUCCESS"), "w").close()
        pq.write_table(table, os.path.join(tmp, "data", "part-00000.parquet"))
        open(os.path.join(tmp, "data", "_SUCCESS"), "w").close()
        if streaming:
            os.makedirs(os.path.join(tmp, "streaming"))
            for name, obj in streaming.items():
                with open(os.path.join(tmp, "streaming", name), "w") as fh:
                    json.dump(obj, fh)
        if os.path.exists(path):
            old = path + ".old"
            shutil.rmtree(old, ignore_errors=True)
            os.replace(path, old)
            os.replace(tmp, path)
            shutil.rmtree(old, ignore_errors=True)
        else:
            os.replace(tmp, path)
    except BaseException:
        shutil.rmtree(tmp, ignore_errors=True)
        raise


def _read_meta(path: str, cls: str) -> dict:
    with open(os.path.join(path, "metadata", "part-00000")) as fh:
        meta = json.loads(fh.readline())
    if meta.get("class") != cls:
        raise ValueError(f"{path}: expected class {cls}, found {meta.get('class')}")
    if meta.get("version") != "1.0":
        raise ValueError(f"{path}: unsupported version {meta.get('version')}")
    return meta


def _read_data(path: str) -> pa.Table:
    d = os.path.join(path, "data")
    files = sorted(f for f in os.listdir(d) if f.endswith(".parquet"))
    return pa.concat_tables([pq.read_table(os.path.join(d, f)) for f in files])


def save_linear_regression(path: str, weights: np.ndarray, intercept: float = 0.0,
                           progress: Optional[dict] = None) -> None:
    w = np.asarray(weights, dtype=np.float64)
    schema = pa.schema([pa.field("weights", vector_udt_type()), pa.field("intercept", pa.float64())])
    table = pa.Table.from_pylist([{"weights": _dense(w), "intercept": float(intercept)}], schema)
    _write_dir(path, {"class": LR_CLASS, "version": "1.0", "numFeatures": int(w.shape[0])}, table,
               {"progress.json": progress} if progress else None)


def load_linear_regression(path: str) -> Tuple[np.ndarray, float]:
    meta = _read_meta(path, LR_CLASS)
    rows = _read_data(path).to_pylist()
    if len(rows) != 1:
        raise ValueError(f"{path}: expected one data row, found {len(rows)}")
    w = _from_udt(rows[0]["weights"])
    if w.shape[0] != int(meta["numFeatures"]):
        raise ValueError(f"{path}: numFeatures {meta['numFeatures']} != {w.shape[0]}")
    return w, float(rows[0]["intercept"])


def save_kmeans(path: str, centers: np.ndarray, weights: Optional[np.ndarray] = None,
                progress: Optional[dict] = None) -> None:
    c = np.asarray(centers, dtype=np.float64)
    schema = pa.schema([pa.field("id", pa.int32()), pa.field("point", vector_udt_type())])
    table = pa.Table.from_pylist([{"id": i, "point": _dense(c[i])} for i in range(c.shape[0])], schema)
    files: Dict[str, dict] = {}
    if weights is not None:
        files["weights.json"] = {"clusterWeights": np.asarray(weights, np.float64).tolist()}
    if progress:
        files["progress.json"] = progress
    _write_dir(path, {"class": KMEANS_CLASS, "version": "1.0", "k": int(c.shape[0])}, table, files)


def load_kmeans(path: str) -> Tuple[np.ndarray, Optional[np.ndarray]]:
    meta = _read_meta(path, KMEANS_CLASS)
    rows = sorted(_read_data(path).to_pylist(), key=lambda r: r["id"])
    centers = np.stack([_from_udt(r["point"]) for r in rows]) if rows else np.zeros((0, 0))
    if centers.shape[0] != int(meta["k"]):
        raise ValueError(f"{path}: k {meta['k']} != {centers.shape[0]}")
    wpath = os.path.join(path, "streaming", "weights.json")
    weights = None
    if os.path.exists(wpath):
        with open(wpath) as fh:
            weights = np.asarray(json.load(fh)["clusterWeights"], np.float64)
    return centers, weights


def load_progress(path: str) -> Optional[dict]:
    """Stream progress stored with a model (``{"batches": t, ...}``) or None."""
    p = os.path.join(path, "streaming", "progress.json")
    if not os.path.exists(p):
        return None
    with open(p) as fh:
        return json.load(fh)
