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
  (sparse: a vector with under 25 % non-zeros -- the usual case for hashed
  text weights at F = 1e8, where only the touched bigrams ever move).  The
  footer carries Spark's ``org.apache.spark.sql.parquet.row.metadata``
  schema JSON with the VectorUDT class, which is what Spark's parquet reader
  uses to turn the struct back into a ``Vector``.  Loading in real Spark is
  parity-unpinned (no Spark here); the layout follows upstream
  ``GLMRegressionModel.SaveLoadV1_0`` / ``VectorUDT.sqlType``.

Vectors are built and read column-wise (numpy <-> arrow buffers), never as
Python lists: a 1e8-weight model saves and loads in seconds.

Streaming k-means also needs the cluster weights, which ``KMeansModel`` does
not store; they go to ``<path>/streaming/weights.json`` (extension, ignored
by Spark).  Writes replace the directory via rename: a crash between the
two renames leaves ``<path>.old`` as the last good model, which
``resolve_resume`` falls back to.
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

__all__ = ["SparseWeights", "save_linear_regression", "load_linear_regression", "save_kmeans", "load_kmeans",
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


SPARSE_DENSITY = 0.25   # sparse VectorUDT (type 0) below this fraction of non-zeros

_UDT_JSON = {
    "type": "udt", "class": "org.apache.spark.mllib.linalg.VectorUDT",
    "pyClass": "pyspark.mllib.linalg.VectorUDT",
    "sqlType": {"type": "struct", "fields": [
        {"name": "type", "type": "byte", "nullable": False, "metadata": {}},
        {"name": "size", "type": "integer", "nullable": True, "metadata": {}},
        {"name": "indices", "type": {"type": "array", "elementType": "integer", "containsNull": False},
         "nullable": True, "metadata": {}},
        {"name": "values", "type": {"type": "array", "elementType": "double", "containsNull": False},
         "nullable": True, "metadata": {}}]},
}


def _spark_row_metadata(fields) -> dict:
    """Spark's parquet footer schema (``org.apache.spark.sql.parquet.row.metadata``)."""
    js = {"type": "struct", "fields": [
        {"name": n, "type": (_UDT_JSON if t == "vector" else t), "nullable": nl, "metadata": {}}
        for n, t, nl in fields]}
    return {b"org.apache.spark.sql.parquet.row.metadata": json.dumps(js, separators=(",", ":")).encode()}


class SparseWeights:
    """A weight vector held as its non-zeros: ``size``, int32 ``indices``
    (ascending) and fp64 ``values`` -- what the device snapshot delivers
    (``DeviceLinearRegression.snapshot_fetch``), saved without densifying."""

    def __init__(self, size: int, indices: np.ndarray, values: np.ndarray):
        self.size = int(size)
        self.indices = np.asarray(indices, np.int32)
        self.values = np.asarray(values, np.float64)
        if self.indices.shape != self.values.shape:
            raise ValueError("indices / values length mismatch")

    def dense(self) -> np.ndarray:
        d = np.zeros(self.size, np.float64)
        d[self.indices] = self.values
        return d


def _udt_array(vecs, sparse_density: float = SPARSE_DENSITY) -> pa.StructArray:
    """VectorUDT column of ``vecs`` from numpy buffers (no Python floats)."""
    types, sizes, size_null = [], [], []
    iv, io, inull = [], [0], []
    vv, vo = [], [0]
    for v in vecs:
        if isinstance(v, SparseWeights):
            if v.size > 0 and v.indices.shape[0] < sparse_density * v.size:
                types.append(0)
                sizes.append(v.size)
                size_null.append(False)
                iv.append(v.indices)
                vv.append(v.values)
                inull.append(False)
                io.append(io[-1] + v.indices.shape[0])
                vo.append(vo[-1] + v.values.shape[0])
                continue
            v = v.dense()
        v = np.asarray(v, dtype=np.float64)
        nz = np.flatnonzero(v)
        sparse = v.shape[0] > 0 and nz.shape[0] < sparse_density * v.shape[0]
        types.append(0 if sparse else 1)
        sizes.append(v.shape[0] if sparse else 0)
        size_null.append(not sparse)
        if sparse:
            iv.append(nz.astype(np.int32))
            vv.append(v[nz])
        else:
            vv.append(v)
        inull.append(not sparse)
        io.append(io[-1] + (nz.shape[0] if sparse else 0))
        vo.append(vo[-1] + vv[-1].shape[0])
    i32 = pa.list_(pa.field("element", pa.int32(), nullable=False))
    f64 = pa.list_(pa.field("element", pa.float64(), nullable=False))

    def cat(parts, dtype):
        # one vector (a model): its buffer as it is -- pa.array of a numpy
        # array is zero-copy, np.concatenate would copy ~MBs holding the GIL
        # on the checkpoint writer thread while the training thread streams
        if not parts:
            return np.zeros(0, dtype)
        return np.ascontiguousarray(parts[0], dtype) if len(parts) == 1 else np.concatenate(parts).astype(dtype, copy=False)

    ind = pa.ListArray.from_arrays(pa.array(np.asarray(io, np.int32)), pa.array(cat(iv, np.int32)),
                                   type=i32, mask=pa.array(np.asarray(inull, bool)))
    if vo[-1] >= 2 ** 31:
        raise ValueError("VectorUDT column: more than 2^31 values")
    val = pa.ListArray.from_arrays(pa.array(np.asarray(vo, np.int32)), pa.array(cat(vv, np.float64)), type=f64)
    siz = pa.array(np.asarray(sizes, np.int32), mask=np.asarray(size_null, bool))
    return pa.StructArray.from_arrays([pa.array(np.asarray(types, np.int8)), siz, ind, val],
                                      fields=list(vector_udt_type()))


def _from_udt_column(col: pa.ChunkedArray) -> list:
    """VectorUDT column -> list of numpy vectors (buffers, not Python lists)."""
    out = []
    for chunk in col.chunks:
        types = chunk.field("type").to_numpy(zero_copy_only=False)
        sizes = chunk.field("size")
        inds, vals = chunk.field("indices"), chunk.field("values")
        for r in range(len(chunk)):
            v = vals[r].values.to_numpy(zero_copy_only=False).astype(np.float64, copy=False)
            if int(types[r]) == 1:
                out.append(np.array(v, dtype=np.float64))
            else:
                dense = np.zeros(int(sizes[r].as_py()), np.float64)
                dense[inds[r].values.to_numpy(zero_copy_only=False).astype(np.int64)] = v
                out.append(dense)
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


def save_linear_regression(path: str, weights, intercept: float = 0.0,
                           progress: Optional[dict] = None) -> None:
    """``weights``: a dense vector or :class:`SparseWeights`."""
    w = weights if isinstance(weights, SparseWeights) else np.asarray(weights, dtype=np.float64)
    size = w.size if isinstance(w, SparseWeights) else int(w.shape[0])
    schema = pa.schema([pa.field("weights", vector_udt_type()), pa.field("intercept", pa.float64(), nullable=False)],
                       metadata=_spark_row_metadata([("weights", "vector", True), ("intercept", "double", False)]))
    table = pa.Table.from_arrays([_udt_array([w]), pa.array([float(intercept)], pa.float64())], schema=schema)
    _write_dir(path, {"class": LR_CLASS, "version": "1.0", "numFeatures": size}, table,
               {"progress.json": progress} if progress else None)


def load_linear_regression(path: str) -> Tuple[np.ndarray, float]:
    meta = _read_meta(path, LR_CLASS)
    t = _read_data(path)
    if t.num_rows != 1:
        raise ValueError(f"{path}: expected one data row, found {t.num_rows}")
    w = _from_udt_column(t.column("weights"))[0]
    if w.shape[0] != int(meta["numFeatures"]):
        raise ValueError(f"{path}: numFeatures {meta['numFeatures']} != {w.shape[0]}")
    return w, float(t.column("intercept")[0].as_py())


def save_kmeans(path: str, centers: np.ndarray, weights: Optional[np.ndarray] = None,
                progress: Optional[dict] = None) -> None:
    c = np.asarray(centers, dtype=np.float64)
    schema = pa.schema([pa.field("id", pa.int32(), nullable=False), pa.field("point", vector_udt_type())],
                       metadata=_spark_row_metadata([("id", "integer", False), ("point", "vector", True)]))
    table = pa.Table.from_arrays([pa.array(np.arange(c.shape[0], dtype=np.int32)),
                                  _udt_array([c[i] for i in range(c.shape[0])], sparse_density=0.0)],
                                 schema=schema)
    files: Dict[str, dict] = {}
    if weights is not None:
        files["weights.json"] = {"clusterWeights": np.asarray(weights, np.float64).tolist()}
    if progress:
        files["progress.json"] = progress
    _write_dir(path, {"class": KMEANS_CLASS, "version": "1.0", "k": int(c.shape[0])}, table, files)


def load_kmeans(path: str) -> Tuple[np.ndarray, Optional[np.ndarray]]:
    meta = _read_meta(path, KMEANS_CLASS)
    t = _read_data(path)
    ids = t.column("id").to_numpy()
    pts = _from_udt_column(t.column("point"))
    order = np.argsort(ids, kind="stable")
    centers = np.stack([pts[i] for i in order]) if len(pts) else np.zeros((0, 0))
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
