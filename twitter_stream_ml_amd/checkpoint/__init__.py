"""Model checkpoints in MLlib's Saveable layout (metadata JSON + parquet) + stream positions."""
from .saveable import (KMEANS_CLASS, LR_CLASS, SparseWeights, load_kmeans, load_linear_regression, load_progress,
                       save_kmeans, save_linear_regression, vector_udt_type)
from .stream_state import StreamPositions, resolve_resume

__all__ = ["KMEANS_CLASS", "LR_CLASS", "SparseWeights", "load_kmeans", "load_linear_regression", "load_progress",
           "save_kmeans", "save_linear_regression", "vector_udt_type", "StreamPositions",
           "resolve_resume"]
