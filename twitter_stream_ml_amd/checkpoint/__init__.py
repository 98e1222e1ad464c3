"""Model checkpoints in MLlib's Saveable layout (metadata JSON + parquet)."""
from .saveable import (KMEANS_CLASS, LR_CLASS, load_kmeans, load_linear_regression, save_kmeans,
                       save_linear_regression, vector_udt_type)

__all__ = ["KMEANS_CLASS", "LR_CLASS", "load_kmeans", "load_linear_regression", "save_kmeans",
           "save_linear_regression", "vector_udt_type"]
