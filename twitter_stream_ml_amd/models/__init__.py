"""Model families: streaming linear regression (SGD), streaming k-means, HashingTF,
StandardScaler, MLlib vectors (all with fp64 CPU semantics; MI355X engines in ops/)."""
from .hashing_tf import HashingTF
from .kmeans import (CpuKMeans, StandardScaler, StandardScalerModel, StreamingKMeans,
                     StreamingKMeansModel, kmeans_features)
from .linear_regression import (CpuLinearRegression, LinearRegressionModel,
                                StreamingLinearRegressionWithSGD, featurize_columnar)
from .mllib_helper import MllibHelper
from .vectors import DenseVector, LabeledPoint, SparseVector, Vector, Vectors

__all__ = ["HashingTF", "CpuKMeans", "StandardScaler", "StandardScalerModel", "StreamingKMeans",
           "StreamingKMeansModel", "kmeans_features", "CpuLinearRegression",
           "LinearRegressionModel", "StreamingLinearRegressionWithSGD", "featurize_columnar",
           "MllibHelper", "DenseVector", "LabeledPoint", "SparseVector", "Vector", "Vectors"]
