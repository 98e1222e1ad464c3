"""fp64 CPU golden oracle of the MLlib 1.6.1 semantics (also the CPU engine)."""
from .mllib import (CONVERGENCE_TOL, KMeansState, SGDResult, StatCounter,
                    decay_factor_from_half_life, find_closest, kmeans_update,
                    least_squares_gradient, round_half_up, round_half_up_array,
                    run_minibatch_sgd, run_minibatch_sgd_active, sgd_uniform, standard_scaler_fit,
                    standard_scaler_transform)
from .featurize import (FeaturizedBatch, featurize_batch, featurize_batch_native, filter_mask,
                        lowered_units)

__all__ = [
    "CONVERGENCE_TOL", "KMeansState", "SGDResult", "StatCounter", "decay_factor_from_half_life",
    "find_closest", "kmeans_update", "least_squares_gradient", "round_half_up",
    "round_half_up_array", "run_minibatch_sgd", "run_minibatch_sgd_active", "sgd_uniform",
    "standard_scaler_fit", "standard_scaler_transform", "FeaturizedBatch", "featurize_batch",
    "featurize_batch_native", "filter_mask", "lowered_units",
]
