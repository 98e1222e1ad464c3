"""Driver programs: ``linear_regression`` (default, twtml-spark main class) and ``kmeans``."""
