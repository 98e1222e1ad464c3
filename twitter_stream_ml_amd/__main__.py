"""``python -m twitter_stream_ml_amd [args]`` = the twtml-spark default main class
(``spark/build.sbt:10``: LinearRegression)."""
import sys

from .apps.linear_regression import main

sys.exit(main())
