"""Micro-batch streaming runtime: RDD-like batches, DStreams, StreamingContext."""
from .rdd import RDD
from .streaming import Accumulator, BatchInfo, DStream, ReceiverDStream, Seconds, StreamingContext

__all__ = ["RDD", "Accumulator", "BatchInfo", "DStream", "ReceiverDStream", "Seconds",
           "StreamingContext"]
