"""twitter_stream_ml_amd -- an MI355X-native streaming-ML engine.

Capabilities of QilinGu/twitter-stream-ml (twtml-spark + twtml-web), rebuilt
for AMD Instinct MI355X (gfx950): tweet-shaped records are ingested into
GPU-resident micro-batches and trained online with a
StreamingLinearRegressionWithSGD-equivalent whose filter / bigram-HashingTF /
predict / gradient / update pipeline is hand-written CDNA4 HIP, data-parallel
over RCCL; plus streaming k-means, the twtml-web reporting server, and
MLlib-layout checkpoints.

Subpackages: config, records, sources, runtime, ops (native engines), models,
oracle (fp64 reference semantics), parallel, checkpoint, report, web, apps,
utils.
"""
__version__ = "0.1.0"
