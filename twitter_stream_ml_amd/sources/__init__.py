"""Tweet sources: synthetic (seeded C++ generator), JSONL replay, live Twitter stream."""
from .replay import JsonlReplaySource, write_jsonl
from .synthetic import SynthConfig, SyntheticTweetSource, generate_batch, generate_into
from .twitter import TwitterSource, TwitterUnavailable

__all__ = ["JsonlReplaySource", "write_jsonl", "SynthConfig", "SyntheticTweetSource",
           "generate_batch", "generate_into", "TwitterSource", "TwitterUnavailable",
           "make_source"]


def make_source(spec: str, rate: float = 0.0, seed: int = 1, profile: str = "twitter",
                shard: int = 0, num_shards: int = 1, start: int = 0):
    """``--source`` value -> source object; ``start`` = records already consumed."""
    if spec in ("", "synthetic"):
        return SyntheticTweetSource(SynthConfig.profile(profile, seed=seed), rate=rate,
                                    shard=shard, num_shards=num_shards, start=start)
    if spec.startswith("replay:"):
        return JsonlReplaySource(spec[len("replay:"):], rate=rate, skip=start, shard=shard,
                                 num_shards=num_shards)
    if spec == "twitter":
        return TwitterSource().start()          # fails fast without OAuth keys
    raise ValueError(f"unknown source {spec!r}")
