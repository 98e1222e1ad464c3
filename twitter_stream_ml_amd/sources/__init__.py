"""Tweet sources: synthetic (seeded C++ generator), JSONL replay, live Twitter stream."""
from .replay import JsonlReplaySource, write_jsonl
from .synthetic import SynthConfig, SyntheticReplaySource, SyntheticTweetSource, generate_batch, generate_into
from .twitter import TwitterSource, TwitterUnavailable

__all__ = ["JsonlReplaySource", "write_jsonl", "SynthConfig", "SyntheticTweetSource",
           "SyntheticReplaySource", "generate_batch", "generate_into", "TwitterSource", "TwitterUnavailable",
           "make_source"]


def make_source(spec: str, rate: float = 0.0, seed: int = 1, profile: str = "twitter",
                shard: int = 0, num_shards: int = 1, start: int = 0, batch_size: int = 0):
    """``--source`` value -> source object; ``start`` = records already consumed.

    ``synthetic[:<profile>]``: the seeded generator, live; ``replay:synthetic
    :<profile>:<batches>``: a pool of ``batches`` pre-generated batches of
    ``batch_size`` tweets replayed from page-locked UTF-8 buffers;
    ``replay:<file.jsonl>``: recorded statuses; ``twitter``: the live stream."""
    if spec in ("", "synthetic") or spec.startswith("synthetic:"):
        prof = spec.split(":", 1)[1] if ":" in spec else profile
        return SyntheticTweetSource(SynthConfig.profile(prof, seed=seed), rate=rate,
                                    shard=shard, num_shards=num_shards, start=start)
    if spec.startswith("replay:synthetic"):
        parts = spec.split(":")
        prof = parts[2] if len(parts) > 2 and parts[2] else profile
        nb = int(parts[3]) if len(parts) > 3 and parts[3] else 8
        if rate > 0:
            raise ValueError("replay:synthetic replays as fast as the job asks (use --sourceRate 0)")
        return SyntheticReplaySource(SynthConfig.profile(prof, seed=seed + 7919 * shard), nb, batch_size,
                                     shard=shard, num_shards=num_shards, start=start)
    if spec.startswith("replay:"):
        return JsonlReplaySource(spec[len("replay:"):], rate=rate, skip=start, shard=shard,
                                 num_shards=num_shards)
    if spec == "twitter":
        return TwitterSource().start()          # fails fast without OAuth keys
    raise ValueError(f"unknown source {spec!r}")
