"""Live Twitter source (``TwitterUtils.createStream(ssc, None)``).

The statuses/sample endpoint the reference reads (twitter4j 4.0.4 with the
``twitter4j.oauth.*`` system properties) no longer exists, and this build has
no network.  The class keeps the OAuth plumbing so the CLI surface is intact
and fails with an actionable message when polled.
"""
from __future__ import annotations

from ..config.hocon import get_property

__all__ = ["TwitterSource", "TwitterUnavailable"]

OAUTH_KEYS = ("consumerKey", "consumerSecret", "accessToken", "accessTokenSecret")


class TwitterUnavailable(RuntimeError):
    pass


class TwitterSource:
    def __init__(self) -> None:
        self.oauth = {k: get_property("twitter4j.oauth." + k, "") for k in OAUTH_KEYS}

    def poll(self, max_n: int, now_ms=None):
        missing = [k for k, v in self.oauth.items() if not v]
        why = f"missing OAuth keys {missing}" if missing else "the v1.1 sample stream is retired"
        raise TwitterUnavailable(
            f"live Twitter ingest is unavailable ({why}); use --source synthetic or "
            "--source replay:FILE.jsonl")
