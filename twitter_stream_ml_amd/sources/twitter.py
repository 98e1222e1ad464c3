"""Live Twitter source (``TwitterUtils.createStream(ssc, None)``).

The reference opens ``statuses/sample`` through twitter4j 4.0.4 with the OAuth
keys that ``ConfArguments`` pushes into the ``twitter4j.oauth.*`` system
properties, in a receiver that restarts itself on errors.  This is the same
receiver, natively in Python:

* OAuth 1.0a request signing (HMAC-SHA1, RFC 5849) from the
  ``twitter4j.oauth.*`` properties;
* a background reader thread on a streaming HTTP connection that parses one
  JSON status per line (``delete``/``limit``/keep-alive lines are skipped)
  into a bounded buffer (oldest records dropped when the job falls behind,
  like a receiver whose block store is full);
* reconnect with twitter4j's back-off (linear 250 ms steps up to 16 s on
  network errors, exponential from 5 s up to 320 s on HTTP errors, from 60 s on
  420/429 rate limiting).

The endpoint defaults to the v1.1 sample stream and can be pointed elsewhere
(``twitterStreamUrl`` config key or ``TWTML_TWITTER_STREAM_URL``) -- e.g. a
compatible relay, or the fake server the tests use.  With missing keys,
``poll`` raises :class:`TwitterUnavailable` with an actionable message.
"""
from __future__ import annotations

import base64
import collections
import hashlib
import hmac
import json
import logging
import os
import secrets
import threading
import time
import urllib.parse
from typing import Deque, Dict, Optional

from ..config.hocon import get_property
from ..records.batch import RawBatch
from ..records.schema import Status, status_from_json

__all__ = ["TwitterSource", "TwitterUnavailable", "oauth1_header", "oauth1_signature",
           "DEFAULT_STREAM_URL"]

log = logging.getLogger("twtml.sources.twitter")
OAUTH_KEYS = ("consumerKey", "consumerSecret", "accessToken", "accessTokenSecret")
DEFAULT_STREAM_URL = "https://stream.twitter.com/1.1/statuses/sample.json"


class TwitterUnavailable(RuntimeError):
    pass


def _pct(s: str) -> str:
    return urllib.parse.quote(str(s), safe="-._~")


def oauth1_signature(method: str, url: str, params: Dict[str, str], consumer_secret: str,
                     token_secret: str) -> str:
    """RFC 5849 §3.4 HMAC-SHA1 signature of a request."""
    parsed = urllib.parse.urlsplit(url)
    base_url = f"{parsed.scheme.lower()}://{parsed.netloc.lower()}{parsed.path}"
    pairs = sorted((_pct(k), _pct(v)) for k, v in params.items())
    norm = "&".join(f"{k}={v}" for k, v in pairs)
    base = "&".join([method.upper(), _pct(base_url), _pct(norm)])
    key = f"{_pct(consumer_secret)}&{_pct(token_secret)}".encode()
    return base64.b64encode(hmac.new(key, base.encode(), hashlib.sha1).digest()).decode()


def oauth1_header(method: str, url: str, oauth: Dict[str, str], query: Optional[Dict[str, str]] = None,
                  nonce: Optional[str] = None, timestamp: Optional[int] = None) -> str:
    """``Authorization: OAuth ...`` value for a request."""
    o = {
        "oauth_consumer_key": oauth["consumerKey"],
        "oauth_nonce": nonce or secrets.token_hex(16),
        "oauth_signature_method": "HMAC-SHA1",
        "oauth_timestamp": str(int(time.time()) if timestamp is None else timestamp),
        "oauth_token": oauth["accessToken"],
        "oauth_version": "1.0",
    }
    params = dict(o)
    params.update(query or {})
    parsed = urllib.parse.urlsplit(url)
    params.update(dict(urllib.parse.parse_qsl(parsed.query)))
    o["oauth_signature"] = oauth1_signature(method, url.split("?")[0], params,
                                            oauth["consumerSecret"], oauth["accessTokenSecret"])
    return "OAuth " + ", ".join(f'{_pct(k)}="{_pct(v)}"' for k, v in sorted(o.items()))


class TwitterSource:
    """Receiver for a streaming statuses endpoint (one JSON status per line)."""

    def __init__(self, url: Optional[str] = None, oauth: Optional[Dict[str, str]] = None,
                 buffer: int = 1 << 20, connect_timeout: float = 10.0, read_timeout: float = 90.0):
        self.oauth = oauth or {k: get_property("twitter4j.oauth." + k, "") for k in OAUTH_KEYS}
        self.url = (url or os.environ.get("TWTML_TWITTER_STREAM_URL")
                    or get_property("twitterStreamUrl", "") or DEFAULT_STREAM_URL)
        self.timeouts = (connect_timeout, read_timeout)
        self._buf: Deque[Status] = collections.deque(maxlen=int(buffer))
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self.connected = threading.Event()
        self.received = 0
        self.dropped = 0
        self.reconnects = 0
        self.last_error: Optional[str] = None

    # ---- receiver lifecycle ---------------------------------------------------
    def _check_keys(self) -> None:
        missing = [k for k, v in self.oauth.items() if not v]
        if missing:
            raise TwitterUnavailable(
                f"live Twitter ingest needs OAuth keys (missing {missing}: set them in "
                "application.conf or with -C/-S/-A/-T); or use --source synthetic / "
                "--source replay:FILE.jsonl")

    def start(self) -> "TwitterSource":
        self._check_keys()
        if self._thread is None:
            self._thread = threading.Thread(target=self._run, name="twitter-receiver", daemon=True)
            self._thread.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5)

    close = stop

    def _run(self) -> None:
        import requests
        net_wait, http_wait = 0.0, 0.0
        while not self._stop.is_set():
            try:
                hdr = {"Authorization": oauth1_header("GET", self.url, self.oauth),
                       "User-Agent": "twtml-mi355x"}
                with requests.get(self.url, headers=hdr, stream=True, timeout=self.timeouts) as r:
                    if r.status_code != 200:
                        self.last_error = f"HTTP {r.status_code}"
                        if r.status_code in (420, 429):
                            http_wait = max(60.0, http_wait * 2)
                        else:
                            http_wait = min(320.0, max(5.0, http_wait * 2))
                        log.warning("twitter stream: %s; retry in %.0f s", self.last_error, http_wait)
                        self._stop.wait(http_wait)
                        continue
                    net_wait, http_wait = 0.0, 0.0
                    self.connected.set()
                    for line in r.iter_lines(chunk_size=1, decode_unicode=False):
                        if self._stop.is_set():
                            return
                        self._on_line(line)
            except Exception as e:  # network error: receiver restart
                self.last_error = repr(e)
                net_wait = min(16.0, net_wait + 0.25)
                log.warning("twitter stream error %s; reconnect in %.2f s", e, net_wait)
                self._stop.wait(net_wait)
            finally:
                self.connected.clear()
            self.reconnects += 1

    def _on_line(self, line: bytes) -> None:
        if not line or not line.strip():
            return                               # keep-alive newline
        try:
            obj = json.loads(line)
        except ValueError:
            return
        if not isinstance(obj, dict) or "text" not in obj and "full_text" not in obj:
            return                               # delete / limit / warning notices
        try:
            st = status_from_json(obj)
        except (KeyError, TypeError, ValueError):
            return
        with self._lock:
            if len(self._buf) == self._buf.maxlen:
                self.dropped += 1
            self._buf.append(st)
            self.received += 1

    # ---- source protocol ------------------------------------------------------
    def poll(self, max_n: int, now_ms: Optional[int] = None) -> RawBatch:
        if self._thread is None:
            self.start()
        out = []
        with self._lock:
            while self._buf and len(out) < int(max_n):
                out.append(self._buf.popleft())
        return RawBatch.from_statuses(out, batch_time_ms=int(now_ms or time.time() * 1000))
