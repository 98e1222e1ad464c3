"""Live Twitter receiver against a fake streaming endpoint (no network).

The fake server checks the OAuth 1.0a signature of every connection, streams
keep-alives, a delete notice and statuses, then drops the connection; the
receiver must reconnect and keep delivering.
"""
import json
import threading
import time
import urllib.parse

import pytest
from aiohttp import web

from twitter_stream_ml_amd.sources.twitter import (TwitterSource, TwitterUnavailable,
                                                   oauth1_signature)

KEYS = {"consumerKey": "ck", "consumerSecret": "cs s", "accessToken": "at",
        "accessTokenSecret": "ats"}


def test_signature_matches_twitter_documentation_example():
    # "Creating a signature" example from Twitter's OAuth 1.0a documentation
    params = {"include_entities": "true", "oauth_consumer_key": "xvz1evFS4wEEPTGEFPHBog",
              "oauth_nonce": "kYjzVBB8Y0ZFabxSWbWovY3uYSQ2pTgmZeNu2VS4cg",
              "oauth_signature_method": "HMAC-SHA1", "oauth_timestamp": "1318622958",
              "oauth_token": "370773112-GmHxMAgYyLbNEtIKZeRNFsMKPR9EyMZeS9weJAEb",
              "oauth_version": "1.0",
              "status": "Hello Ladies + Gentlemen, a signed OAuth request!"}
    sig = oauth1_signature("POST", "https://api.twitter.com/1.1/statuses/update.json", params,
                           "kAcSOqF21Fu85e7zjz7ZN2U4ZRhfV3WpwPAoE3Z7kBw",
                           "LswwdoUaIvS8ltyTt5jkRh4J50vUPVVHtR2YPi5kE")
    assert sig == "hCtSmYh+iHYCEqBWrE7C7hYmtUk="


def _status(i, rt=True):
    s = {"id": i, "text": f"tweet number {i} ünïcode", "retweet_count": 0,
         "created_at_ms": 1_700_000_000_000 + i, "user": {"followers_count": i}}
    if rt:
        s["retweeted_status"] = {"id": 10_000 + i, "text": f"original {i}", "retweet_count": 150 + i,
                                 "created_at_ms": 1_699_999_000_000,
                                 "user": {"followers_count": 1000 + i, "favourites_count": 5,
                                          "friends_count": 7}}
    return s


class FakeStream:
    def __init__(self):
        self.connections = 0
        self.bad_auth = 0
        self.runner = None
        self.url = None

    def _check_auth(self, request):
        auth = request.headers.get("Authorization", "")
        assert auth.startswith("OAuth ")
        fields = dict(urllib.parse.unquote(p.strip()).split("=", 1) for p in auth[6:].split(","))
        fields = {k: v.strip('"') for k, v in fields.items()}
        sig = fields.pop("oauth_signature")
        url = f"http://{request.host}{request.path}"
        want = oauth1_signature("GET", url, fields, KEYS["consumerSecret"], KEYS["accessTokenSecret"])
        return sig == want and fields["oauth_consumer_key"] == "ck" and fields["oauth_token"] == "at"

    async def handler(self, request):
        if not self._check_auth(request):
            self.bad_auth += 1
            return web.Response(status=401)
        self.connections += 1
        resp = web.StreamResponse()
        await resp.prepare(request)
        base = self.connections * 100
        await resp.write(b"\r\n")                                     # keep-alive
        await resp.write(json.dumps({"delete": {"status": {"id": 1}}}).encode() + b"\r\n")
        for i in range(5):
            await resp.write(json.dumps(_status(base + i, rt=i % 2 == 0)).encode() + b"\r\n")
        return resp                                                   # connection closes

    def start(self):
        import asyncio
        loop = asyncio.new_event_loop()
        ready = threading.Event()

        async def boot():
            app = web.Application()
            app.router.add_get("/1.1/statuses/sample.json", self.handler)
            self.runner = web.AppRunner(app)
            await self.runner.setup()
            site = web.TCPSite(self.runner, "127.0.0.1", 0)
            await site.start()
            port = site._server.sockets[0].getsockname()[1]
            self.url = f"http://127.0.0.1:{port}/1.1/statuses/sample.json"
            ready.set()

        def run():
            asyncio.set_event_loop(loop)
            loop.run_until_complete(boot())
            loop.run_forever()

        threading.Thread(target=run, daemon=True).start()
        ready.wait(10)
        self.loop = loop
        return self

    def stop(self):
        import asyncio
        fut = asyncio.run_coroutine_threadsafe(self.runner.cleanup(), self.loop)
        fut.result(10)
        self.loop.call_soon_threadsafe(self.loop.stop)


def test_receiver_streams_reconnects_and_batches():
    fake = FakeStream().start()
    try:
        src = TwitterSource(url=fake.url, oauth=dict(KEYS)).start()
        deadline = time.time() + 20
        while src.received < 10 and time.time() < deadline:
            time.sleep(0.05)
        assert fake.bad_auth == 0
        assert src.received >= 10 and fake.connections >= 2 and src.reconnects >= 1
        b = src.poll(7, now_ms=123)
        assert b.n == 7 and b.batch_time_ms == 123
        sts = b.to_statuses()
        # RawBatch keeps what the features need: the original's text/counts for retweets
        assert sts[0].isRetweet() and sts[0].getRetweetedStatus().getRetweetCount() == 150 + 100
        assert sts[0].getRetweetedStatus().getText() == "original 100"
        assert not sts[1].isRetweet() and sts[1].getText() == "tweet number 101 ünïcode"
        src.stop()
    finally:
        fake.stop()


def test_missing_keys_fail_fast():
    with pytest.raises(TwitterUnavailable, match="OAuth"):
        TwitterSource(url="http://127.0.0.1:9/x", oauth={k: "" for k in KEYS}).start()
