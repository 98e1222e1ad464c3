"""The report sinks' native POST (``csrc/host/http_post.cpp`` via
``report/http.py``): the whole exchange runs without the GIL.  Checked
against a local aiohttp server: Content-Length and chunked bodies, an error
status, basic auth, a refused connection and a server that never answers."""
import asyncio
import socket
import threading
import time

import pytest
import requests
from aiohttp import web

from twitter_stream_ml_amd.report.http import post


class _Server:
    def __init__(self):
        self.seen = []
        self._ready = threading.Event()

    def start(self):
        async def echo(request):
            body = await request.read()
            self.seen.append((request.path, dict(request.headers), body))
            return web.json_response({"n": len(body)})

        async def chunked(request):
            await request.read()
            resp = web.StreamResponse()
            resp.enable_chunked_encoding()
            await resp.prepare(request)
            for part in (b'{"a":', b' [1, 2', b', 3]}'):
                await resp.write(part)
            await resp.write_eof()
            return resp

        async def fail(request):
            await request.read()
            return web.Response(status=503, text="busy")

        async def slow(request):
            await asyncio.sleep(5)
            return web.json_response({})

        def run():
            self.loop = asyncio.new_event_loop()
            asyncio.set_event_loop(self.loop)
            app = web.Application(client_max_size=64 << 20)
            app.router.add_post("/echo", echo)
            app.router.add_post("/chunked", chunked)
            app.router.add_post("/fail", fail)
            app.router.add_post("/slow", slow)
            runner = web.AppRunner(app, access_log=None)
            self.loop.run_until_complete(runner.setup())
            site = web.TCPSite(runner, "127.0.0.1", 0)
            self.loop.run_until_complete(site.start())
            self.port = site._server.sockets[0].getsockname()[1]
            self._ready.set()
            self.loop.run_forever()

        self.th = threading.Thread(target=run, daemon=True)
        self.th.start()
        self._ready.wait(10)
        return self

    def stop(self):
        self.loop.call_soon_threadsafe(self.loop.stop)
        self.th.join(5)


@pytest.fixture(scope="module")
def srv():
    s = _Server().start()
    yield s
    s.stop()


def test_post_content_length_and_big_body(srv):
    body = b'{"x":"' + b"y" * (3 << 20) + b'"}'          # a few MB: many send() rounds
    status, content = post(f"http://127.0.0.1:{srv.port}/echo?q=1", body)
    assert status == 200 and content == b'{"n": %d}' % len(body)
    path, headers, got = srv.seen[-1]
    assert path == "/echo" and got == body
    assert headers["Content-Type"] == "application/json"


def test_post_chunked_response(srv):
    status, content = post(f"http://127.0.0.1:{srv.port}/chunked", b"{}")
    assert status == 200 and content == b'{"a": [1, 2, 3]}'


def test_post_error_status_is_a_response(srv):
    status, content = post(f"http://127.0.0.1:{srv.port}/fail", b"{}")
    assert status == 503 and content == b"busy"


def test_post_basic_auth_header(srv):
    post(f"http://127.0.0.1:{srv.port}/echo", b"{}", auth=("user", "pa:ss"))
    assert srv.seen[-1][1]["Authorization"] == "Basic dXNlcjpwYTpzcw=="


def test_post_refused_and_timeout(srv):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()                                            # nothing listens there
    with pytest.raises(requests.ConnectionError):
        post(f"http://127.0.0.1:{port}/x", b"{}", timeout=2.0)
    t = time.perf_counter()
    with pytest.raises(requests.ConnectionError, match="timed out"):
        post(f"http://127.0.0.1:{srv.port}/slow", b"{}", timeout=0.3)
    assert time.perf_counter() - t < 2.0


def test_post_releases_the_gil(srv):
    """Another Python thread keeps running while a request waits on the
    server (the whole exchange is one GIL-released native call)."""
    ticks = []
    stop = threading.Event()

    def spin():
        while not stop.is_set():
            ticks.append(time.perf_counter())
            time.sleep(0.001)

    th = threading.Thread(target=spin)
    th.start()
    with pytest.raises(requests.ConnectionError):
        post(f"http://127.0.0.1:{srv.port}/slow", b"{}", timeout=0.5)
    stop.set()
    th.join()
    gaps = [b - a for a, b in zip(ticks, ticks[1:])]
    assert len(ticks) > 100 and max(gaps) < 0.1


def _raw_server(response: bytes):
    """One-shot TCP server that answers any request with `response` bytes."""
    ls = socket.socket()
    ls.bind(("127.0.0.1", 0))
    ls.listen(1)

    def run():
        c, _ = ls.accept()
        c.settimeout(5)
        try:
            c.recv(65536)
            c.sendall(response)
        finally:
            c.close()
            ls.close()

    threading.Thread(target=run, daemon=True).start()
    return ls.getsockname()[1]


@pytest.mark.parametrize("response", [
    b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\nConnection: close\r\n\r\nZZ\r\nabc\r\n0\r\n\r\n",
    b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\nConnection: close\r\n\r\nffffffffffffffffff\r\nabc\r\n",
    b"HTTP/1.1 200 OK\r\nContent-Length: 12abc\r\nConnection: close\r\n\r\nhello",
    b"HTTP/1.1 200 OK\r\nContent-Length: 99999999999999999999999\r\nConnection: close\r\n\r\nhello",
], ids=["bad-chunk", "huge-chunk", "bad-length", "huge-length"])
def test_post_malformed_response_is_a_connection_error(response):
    """a malformed chunk size or Content-Length is an HttpError
    (-> requests.ConnectionError, what the Lightning / twtml-web clients
    catch), not a ValueError / IndexError leaking from std::stoul."""
    port = _raw_server(response)
    with pytest.raises(requests.ConnectionError, match="malformed|range|truncated"):
        post(f"http://127.0.0.1:{port}/x", b"{}", timeout=5.0)


def test_chunk_extension_is_accepted():
    port = _raw_server(b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\nConnection: close\r\n\r\n"
                       b"3;ext=1\r\nabc\r\n0\r\n\r\n")
    assert post(f"http://127.0.0.1:{port}/x", b"{}", timeout=5.0) == (200, b"abc")
