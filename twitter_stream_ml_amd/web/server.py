"""twtml-web HTTP/WebSocket server (``Server.scala``, ``ApiHandler.scala``; C10-C11).

Routes (``Server.scala:22-64``):

* WebSocket handshake on ``/api`` -> on completion the current config is sent
  to that socket only (``ApiHandler.scala:68-73``); every text frame is cached
  and broadcast verbatim to all sockets (``:59-67``).
* ``POST /api`` -> cache, reply ``{"status":"OK"}``, broadcast the raw posted
  JSON to every socket (``:50-57``).
* ``GET /api/config`` / ``GET /api/stats`` -> cached JSON, ``application/json``.
* ``/`` -> ``index.html``; any other path -> static file under the asset dir;
  else 404.

Built on aiohttp with one asyncio loop (no actor per request); the server can
run in the foreground (``Main``) or on a background thread (tests, embedding
in the streaming job).  An unknown ``jsonClass`` is answered with HTTP 400
instead of the reference's dropped request.
"""
from __future__ import annotations

import asyncio
import json
import logging
import os
import threading
import weakref
from typing import Optional, Set

from aiohttp import WSMsgType, web

from .cache import ApiCache

__all__ = ["TwtmlWebServer", "ASSET_DIR", "make_app"]

log = logging.getLogger("com.giorgioinf.twtml.web.Server")
ASSET_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "assets")
OK = json.dumps({"status": "OK"}, separators=(",", ":"))
SOCKETS = web.AppKey("sockets", object)
CACHE = web.AppKey("cache", ApiCache)


def make_app(cache: ApiCache, asset_dir: str = ASSET_DIR) -> web.Application:
    app = web.Application()
    sockets: Set[web.WebSocketResponse] = weakref.WeakSet()  # type: ignore[assignment]
    app[SOCKETS] = sockets
    app[CACHE] = cache

    async def broadcast(text: str) -> None:
        for ws in list(sockets):
            if not ws.closed:
                try:
                    await ws.send_str(text)
                except (ConnectionResetError, RuntimeError):
                    pass

    async def api(request: web.Request) -> web.StreamResponse:
        if request.method == "GET":
            ws = web.WebSocketResponse()
            if not ws.can_prepare(request).ok:
                raise web.HTTPNotFound()
            await ws.prepare(request)
            sockets.add(ws)
            log.debug("websocket - connected, send config")
            await ws.send_str(cache.config())
            try:
                async for msg in ws:
                    if msg.type == WSMsgType.TEXT:
                        try:
                            cache.cache(msg.data)
                        except ValueError as e:
                            log.error("json not recognized: %s (%s)", msg.data, e)
                            continue
                        await broadcast(msg.data)
                    elif msg.type == WSMsgType.ERROR:
                        break
            finally:
                sockets.discard(ws)
            return ws
        # POST
        body = await request.text()
        log.debug("http - post data %s", body)
        try:
            cache.cache(body)
        except ValueError as e:
            return web.Response(status=400, text=json.dumps({"status": "ERROR", "error": str(e)}),
                                content_type="application/json")
        await broadcast(body)
        return web.Response(text=OK, content_type="application/json")

    async def get_config(request: web.Request) -> web.Response:
        return web.Response(text=cache.config(), content_type="application/json")

    async def get_stats(request: web.Request) -> web.Response:
        return web.Response(text=cache.stats(), content_type="application/json")

    async def static(request: web.Request) -> web.StreamResponse:
        rel = request.match_info.get("path", "") or "index.html"
        full = os.path.realpath(os.path.join(asset_dir, rel))
        root = os.path.realpath(asset_dir)
        if not full.startswith(root + os.sep) or not os.path.isfile(full):
            raise web.HTTPNotFound()
        return web.FileResponse(full)

    app.router.add_route("GET", "/api", api)
    app.router.add_route("POST", "/api", api)
    app.router.add_route("GET", "/api/config", get_config)
    app.router.add_route("GET", "/api/stats", get_stats)
    app.router.add_route("GET", "/", static)
    app.router.add_route("GET", "/{path:.*}", static)
    return app


class TwtmlWebServer:
    """Owns the asyncio loop; ``start()`` serves on a background thread."""

    def __init__(self, host: str = "0.0.0.0", port: Optional[int] = None,
                 cache: Optional[ApiCache] = None, asset_dir: str = ASSET_DIR):
        self.host = host
        self.port = int(port if port is not None else os.environ.get("PORT", "8888"))
        self.cache = cache or ApiCache()
        self.asset_dir = asset_dir
        self._loop: Optional[asyncio.AbstractEventLoop] = None
        self._runner: Optional[web.AppRunner] = None
        self._thread: Optional[threading.Thread] = None
        self._ready = threading.Event()
        self._error: Optional[BaseException] = None

    async def _start_async(self) -> None:
        self.app = make_app(self.cache, self.asset_dir)
        self._runner = web.AppRunner(self.app, access_log=None)
        await self._runner.setup()
        site = web.TCPSite(self._runner, self.host, self.port)
        await site.start()
        if self.port == 0:  # ephemeral port (tests)
            self.port = site._server.sockets[0].getsockname()[1]  # type: ignore[union-attr]
        log.info("Open your browser and navigate to http://%s:%s", self.host, self.port)

    async def _stop_async(self) -> None:
        for ws in list(self.app[SOCKETS]):
            await ws.close()
        if self._runner is not None:
            await self._runner.cleanup()

    def start(self) -> "TwtmlWebServer":
        def run() -> None:
            self._loop = asyncio.new_event_loop()
            asyncio.set_event_loop(self._loop)
            try:
                self._loop.run_until_complete(self._start_async())
            except BaseException as e:  # pragma: no cover - surfaced in start()
                self._error = e
                self._ready.set()
                return
            self._ready.set()
            self._loop.run_forever()
            self._loop.run_until_complete(self._stop_async())
            self._loop.close()

        self._thread = threading.Thread(target=run, name="twtml-web", daemon=True)
        self._thread.start()
        self._ready.wait(30)
        if self._error is not None:
            raise self._error
        return self

    def stop(self) -> None:
        if self._loop is not None and self._thread is not None:
            self._loop.call_soon_threadsafe(self._loop.stop)
            self._thread.join(timeout=10)
            self._thread = None

    def serve_forever(self) -> None:
        self.start()
        try:
            while self._thread is not None and self._thread.is_alive():
                self._thread.join(1.0)
        except KeyboardInterrupt:
            pass
        finally:
            self.stop()

    @property
    def url(self) -> str:
        host = "127.0.0.1" if self.host in ("0.0.0.0", "") else self.host
        return f"http://{host}:{self.port}"
