"""Test doubles: a fake Lightning server that records every REST call.

The reference has no Lightning fake ("no mock HTTP server"); this
one implements the three endpoints the client uses and remembers payloads.
"""
from __future__ import annotations

import asyncio
import itertools
import threading
from typing import Any, Dict, List, Tuple

from aiohttp import web


class FakeLightning:
    def __init__(self, fail: bool = False):
        self.calls: List[Tuple[str, str, Any]] = []
        self.fail = fail
        self._ids = itertools.count(1)
        self.port = 0
        self._loop = None
        self._thread = None
        self._ready = threading.Event()

    def _app(self) -> web.Application:
        app = web.Application()

        async def handler(request: web.Request) -> web.Response:
            body = await request.json() if request.can_read_body else None
            self.calls.append((request.method, request.path, body))
            if self.fail:
                return web.Response(status=500, text="boom")
            if request.path == "/sessions/":
                return web.json_response({"id": f"s{next(self._ids)}"})
            if request.path.endswith("/visualizations/"):
                return web.json_response({"id": f"v{next(self._ids)}"})
            return web.json_response({})

        app.router.add_route("POST", "/{tail:.*}", handler)
        return app

    def start(self) -> "FakeLightning":
        def run():
            self._loop = asyncio.new_event_loop()
            asyncio.set_event_loop(self._loop)
            runner = web.AppRunner(self._app(), access_log=None)
            self._loop.run_until_complete(runner.setup())
            site = web.TCPSite(runner, "127.0.0.1", 0)
            self._loop.run_until_complete(site.start())
            self.port = site._server.sockets[0].getsockname()[1]
            self._ready.set()
            self._loop.run_forever()
            self._loop.run_until_complete(runner.cleanup())

        self._thread = threading.Thread(target=run, daemon=True)
        self._thread.start()
        self._ready.wait(10)
        return self

    @property
    def url(self) -> str:
        return f"http://127.0.0.1:{self.port}"

    def stop(self) -> None:
        if self._loop:
            self._loop.call_soon_threadsafe(self._loop.stop)
            self._thread.join(5)

    def appends(self) -> List[Dict[str, Any]]:
        return [b for (m, p, b) in self.calls if p.endswith("/data/")]
