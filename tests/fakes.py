"""Test doubles: a fake Lightning server that records every REST call.

The reference has no Lightning fake ("no mock HTTP server"); this
one implements the three endpoints the client uses and remembers payloads.
``FakeLightningProcess`` serves the same endpoints from a child process (so
its JSON parsing does not share the test's GIL) and reports a summary of the
appends over ``GET /_summary``.
"""
from __future__ import annotations

import asyncio
import itertools
import json
import os
import subprocess
import sys
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

        async def summary(request: web.Request) -> web.Response:
            apps = self.appends()
            return web.json_response({
                "calls": len(self.calls), "appends": len(apps),
                "last_series_lens": [len(s) for s in apps[-1]["data"]["series"]] if apps else []})

        app.router.add_route("GET", "/_summary", summary)
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


class FakeLightningProcess:
    """``FakeLightning`` in a child process; ``summary()`` -> ``{"calls",
    "appends", "last_series_lens"}``."""

    def __init__(self):
        self.proc = None
        self.port = 0

    def start(self) -> "FakeLightningProcess":
        env = dict(os.environ, PYTHONPATH=os.path.dirname(os.path.abspath(__file__)))
        self.proc = subprocess.Popen([sys.executable, "-c", "import fakes; fakes._serve()"],
                                     stdout=subprocess.PIPE, env=env, text=True)
        self.port = int(self.proc.stdout.readline())
        return self

    @property
    def url(self) -> str:
        return f"http://127.0.0.1:{self.port}"

    def summary(self) -> Dict[str, Any]:
        import requests
        return requests.get(self.url + "/_summary", timeout=10).json()

    def stop(self) -> None:
        if self.proc is not None:
            self.proc.terminate()
            try:
                self.proc.wait(10)
            except subprocess.TimeoutExpired:
                self.proc.kill()
            self.proc = None


def _serve() -> None:
    srv = FakeLightning().start()
    print(srv.port, flush=True)
    srv._thread.join()
