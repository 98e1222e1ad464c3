"""HTTP client of twtml-web (``WebClient.scala:9-56``).

``POST {server}/api`` with the json4s body of a ``Config``/``Stats``;
``GET {server}/api/config`` and ``GET {server}/api/stats``.  Headers
``content-type`` and ``accept`` are ``application/json``; the default server
is ``http://localhost:8888``.  Timeouts are explicit so a dead server never
stalls a caller for long (the reference's scalaj-http defaults are 1 s
connect / 5 s read).
"""
from __future__ import annotations

from typing import List, Optional

import requests

from .http import post as http_post
from .api_types import Config, Stats, TypeData, parse_type_data

__all__ = ["WebClient"]

_HEADERS = {"content-type": "application/json", "accept": "application/json"}


class WebClient:
    def __init__(self, server: str = "http://localhost:8888", timeout: float = 5.0):
        self.server = (server or "http://localhost:8888").rstrip("/")
        self.timeout = timeout
        self._session = requests.Session()

    @classmethod
    def apply(cls, host: str = "") -> "WebClient":
        """``WebClient(host)`` companion: empty host -> default server."""
        return cls() if host == "" else cls(host)

    def _url(self, kind: str = "") -> str:
        return self.server + "/api" + kind

    def post(self, data: TypeData) -> str:
        status, content = http_post(self._url(), data.to_json().encode("utf-8"), timeout=self.timeout,
                                    session=self._session)
        if status >= 400:
            raise requests.HTTPError(f"{status} posting to {self._url()}")
        return content.decode("utf-8", "replace")

    def get(self, kind: str) -> TypeData:
        r = self._session.get(self._url(kind), headers=_HEADERS, timeout=self.timeout)
        r.raise_for_status()
        return parse_type_data(_text(r))

    # -- the reference's four calls (WebClient.scala:31-46) ----------------
    def config(self, id: Optional[str] = None, host: Optional[str] = None,
               viz: Optional[List[str]] = None):
        if id is None and host is None and viz is None:
            return self.get("/config")
        return self.post(Config(id or "", host or "", list(viz or [])))

    def stats(self, count: Optional[int] = None, batch: int = 0, mse: int = 0,
              realStddev: int = 0, predStddev: int = 0):
        if count is None:
            return self.get("/stats")
        return self.post(Stats(int(count), int(batch), int(mse), int(realStddev), int(predStddev)))

    def close(self) -> None:
        self._session.close()


def _text(r: "requests.Response") -> str:
    # UTF-8 JSON: decoded directly; ``Response.text`` guesses an encoding
    # when the server names none, and its first use imports a charset
    # detector on the reporting thread while the training thread waits on
    # the GIL
    return r.content.decode("utf-8", "replace")
