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
        r = self._session.post(self._url(), data=data.to_json().encode("utf-8"), headers=_HEADERS,
                               timeout=self.timeout)
        r.raise_for_status()
        return r.text

    def get(self, kind: str) -> TypeData:
        r = self._session.get(self._url(kind), headers=_HEADERS, timeout=self.timeout)
        r.raise_for_status()
        return parse_type_data(r.text)

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
