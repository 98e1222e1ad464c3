"""POST for the report sinks (Lightning, twtml-web), off the GIL.

``post(url, body)`` sends a JSON body and returns ``(status, content)``.  For
``http://`` URLs it runs ``_twtml_host.http_post`` (``csrc/host/http_post.cpp``)
with the GIL released for the whole exchange: through ``requests`` the
reporting thread gives up and re-takes the GIL around every socket call,
CPython does not hand it fairly to a waiting thread, and the training thread
was measured stalling up to ~9 ms behind one plot append.  ``https://`` (or a
missing host extension) goes through ``requests``.  Connection failures raise
``requests.ConnectionError`` either way.
"""
from __future__ import annotations

import base64
from typing import Optional, Tuple
from urllib.parse import urlsplit

import requests

__all__ = ["post"]


def _native():
    try:
        from ..ops._native import NativeUnavailable, host
        return host()
    except (ImportError, NativeUnavailable):
        return None


def post(url: str, body: bytes, auth: Optional[tuple] = None, timeout: float = 5.0,
         session: Optional[requests.Session] = None) -> Tuple[int, bytes]:
    u = urlsplit(url)
    h = _native() if u.scheme == "http" and u.hostname else None
    if h is None:
        r = (session or requests).post(url, data=body, auth=auth, timeout=timeout,
                                       headers={"Content-Type": "application/json",
                                                "Accept": "application/json"})
        return r.status_code, r.content
    headers = ""
    if auth:
        tok = base64.b64encode(f"{auth[0]}:{auth[1]}".encode()).decode()
        headers = f"Authorization: Basic {tok}\r\n"
    path = (u.path or "/") + (f"?{u.query}" if u.query else "")
    try:
        return h.http_post(u.hostname, u.port or 80, path, body, headers, float(timeout))
    except ConnectionError as e:
        raise requests.ConnectionError(f"{url}: {e}") from e
