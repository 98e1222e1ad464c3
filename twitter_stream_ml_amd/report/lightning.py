"""REST client for a Lightning visualization server.

Re-implements the slice of the vendored ``lightning-scala`` jar the reference
uses (``SessionStats.scala:11,31-33,49-52``; endpoints inferred from the jar's
constant pool):

* ``POST {host}/sessions/`` ``{"name": ...}`` -> ``{"id": ...}`` (createSession;
  done lazily on first plot, the jar's ``checkSession``)
* ``POST {host}/sessions/{s}/visualizations/`` ``{"type": "line-streaming",
  "data": {...}}`` -> ``{"id": ...}``
* ``POST {host}/sessions/{s}/visualizations/{id}/data/`` ``{"data": {...}}``
  (append to a streaming viz)
* embed URL ``{host}/visualizations/{id}/pym``

Optional HTTP basic auth as in the jar.  Default host ``http://localhost:3000``.

Series given as numpy arrays are encoded by the host extension
(``_twtml_host.json_floats``, GIL released) and posted as a pre-built body:
an append carries tens of thousands of numbers, and ``json.dumps`` of them
holds the GIL long enough to stall the training thread's host work.
"""
from __future__ import annotations

import json
from dataclasses import dataclass
from typing import Any, Dict, List, Optional, Sequence, Union

import numpy as np
import requests

from .http import post as http_post

__all__ = ["Lightning", "Visualization", "LightningError"]


class LightningError(RuntimeError):
    pass


@dataclass
class Visualization:
    lgn: "Lightning"
    id: str
    type: str = "line-streaming"

    def append(self, data: Union[Dict[str, Any], bytes]) -> Dict[str, Any]:
        body = b'{"data":' + data + b"}" if isinstance(data, bytes) else {"data": data}
        return self.lgn._post(f"/sessions/{self.lgn.session}/visualizations/{self.id}/data/", body)

    def get_pym_link(self) -> str:
        return f"{self.lgn.host}/visualizations/{self.id}/pym"

    getPymLink = get_pym_link


class Lightning:
    def __init__(self, host: str = "http://localhost:3000", auth: Optional[tuple] = None,
                 timeout: float = 5.0):
        self.host = (host or "http://localhost:3000").rstrip("/")
        self.auth = auth
        self.timeout = timeout
        self.session: str = ""
        self._http = requests.Session()

    # ------------------------------------------------------------------
    def _post(self, path: str, payload: Union[Dict[str, Any], bytes]) -> Dict[str, Any]:
        body = payload if isinstance(payload, bytes) else json.dumps(payload).encode()   # bytes: pre-encoded
        try:
            status, content = http_post(self.host + path, body, auth=self.auth, timeout=self.timeout,
                                        session=self._http)
        except requests.RequestException as e:
            raise LightningError(f"lightning unreachable at {self.host}: {e}") from e
        if status >= 400:
            raise LightningError(f"lightning {path}: HTTP {status} {content[:200].decode('utf-8', 'replace')}")
        try:
            return json.loads(content) if content else {}
        except ValueError:
            return {}

    def create_session(self, name: str = "") -> str:
        body = {"name": name} if name else {}
        res = self._post("/sessions/", body)
        self.session = str(res.get("id", ""))
        if not self.session:
            raise LightningError("lightning did not return a session id")
        return self.session

    createSession = create_session

    def check_session(self) -> None:
        if not self.session:
            self.create_session()

    def plot(self, type: str, data: Dict[str, Any]) -> Visualization:
        self.check_session()
        res = self._post(f"/sessions/{self.session}/visualizations/", {"type": type, "data": data})
        vid = res.get("id")
        if vid is None:
            raise LightningError("lightning did not return a visualization id")
        return Visualization(self, str(vid), type)

    def line_streaming(self, series: Sequence[Sequence[float]], size: Sequence[float] = (),
                       color: Sequence[Sequence[float]] = (), alpha: Sequence[float] = (),
                       label: Sequence[int] = (), xaxis: str = "", yaxis: str = "",
                       viz: Optional[Visualization] = None):
        if viz is not None and series and all(isinstance(x, np.ndarray) for x in series):
            # the append fast path: native encoding of the numbers, GIL released
            rest: Dict[str, Any] = {}
            if xaxis:
                rest["xaxis"] = xaxis
            if yaxis:
                rest["yaxis"] = yaxis
            body = b'{"series":[' + b",".join(_json_floats(x) for x in series) + b"]"
            for key, val in (("size", size), ("color", color), ("alpha", alpha), ("label", label)):
                if len(val):
                    body += b',"' + key.encode() + b'":' + json.dumps(np.asarray(val).tolist()).encode()
            for key, val in rest.items():
                body += b',"' + key.encode() + b'":' + json.dumps(val).encode()
            viz.append(body + b"}")
            return viz
        data: Dict[str, Any] = {"series": [list(map(float, s)) for s in series]}
        if size:
            data["size"] = list(size)
        if color:
            data["color"] = [list(c) for c in color]
        if alpha:
            data["alpha"] = list(alpha)
        if label:
            data["label"] = list(label)
        if xaxis:
            data["xaxis"] = xaxis
        if yaxis:
            data["yaxis"] = yaxis
        if viz is None:
            return self.plot("line-streaming", data)
        viz.append(data)
        return viz

    lineStreaming = line_streaming


def _json_floats(x: np.ndarray) -> bytes:
    """JSON array of ``x`` as float64 (non-finite -> null)."""
    x = np.ascontiguousarray(x, dtype=np.float64).ravel()
    try:
        from ..ops._native import NativeUnavailable, host
        return host().json_floats(x)
    except (ImportError, NativeUnavailable):
        return json.dumps([v if np.isfinite(v) else None for v in x.tolist()]).encode()
