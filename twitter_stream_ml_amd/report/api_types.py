"""Wire schema between the streaming job and twtml-web.

The reference's ``ApiTypes.scala:3-17`` (three identical copies) defines
``Config(id, host, viz)`` and ``Stats(count, batch, mse, realStddev,
predStddev)`` (all Longs), serialised by json4s with ``ShortTypeHints`` —
i.e. a leading ``"jsonClass": "<SimpleName>"`` field followed by the fields
in declaration order.  This module is the single copy.
"""
from __future__ import annotations

import json
from dataclasses import dataclass, field
from typing import Any, Dict, List, Union

__all__ = ["TypeData", "Config", "Stats", "parse_type_data", "TYPE_HINT"]

TYPE_HINT = "jsonClass"


class TypeData:
    """Marker base (``trait TypeData``)."""

    def to_dict(self) -> Dict[str, Any]:  # pragma: no cover - abstract
        raise NotImplementedError

    def to_json(self) -> str:
        return json.dumps(self.to_dict(), separators=(",", ":"), ensure_ascii=False)


def _to_long(v: Any) -> int:
    """json4s reads a JSON number into a Scala Long (truncating a double)."""
    if isinstance(v, bool):
        raise ValueError("boolean is not a Long")
    if isinstance(v, (int,)):
        return int(v)
    if isinstance(v, float):
        return int(v)
    if isinstance(v, str):
        return int(float(v)) if "." in v or "e" in v.lower() else int(v)
    raise ValueError(f"not a number: {v!r}")


@dataclass
class Config(TypeData):
    id: str = ""
    host: str = ""
    viz: List[str] = field(default_factory=list)

    def to_dict(self) -> Dict[str, Any]:
        return {TYPE_HINT: "Config", "id": self.id, "host": self.host, "viz": list(self.viz)}

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "Config":
        viz = d.get("viz", [])
        if isinstance(viz, str):
            viz = [viz]
        return cls(str(d.get("id", "")), str(d.get("host", "")), [str(v) for v in viz])


@dataclass
class Stats(TypeData):
    count: int = 0
    batch: int = 0
    mse: int = 0
    realStddev: int = 0
    predStddev: int = 0

    def to_dict(self) -> Dict[str, Any]:
        return {TYPE_HINT: "Stats", "count": int(self.count), "batch": int(self.batch),
                "mse": int(self.mse), "realStddev": int(self.realStddev),
                "predStddev": int(self.predStddev)}

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "Stats":
        return cls(*(_to_long(d.get(k, 0)) for k in
                     ("count", "batch", "mse", "realStddev", "predStddev")))


_TYPES = {"Config": Config, "Stats": Stats}


def parse_type_data(payload: Union[str, bytes, Dict[str, Any]]) -> TypeData:
    """``read[TypeData](json)``: dispatch on the ``jsonClass`` hint.

    Raises ``ValueError`` for malformed JSON or an unknown/missing hint (the
    reference's actor dies without replying in that case, ApiCache.scala:42).
    """
    if isinstance(payload, (bytes, bytearray)):
        payload = payload.decode("utf-8")
    d = json.loads(payload) if isinstance(payload, str) else payload
    if not isinstance(d, dict):
        raise ValueError("expected a JSON object")
    kind = d.get(TYPE_HINT)
    if kind not in _TYPES:
        raise ValueError(f"json not recognized: unknown {TYPE_HINT} {kind!r}")
    return _TYPES[kind].from_dict(d)
