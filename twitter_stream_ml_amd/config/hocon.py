"""HOCON-subset loader with Typesafe-Config precedence.

The reference loads its tunables through ``ConfigFactory.load`` (reference:
``spark/src/main/scala/com/giorgioinf/twtml/spark/ConfArguments.scala:8``),
whose precedence is: JVM system properties > ``application.conf`` >
``reference.conf``.  pyhocon is not available, so this module
implements the subset of HOCON the reference's files actually use
(``spark/src/main/resources/reference.conf:1-13``,
``spark/src/test/resources/application.conf:1-4``): ``key = value`` /
``key: value`` / ``key="value"`` lines, ``#`` and ``//`` comments, and nested
``a { b = 1 }`` objects flattened to dotted paths.  Values are kept as strings
and converted on access, exactly like Typesafe's ``getInt("seconds")`` on the
string ``"5"``.

System properties are emulated by a process-global dictionary
(:data:`system_properties`) that also receives the ``twitter4j.oauth.*`` keys
the reference pushes with ``System.setProperty``
(``ConfArguments.scala:58-76,103-118``).  ``-Dkey=value`` tokens and the
``TWTML_JAVA_OPTS`` environment variable seed it, mirroring ``java -Dk=v``.
"""
from __future__ import annotations

import os
import re
import shlex
from importlib import resources
from typing import Dict, Iterable, List, Optional

__all__ = [
    "Config",
    "ConfigError",
    "ConfigFactory",
    "parse_hocon",
    "system_properties",
    "get_property",
    "set_property",
    "clear_property",
    "load_java_opts",
]


class ConfigError(KeyError):
    """Missing or malformed configuration key (Typesafe ``ConfigException``)."""


# --------------------------------------------------------------------------
# System properties (JVM ``System.getProperty`` emulation)
# --------------------------------------------------------------------------
system_properties: Dict[str, str] = {}


def get_property(key: str, default: Optional[str] = None) -> Optional[str]:
    return system_properties.get(key, default)


def set_property(key: str, value: str) -> None:
    system_properties[key] = str(value)


def clear_property(key: str) -> None:
    system_properties.pop(key, None)


def load_java_opts(tokens: Optional[Iterable[str]] = None) -> List[str]:
    """Absorb ``-Dkey=value`` tokens into :data:`system_properties`.

    ``tokens`` defaults to ``shlex.split($TWTML_JAVA_OPTS)``.  Returns the
    tokens that were *not* ``-D`` definitions so callers can pass them on.
    """
    if tokens is None:
        tokens = shlex.split(os.environ.get("TWTML_JAVA_OPTS", ""))
    rest: List[str] = []
    for tok in tokens:
        if tok.startswith("-D") and "=" in tok:
            k, v = tok[2:].split("=", 1)
            set_property(k, v)
        else:
            rest.append(tok)
    return rest


# --------------------------------------------------------------------------
# Parser
# --------------------------------------------------------------------------
_KEY_RE = re.compile(r'\s*("(?:[^"\\]|\\.)*"|[A-Za-z0-9_.\-]+)\s*')


def _strip_comment(line: str) -> str:
    out = []
    in_str = False
    i = 0
    while i < len(line):
        c = line[i]
        if c == '"' and (i == 0 or line[i - 1] != "\\"):
            in_str = not in_str
        if not in_str:
            if c == "#":
                break
            if c == "/" and i + 1 < len(line) and line[i + 1] == "/":
                break
        out.append(c)
        i += 1
    return "".join(out)


def _unquote(v: str) -> str:
    v = v.strip()
    if len(v) >= 2 and v[0] == '"' and v[-1] == '"':
        body = v[1:-1]
        return bytes(body, "utf-8").decode("unicode_escape") if "\\" in body else body
    return v


def parse_hocon(text: str) -> Dict[str, str]:
    """Parse the HOCON subset into a flat ``{dotted.key: str}`` map.

    Later definitions override earlier ones (HOCON semantics for scalars).
    Lists (``[a, b]``) are kept as their raw text.
    """
    flat: Dict[str, str] = {}
    stack: List[str] = []
    for lineno, raw in enumerate(text.splitlines(), 1):
        line = _strip_comment(raw).strip()
        if not line:
            continue
        while line:
            if line.startswith("}"):
                if not stack:
                    raise ConfigError(f"line {lineno}: unbalanced '}}'")
                stack.pop()
                line = line[1:].strip().lstrip(",").strip()
                continue
            m = _KEY_RE.match(line)
            if not m:
                raise ConfigError(f"line {lineno}: cannot parse {raw!r}")
            key = _unquote(m.group(1))
            rest = line[m.end():]
            if rest.startswith("{"):
                stack.append(key)
                line = rest[1:].strip()
                continue
            if rest[:1] in ("=", ":"):
                rest = rest[1:].strip()
                if rest.startswith("{"):
                    stack.append(key)
                    line = rest[1:].strip()
                    continue
            elif rest.startswith("+="):
                rest = rest[2:].strip()
            else:
                raise ConfigError(f"line {lineno}: expected '=' after {key!r}")
            # value runs to end of line (or a closing brace outside quotes)
            value, tail = _split_value(rest)
            full = ".".join(stack + [key])
            flat[full] = _unquote(value)
            line = tail.strip()
    if stack:
        raise ConfigError("unterminated object: " + ".".join(stack))
    return flat


def _split_value(s: str):
    in_str = False
    depth = 0
    for i, c in enumerate(s):
        if c == '"' and (i == 0 or s[i - 1] != "\\"):
            in_str = not in_str
        elif not in_str:
            if c == "[":
                depth += 1
            elif c == "]":
                depth -= 1
            elif c == "}" and depth == 0:
                return s[:i].rstrip().rstrip(","), s[i:]
            elif c == "," and depth == 0:
                return s[:i], s[i + 1:]
    return s.rstrip().rstrip(","), ""


# --------------------------------------------------------------------------
# Config object
# --------------------------------------------------------------------------
class Config:
    """Read-only view with Typesafe-style typed getters."""

    def __init__(self, values: Dict[str, str], origin: str = "merged"):
        self._values = dict(values)
        self.origin = origin

    def has_path(self, path: str) -> bool:
        return path in self._values

    hasPath = has_path

    def _raw(self, path: str) -> str:
        try:
            return self._values[path]
        except KeyError:
            raise ConfigError(f"No configuration setting found for key '{path}'") from None

    def get_string(self, path: str) -> str:
        return self._raw(path)

    def get_int(self, path: str) -> int:
        v = self._raw(path).strip()
        try:
            return int(v)
        except ValueError:
            f = float(v)
            if f != int(f):
                raise ConfigError(f"{path} has type DOUBLE rather than INT: {v}") from None
            return int(f)

    def get_long(self, path: str) -> int:
        return self.get_int(path)

    def get_double(self, path: str) -> float:
        return float(self._raw(path))

    def get_boolean(self, path: str) -> bool:
        v = self._raw(path).strip().lower()
        if v in ("true", "yes", "on"):
            return True
        if v in ("false", "no", "off"):
            return False
        raise ConfigError(f"{path} is not a boolean: {v}")

    # camelCase aliases matching the reference's call sites
    getString = get_string
    getInt = get_int
    getLong = get_long
    getDouble = get_double
    getBoolean = get_boolean

    def as_dict(self) -> Dict[str, str]:
        return dict(self._values)

    def with_fallback(self, other: "Config") -> "Config":
        merged = dict(other._values)
        merged.update(self._values)
        return Config(merged, f"{self.origin} < {other.origin}")

    withFallback = with_fallback

    def __repr__(self) -> str:  # pragma: no cover - debugging aid
        return f"Config({self.origin}, {len(self._values)} keys)"


def _config_search_path() -> List[str]:
    """Directories searched for ``application.conf`` ("the classpath").

    ``TWTML_CONFIG_PATH`` (os.pathsep separated) first, then the working
    directory.  Tests point it at ``tests/resources`` the way sbt puts
    ``src/test/resources`` on the test classpath.
    """
    env = os.environ.get("TWTML_CONFIG_PATH")
    dirs = [d for d in env.split(os.pathsep) if d] if env else []
    dirs.append(os.getcwd())
    return dirs


class ConfigFactory:
    """``com.typesafe.config.ConfigFactory`` subset."""

    @staticmethod
    def parse_string(text: str, origin: str = "string") -> Config:
        return Config(parse_hocon(text), origin)

    parseString = parse_string

    @staticmethod
    def parse_file(path: str) -> Config:
        with open(path, "r", encoding="utf-8") as fh:
            return Config(parse_hocon(fh.read()), path)

    parseFile = parse_file

    @staticmethod
    def reference() -> Config:
        text = resources.files("twitter_stream_ml_amd.config").joinpath("reference.conf").read_text("utf-8")
        return Config(parse_hocon(text), "reference.conf")

    @staticmethod
    def application() -> Config:
        for d in _config_search_path():
            p = os.path.join(d, "application.conf")
            if os.path.isfile(p):
                return ConfigFactory.parse_file(p)
        return Config({}, "application.conf (absent)")

    @staticmethod
    def system() -> Config:
        return Config(dict(system_properties), "system properties")

    @staticmethod
    def load(resource: Optional[str] = None) -> Config:
        """``ConfigFactory.load()`` / ``ConfigFactory.load("reference")``.

        With no argument: system properties > application.conf > reference.conf.
        With ``"reference"``: just reference.conf (the test oracle at
        ``ConfArgumentsSuite.scala:35``).
        """
        if resource == "reference":
            return ConfigFactory.reference()
        if resource not in (None, "application"):
            for d in _config_search_path():
                p = os.path.join(d, resource if resource.endswith(".conf") else resource + ".conf")
                if os.path.isfile(p):
                    return ConfigFactory.system().with_fallback(
                        ConfigFactory.parse_file(p)).with_fallback(ConfigFactory.reference())
            raise ConfigError(f"resource {resource!r} not found")
        return (ConfigFactory.system()
                .with_fallback(ConfigFactory.application())
                .with_fallback(ConfigFactory.reference()))
