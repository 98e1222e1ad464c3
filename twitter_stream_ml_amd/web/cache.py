"""twtml-web state and persistence (``ApiCache.scala:11-56``).

Holds the last ``Stats`` and ``Config``.  ``cache(json)`` dispatches on the
``jsonClass`` hint; only ``Config`` is persisted, to
``${tmpdir}/twtml-web.json``, on every config post, and ``restore()`` reloads
it best-effort at startup.  Unlike the reference's unsynchronised globals
(a benign race), state is per server instance and guarded by a
lock.
"""
from __future__ import annotations

import logging
import os
import tempfile
import threading
from typing import Optional, Union

from ..report.api_types import Config, Stats, TypeData, parse_type_data

__all__ = ["ApiCache", "default_backup_file"]

log = logging.getLogger("com.giorgioinf.twtml.web.ApiCache")


def default_backup_file() -> str:
    return os.path.join(tempfile.gettempdir(), "twtml-web.json")


class ApiCache:
    def __init__(self, backup_file: Optional[str] = None):
        self.backup_file = backup_file or default_backup_file()
        self._stats = Stats()
        self._config = Config()
        self._lock = threading.Lock()

    def config(self) -> str:
        with self._lock:
            return self._config.to_json()

    def stats(self) -> str:
        with self._lock:
            return self._stats.to_json()

    def config_obj(self) -> Config:
        with self._lock:
            return self._config

    def stats_obj(self) -> Stats:
        with self._lock:
            return self._stats

    def cache(self, payload: Union[str, bytes]) -> TypeData:
        data = parse_type_data(payload)
        if isinstance(data, Stats):
            log.debug("caching stats")
            with self._lock:
                self._stats = data
        elif isinstance(data, Config):
            log.debug("caching config")
            with self._lock:
                self._config = data
            self.backup()
        return data

    def restore(self) -> bool:
        try:
            with open(self.backup_file, "r", encoding="utf-8") as fh:
                self.cache(fh.read())
            return True
        except Exception as e:  # Try(...) in the reference
            log.debug("no cached config restored: %s", e)
            return False

    def backup(self) -> None:
        tmp = self.backup_file + ".tmp"
        with open(tmp, "w", encoding="utf-8") as fh:
            fh.write(self.config())
        os.replace(tmp, self.backup_file)
