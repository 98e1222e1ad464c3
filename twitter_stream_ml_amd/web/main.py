"""twtml-web entry point (``Main.scala:5-23``).

``-nocache`` skips restoring the cached Config from ``${tmpdir}/twtml-web.json``;
the port comes from ``$PORT`` (default 8888, Heroku style, ``Server.scala:66``);
SIGTERM/SIGINT close every WebSocket and stop the server (the reference's
shutdown hook, ``Main.scala:18-20``).
"""
from __future__ import annotations

import logging
import signal
import sys
from typing import List, Optional

from .cache import ApiCache
from .server import TwtmlWebServer

__all__ = ["main", "build_server"]


def build_server(args: List[str], port: Optional[int] = None, host: str = "0.0.0.0",
                 backup_file: Optional[str] = None) -> TwtmlWebServer:
    nocache = any(a in ("-nocache", "--nocache") for a in args)
    cache = ApiCache(backup_file)
    if not nocache:
        cache.restore()
    return TwtmlWebServer(host=host, port=port, cache=cache)


def main(argv: Optional[List[str]] = None) -> int:
    logging.basicConfig(level=logging.INFO,
                        format="%(asctime)s %(levelname)-5s %(name)s: %(message)s")
    logging.getLogger("com.giorgioinf").setLevel(logging.DEBUG)
    args = list(sys.argv[1:] if argv is None else argv)
    server = build_server(args)
    server.start()

    def _stop(signum, frame):  # shutdown hook
        server.stop()
        sys.exit(0)

    signal.signal(signal.SIGTERM, _stop)
    server.serve_forever()
    return 0


if __name__ == "__main__":
    sys.exit(main())
