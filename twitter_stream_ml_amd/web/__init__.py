"""twtml-web: reporting HTTP/WebSocket server and dashboard (reference ``web/`` module)."""
from .cache import ApiCache
from .server import ASSET_DIR, TwtmlWebServer, make_app

__all__ = ["ApiCache", "TwtmlWebServer", "make_app", "ASSET_DIR"]
