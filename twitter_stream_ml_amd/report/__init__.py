"""Report clients: twtml-web wire types + client, Lightning REST client, SessionStats."""
from .api_types import Config, Stats, TypeData, parse_type_data
from .lightning import Lightning, LightningError, Visualization
from .session_stats import SessionStats
from .webclient import WebClient

__all__ = ["Config", "Stats", "TypeData", "parse_type_data", "Lightning", "LightningError",
           "Visualization", "SessionStats", "WebClient"]
