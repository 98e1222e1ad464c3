"""Tweet records: row schema (twitter4j ``Status`` subset) and columnar batches."""
from .schema import Status, User, status_from_json, status_to_json
from .batch import (CREATED_AT, FAVOURITES, FOLLOWERS, FRIENDS, RETWEET_COUNT, SCALAR_FIELDS,
                    RawBatch, units_to_str, utf16_units)

__all__ = ["Status", "User", "status_from_json", "status_to_json", "RawBatch", "SCALAR_FIELDS",
           "RETWEET_COUNT", "FOLLOWERS", "FAVOURITES", "FRIENDS", "CREATED_AT", "utf16_units",
           "units_to_str"]
