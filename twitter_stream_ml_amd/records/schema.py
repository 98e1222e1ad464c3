"""Tweet-shaped record schema (the twitter4j ``Status`` fields the app reads).

The reference reads, from a twitter4j 4.0.4 ``Status``: ``isRetweet``,
``getRetweetedStatus`` and, on that original tweet, ``getText``,
``getRetweetCount``, ``getCreatedAt`` and ``getUser.{getFollowersCount,
getFavouritesCount, getFriendsCount}`` (``MllibHelper.scala:43-45,59-66,81,85,
91``; ``KMeans.scala:21,26-27,79``).  SURVEY Appendix B fixes this as the
record schema every source must produce.  The camelCase accessor methods keep
call sites reading like the reference; the data lives in plain fields.
"""
from __future__ import annotations

import json
from dataclasses import dataclass, field
from typing import Any, Dict, Optional

__all__ = ["User", "Status", "status_from_json", "status_to_json"]


@dataclass
class User:
    followersCount: int = 0
    favouritesCount: int = 0
    friendsCount: int = 0
    screenName: str = ""

    def getFollowersCount(self) -> int:
        return self.followersCount

    def getFavouritesCount(self) -> int:
        return self.favouritesCount

    def getFriendsCount(self) -> int:
        return self.friendsCount


@dataclass
class Status:
    """A tweet.  ``retweetedStatus`` is the original when this is a retweet."""

    text: str = ""
    retweetCount: int = 0
    createdAt: int = 0            # epoch milliseconds (``Date.getTime``)
    user: User = field(default_factory=User)
    retweetedStatus: Optional["Status"] = None
    id: int = 0
    lang: str = "en"

    # twitter4j-style accessors ------------------------------------------
    def isRetweet(self) -> bool:
        return self.retweetedStatus is not None

    def getRetweetedStatus(self) -> Optional["Status"]:
        return self.retweetedStatus

    def getText(self) -> str:
        return self.text

    def getRetweetCount(self) -> int:
        return self.retweetCount

    def getCreatedAt(self) -> int:
        return self.createdAt

    def getUser(self) -> User:
        return self.user

    def getLang(self) -> str:
        return self.lang


def status_to_json(s: Status) -> Dict[str, Any]:
    d: Dict[str, Any] = {
        "id": s.id,
        "text": s.text,
        "retweet_count": s.retweetCount,
        "created_at_ms": s.createdAt,
        "lang": s.lang,
        "user": {
            "followers_count": s.user.followersCount,
            "favourites_count": s.user.favouritesCount,
            "friends_count": s.user.friendsCount,
            "screen_name": s.user.screenName,
        },
    }
    if s.retweetedStatus is not None:
        d["retweeted_status"] = status_to_json(s.retweetedStatus)
    return d


def status_from_json(d: Dict[str, Any]) -> Status:
    """Build a :class:`Status` from a Twitter-API-v1.1-like JSON object.

    Accepts both the field names above and the v1.1 names (``favourites_count``
    etc.); ``created_at_ms`` (epoch ms) is preferred over ``created_at``.
    """
    if isinstance(d, str):
        d = json.loads(d)
    u = d.get("user") or {}
    user = User(
        followersCount=int(u.get("followers_count", 0)),
        favouritesCount=int(u.get("favourites_count", 0)),
        friendsCount=int(u.get("friends_count", 0)),
        screenName=str(u.get("screen_name", "")),
    )
    created = d.get("created_at_ms")
    if created is None:
        created = _parse_twitter_date(d.get("created_at"))
    rt = d.get("retweeted_status")
    return Status(
        text=str(d.get("text", d.get("full_text", ""))),
        retweetCount=int(d.get("retweet_count", 0)),
        createdAt=int(created or 0),
        user=user,
        retweetedStatus=status_from_json(rt) if rt else None,
        id=int(d.get("id", 0)),
        lang=str(d.get("lang", "")),
    )


def _parse_twitter_date(s: Optional[str]) -> int:
    if not s:
        return 0
    from email.utils import parsedate_to_datetime
    try:
        # "Wed Oct 10 20:19:24 +0000 2018"
        import datetime as _dt
        dt = _dt.datetime.strptime(s, "%a %b %d %H:%M:%S %z %Y")
        return int(dt.timestamp() * 1000)
    except ValueError:
        return int(parsedate_to_datetime(s).timestamp() * 1000)
