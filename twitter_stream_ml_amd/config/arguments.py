"""``ConfArguments``: the twtml-spark command line and tunables.

Behaviour of the reference (``spark/src/main/scala/com/giorgioinf/twtml/spark/
ConfArguments.scala:6-164``) kept here:

* defaults come from :class:`ConfigFactory.load` (reference.conf <
  application.conf < system properties, ``:8-28``);
* the usage text lists the same 15 flags + help (``:30-52``);
* the master defaults to ``local[*]`` unless the ``SPARK_SUBMIT`` system
  property is ``"true"`` (``:54-56``);
* non-empty OAuth keys from the config are pushed into the
  ``twitter4j.oauth.*`` system properties (``:58-76``);
* ``parse`` consumes ``flag value`` pairs left to right; ``-h/--help`` prints
  the usage and exits 0; anything unrecognised (or a flag missing its value)
  prints the usage and exits 1 (``:91-163``).

Extensions for the MI355X engine are long flags only (the reference's 16
short letters keep their meaning): ``--source``, ``--batchSize``,
``--numBatches``, ``--hash``, ``--checkpoint``, ``--checkpointInterval``,
``--resume``, ``--sourceRate``, ``--plotPoints``, ``--legacyNumTextFeatures``,
``--batchTimeout``, ``--checkReplicas``.
The master accepts, besides Spark's ``local``, ``local[N]``, ``local[*]``
(CPU plumbing engine, fp64), the device masters ``rocm``, ``rocm[N]``,
``rocm[*]`` and ``rocm:0,1,...`` (HIP engine, one process per GPU).
"""
from __future__ import annotations

import re
import sys
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence

from .hocon import ConfigFactory, get_property, set_property

__all__ = ["ConfArguments", "SparkConf", "MasterSpec", "parse_master"]


class SparkConf:
    """Minimal ``org.apache.spark.SparkConf``: a string map with setters."""

    def __init__(self) -> None:
        self._settings: Dict[str, str] = {}

    def set(self, key: str, value: str) -> "SparkConf":
        self._settings[key] = str(value)
        return self

    def get(self, key: str, default: Optional[str] = None) -> str:
        if key in self._settings:
            return self._settings[key]
        if default is not None:
            return default
        raise KeyError(key)

    def contains(self, key: str) -> bool:
        return key in self._settings

    def setMaster(self, master: str) -> "SparkConf":
        return self.set("spark.master", master)

    def setAppName(self, name: str) -> "SparkConf":
        return self.set("spark.app.name", name)

    def getAll(self):
        return sorted(self._settings.items())


@dataclass(frozen=True)
class MasterSpec:
    """Decoded ``--master``: which engine and how many workers/devices."""

    kind: str                 # "local" (CPU engine) or "rocm" (HIP engine) or "cluster"
    workers: Optional[int]    # None = all available ("*")
    devices: Optional[tuple] = None  # explicit device ids for rocm:0,1,...
    url: str = ""

    @property
    def is_gpu(self) -> bool:
        return self.kind == "rocm"


_LOCAL_RE = re.compile(r"^local(?:\[(\*|\d+)(?:,\s*\d+)?\])?$")
_ROCM_RE = re.compile(r"^rocm(?:\[(\*|\d+)\])?$")
_ROCM_IDS_RE = re.compile(r"^rocm:(\d+(?:,\d+)*)$")


def parse_master(master: str) -> MasterSpec:
    m = _LOCAL_RE.match(master)
    if m:
        n = m.group(1)
        workers = None if n == "*" else (1 if n is None else int(n))
        return MasterSpec("local", workers, url=master)
    m = _ROCM_RE.match(master)
    if m:
        n = m.group(1)
        workers = None if n in (None, "*") else int(n)
        return MasterSpec("rocm", workers, url=master)
    m = _ROCM_IDS_RE.match(master)
    if m:
        ids = tuple(int(x) for x in m.group(1).split(","))
        return MasterSpec("rocm", len(ids), ids, url=master)
    # spark://, mesos://, yarn: accepted for compatibility; executed by the
    # torch.distributed launcher on the CPU engine.
    return MasterSpec("cluster", None, url=master)


# flag -> (attribute, converter); the reference's 15 value flags
_VALUE_FLAGS = {
    ("--master", "-m"): "master",
    ("--name", "-n"): "name",
    ("--consumerKey", "-C"): "consumerKey",
    ("--consumerSecret", "-S"): "consumerSecret",
    ("--accessToken", "-A"): "accessToken",
    ("--accessTokenSecret", "-T"): "accessTokenSecret",
    ("--lightning", "-l"): "lightning",
    ("--twtweb", "-w"): "twtweb",
    ("--seconds", "-s"): "seconds",
    ("--stepSize", "-p"): "stepSize",
    ("--numIterations", "-i"): "numIterations",
    ("--miniBatchFraction", "-b"): "miniBatchFraction",
    ("--numRetweetBegin", "-B"): "numRetweetBegin",
    ("--numRetweetEnd", "-E"): "numRetweetEnd",
    ("--numTextFeatures", "-f"): "numTextFeatures",
}

# MI355X-engine extension flags (long form only)
_EXT_FLAGS = {
    "--source": ("source", str),
    "--sourceRate": ("sourceRate", float),
    "--batchSize": ("batchSize", int),
    "--numBatches": ("numBatches", int),
    "--hash": ("hash", str),
    "--checkpoint": ("checkpoint", str),
    "--checkpointInterval": ("checkpointInterval", int),
    "--resume": ("resume", str),
    "--plotPoints": ("plotPoints", int),
    "--seed": ("seed", int),
    "--batchTimeout": ("batchTimeout", float),
    "--checkReplicas": ("checkReplicas", int),
}

_FLAG_LOOKUP = {}
for _names, _attr in _VALUE_FLAGS.items():
    for _n in _names:
        _FLAG_LOOKUP[_n] = _attr

_OAUTH = ("consumerKey", "consumerSecret", "accessToken", "accessTokenSecret")


class ConfArguments:
    """CLI + config for the streaming jobs (``ConfArguments.scala:6``)."""

    def __init__(self) -> None:
        self.conf = ConfigFactory.load()
        self.sparkConf = SparkConf()
        c = self.conf
        self.lightningDef = c.getString("lightning")
        self.twtwebDef = c.getString("twtweb")
        self.secondsDef = c.getInt("seconds")
        self.stepSizeDef = c.getDouble("stepSize")
        self.numIterationsDef = c.getInt("numIterations")
        self.miniBatchFractionDef = c.getDouble("miniBatchFraction")
        self.numRetweetBeginDef = c.getInt("numRetweetBegin")
        self.numRetweetEndDef = c.getInt("numRetweetEnd")
        self.numTextFeaturesDef = c.getInt("numTextFeatures")

        self.lightning = self.lightningDef
        self.twtweb = self.twtwebDef
        self.seconds = self.secondsDef
        self.stepSize = self.stepSizeDef
        self.numIterations = self.numIterationsDef
        self.miniBatchFraction = self.miniBatchFractionDef
        self.numRetweetBegin = self.numRetweetBeginDef
        self.numRetweetEnd = self.numRetweetEndDef
        self.numTextFeatures = self.numTextFeaturesDef

        # extension tunables (reference.conf of this package provides them)
        self.source = c.getString("source") if c.hasPath("source") else "synthetic"
        self.sourceRate = c.getDouble("sourceRate") if c.hasPath("sourceRate") else 50.0
        self.batchSize = c.getInt("batchSize") if c.hasPath("batchSize") else 0
        self.numBatches = 0
        self.hash = c.getString("hash") if c.hasPath("hash") else "java"
        self.honourNumTextFeatures = (c.getBoolean("honourNumTextFeatures")
                                      if c.hasPath("honourNumTextFeatures") else True)
        self.checkpoint = c.getString("checkpoint") if c.hasPath("checkpoint") else ""
        self.checkpointInterval = (c.getInt("checkpointInterval")
                                   if c.hasPath("checkpointInterval") else 10)
        self.resume = ""
        # bounded by default: at the reference's batch sizes (~11
        # tweets per 5 s batch) 10000 is every row, as
        # LinearRegression.scala:76-77 appends them; at 1M-tweet batches the
        # device samples 10000 evenly spaced pairs.  0 = every row.
        self.plotPoints = c.getInt("plotPoints") if c.hasPath("plotPoints") else 10000
        self.seed = 42
        self.batchTimeout = 0.0
        self.checkReplicas = 0

        self.usage = f"""
Usage: python -m twitter_stream_ml_amd.apps.linear_regression
Usage: python -m twitter_stream_ml_amd.apps.linear_regression [options]
Usage: twtml-spark [options]

  Options:
  -h, --help
  -m, --master <master_url>                    local[N], rocm[N], rocm:0,1,.. (also spark://host:port, mesos://host:port, yarn).
  -n, --name <name>                            A name of your application.
  -C, --consumerKey <consumerKey>              Twitter's consumer key
  -S, --consumerSecret <consumerSecret>        Twitter's consumer secret
  -A, --accessToken <accessToken>              Twitter's access token
  -T, --accessTokenSecret <accessTokenSecret>  Twitter's access token secret
  -l, --lightning <lightning_url>              {self.lightningDef}
  -w, --twtweb <twtweb_url>                    {self.twtwebDef}
  -s, --seconds <integer number>               Default: {self.secondsDef}
  -p, --stepSize <float number>                Default: {self.stepSizeDef}
  -i, --numIterations <integer number>         Default: {self.numIterationsDef}
  -b, --miniBatchFraction <float number>       Default: {self.miniBatchFractionDef}
  -B, --numRetweetBegin <integer number>       Default: {self.numRetweetBeginDef}
  -E, --numRetweetEnd <integer number>         Default: {self.numRetweetEndDef}
  -f, --numTextFeatures <integer number>       Default: {self.numTextFeaturesDef}

  MI355X engine options:
  --source <synthetic|replay:FILE.jsonl|twitter>  Default: {self.source}
  --sourceRate <tweets per second, 0 = max>       Default: {self.sourceRate:g}
  --batchSize <max tweets per micro-batch>        Default: {self.batchSize}
  --numBatches <stop after N batches, 0 = never>  Default: 0
  --hash <java|murmur3>                           Default: {self.hash}
  --checkpoint <dir>  --checkpointInterval <n>    Default: off / {self.checkpointInterval}
  --resume <dir|auto>                             warm start from an MLlib model dir
                                                  (auto: the --checkpoint dir if present,
                                                  continuing its stream position)
  --batchTimeout <seconds>                        abort the process if a batch hangs (0 = off)
  --checkReplicas <n>                             verify DP replicas agree every n batches
  --plotPoints <n>                                points per Lightning append (default 10000; 0 = all)
  --legacyNumTextFeatures                         reproduce the reference bug: ignore -f
  """

        if get_property("SPARK_SUBMIT") != "true":
            self.sparkConf.setMaster("local[*]")

        for key in _OAUTH:
            if c.hasPath(key) and c.getString(key) != "":
                set_property("twitter4j.oauth." + key, c.getString(key))

    # -- accessors mirroring ConfArguments.scala:78-89 --------------------
    def appName(self) -> str:
        return self.sparkConf.get("spark.app.name")

    def setAppName(self, appName: str) -> "ConfArguments":
        self.sparkConf.setAppName(appName)
        return self

    def master(self) -> str:
        return self.sparkConf.get("spark.master")

    def master_spec(self) -> MasterSpec:
        return parse_master(self.master())

    @property
    def effectiveNumTextFeatures(self) -> int:
        """Width of the text hash space actually used by the model.

        The reference's ``MllibHelper.reset`` shadows its fields with locals
        (``MllibHelper.scala:27-29``), so its HashingTF always stays at 1000.
        We honour ``-f`` unless ``--legacyNumTextFeatures`` is given.
        """
        return self.numTextFeatures if self.honourNumTextFeatures else 1000

    # -- parse (ConfArguments.scala:91-158) --------------------------------
    def parse(self, args: Sequence[str]) -> "ConfArguments":
        lst: List[str] = list(args)
        i = 0
        while i < len(lst):
            flag = lst[i]
            if flag in ("--help", "-h"):
                self.printUsage(0)
            if flag == "--legacyNumTextFeatures":
                self.honourNumTextFeatures = False
                i += 1
                continue
            if flag in _FLAG_LOOKUP and i + 1 < len(lst):
                value = lst[i + 1]
                try:
                    self._apply(_FLAG_LOOKUP[flag], value)
                except ValueError:
                    # Scala's value.toInt throws NumberFormatException; the
                    # job dies with a non-zero status.
                    self.printUsage(1)
                i += 2
                continue
            if flag in _EXT_FLAGS and i + 1 < len(lst):
                attr, conv = _EXT_FLAGS[flag]
                try:
                    setattr(self, attr, conv(lst[i + 1]))
                except ValueError:
                    self.printUsage(1)
                i += 2
                continue
            self.printUsage(1)
        return self

    def _apply(self, attr: str, value: str) -> None:
        if attr == "master":
            self.sparkConf.setMaster(value)
        elif attr == "name":
            self.sparkConf.setAppName(value)
        elif attr in _OAUTH:
            set_property("twitter4j.oauth." + attr, value)
        elif attr in ("lightning", "twtweb"):
            setattr(self, attr, value)
        elif attr == "seconds":
            # extension: sub-second intervals ("0.5"); integers parse as in Scala;
            # 0 = no timer, batches are sealed by --batchSize alone
            v = _java_int(value) if value.strip().lstrip("+-").isdigit() else float(value)
            if v < 0:
                raise ValueError(value)
            self.seconds = v
        elif attr in ("numIterations", "numRetweetBegin", "numRetweetEnd",
                      "numTextFeatures"):
            setattr(self, attr, _java_int(value))
        elif attr in ("stepSize", "miniBatchFraction"):
            setattr(self, attr, float(value))
        else:  # pragma: no cover
            raise AssertionError(attr)

    def printUsage(self, exitNumber: int):
        print(self.usage)
        sys.exit(exitNumber)

    def describe(self) -> Dict[str, object]:
        return {
            "appName": self.sparkConf.get("spark.app.name", ""),
            "master": self.master(),
            "lightning": self.lightning,
            "twtweb": self.twtweb,
            "seconds": self.seconds,
            "stepSize": self.stepSize,
            "numIterations": self.numIterations,
            "miniBatchFraction": self.miniBatchFraction,
            "numRetweetBegin": self.numRetweetBegin,
            "numRetweetEnd": self.numRetweetEnd,
            "numTextFeatures": self.effectiveNumTextFeatures,
            "source": self.source,
            "batchSize": self.batchSize,
            "hash": self.hash,
        }


def _java_int(value: str) -> int:
    """Scala ``String.toInt``: decimal digits with optional sign, 32-bit."""
    v = value.strip()
    if not re.fullmatch(r"[+-]?\d+", v):
        raise ValueError(value)
    n = int(v)
    if not -(2 ** 31) <= n < 2 ** 31:
        raise ValueError(value)
    return n
