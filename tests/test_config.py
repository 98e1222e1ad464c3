"""ConfArguments tests: ``ConfArgumentsSuite.scala:6-144`` ported 1:1, plus
HOCON precedence, the help/unknown-flag exit codes and the master parser.

The test "classpath" application.conf (tests/resources, set in conftest.py)
carries the dummy OAuth keys, exactly like ``spark/src/test/resources``.
"""
import pytest

from twitter_stream_ml_amd.config import (ConfArguments, ConfigFactory, clear_property,
                                          get_property, load_java_opts, parse_hocon,
                                          parse_master, set_property, system_properties)

lightningDef = "http://public.lightning-viz.org"
twtwebDef = "http://localhost:8888"
consumerKeyApp = "xxxxxxxxxxxxxxxxxxxxxxxxx"
consumerSecretApp = "xxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxx"
accessTokenApp = "xxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxx"
accessTokenSecretApp = "xxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxx"

master = "local[4]"
name = "twtml-spark-test"
lightning = "http://lightninghost"
twtweb = "http://twtwebhost"
seconds = 123
stepSize = 0.01234
numIterations = 123
miniBatchFraction = 1.23
numRetweetBegin = 1234
numRetweetEnd = 12345678
numTextFeatures = 123456
consumerKey = "1234567"
consumerSecret = "12345678"
accessToken = "123456789"
accessTokenSecret = "1234567890"

ref = ConfigFactory.load("reference")


def twt(key):
    return get_property("twitter4j.oauth." + key)


@pytest.fixture(autouse=True)
def clean_props():
    saved = dict(system_properties)
    yield
    system_properties.clear()
    system_properties.update(saved)


def test_config_initialization_reference_conf():
    conf = ConfArguments().setAppName(name)
    assert conf.appName() == name
    assert conf.lightning == lightningDef
    assert ref.getString("lightning") == lightningDef
    assert conf.twtweb == twtwebDef
    assert ref.getString("twtweb") == twtwebDef


def test_config_twitter_application_conf():
    ConfArguments()
    assert twt("consumerKey") == consumerKeyApp
    assert twt("consumerSecret") == consumerSecretApp
    assert twt("accessToken") == accessTokenApp
    assert twt("accessTokenSecret") == accessTokenSecretApp


def test_config_reference_conf():
    conf = ConfArguments()
    assert conf.seconds == ref.getInt("seconds")
    assert conf.stepSize == ref.getDouble("stepSize")
    assert conf.numIterations == ref.getInt("numIterations")
    assert conf.miniBatchFraction == ref.getDouble("miniBatchFraction")
    assert conf.numRetweetBegin == ref.getInt("numRetweetBegin")
    assert conf.numRetweetEnd == ref.getInt("numRetweetEnd")
    assert conf.numTextFeatures == ref.getInt("numTextFeatures")


def _check_parsed(conf):
    assert conf.master() == master
    assert conf.lightning == lightning
    assert conf.twtweb == twtweb
    assert conf.seconds == seconds
    assert conf.stepSize == stepSize
    assert conf.numIterations == numIterations
    assert conf.miniBatchFraction == miniBatchFraction
    assert conf.numRetweetBegin == numRetweetBegin
    assert conf.numRetweetEnd == numRetweetEnd
    assert conf.numTextFeatures == numTextFeatures
    assert twt("consumerKey") == consumerKey
    assert twt("consumerSecret") == consumerSecret
    assert twt("accessToken") == accessToken
    assert twt("accessTokenSecret") == accessTokenSecret


def test_config_long_arguments():
    conf = ConfArguments().parse([
        "--master", master, "--lightning", lightning, "--twtweb", twtweb,
        "--seconds", str(seconds), "--stepSize", str(stepSize),
        "--numIterations", str(numIterations), "--miniBatchFraction", str(miniBatchFraction),
        "--numRetweetBegin", str(numRetweetBegin), "--numRetweetEnd", str(numRetweetEnd),
        "--numTextFeatures", str(numTextFeatures), "--consumerKey", consumerKey,
        "--consumerSecret", consumerSecret, "--accessToken", accessToken,
        "--accessTokenSecret", accessTokenSecret])
    _check_parsed(conf)


def test_config_small_arguments():
    conf = ConfArguments().parse([
        "-m", master, "-n", name, "-l", lightning, "-w", twtweb, "-s", str(seconds),
        "-p", str(stepSize), "-i", str(numIterations), "-b", str(miniBatchFraction),
        "-B", str(numRetweetBegin), "-E", str(numRetweetEnd), "-f", str(numTextFeatures),
        "-C", consumerKey, "-S", consumerSecret, "-A", accessToken, "-T", accessTokenSecret])
    _check_parsed(conf)
    assert conf.appName() == name


# ---- beyond the reference suite --------------------------------------------
@pytest.mark.parametrize("argv,code", [(["-h"], 0), (["--help"], 0), (["--bogus"], 1),
                                       (["--seconds"], 1), (["--seconds", "x"], 1),
                                       (["-s", "5", "extra"], 1)])
def test_help_and_bad_flags_exit_codes(argv, code, capsys):
    with pytest.raises(SystemExit) as e:
        ConfArguments().parse(argv)
    assert e.value.code == code
    assert "--numTextFeatures" in capsys.readouterr().out


def test_default_master_and_spark_submit():
    assert ConfArguments().master() == "local[*]"
    set_property("SPARK_SUBMIT", "true")
    conf = ConfArguments()
    with pytest.raises(KeyError):
        conf.master()
    clear_property("SPARK_SUBMIT")


def test_system_properties_override_files():
    load_java_opts(["-Dseconds=9", "-DstepSize=0.5", "--keep"])
    conf = ConfArguments()
    assert conf.seconds == 9 and conf.stepSize == 0.5
    clear_property("seconds")
    clear_property("stepSize")


def test_hocon_subset():
    d = parse_hocon('''
        # comment
        a = 1
        b: "two" // trailing
        c { d = "x#y", e = 3 }
        f = [1, 2]
        g = "q\\"uote"
    ''')
    assert d == {"a": "1", "b": "two", "c.d": "x#y", "c.e": "3", "f": "[1, 2]", "g": 'q"uote'}


def test_master_spec():
    assert parse_master("local[*]").kind == "local" and parse_master("local[*]").workers is None
    assert parse_master("local[2]").workers == 2
    assert parse_master("local").workers == 1
    assert parse_master("rocm").is_gpu and parse_master("rocm[8]").workers == 8
    m = parse_master("rocm:0,2")
    assert m.devices == (0, 2) and m.workers == 2
    assert parse_master("spark://h:7077").kind == "cluster"


def test_num_text_features_honoured_unless_legacy():
    conf = ConfArguments().parse(["-f", "4096"])
    assert conf.effectiveNumTextFeatures == 4096
    conf = ConfArguments().parse(["-f", "4096", "--legacyNumTextFeatures"])
    assert conf.effectiveNumTextFeatures == 1000


def test_extension_flags():
    conf = ConfArguments().parse(["--source", "replay:x.jsonl", "--batchSize", "64",
                                  "--hash", "murmur3", "--numBatches", "3"])
    assert (conf.source, conf.batchSize, conf.hash, conf.numBatches) == ("replay:x.jsonl", 64,
                                                                        "murmur3", 3)


def test_plot_points_default_is_bounded():
    """a bounded default (10000 pairs per batch, sampled on the
    device) -- at the reference's batch sizes that is every kept row
    (LinearRegression.scala:76-77); 0 (= all rows) is opt-in."""
    assert ConfArguments().parse([]).plotPoints == 10000
    assert ConfArguments().parse(["--plotPoints", "0"]).plotPoints == 0
