"""twtml-web server tests.

Ports ``WebTestSuite.scala:7-53`` 1:1 (post/get Config and Stats round trips
through the real server started in-process with ``-nocache``) and adds what the
reference leaves untested: WebSocket connect-time config, WS and
POST broadcast, the config backup/restore, static files, 404 and malformed
payloads.
"""
import asyncio
import json
import os

import aiohttp
import pytest
import requests

from twitter_stream_ml_amd.report.api_types import Config, Stats, parse_type_data
from twitter_stream_ml_amd.report.webclient import WebClient
from twitter_stream_ml_amd.web.main import build_server


@pytest.fixture(scope="module")
def server(tmp_path_factory):
    backup = str(tmp_path_factory.mktemp("web") / "twtml-web.json")
    srv = build_server(["-nocache"], port=0, host="127.0.0.1", backup_file=backup).start()
    yield srv
    srv.stop()


# ---- WebTestSuite (order-dependent in the reference: a get reads what the
# previous test posted; each get here posts first, so the pair also holds
# when pytest-xdist runs the tests on different workers) ------------------
config_test = Config("100", "http://localhost:8888", ["101", "102"])
stats_test = Stats(1000, 10, 2000, 15, 25)


def test_client_posts_config(server):
    WebClient(server.url).config(config_test.id, config_test.host, config_test.viz)


def test_client_gets_correct_config(server):
    test_client_posts_config(server)
    assert WebClient(server.url).config() == config_test


def test_client_posts_stats(server):
    c = stats_test
    WebClient(server.url).stats(c.count, c.batch, c.mse, c.realStddev, c.predStddev)


def test_client_gets_correct_stats(server):
    test_client_posts_stats(server)
    assert WebClient(server.url).stats() == stats_test


# ---- beyond the reference ---------------------------------------------------
def test_wire_format_has_leading_type_hint():
    s = Stats(1, 2, 3, 4, 5).to_json()
    assert s.startswith('{"jsonClass":"Stats","count":1')
    assert json.loads(Config("a", "h", ["v"]).to_json()) == {
        "jsonClass": "Config", "id": "a", "host": "h", "viz": ["v"]}
    assert parse_type_data('{"jsonClass":"Stats","count":7.9}') == Stats(7, 0, 0, 0, 0)
    with pytest.raises(ValueError):
        parse_type_data('{"jsonClass":"Nope"}')


def test_post_reply_and_bad_payload(server):
    r = requests.post(server.url + "/api", data=Stats(1, 1, 1, 1, 1).to_json())
    assert r.status_code == 200 and r.json() == {"status": "OK"}
    assert r.headers["content-type"].startswith("application/json")
    bad = requests.post(server.url + "/api", data='{"jsonClass":"Bogus"}')
    assert bad.status_code == 400


def test_static_and_404(server):
    r = requests.get(server.url + "/")
    assert r.status_code == 200 and "<title>Twitter Stream ML</title>" in r.text
    assert requests.get(server.url + "/test.html").status_code == 200
    assert requests.get(server.url + "/js/api.js").status_code == 200
    assert requests.get(server.url + "/nothing-here").status_code == 404
    assert requests.get(server.url + "/../../etc/passwd").status_code == 404
    assert requests.get(server.url + "/api").status_code == 404  # no WS upgrade


def test_websocket_config_on_connect_and_broadcast(server):
    async def scenario():
        async with aiohttp.ClientSession() as s:
            ws1 = await s.ws_connect(server.url + "/api")
            first = json.loads((await ws1.receive(timeout=5)).data)
            assert first["jsonClass"] == "Config"
            ws2 = await s.ws_connect(server.url + "/api")
            await ws2.receive(timeout=5)
            # HTTP POST is broadcast verbatim to every socket
            body = Stats(5, 6, 7, 8, 9).to_json()
            async with s.post(server.url + "/api", data=body) as r:
                assert r.status == 200
            assert (await ws1.receive(timeout=5)).data == body
            assert (await ws2.receive(timeout=5)).data == body
            # a WS frame is cached and broadcast (to the sender too)
            frame = Config("7", "http://lgn", ["9"]).to_json()
            await ws2.send_str(frame)
            assert (await ws1.receive(timeout=5)).data == frame
            assert (await ws2.receive(timeout=5)).data == frame
            await ws1.close()
            await ws2.close()

    asyncio.run(scenario())
    assert WebClient(server.url).config() == Config("7", "http://lgn", ["9"])
    assert WebClient(server.url).stats() == Stats(5, 6, 7, 8, 9)


def test_config_backup_and_restore(tmp_path):
    backup = str(tmp_path / "twtml-web.json")
    srv = build_server(["-nocache"], port=0, host="127.0.0.1", backup_file=backup).start()
    try:
        WebClient(srv.url).config("s1", "http://l", ["v1"])
    finally:
        srv.stop()
    assert json.load(open(backup))["id"] == "s1"
    srv2 = build_server([], port=0, host="127.0.0.1", backup_file=backup).start()
    try:
        assert WebClient(srv2.url).config() == Config("s1", "http://l", ["v1"])
    finally:
        srv2.stop()
    srv3 = build_server(["-nocache"], port=0, host="127.0.0.1", backup_file=backup).start()
    try:
        assert WebClient(srv3.url).config() == Config()
    finally:
        srv3.stop()
