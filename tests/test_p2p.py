"""Federation (reference: core/p2p/federated.go selection + request table, federated_server.go
503 when no node, node.go 40 s liveness; the reference has no test for p2p — its transport is
libp2p — so these pin the selection/proxy semantics with loopback instances)."""
import asyncio
import json
import threading
import time
import urllib.request

import pytest

from localai_tfp_amd import p2p as P


def test_registry_liveness_and_token():
    r = P.Registry("tok", "net")
    r.add(P.NodeData(id="a", address="127.0.0.1:1"))
    r.add(P.NodeData(id="b", address="127.0.0.1:2"))
    r._nodes["net_federated"]["b"].last_seen = time.time() - 41
    assert [n.id for n in r.nodes("federated") if n.is_online()] == ["a"]
    assert r.authorised("Bearer tok") and not r.authorised("Bearer nope") and not r.authorised(None)
    assert P.network_id("", "worker") == "worker" and P.network_id("n", "worker") == "n_worker"


def test_least_used_and_target_selection():
    r = P.Registry()
    for i in "abc":
        r.add(P.NodeData(id=i, address="127.0.0.1:1"))
    fs = P.FederatedServer("127.0.0.1:0", r, load_balanced=True)
    seen = []
    for _ in range(6):
        n = fs.pick()
        fs.record_request(n)
        seen.append(n)
    assert sorted(seen) == ["a", "a", "b", "b", "c", "c"]
    r._nodes["federated"]["a"].last_seen = 0  # offline nodes leave the table
    assert fs.pick() in ("b", "c") and "a" not in fs.request_table
    assert P.FederatedServer("x:1", r, worker_target="zz").pick() == "zz"
    assert P.FederatedServer("x:1", P.Registry()).pick() == ""


def _serve_http(body: bytes):
    import http.server

    class H(http.server.BaseHTTPRequestHandler):
        def do_GET(self):
            self.send_response(200)
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

        def log_message(self, *a):
            pass
    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), H)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    return srv


def test_proxy_register_forward_and_503():
    backends = [_serve_http(b"node-%d" % i) for i in range(2)]
    reg = P.Registry("secret")
    fs = P.FederatedServer("127.0.0.1:0", reg, load_balanced=True)
    loop = asyncio.new_event_loop()
    srv = loop.run_until_complete(fs.start())
    port = srv.sockets[0].getsockname()[1]
    threading.Thread(target=loop.run_forever, daemon=True).start()
    base = f"http://127.0.0.1:{port}"
    try:
        with pytest.raises(urllib.error.HTTPError) as e:
            urllib.request.urlopen(base + "/v1/models", timeout=5)
        assert e.value.code == 503
        bad = P.Announcer(P.NodeData(id="x", address="127.0.0.1:1"), [base], "wrong")
        assert bad.announce_once() == 0
        for i, b in enumerate(backends):
            a = P.Announcer(P.NodeData(id=f"n{i}", address=f"127.0.0.1:{b.server_address[1]}"), [base], "secret")
            assert a.announce_once() == 1
        listing = json.loads(urllib.request.urlopen(base + "/api/p2p", timeout=5).read())
        assert sorted(n["id"] for n in listing["federated_nodes"]) == ["n0", "n1"]
        got = {urllib.request.urlopen(base + "/v1/models", timeout=5).read() for _ in range(4)}
        assert got == {b"node-0", b"node-1"}  # least-used alternates between the two nodes
    finally:
        loop.call_soon_threadsafe(srv.close)
        for b in backends:
            b.shutdown()


def test_gateway_register_route(tmp_path):
    from fastapi.testclient import TestClient

    from localai_tfp_amd.config.app_config import ApplicationConfig
    from localai_tfp_amd.gateway.app import create_app
    cfg = ApplicationConfig(models_path=str(tmp_path), generated_content_dir=str(tmp_path / "g"),
                            upload_dir=str(tmp_path / "u"), config_dir=str(tmp_path / "c"), api_keys=[],
                            p2p=True, p2p_token="t0k")
    app = create_app(cfg, inproc=True)
    with TestClient(app) as c:
        assert c.post("/api/p2p/register", json={"id": "w1", "address": "127.0.0.1:9"},
                      headers={"Authorization": "Bearer bad"}).status_code == 401
        assert c.post("/api/p2p/register", json={"id": "w1", "address": "127.0.0.1:9"},
                      headers={"Authorization": "Bearer t0k"}).status_code == 200
        j = c.get("/api/p2p").json()
        assert [n["id"] for n in j["nodes"]] == ["w1"] and j["nodes"][0]["online"]
        assert c.get("/api/p2p/token").text == "t0k"
    app.state.localai.shutdown()


def test_explorer_db_discovery_and_routes(tmp_path):
    from fastapi.testclient import TestClient

    from localai_tfp_amd.p2p import explorer as X
    backend = _serve_http(b"x")
    reg = P.Registry("k3y")
    fs = P.FederatedServer("127.0.0.1:0", reg)
    loop = asyncio.new_event_loop()
    srv = loop.run_until_complete(fs.start())
    threading.Thread(target=loop.run_forever, daemon=True).start()
    fed = f"http://127.0.0.1:{srv.sockets[0].getsockname()[1]}"
    try:
        db = X.Database(str(tmp_path / "pool.json"))
        c = TestClient(X.create_explorer_app(db))
        good = X.make_network_token(fed, "k3y")
        dead = X.make_network_token("http://127.0.0.1:9", "k")
        assert c.post("/network/add", json={"token": good, "name": "n"}).status_code == 400  # description missing
        assert c.post("/network/add", json={"token": "***", "name": "n", "description": "d"}).json()["error"] == "Invalid token"
        for t in (good, dead):
            assert c.post("/network/add", json={"token": t, "name": "n", "description": "d"}).status_code == 200
        assert c.post("/network/add", json={"token": good, "name": "n", "description": "d"}).status_code == 400
        assert c.get("/networks").json() == []  # no workers seen yet
        P.Announcer(P.NodeData(id="w0", address=f"127.0.0.1:{backend.server_address[1]}", service="worker"),
                    [fed], "k3y").announce_once()
        ds = X.DiscoveryServer(db, 5, 1)
        ds.run_once()
        nets = c.get("/networks").json()
        assert len(nets) == 1 and nets[0]["token"] == good and nets[0]["Clusters"][0]["Workers"] == ["w0"]
        ds.run_once()  # the dead network exceeds the failure threshold and is removed
        assert db.token_list() == [good]
        assert c.get("/", headers={"content-type": "application/json"}).json()["Version"]
    finally:
        loop.call_soon_threadsafe(srv.close)
        backend.shutdown()


def test_token_has_the_reference_edgevpn_shape():
    """generate_token mirrors core/p2p/p2p.go:33-66: base64 of the edgevpn connection YAML with 43-letter names and
    OTP keys, DHT / crypto intervals (defaults 360 / 9000, overridable like --p2p-dht-interval / --p2p-otp-interval)
    and the 20 MB message cap."""
    import base64
    import re

    import yaml
    cfg = yaml.safe_load(base64.b64decode(P.generate_token()))
    assert cfg["max_message_size"] == 20 << 20
    for k in ("room", "rendezvous", "mdns"):
        assert re.fullmatch(r"[A-Za-z]{43}", cfg[k])
    assert cfg["otp"]["dht"]["interval"] == 360 and cfg["otp"]["crypto"]["interval"] == 9000
    for o in ("dht", "crypto"):
        assert re.fullmatch(r"[A-Za-z]{43}", cfg["otp"][o]["key"]) and cfg["otp"][o]["length"] == 43
    c2 = P.parse_token(P.generate_token(100, 200))
    assert c2["otp"]["dht"]["interval"] == 100 and c2["otp"]["crypto"]["interval"] == 200
    assert P.generate_token() != P.generate_token()


def test_reference_token_parses_and_keys_the_network():
    """A token written the way the reference writes one (Go yaml of node.YAMLConnectionConfig, standard base64) is
    accepted: its crypto OTP key + room are the network secret, so two nodes holding it authenticate each other's
    beacons and a node with another token does not. Opaque tokens keep working as their own secret."""
    import base64

    from localai_tfp_amd.p2p import discovery as D
    go_yaml = ("otp:\n  dht:\n    interval: 360\n    key: " + "A" * 43 + "\n    length: 43\n"
               "  crypto:\n    interval: 9000\n    key: " + "B" * 43 + "\n    length: 43\n"
               "room: " + "C" * 43 + "\nrendezvous: " + "D" * 43 + "\nmdns: " + "E" * 43 + "\n"
               "max_message_size: 20971520\n")
    tok = base64.b64encode(go_yaml.encode()).decode()
    cfg = P.parse_token(tok)
    assert cfg is not None and cfg["room"] == "C" * 43
    assert P.token_secret(tok) == "B" * 43 + ":" + "C" * 43
    assert P.parse_token("tok") is None and P.token_secret("tok") == "tok"
    assert P.parse_token(base64.b64encode(b"just: text").decode()) is None
    node = P.NodeData(id="n1", address="127.0.0.1:9", service="worker")
    beacon = D.encode_beacon(node, tok, "net")
    assert D.decode_beacon(beacon, tok, "net").id == "n1"
    assert D.decode_beacon(beacon, P.generate_token(), "net") is None


def test_cli_p2p_intervals_reach_the_config():
    import argparse

    from localai_tfp_amd.cli import add_run_args, app_config_from_args
    ap = argparse.ArgumentParser()
    add_run_args(ap)
    a = ap.parse_args(["--p2p-dht-interval", "120", "--p2p-otp-interval", "600"])
    c = app_config_from_args(a)
    assert c.p2p_dht_interval == 120 and c.p2p_otp_interval == 600
