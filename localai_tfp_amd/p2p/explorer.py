"""Explorer: a public directory of p2p networks — a JSON token database, a
discovery loop that keeps each network's cluster list fresh, and the HTTP API
(core/explorer/database.go, discovery.go; core/http/endpoints/explorer/dashboard.go; routes
`GET /`, `GET /networks`, `POST /network/add`).

Tokens: where the reference's token is a base64 edgevpn config that lets the explorer join the
libp2p ledger, a network token here is base64(JSON {"federator": url, "key": secret}) — the
federator's `/api/p2p` listing (authorised with the key) plays the ledger's role. Discovery
semantics follow the reference: a token whose network shows online workers gets its clusters
refreshed and its failure count reset; otherwise the failure count grows and the token is
dropped once it exceeds the threshold (default 3).
"""
from __future__ import annotations

import base64
import fcntl
import json
import logging
import os
import threading
import time
import urllib.request

from fastapi import FastAPI, Request
from fastapi.responses import HTMLResponse, JSONResponse

log = logging.getLogger("localai_tfp_amd.p2p.explorer")


def make_network_token(federator_url: str, key: str) -> str:
    return base64.b64encode(json.dumps({"federator": federator_url, "key": key}).encode()).decode()


def parse_network_token(token: str) -> dict:
    return json.loads(base64.b64decode(token, validate=True))


class Database:
    """token -> {name, description, Clusters: [{Workers, Type, NetworkID}], Failures}; a JSON file
    guarded by an fcntl lock (the reference uses flock the same way) so several processes share it."""

    def __init__(self, path: str):
        self.path = path
        self._lock = threading.Lock()
        if os.path.dirname(path):
            os.makedirs(os.path.dirname(path), exist_ok=True)

    def _locked(self, fn):
        with self._lock, open(self.path + ".lock", "a+") as lf:
            fcntl.flock(lf, fcntl.LOCK_EX)
            try:
                data = {}
                if os.path.exists(self.path):
                    with open(self.path) as f:
                        data = json.load(f) or {}
                out, changed = fn(data)
                if changed:
                    tmp = self.path + ".tmp"
                    with open(tmp, "w") as f:
                        json.dump(data, f)
                    os.replace(tmp, self.path)
                return out
            finally:
                fcntl.flock(lf, fcntl.LOCK_UN)

    def get(self, token: str):
        return self._locked(lambda d: (d.get(token), False))

    def set(self, token: str, td: dict):
        def f(d):
            d[token] = td
            return None, True
        self._locked(f)

    def delete(self, token: str):
        def f(d):
            d.pop(token, None)
            return None, True
        self._locked(f)

    def token_list(self) -> list[str]:
        return self._locked(lambda d: (sorted(d), False))


class DiscoveryServer:
    def __init__(self, db: Database, timeout_s: float = 50.0, failure_threshold: int = 3):
        self.db, self.timeout, self.threshold = db, timeout_s or 50.0, failure_threshold or 3

    def clusters_of(self, token: str) -> list[dict]:
        t = parse_network_token(token)
        req = urllib.request.Request(t["federator"].rstrip("/") + "/api/p2p",
                                     headers={"Authorization": f"Bearer {t.get('key', '')}"})
        with urllib.request.urlopen(req, timeout=min(self.timeout, 30)) as r:
            listing = json.loads(r.read())
        out = []
        for key, typ in (("nodes", "worker"), ("federated_nodes", "federated")):
            workers = [n["id"] for n in listing.get(key, []) if n.get("online", True)]
            if workers:
                out.append({"Workers": workers, "Type": typ, "NetworkID": ""})
        return out

    def run_once(self):
        for token in self.db.token_list():
            td = self.db.get(token) or {}
            try:
                clusters = self.clusters_of(token)
            except Exception as ex:
                log.debug("network %s unreachable: %s", token[:12], ex)
                clusters = []
            if any(c["Workers"] for c in clusters):
                td["Clusters"], td["Failures"] = clusters, 0
            else:
                td["Failures"] = int(td.get("Failures", 0)) + 1
            self.db.set(token, td)
        for token in self.db.token_list():
            if int((self.db.get(token) or {}).get("Failures", 0)) > self.threshold:
                log.info("token %s removed from the database", token[:12])
                self.db.delete(token)

    def start(self, interval: float = 5.0):
        def loop():
            while True:
                self.run_once()
                time.sleep(interval)
        threading.Thread(target=loop, daemon=True, name="explorer-discovery").start()
        return self


def create_explorer_app(db: Database):
    from .. import __version__
    app = FastAPI(title="LocalAI explorer")

    @app.get("/")
    async def dashboard(request: Request):
        summary = {"Title": f"LocalAI API - {__version__}", "Version": __version__,
                   "BaseURL": str(request.base_url)}
        accept = request.headers.get("accept", "")
        if request.headers.get("content-type") == "application/json" or "html" not in accept:
            return summary
        return HTMLResponse("<html><body><h1>LocalAI explorer</h1><p>Networks: <a href='/networks'>/networks</a></p>"
                            "</body></html>")

    @app.get("/networks")
    async def networks():
        res = []
        for t in db.token_list():
            d = db.get(t) or {}
            if any(c.get("Workers") for c in d.get("Clusters") or []):
                res.append({**d, "token": t})
        res.sort(key=lambda n: -len(n.get("Clusters") or []))
        return res

    @app.post("/network/add")
    async def add_network(request: Request):
        try:
            b = await request.json()
        except Exception:
            return JSONResponse({"error": "Cannot parse JSON"}, status_code=400)
        for k, msg in (("token", "Token is required"), ("name", "Name is required"),
                       ("description", "Description is required")):
            if not b.get(k):
                return JSONResponse({"error": msg}, status_code=400)
        try:
            base64.b64decode(b["token"], validate=True)
        except Exception:
            return JSONResponse({"error": "Invalid token"}, status_code=400)
        if db.get(b["token"]) is not None:
            return JSONResponse({"error": "Token already exists"}, status_code=400)
        db.set(b["token"], {"name": b["name"], "description": b["description"], "Clusters": [], "Failures": 0})
        return {"message": "Token added"}

    return app
