"""Federation / p2p: a token-scoped node registry, node announcement and
the federated load-balancing TCP proxy.

Reference behaviour (core/p2p/federated.go, federated_server.go, node.go, p2p.go):
  * nodes of one network share a token; each announces itself under a service ("worker" for
    distributed inference workers, "federated" for full LocalAI instances) and counts as online
    while it has been seen in the last 40 s (node.go:21-25);
  * `local-ai federated` listens on one address and forwards every incoming TCP connection to an
    online instance: a fixed target worker, the least-used node when load balancing (request
    counters per node, federated.go:77-108), or a random one; no node -> an HTML 503
    (federated_server.go:84-87).
Transport: the reference rides libp2p/edgevpn tunnels, which this image does not have. Nodes
announce to the federator over plain HTTP (`POST /api/p2p/register`, bearer token = the network
token, constant-time compared), find each other on the local link with HMAC-authenticated UDP
multicast beacons (p2p/discovery.py, the reference's mDNS discovery), and connections are proxied
over TCP directly. No DHT / NAT traversal. Selection, the
liveness window, request accounting and the 503 behaviour follow the reference.
"""
from __future__ import annotations

import asyncio
import base64
import hmac
import json
import logging
import os
import random
import secrets
import threading
import time
import urllib.request
from dataclasses import asdict, dataclass, field

log = logging.getLogger("localai_tfp_amd.p2p")

ONLINE_WINDOW_S = 40.0
ANNOUNCE_INTERVAL_S = 10.0
WORKER_ID = "worker"
FEDERATED_ID = "federated"


def network_id(network: str, service: str) -> str:
    """federated.go:13-18."""
    return f"{network}_{service}" if network else service


def generate_token() -> str:
    return base64.urlsafe_b64encode(secrets.token_bytes(32)).decode().rstrip("=")


@dataclass
class NodeData:
    id: str
    name: str = ""
    address: str = ""  # host:port the node serves on
    service: str = FEDERATED_ID
    last_seen: float = field(default_factory=time.time)

    def is_online(self, now: float | None = None) -> bool:
        return ((now or time.time()) - self.last_seen) < ONLINE_WINDOW_S

    def to_json(self) -> dict:
        d = asdict(self)
        d["online"] = self.is_online()
        return d


class Registry:
    """Nodes per service (the reference's AddNode / GetAvailableNodes / GetNode)."""

    def __init__(self, token: str = "", network: str = ""):
        self.token = token
        self.network = network
        self._nodes: dict[str, dict[str, NodeData]] = {}
        self._lock = threading.Lock()

    def authorised(self, header: str | None) -> bool:
        if not self.token:
            return True
        got = (header or "").removeprefix("Bearer ").strip()
        return hmac.compare_digest(got.encode(), self.token.encode())

    def add(self, node: NodeData) -> None:
        with self._lock:
            node.last_seen = time.time()
            self._nodes.setdefault(network_id(self.network, node.service), {})[node.id] = node

    def nodes(self, service: str) -> list[NodeData]:
        with self._lock:
            return list(self._nodes.get(network_id(self.network, service), {}).values())

    def get(self, service: str, node_id: str) -> NodeData | None:
        with self._lock:
            return self._nodes.get(network_id(self.network, service), {}).get(node_id)

    def json_nodes(self, service: str) -> list[dict]:
        return [n.to_json() for n in self.nodes(service)]


class Announcer:
    """Periodically registers this instance with every federator / peer URL (nodeAnnounce)."""

    def __init__(self, node: NodeData, peers: list[str], token: str, interval: float = ANNOUNCE_INTERVAL_S):
        self.node, self.token, self.interval = node, token, interval
        self.peers = [p.rstrip("/") for p in peers if p]
        self._stop = threading.Event()

    def announce_once(self) -> int:
        ok = 0
        body = json.dumps(asdict(self.node)).encode()
        for p in self.peers:
            req = urllib.request.Request(p + "/api/p2p/register", data=body, method="POST",
                                         headers={"Content-Type": "application/json",
                                                  "Authorization": f"Bearer {self.token}"})
            try:
                with urllib.request.urlopen(req, timeout=5) as r:
                    ok += r.status == 200
            except Exception as ex:  # a federator being down is routine
                log.debug("announce to %s failed: %s", p, ex)
        return ok

    def start(self) -> "Announcer":
        def loop():
            while not self._stop.is_set():
                self.announce_once()
                self._stop.wait(self.interval)
        threading.Thread(target=loop, daemon=True, name="p2p-announce").start()
        return self

    def stop(self):
        self._stop.set()


class P2PNode:
    """Per-instance p2p state behind /api/p2p (what `local-ai run --p2p` sets up): the registry, HTTP
    announcements to configured peers, and LAN discovery beacons (p2p/discovery.py; the reference's mDNS)
    unless `lan_discovery` is False."""

    def __init__(self, token: str, network: str = "", peers: list[str] | None = None,
                 self_node: NodeData | None = None, lan_discovery: bool = False, discovery_targets=None,
                 discovery_port: int | None = None):
        self.registry = Registry(token, network)
        self.announcer = Announcer(self_node, peers or [], token).start() if (self_node and peers) else None
        self.discovery = None
        if lan_discovery and token:
            from .discovery import PORT, LanDiscovery
            try:
                self.discovery = LanDiscovery(self.registry, self_node, token, network,
                                              port=discovery_port if discovery_port is not None else PORT,
                                              targets=list(discovery_targets or [])).start()
            except OSError as ex:  # port taken / no network: the HTTP announcements still work
                log.warning("p2p LAN discovery disabled: %s", ex)

    def nodes(self, service: str) -> list[dict]:
        return self.registry.json_nodes(service)

    def stop(self):
        if self.announcer:
            self.announcer.stop()
        if self.discovery:
            self.discovery.stop()


# ------------------------------------------------------------------------------------------------
class FederatedServer:
    """Load-balancing TCP proxy over the online nodes of one service (federated.go +
    federated_server.go). The federator also serves `/api/p2p` (listing) and
    `/api/p2p/register` (announcements) itself."""

    def __init__(self, listen: str, registry: Registry, service: str = FEDERATED_ID, load_balanced: bool = False,
                 worker_target: str = ""):
        self.listen, self.registry, self.service = listen, registry, service
        self.load_balanced, self.worker_target = load_balanced, worker_target
        self.request_table: dict[str, int] = {}
        self._lock = threading.Lock()
        self.server: asyncio.base_events.Server | None = None

    # ---- selection (federated.go:39-118) ----
    def random_server(self) -> str:
        online = []
        for n in self.registry.nodes(self.service):
            if n.is_online():
                online.append(n.id)
            else:
                with self._lock:
                    self.request_table.pop(n.id, None)
        return random.choice(online) if online else ""

    def _sync_table(self):
        with self._lock:
            live = {n.id for n in self.registry.nodes(self.service) if n.is_online()}
            for i in live:
                self.request_table.setdefault(i, 0)
            for i in list(self.request_table):
                if i not in live:
                    del self.request_table[i]

    def select_least_used(self) -> str:
        self._sync_table()
        with self._lock:
            if not self.request_table:
                return ""
            return min(self.request_table.items(), key=lambda kv: (kv[1], kv[0]))[0]

    def record_request(self, node_id: str):
        with self._lock:
            self.request_table[node_id] = self.request_table.get(node_id, 0) + 1

    def pick(self) -> str:
        if self.worker_target:
            return self.worker_target
        if self.load_balanced:
            return self.select_least_used() or self.random_server()
        return self.random_server()

    # ---- proxy ----
    @staticmethod
    def html_response(code: int, msg: str) -> bytes:
        text = {503: "Service Unavailable", 404: "Not Found", 200: "OK"}.get(code, "Unknown Status")
        body = f"<html><body><h1>{msg}</h1></body></html>\r\n"
        return f"HTTP/1.1 {code} {text}\r\nContent-Type: text/html\r\nConnection: close\r\n\r\n{body}".encode()

    async def _handle_local(self, head: bytes, reader, writer) -> bool:
        lines = head.split(b"\r\n")
        parts = lines[0].decode("latin1").split()
        if len(parts) < 2 or not parts[1].startswith("/api/p2p"):
            return False
        hdrs = {}
        for h in lines[1:]:
            k, _, v = h.decode("latin1").partition(":")
            hdrs[k.strip().lower()] = v.strip()
        n = int(hdrs.get("content-length", "0") or 0)
        body = await reader.readexactly(n) if n else b""
        code = 200
        if parts[0] == "POST" and parts[1].startswith("/api/p2p/register"):
            if not self.registry.authorised(hdrs.get("authorization")):
                resp, code = {"error": "invalid token"}, 401
            else:
                d = json.loads(body or b"{}")
                self.registry.add(NodeData(id=str(d["id"]), name=d.get("name", ""), address=d.get("address", ""),
                                           service=d.get("service", self.service)))
                resp = {"ok": True}
        else:
            resp = {"nodes": self.registry.json_nodes(WORKER_ID),
                    "federated_nodes": self.registry.json_nodes(FEDERATED_ID)}
        payload = json.dumps(resp).encode()
        writer.write(f"HTTP/1.1 {code} {'OK' if code == 200 else 'Unauthorized'}\r\nContent-Type: application/json\r\n"
                     f"Content-Length: {len(payload)}\r\nConnection: close\r\n\r\n".encode() + payload)
        await writer.drain()
        writer.close()
        return True

    @staticmethod
    async def _pipe(r, w):
        try:
            while True:
                data = await r.read(65536)
                if not data:
                    break
                w.write(data)
                await w.drain()
        except (ConnectionError, asyncio.CancelledError):
            pass
        finally:
            try:
                w.close()
            except Exception:
                pass

    async def _reply(self, writer, code: int, msg: str):
        writer.write(self.html_response(code, msg))
        await writer.drain()
        writer.close()

    async def _conn(self, reader, writer):
        try:
            head = await reader.readuntil(b"\r\n\r\n")
        except Exception:
            writer.close()
            return
        if await self._handle_local(head, reader, writer):
            return
        node_id = self.pick()
        if not node_id:
            await self._reply(writer, 503, "Sorry, waiting for nodes to connect")
            return
        nd = self.registry.get(self.service, node_id)
        if nd is None:
            await self._reply(writer, 404, "Node not found")
            return
        host, _, port = nd.address.rpartition(":")
        try:
            ur, uw = await asyncio.open_connection(host or "127.0.0.1", int(port))
        except (OSError, ValueError):
            await self._reply(writer, 503, f"Node {node_id} unreachable")
            return
        uw.write(head)
        await uw.drain()
        await asyncio.gather(self._pipe(reader, uw), self._pipe(ur, writer))
        if self.load_balanced:
            self.record_request(node_id)

    async def start(self):
        host, _, port = self.listen.rpartition(":")
        self.server = await asyncio.start_server(self._conn, host or "0.0.0.0", int(port))
        return self.server

    def serve_forever(self):
        async def main():
            srv = await self.start()
            log.info("federated proxy for service %r on %s", self.service, self.listen)
            async with srv:
                await srv.serve_forever()
        asyncio.run(main())


def self_node(address: str, service: str = FEDERATED_ID) -> NodeData:
    """This instance's announcement: LOCALAI_P2P_ADVERTISE overrides the served host:port."""
    adv = os.environ.get("LOCALAI_P2P_ADVERTISE", "")
    if not adv:
        host, _, port = address.rpartition(":")
        adv = f"{host if host not in ('', '0.0.0.0') else '127.0.0.1'}:{port}"
    nid = os.environ.get("LOCALAI_P2P_NODE_ID") or f"{os.uname().nodename}-{adv}"
    return NodeData(id=nid, name=os.uname().nodename, address=adv, service=service)
