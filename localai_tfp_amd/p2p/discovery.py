"""LAN peer discovery for the p2p network (the reference's edgevpn runs libp2p mDNS discovery on every
node, every 10 s: core/p2p/p2p.go:431-436 `Discovery{MDNS: true, Interval: 10s}`).

libp2p is not in this image, so nodes find each other with their own beacon instead: every `interval`
seconds a node sends one UDP datagram to the multicast group (default 239.255.77.77:47777, TTL 1, i.e. the
local link — the reach of mDNS) describing itself ({service, id, name, address}). The datagram is
authenticated with HMAC-SHA256 keyed by the network token, so the token never crosses the wire, nodes of
other networks (or without the token) are ignored, and a timestamp window rejects replays older than
`max_skew` seconds. Every valid beacon from another node is added to the local Registry, which is exactly
what an announcement over HTTP does (same liveness window).

`targets` replaces the multicast group with unicast host:port destinations (networks without multicast,
and the tests: a container's loopback usually has no multicast route).
"""
from __future__ import annotations

import hashlib
import hmac
import json
import logging
import socket
import struct
import threading
import time

from . import NodeData, Registry, token_secret

log = logging.getLogger("localai_tfp_amd.p2p.discovery")

GROUP, PORT = "239.255.77.77", 47777
VERSION = 1


def _mac(token: str, payload: bytes) -> str:
    return hmac.new(token_secret(token).encode(), payload, hashlib.sha256).hexdigest()


def encode_beacon(node: NodeData, token: str, network: str, now: float | None = None) -> bytes:
    body = json.dumps({"v": VERSION, "net": network, "ts": round(now if now is not None else time.time(), 3),
                       "node": {"id": node.id, "name": node.name, "address": node.address, "service": node.service}},
                      separators=(",", ":"), sort_keys=True).encode()
    return json.dumps({"b": body.decode(), "mac": _mac(token, body)}, separators=(",", ":")).encode()


def decode_beacon(data: bytes, token: str, network: str, max_skew: float = 60.0,
                  now: float | None = None) -> NodeData | None:
    """-> the announced node, or None for a malformed / foreign / forged / stale beacon."""
    try:
        outer = json.loads(data.decode())
        body = outer["b"].encode()
        if not hmac.compare_digest(_mac(token, body), str(outer["mac"])):
            return None
        b = json.loads(body)
        if b.get("v") != VERSION or b.get("net", "") != network:
            return None
        if abs((now if now is not None else time.time()) - float(b["ts"])) > max_skew:
            return None
        n = b["node"]
        return NodeData(id=str(n["id"]), name=str(n.get("name", "")), address=str(n.get("address", "")),
                        service=str(n.get("service", "")))
    except (ValueError, KeyError, TypeError, UnicodeDecodeError):
        return None


_LOCAL_HOSTS = ("", "0.0.0.0", "::", "localhost")


def reachable_address(advertised: str, sender_ip: str) -> str:
    """The address a peer's beacon should be registered under. A node bound to 0.0.0.0 with no
    LOCALAI_P2P_ADVERTISE advertises a loopback / unspecified host (p2p.self_node); taken literally, every
    LAN peer would register that worker at ITS OWN loopback and proxy to itself. Such hosts are replaced
    by the datagram's source IP (the only address known to reach the sender); routable hosts are kept."""
    host, sep, port = advertised.rpartition(":")
    if not sep:
        host, port = advertised, ""
    h = host.strip("[]")
    if h in _LOCAL_HOSTS or h.startswith("127.") or h == "::1":
        if not sender_ip:
            return advertised
        return f"{sender_ip}:{port}" if port else sender_ip
    return advertised


class LanDiscovery:
    """Beacon sender + listener for one node (started by p2p.P2PNode when p2p is on)."""

    def __init__(self, registry: Registry, me: NodeData | None, token: str, network: str = "",
                 group: str = GROUP, port: int = PORT, targets: list[str] | None = None, interval: float = 10.0,
                 bind_host: str = ""):
        self.registry, self.me, self.token, self.network = registry, me, token, network
        self.group, self.port, self.interval = group, int(port), interval
        self.targets = [self._split(t) for t in (targets or []) if t]
        self._stop = threading.Event()
        self.received = 0
        self.rx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM, socket.IPPROTO_UDP)
        self.rx.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        if hasattr(socket, "SO_REUSEPORT"):
            try:
                self.rx.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEPORT, 1)
            except OSError:
                pass
        self.rx.bind((bind_host, self.port))
        self.port = self.rx.getsockname()[1]
        self.rx.settimeout(0.5)
        if not self.targets:
            try:
                mreq = struct.pack("4s4s", socket.inet_aton(self.group), socket.inet_aton("0.0.0.0"))
                self.rx.setsockopt(socket.IPPROTO_IP, socket.IP_ADD_MEMBERSHIP, mreq)
            except OSError as ex:  # no multicast route (containers): unicast targets still work
                log.warning("p2p LAN discovery: cannot join %s (%s)", self.group, ex)
        self.tx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM, socket.IPPROTO_UDP)
        self.tx.setsockopt(socket.IPPROTO_IP, socket.IP_MULTICAST_TTL, 1)

    @staticmethod
    def _split(t: str) -> tuple[str, int]:
        host, _, port = t.rpartition(":")
        return host or "127.0.0.1", int(port)

    def beacon_once(self) -> int:
        if self.me is None:
            return 0
        data = encode_beacon(self.me, self.token, self.network)
        sent = 0
        for dst in (self.targets or [(self.group, self.port)]):
            try:
                self.tx.sendto(data, dst)
                sent += 1
            except OSError as ex:
                log.debug("p2p beacon to %s failed: %s", dst, ex)
        return sent

    def poll_once(self) -> NodeData | None:
        try:
            data, src = self.rx.recvfrom(4096)
        except (socket.timeout, OSError):
            return None
        node = decode_beacon(data, self.token, self.network)
        if node is None or (self.me is not None and node.id == self.me.id):
            return None
        node.address = reachable_address(node.address, src[0])
        self.registry.add(node)
        self.received += 1
        return node

    def start(self) -> "LanDiscovery":
        def send_loop():
            while not self._stop.is_set():
                self.beacon_once()
                self._stop.wait(self.interval)

        def recv_loop():
            while not self._stop.is_set():
                self.poll_once()

        threading.Thread(target=send_loop, daemon=True, name="p2p-beacon").start()
        threading.Thread(target=recv_loop, daemon=True, name="p2p-listen").start()
        return self

    def stop(self):
        self._stop.set()
        for s in (self.rx, self.tx):
            try:
                s.close()
            except OSError:
                pass
