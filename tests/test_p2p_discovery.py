"""LAN discovery beacons (p2p/discovery.py; the reference's libp2p mDNS discovery, core/p2p/p2p.go:431-436):
nodes sharing a network token find each other without configured peer URLs; beacons of another token,
another network id, forged or replayed ones are ignored. Unicast targets on loopback stand in for the
multicast group (a container's loopback has no multicast route): the multicast join itself is unpinned here."""
import time

from localai_tfp_amd.p2p import FEDERATED_ID, WORKER_ID, NodeData, P2PNode, Registry
from localai_tfp_amd.p2p.discovery import LanDiscovery, decode_beacon, encode_beacon


def test_beacon_auth_network_and_replay():
    me = NodeData(id="n1", name="a", address="10.0.0.1:8080", service=WORKER_ID)
    b = encode_beacon(me, "tok", "net")
    n = decode_beacon(b, "tok", "net")
    assert n is not None and (n.id, n.address, n.service) == ("n1", "10.0.0.1:8080", WORKER_ID)
    assert decode_beacon(b, "other-token", "net") is None
    assert decode_beacon(b, "tok", "other-net") is None
    assert decode_beacon(b.replace(b"10.0.0.1", b"10.6.6.6"), "tok", "net") is None  # tampered body
    assert decode_beacon(encode_beacon(me, "tok", "net", now=time.time() - 3600), "tok", "net") is None  # replay
    assert decode_beacon(b"not json", "tok", "net") is None


def test_two_nodes_discover_each_other_over_udp():
    ra, rb, rc = Registry("tok"), Registry("tok"), Registry("other")
    a = LanDiscovery(ra, NodeData(id="A", address="127.0.0.1:1111", service=FEDERATED_ID), "tok", port=0,
                     targets=[], bind_host="127.0.0.1")
    b = LanDiscovery(rb, NodeData(id="B", address="127.0.0.1:2222", service=FEDERATED_ID), "tok", port=0,
                     bind_host="127.0.0.1")
    c = LanDiscovery(rc, NodeData(id="C", address="127.0.0.1:3333", service=FEDERATED_ID), "other", port=0,
                     bind_host="127.0.0.1")
    try:
        a.targets = [("127.0.0.1", b.port), ("127.0.0.1", c.port)]
        b.targets = [("127.0.0.1", a.port)]
        c.targets = [("127.0.0.1", a.port), ("127.0.0.1", b.port)]
        for d in (a, b, c):
            d.start()
        deadline = time.time() + 5
        while time.time() < deadline and not (ra.nodes(FEDERATED_ID) and rb.nodes(FEDERATED_ID)):
            time.sleep(0.05)
        assert [n.id for n in ra.nodes(FEDERATED_ID)] == ["B"]  # C's beacons carry another token's MAC
        assert [n.id for n in rb.nodes(FEDERATED_ID)] == ["A"]
        assert rc.nodes(FEDERATED_ID) == [] and ra.get(FEDERATED_ID, "B").is_online()
    finally:
        for d in (a, b, c):
            d.stop()


def test_p2p_node_starts_discovery_with_token():
    n = P2PNode("tok", "", [], NodeData(id="me", address="127.0.0.1:9"), lan_discovery=True,
                discovery_targets=["127.0.0.1:9"], discovery_port=0)
    try:
        assert n.discovery is not None and n.discovery.beacon_once() == 1
    finally:
        n.stop()
    assert P2PNode("", "", [], None, lan_discovery=True).discovery is None  # no token: no beacons


def test_loopback_advertisement_replaced_by_sender_ip():
    """A node bound to 0.0.0.0 without LOCALAI_P2P_ADVERTISE advertises 127.0.0.1:<port>; the receiver must
    register it at the datagram's source address, never at its own loopback (which would proxy to itself)."""
    from localai_tfp_amd.p2p.discovery import reachable_address
    assert reachable_address("127.0.0.1:8080", "10.1.2.3") == "10.1.2.3:8080"
    assert reachable_address("0.0.0.0:8080", "10.1.2.3") == "10.1.2.3:8080"
    assert reachable_address("localhost:9", "10.1.2.3") == "10.1.2.3:9"
    assert reachable_address("[::1]:9", "10.1.2.3") == "10.1.2.3:9"
    assert reachable_address("10.0.0.7:8080", "10.1.2.3") == "10.0.0.7:8080"  # routable: kept
    assert reachable_address("node-b.lan:8080", "10.1.2.3") == "node-b.lan:8080"
    # over the wire: the advertised host differs from the sender's address
    ra = Registry("tok")
    a = LanDiscovery(ra, NodeData(id="A", address="10.9.9.9:1", service=FEDERATED_ID), "tok", port=0,
                     bind_host="127.0.0.1")
    b = LanDiscovery(Registry("tok"), NodeData(id="B", address="0.0.0.0:2222", service=FEDERATED_ID), "tok",
                     port=0, bind_host="127.0.0.1")
    try:
        b.targets = [("127.0.0.1", a.port)]
        assert b.beacon_once() == 1
        deadline = time.time() + 5
        node = None
        while node is None and time.time() < deadline:
            node = a.poll_once()
        assert node is not None and node.address == "127.0.0.1:2222"  # the sender's IP, its advertised port
        assert ra.get(FEDERATED_ID, "B").address == "127.0.0.1:2222"
    finally:
        a.stop()
        b.stop()
