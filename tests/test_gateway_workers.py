"""Multi-process gateway (`local-ai run --gateway-workers N`, cli.py + serving/shared_backends.py): N gateway
processes accept on one SO_REUSEPORT address and share the data-parallel replicas through the backend registry.
Checked end to end with fake mxstream workers (tools/gateway_bench.py): every request completes, the replicas are
spawned once (not once per gateway process), and the registry entry follows its owner."""
import os

from localai_tfp_amd.serving.shared_backends import SharedBackends
from localai_tfp_amd.tools.gateway_bench import run_bench


class _R:
    def __init__(self, a, p):
        self.address, self.mx_path = a, p


def test_registry_publish_read_withdraw(tmp_path):
    reg = SharedBackends(str(tmp_path))
    assert reg.read("m") is None
    with reg.locked("m"):
        e = reg.publish("m", "llama-cpp", [_R("127.0.0.1:1", "/x.sock")])
    got = reg.read("m")
    assert SharedBackends.same(got, e) and got["owner"] == os.getpid()
    other = SharedBackends(str(tmp_path))
    other.pid = -1  # not the owner: withdraw is a no-op
    other.withdraw("m")
    assert reg.read("m") is not None
    reg.withdraw("m")
    assert reg.read("m") is None


def test_dead_owner_entry_is_ignored(tmp_path):
    reg = SharedBackends(str(tmp_path))
    reg.pid = 2 ** 22 + 12345  # no such process
    reg.publish("m", "llama-cpp", [])
    assert reg.read("m") is None


def test_gateway_workers_share_replicas():
    r = run_bench(replicas=2, concurrency=24, tokens=16, step_ms=5.0, duration=3.0, loadgen_procs=1,
                  gateway_workers=2)
    assert r["workers_started"] == 2, r  # one model load, shared by both gateway processes
    assert r["requests_ok"] > 20 and r["chunks_per_s"] > 0, r
