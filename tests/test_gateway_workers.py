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


def test_owner_watchdog_counts_sibling_activity(tmp_path):
    """the owner's idle watchdog must not kill a replica that an attached sibling process is
    serving — siblings report use through the registry and the owner folds it into its idle / busy checks."""
    import subprocess
    import sys
    import time

    from localai_tfp_amd.serving.model_loader import WatchDog
    from localai_tfp_amd.serving.shared_backends import ActivityReporter

    owner = SharedBackends(str(tmp_path))

    class _Loader:
        shared = owner
        killed: list = []

        def shutdown_model(self, m, force=False):
            self.killed.append(m)

    ld = _Loader()
    wd = WatchDog(ld, busy_timeout=1e9, idle_timeout=10.0, interval=1e9)
    wd.add("127.0.0.1:9", "m")
    wd.last_used["127.0.0.1:9"] = time.time() - 100  # the owner itself has not used it for 100 s
    # a live sibling process (not this pid) reports a request in flight
    sib = subprocess.Popen([sys.executable, "-c", "import time; time.sleep(30)"])
    try:
        rep = ActivityReporter(SharedBackends(str(tmp_path)))
        rep.shared.pid = sib.pid
        rep.mark("127.0.0.1:9")
        assert wd.check_once() == [] and ld.killed == []           # busy in a sibling: not idle
        rep.unmark("127.0.0.1:9")
        assert wd.check_once() == []                               # used by the sibling just now
        assert wd.check_once(now=time.time() + 60) == ["m"]        # nobody used it for 60 s
    finally:
        sib.kill()
        sib.wait()
