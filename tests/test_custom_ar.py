"""One-shot IPC all-reduce (csrc/kernels/allreduce.hip): several processes exchange hipIpc handles over gloo
and reduce 16-bit tensors (sizes 2 .. 1 MB, f16 / bf16, eager and hipGraph replay) against an fp32 sum.
On the 1-GPU box the ranks share the GPU (same protocol: uncached receive buffers, 8-byte tagged granules)."""
import os
import socket
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4, 8])
def test_one_shot_allreduce_multiprocess(world):
    port = _port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "_ar_worker.py")], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=100)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(out)
    for r, (p, o) in enumerate(zip(procs, outs)):
        assert p.returncode == 0, f"rank {r} rc={p.returncode}\n{o[-3000:]}"
    for ln in outs[0].splitlines():  # rank 0's latency lines into the test log
        if "us/call" in ln:
            print(ln)


@pytest.mark.gpu
def test_one_shot_allreduce_single_rank_graph():
    """World-1 instance (the --tp-rehearsal stand-in): identity all-reduce and residual add, eager and replayed from a
    hipGraph many times — the in-kernel epoch bump (last workgroup's ticket) must advance once per call."""
    import torch
    from localai_tfp_amd.parallel.custom_ar import OneShotAllReduce
    ar = OneShotAllReduce(None, "cuda", 1 << 20, world=1)
    g = torch.Generator(device="cuda").manual_seed(0)
    for n in (2, 4096, 1 << 19):  # 1 .. 128 workgroups
        t = torch.randn(n, device="cuda", generator=g).to(torch.float16)
        res = torch.randn(n, device="cuda", generator=g)
        ref = res + t.float()
        ar.add_into(t, res)
        out = torch.empty_like(t)
        ar(t, out)
        torch.cuda.synchronize()
        assert torch.equal(out, t)
        assert torch.allclose(res, ref, atol=1e-6)
    e0 = int(ar.epoch[0])
    assert int(ar.epoch[1]) == 0  # ticket re-armed
    t = torch.randn(8192, device="cuda", generator=g).to(torch.float16)
    res = torch.zeros(8192, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ar.add_into(t, res)  # warm-up outside capture
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s):
        ar.add_into(t, res)
    res.zero_()
    for _ in range(50):
        graph.replay()
    torch.cuda.synchronize()
    assert torch.allclose(res, 50 * t.float(), atol=1e-3)
    assert int(ar.epoch[0]) == e0 + 51  # the warm-up call + 50 replays (capture launches nothing)
    assert int(ar.epoch[1]) == 0
