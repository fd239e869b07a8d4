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
