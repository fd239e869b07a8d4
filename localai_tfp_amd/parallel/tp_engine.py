"""Tensor-parallel serving: one process per GPU, rank 0 leads.

The leader owns the scheduler, sampler, gRPC server and block manager; every engine step it sends
the step plan (engine._plan: token ids, positions, KV slots, block tables — a few KB of int32) to
the followers, and all ranks run the same forward (RCCL all-reduces over xGMI inside the model,
parallel/tp.py). Only the leader samples. Control messages (model load / unload) travel on the same
channel, so ranks stay in lock-step by construction.

Channel: a gloo (CPU/TCP) process group next to the RCCL one — plans are host data the followers
need on the host anyway, and a CPU broadcast never queues behind GPU work on the RCCL stream.
Behavioural parity: the reference's only TP is inside vLLM (backend/python/vllm/backend.py:106-107).
"""
from __future__ import annotations

import datetime
import logging
import os

import torch

log = logging.getLogger("localai_tfp_amd.tp")

STOP = None


class TPLink:
    def __init__(self, rank: int, world: int, cpu_group, gpu_group=None):
        self.rank, self.world = rank, world
        self.cpu_group, self.gpu_group = cpu_group, gpu_group
        self.is_leader = rank == 0

    # -------------------------------------------------------------- messages (leader -> followers)
    def _bcast(self, obj=None):
        import torch.distributed as dist
        buf = [obj]
        dist.broadcast_object_list(buf, src=0, group=self.cpu_group)
        return buf[0]

    def send_plan(self, plan):
        assert self.is_leader
        self._bcast(plan)

    def recv_plan(self):
        return self._bcast(None)

    def send_control(self, kind: str, payload=None):
        self._bcast(("ctl", kind, payload))

    def recv_control(self):
        msg = self._bcast(None)
        if not (isinstance(msg, tuple) and msg and msg[0] == "ctl"):
            raise RuntimeError(f"tensor-parallel follower expected a control message, got {type(msg)}")
        return msg[1], msg[2]

    # -------------------------------------------------------------- collectives on host ints
    def allreduce_min(self, x: int) -> int:
        import torch.distributed as dist
        t = torch.tensor([int(x)], dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.cpu_group)
        return int(t.item())


def init_from_env():
    """torch.distributed.run environment -> (TPLink, local device). RCCL for the model's
    all-reduces, gloo (no timeout in practice: idle followers wait on it) for plans."""
    import torch.distributed as dist
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    cpu = dist.new_group(backend="gloo", timeout=datetime.timedelta(days=365))
    return TPLink(rank, world, cpu, None), dev


def follower_main(link: TPLink, device):
    """Non-leader ranks: wait for control messages; on `load` build the same model shard + engine
    and replay plans until the leader unloads / stops."""
    from ..engine.engine import EngineConfig, LLMEngine
    from ..models.loader import load_llm
    while True:
        kind, payload = link.recv_control()
        if kind == "stop":
            return
        if kind != "load":
            continue
        path, overrides, ecfg_dict = payload
        model, tok, _, _ = load_llm(path, device, link.rank, link.world, None, overrides)
        ec = EngineConfig(**ecfg_dict)
        eng = LLMEngine(model, tok, ec, tp=link)
        log.info("rank %d: model shard loaded, following", link.rank)
        eng.follow()
        del eng, model
        torch.cuda.empty_cache()
