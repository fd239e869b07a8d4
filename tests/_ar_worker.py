"""Helper process for test_custom_ar.py: one rank of a one-shot all-reduce group (gloo for the handle
exchange and the reference; all ranks may share one GPU)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ndev = torch.cuda.device_count()
    dev = torch.device("cuda", rank % ndev)
    torch.cuda.set_device(dev)
    from localai_tfp_amd.parallel.custom_ar import OneShotAllReduce
    ar = OneShotAllReduce(dist.group.WORLD, dev, max_bytes=1 << 20)
    ok = True
    for it, (n, dt) in enumerate([(2, torch.float16), (4096, torch.bfloat16), (8192 * 4, torch.float16),
                                  (131072, torch.bfloat16), (524288, torch.float16), (4096, torch.float16)]):
        g = torch.Generator().manual_seed(1000 * it + rank)
        x = torch.randn(n, generator=g)
        parts = [torch.randn(n, generator=torch.Generator().manual_seed(1000 * it + r)) for r in range(world)]
        ref = sum(p.to(dt).float() for p in parts)
        t = x.to(dev, dt)
        ar(t)
        torch.cuda.synchronize()
        ar.check(block=True)
        err = (t.float().cpu() - ref).abs().max().item()
        tol = 1e-2 if dt == torch.float16 else 6e-2
        ok &= err < tol * max(1.0, ref.abs().max().item())
        print(f"rank {rank} n={n} {dt} err={err:.3g}", flush=True)
    # fused all-reduce + fp32 residual add (row-parallel projection epilogue)
    for n in (4096, 8192 * 4):
        parts = [torch.randn(n, generator=torch.Generator().manual_seed(77 + r)) for r in range(world)]
        ref = sum(p.half().float() for p in parts) + 1.5
        res = torch.full((n,), 1.5, device=dev)
        ar.add_into(parts[rank].to(dev, torch.float16), res)
        torch.cuda.synchronize()
        ar.check(block=True)
        err = (res.cpu() - ref).abs().max().item()
        ok &= err < 1e-2 * max(1.0, ref.abs().max().item())
        print(f"rank {rank} add_into n={n} err={err:.3g}", flush=True)
    # hipGraph capture + replays (epoch counter lives on the device)
    t = torch.zeros(8192, device=dev, dtype=torch.float16)
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        t.fill_(rank + 1)
        ar(t)
    torch.cuda.current_stream(dev).wait_stream(s)
    torch.cuda.synchronize()
    dist.barrier()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        t.fill_(rank + 1)
        ar(t)
    for _ in range(5):
        graph.replay()
        torch.cuda.synchronize()
        ar.check(block=True)
        ok &= bool((t.float() == world * (world + 1) / 2).all())
    print(f"rank {rank} graph ok={ok}", flush=True)
    # check() never blocks on queued work: a long kernel queued after the snapshot leaves it pending,
    # and the host call returns at once (the overlap pipeline calls it between two launched steps)
    import time
    ar(t)
    ar.snapshot()
    torch.cuda._sleep(int(1e9))  # ~0.4-0.5 s of device time queued behind the snapshot
    t0 = time.perf_counter()
    ar.check()
    dt = time.perf_counter() - t0
    busy = not torch.cuda.current_stream(dev).query()
    torch.cuda.synchronize()
    ar.check(block=True)
    ok &= dt < 0.02 and busy
    print(f"rank {rank} nonblocking check {dt * 1e3:.2f} ms (stream busy={busy}) ok={ok}", flush=True)
    # per-call latency at 16 KB and 1 MB (all ranks issue back to back; on the 1-GPU box the ranks share one GPU,
    # so this measures the protocol, not xGMI)
    for nbytes in (16 << 10, 1 << 20):
        t = torch.ones(nbytes // 2, device=dev, dtype=torch.float16)
        dist.barrier()
        for _ in range(5):
            ar(t)
        torch.cuda.synchronize()
        dist.barrier()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            ar(t)
        e1.record()
        torch.cuda.synchronize()
        ar.check(block=True)
        print(f"rank {rank} world {world} allreduce {nbytes >> 10} KB: {e0.elapsed_time(e1) / 20 * 1e3:.1f} us/call",
              flush=True)
    dist.barrier()
    ar.close()
    dist.destroy_process_group()
    sys.exit(0 if ok else 3)


if __name__ == "__main__":
    main()
