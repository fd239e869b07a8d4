#!/usr/bin/env python3
"""BASELINE config #5 through the API: Stable-Diffusion-3 `/v1/images/generations` with data parallelism
(one diffusion worker process per GPU — model YAML `data_parallel: N` — the gateway spreading concurrent
requests over the replicas). Random-init SD3-medium weights (MMDiT 2B + CLIP-L/G + T5-XXL + VAE).

Starts the real gateway (uvicorn on 127.0.0.1) with worker subprocesses, warms every replica, then
sends `--images` requests from `--concurrency` clients and reports images/s and per-request latency.

    python tools/bench_images_http.py --gpus 1 --size 1024 --steps 28 --images 8 --concurrency 2
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import socket
import sys
import tempfile
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--model", default="sd3-medium")
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=28)
    ap.add_argument("--images", type=int, default=8)
    ap.add_argument("--concurrency", type=int, default=0, help="default: 2 per GPU")
    ap.add_argument("--timeout", type=float, default=900.0)
    a = ap.parse_args()
    import httpx
    import uvicorn
    import yaml

    from localai_tfp_amd.config.app_config import ApplicationConfig
    from localai_tfp_amd.gateway.app import create_app
    conc = a.concurrency or 2 * a.gpus
    tmp = tempfile.mkdtemp(prefix="bench_img_")
    models = os.path.join(tmp, "models")
    os.makedirs(models)
    with open(os.path.join(models, "sd3.yaml"), "w") as f:
        yaml.safe_dump({"name": "sd3", "backend": "diffusers", "parameters": {"model": f"synthetic:{a.model}"},
                        "step": a.steps, "data_parallel": a.gpus, "options": ["sampler:euler"]}, f)
    cfg = ApplicationConfig(models_path=models, generated_content_dir=os.path.join(tmp, "g"),
                            upload_dir=os.path.join(tmp, "u"), config_dir=os.path.join(tmp, "c"), api_keys=[])
    app = create_app(cfg, inproc=False)
    port = _free_port()
    server = uvicorn.Server(uvicorn.Config(app, host="127.0.0.1", port=port, log_level="warning"))
    th = threading.Thread(target=server.run, daemon=True)
    th.start()
    url = f"http://127.0.0.1:{port}"
    t_start = time.time()
    while not server.started:
        time.sleep(0.1)
        if time.time() - t_start > 60:
            raise SystemExit("gateway did not start")
    body = {"model": "sd3", "prompt": "a lighthouse on a cliff at dusk, oil painting", "size": f"{a.size}x{a.size}",
            "step": a.steps}

    async def one(client, i):
        t0 = time.time()
        r = await client.post(url + "/v1/images/generations", json={**body, "seed": 1 + i}, timeout=a.timeout)
        if r.status_code != 200:
            raise RuntimeError(f"HTTP {r.status_code}: {r.text[:300]}")
        return time.time() - t0

    async def run():
        async with httpx.AsyncClient() as client:
            t0 = time.time()
            # warm-up: one request per replica (model load + first-call kernel setup)
            await asyncio.gather(*[one(client, 1000 + i) for i in range(a.gpus)])
            warm = time.time() - t0
            sem = asyncio.Semaphore(conc)

            async def limited(i):
                async with sem:
                    return await one(client, i)
            t1 = time.time()
            lat = await asyncio.gather(*[limited(i) for i in range(a.images)])
            return warm, time.time() - t1, sorted(lat)
    warm, wall, lat = asyncio.run(run())
    server.should_exit = True
    th.join(timeout=30)
    app.state.localai.shutdown()
    ips = a.images / wall
    print(json.dumps({
        "metric": "images/s, Stable-Diffusion-3 /v1/images/generations (DP replicas)", "value": round(ips, 4),
        "unit": "images/s", "n_gpus": a.gpus, "images": a.images, "concurrency": conc, "size": a.size,
        "steps": a.steps, "s_per_image_per_gpu": round(a.gpus / ips, 3), "latency_p50_s": round(lat[len(lat) // 2], 3),
        "latency_max_s": round(lat[-1], 3), "warmup_s": round(warm, 1), "dtype": "fp16",
        "data": "synthetic (random-init SD3-medium weights)", "model": a.model}), flush=True)


if __name__ == "__main__":
    main()
