"""SDXL (UNet) image generation benchmark on the implicit-GEMM conv kernel (or MIOpen with MX_CONV=miopen).

Random-init SDXL weights (UNet 2.6B + CLIP-L + OpenCLIP-G + VAE; no checkpoint download). Reports the UNet
step (CFG batch of 2), VAE decode and end-to-end seconds per image at --size.

    python tools/bench_sdxl.py --size 1024 --steps 20
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="sdxl")
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--images", type=int, default=1)
    a = ap.parse_args()
    from localai_tfp_amd.models.diffusion.pipeline import GenParams
    from localai_tfp_amd.models.diffusion.sd_pipeline import UNetPipeline
    dev = "cuda:0"
    t0 = time.perf_counter()
    p = UNetPipeline.synthetic(a.model, dev)
    torch.cuda.synchronize()
    res = {"model": a.model, "size": a.size, "steps": a.steps, "conv": os.environ.get("MX_CONV", "mfma-igemm"),
           "build_s": round(time.perf_counter() - t0, 1)}

    def timed(fn, n=3):
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / n * 1e3

    ctx, pooled = p.encode_prompts(["a photo of an astronaut riding a horse", ""])
    L = a.size // 8
    lat = torch.randn(2, 4, L, L, device=dev, dtype=torch.float32)
    t = torch.full((2,), 500.0, device=dev)
    added = None
    if p.xl:
        tid = torch.tensor([[a.size, a.size, 0, 0, a.size, a.size]], dtype=torch.float32, device=dev)
        added = {"text_embeds": pooled, "time_ids": tid.expand(2, 6)}
    res["unet_step_ms_cfg2"] = round(timed(lambda: p.unet(lat, t, ctx, added, ctx), 5), 2)
    z = torch.randn(1, 4, L, L, device=dev)
    res["vae_decode_ms"] = round(timed(lambda: p.vae.decode(z)), 2)
    gp = GenParams(width=a.size, height=a.size, steps=a.steps, seed=1)
    p.generate("warmup", GenParams(width=a.size, height=a.size, steps=2, seed=0))
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for i in range(a.images):
        gp.seed = i
        img = p.generate("a photo of an astronaut riding a horse", gp)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t1) / a.images
    res.update({"s_per_image": round(dt, 3), "images_per_s_per_gpu": round(1 / dt, 3),
                "finite": bool(torch.isfinite(img).all())})
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
