"""SD3 image generation benchmark (BASELINE config #5: Stable-Diffusion-3 /v1/images/generations,
data parallel across GPUs — one replica per GPU, so per-GPU images/s x N is the DP throughput).

Random-init SD3-medium weights (MMDiT 2B + CLIP-L + CLIP-G + T5-XXL + 16-ch VAE; no checkpoint
download). Reports text-encode, per-step transformer (CFG batch of 2) and VAE-decode latencies and
the end-to-end seconds per image.

    python tools/bench_sd3.py --size 1024 --steps 28
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
    ap.add_argument("--model", default="sd3-medium")
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=28)
    ap.add_argument("--images", type=int, default=2)
    ap.add_argument("--sampler", default="euler")
    a = ap.parse_args()
    from localai_tfp_amd.models.diffusion.pipeline import GenParams, SD3Pipeline
    dev = "cuda:0"
    t0 = time.perf_counter()
    p = SD3Pipeline.synthetic(a.model, dev)
    torch.cuda.synchronize()
    res = {"model": a.model, "size": a.size, "steps": a.steps, "build_s": round(time.perf_counter() - t0, 1)}

    def timed(fn, n=3):
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / n * 1e3

    ctx, pooled = p.encode_prompts(["a photo of an astronaut riding a horse", ""])
    res["text_encode_ms"] = round(timed(lambda: p.encode_prompts(["a photo of an astronaut riding a horse", ""])), 2)
    lat = torch.randn(2, 16, a.size // 8, a.size // 8, device=dev)
    t = torch.full((2,), 500.0, device=dev)
    res["mmdit_step_ms_cfg2"] = round(timed(lambda: p.mmdit(lat, t, ctx, pooled), 5), 2)
    z = torch.randn(1, 16, a.size // 8, a.size // 8, device=dev)
    res["vae_decode_ms"] = round(timed(lambda: p.vae.decode(z)), 2)
    gp = GenParams(width=a.size, height=a.size, steps=a.steps, seed=1, sampler=a.sampler)
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
    # FLOP estimate of the transformer step (2 x params x tokens + attention), for MFMA utilisation
    c = p.mmdit.cfg
    S_img = (a.size // 16) ** 2
    T = 77 + p.p.t5_tokens
    n_par = sum(x.numel() for x in p.mmdit.transformer_blocks.parameters())
    fl = 2 * 2 * n_par * (S_img + T) + 2 * c.layers * 4 * (S_img + T) ** 2 * c.dim
    res["mmdit_tflops"] = round(fl / (res["mmdit_step_ms_cfg2"] * 1e-3) / 1e12, 1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
