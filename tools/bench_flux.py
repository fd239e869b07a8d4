"""Flux.1 image generation benchmark (diffusers / stablediffusion-ggml Flux path).

Random-init Flux.1-dev (or schnell) weights — 12B transformer + CLIP-L + T5-XXL + 16-ch VAE; no
checkpoint download. Reports text-encode, per-step transformer, VAE-decode latencies, transformer
TFLOP/s (dense GEMM + attention FLOPs) and the end-to-end seconds per image.

    python tools/bench_flux.py --model flux-dev --size 1024 --steps 28
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
    ap.add_argument("--model", default="flux-dev")
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=28)
    ap.add_argument("--images", type=int, default=1)
    a = ap.parse_args()
    from localai_tfp_amd.models.diffusion import flux as FX
    from localai_tfp_amd.models.diffusion.pipeline import GenParams
    dev = "cuda:0"
    t0 = time.perf_counter()
    p = FX.FluxPipeline.synthetic(a.model, dev)
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

    prompt = "a photo of an astronaut riding a horse"
    ctx, pooled = p.encode_prompts([prompt])
    res["text_encode_ms"] = round(timed(lambda: p.encode_prompts([prompt])), 2)
    h = w = a.size // 8
    S = (h // 2) * (w // 2)
    x = torch.randn(1, S, 64, device=dev)
    ids = FX.image_ids(h // 2, w // 2, dev)
    t = torch.full((1,), 0.5, device=dev)
    g = torch.full((1,), 3.5, device=dev)
    step_ms = timed(lambda: p.tr(x, ids, t, ctx, pooled, g), 5)
    res["transformer_step_ms"] = round(step_ms, 2)
    c = p.cfg
    D, L = c.dim, S + ctx.shape[1]
    params = sum(v.numel() for k, v in p.tr.state_dict().items() if v.dim() == 2)
    flops = 2 * params * L + (c.layers + c.single_layers) * 4 * L * L * D
    res["transformer_tflops"] = round(flops / (step_ms * 1e-3) / 1e12, 1)
    z = torch.randn(1, 16, h, w, device=dev)
    res["vae_decode_ms"] = round(timed(lambda: p.vae.decode(z)), 2)
    gp = GenParams(width=a.size, height=a.size, steps=a.steps, seed=1)
    p.generate("warmup", GenParams(width=a.size, height=a.size, steps=1, seed=0))
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for i in range(a.images):
        gp.seed = i
        p.generate(prompt, gp)
    torch.cuda.synchronize()
    res["s_per_image"] = round((time.perf_counter() - t1) / a.images, 3)
    res["images_per_s_per_gpu"] = round(1.0 / res["s_per_image"], 4)
    res["data"] = "synthetic (random-init Flux.1 weights, bf16)"
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
