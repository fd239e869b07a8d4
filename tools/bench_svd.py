#!/usr/bin/env python3
"""Stable Video Diffusion img2vid timing (the reference's StableVideoDiffusionPipeline,
backend/python/diffusers/backend.py:175-179): random-init SVD weights of the real architecture
(1.52B-parameter spatio-temporal UNet, temporal-decoder VAE, ViT-H image encoder), one start image.
Reports the UNet step (CFG batch of 2 x frames), VAE decode per frame and end-to-end seconds per clip.

    python tools/bench_svd.py --model svd --width 1024 --height 576 --steps 4
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="svd", choices=["svd", "svd-xt"])
    ap.add_argument("--width", type=int, default=1024)
    ap.add_argument("--height", type=int, default=576)
    ap.add_argument("--steps", type=int, default=4)
    a = ap.parse_args()
    from PIL import Image

    from localai_tfp_amd.models.diffusion import svd as SV
    dev = "cuda:0"
    t0 = time.time()
    p = SV.SVDPipeline.synthetic(a.model, dev)
    build_s = time.time() - t0
    c = p.cfg
    Fr = c.num_frames
    h, w = a.height // 8, a.width // 8
    x = torch.randn(2, Fr, c.in_channels, h, w, device=dev)
    t = torch.full((2,), 0.5, device=dev)
    ctx = torch.randn(2, 1, c.cross_dim, device=dev)
    tid = torch.tensor([[6.0, 127.0, 0.02]] * 2, device=dev)
    key = object()
    p.unet(x, t, ctx, tid, ctx_key=key)
    torch.cuda.synchronize()
    t1 = time.time()
    n = 3
    for _ in range(n):
        p.unet(x, t, ctx, tid, ctx_key=key)
    torch.cuda.synchronize()
    step_ms = (time.time() - t1) / n * 1e3
    z = torch.randn(8, 4, h, w, device=dev)
    p.vae.decode(z, 8)
    torch.cuda.synchronize()
    t2 = time.time()
    p.vae.decode(z, 8)
    torch.cuda.synchronize()
    dec_ms_frame = (time.time() - t2) / 8 * 1e3
    im = Image.fromarray((np.random.RandomState(0).rand(a.height, a.width, 3) * 255).astype("uint8"))
    t3 = time.time()
    frames = p.generate(im, SV.VideoParams(width=a.width, height=a.height, steps=a.steps, seed=1))
    clip_s = time.time() - t3
    print(json.dumps({"model": a.model, "frames": Fr, "size": f"{a.width}x{a.height}", "steps": a.steps,
                      "build_s": round(build_s, 1), "unet_step_ms_cfg2": round(step_ms, 1),
                      "vae_decode_ms_per_frame": round(dec_ms_frame, 2), "clip_s": round(clip_s, 2),
                      "clip_s_25_steps_est": round(clip_s + (25 - a.steps) * step_ms / 1e3, 1),
                      "n_frames_out": len(frames), "dtype": "fp16", "data": "synthetic (random-init SVD weights)"}),
          flush=True)


if __name__ == "__main__":
    main()
