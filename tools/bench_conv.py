"""Implicit-GEMM MFMA conv (ops/conv.py) vs F.conv2d (MIOpen) on UNet / VAE shapes (MI355X).

python tools/bench_conv.py [--dtype f16|bf16] [--sweep]  -> one JSON line per shape
"""
import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from localai_tfp_amd.ops import conv as CV  # noqa: E402

# name, n, cin, cout, h, w, k, stride, up
SHAPES = [
    ("sdxl_l0_conv", 2, 320, 320, 128, 128, 3, 1, False),
    ("sdxl_l1_conv", 2, 640, 640, 64, 64, 3, 1, False),
    ("sdxl_l2_conv", 2, 1280, 1280, 32, 32, 3, 1, False),
    ("sdxl_up_cat_conv", 2, 960, 320, 128, 128, 3, 1, False),
    ("sdxl_upsample", 2, 640, 640, 64, 64, 3, 1, True),
    ("sd15_l3_conv", 2, 1280, 1280, 8, 8, 3, 1, False),
    ("vae_512_conv", 1, 512, 512, 128, 128, 3, 1, False),
    ("vae_256_conv", 1, 256, 256, 512, 512, 3, 1, False),
    ("vae_128_conv", 1, 128, 128, 1024, 1024, 3, 1, False),
    ("vae_conv_out", 1, 128, 3, 1024, 1024, 3, 1, False),
    ("shortcut_1x1", 2, 320, 640, 64, 64, 1, 1, False),
]


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="f16")
    ap.add_argument("--sweep", action="store_true", help="time every tile config")
    a = ap.parse_args()
    dt = torch.float16 if a.dtype == "f16" else torch.bfloat16
    for name, n, cin, cout, h, w, k, s, up in SHAPES:
        m = torch.nn.Conv2d(cin, cout, k, s, k // 2).cuda().to(dt)
        m.weight.data = m.weight.data.contiguous(memory_format=torch.channels_last)
        x = torch.randn(n, cin, h, w, device="cuda", dtype=dt).contiguous(memory_format=torch.channels_last)
        ho, wo = (2 * h, 2 * w) if up else (h // s, w // s)
        flop = 2.0 * n * ho * wo * cout * cin * k * k

        def miopen():
            xi = F.interpolate(x, scale_factor=2.0, mode="nearest") if up else x
            return F.conv2d(xi, m.weight, m.bias, s, k // 2)

        ref = miopen().float()
        y = CV.conv2d(x, m, upsample=up)
        err = float((y.float() - ref).norm() / ref.norm())
        t_mx = timeit(lambda: CV.conv2d(x, m, upsample=up))
        t_mi = timeit(miopen)
        rec = {"shape": name, "mx_us": round(t_mx, 1), "miopen_us": round(t_mi, 1),
               "mx_tflops": round(flop / t_mx / 1e6, 1), "miopen_tflops": round(flop / t_mi / 1e6, 1),
               "speedup": round(t_mi / t_mx, 2), "rel_err": round(err, 5),
               "auto_cfg": hex(CV.N.kernels().mxk_conv_tile_auto(n * ho * wo, cout))}
        if a.sweep:
            for cfg in (0x22, 0x14, 0x12, 0x11, 0x21):
                rec[hex(cfg)] = round(timeit(lambda: CV.conv2d(x, m, upsample=up, cfg=cfg)), 1)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
