"""Run one qgemm32 / qgemm16 / dense configuration in a loop (for rocprofv3 counter collection)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from localai_tfp_amd.formats.gguf import QType  # noqa: E402
from localai_tfp_amd.ops import linear as L  # noqa: E402
from localai_tfp_amd.ops.quant import random_quantized  # noqa: E402

N, K, M = int(os.environ.get("N", 28672)), int(os.environ.get("K", 4096)), int(os.environ.get("M", 128))
epi = {"swiglu": L.EPI_SWIGLU, "add": L.EPI_ADD_F32, "f32": L.EPI_F32}[os.environ.get("EPI", "swiglu")]
W = L.QWeight.from_ggml(random_quantized(np.random.default_rng(1), int(QType.Q4_K), N, K), int(QType.Q4_K), N, K,
                        torch.device("cuda"))
x = torch.randn(M, K, device="cuda").half()
out = torch.empty(M, N // 2, device="cuda", dtype=torch.float16) if epi == L.EPI_SWIGLU else \
    torch.zeros(M, N, device="cuda")
path = os.environ.get("PATH_", "q32")
L.BF16_CACHE_MIN_M = 10**9
L.Q32_MIN_M = 1 if path == "q32" else 10**9
for _ in range(int(os.environ.get("IT", 20))):
    L.qmatmul(W, x, epi, out, out_zeroed=True)
torch.cuda.synchronize()
print("done")
