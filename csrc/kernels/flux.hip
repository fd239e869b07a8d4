// flux.hip — fused per-head QK RMSNorm + 3-axis rotary embedding for the Flux transformer.
//
// Reference: the diffusers backend's FluxPipeline (backend/python/diffusers/backend.py:139-270) and
// stable-diffusion.cpp's Flux graph behind stablediffusion-ggml (gosd.cpp:56-162); SURVEY.md §2.3
// N4/N5. Every Flux attention (19 double-stream + 38 single-stream blocks) normalises q and k per
// head with a learned RMSNorm and rotates them with RoPE over (text | row | col) position ids
// (axes 16/56/56 of the 128-wide head). Done in place on the fused QKV GEMM output: one wave64 per
// (row, head, q|k), lane l owns the rotary pair (2l, 2l+1) — one dword load, a 6-step shuffle
// reduction for the RMS, the (cos, sin) pair for that position and lane from a [L, 64, 2] table,
// one dword store. Replaces ~8 elementwise launches (norm, weight, rope split/rotate/cat) per
// attention with one.
#include "mx_common.h"

// one wave per (row, head): RMSNorm over the head (weight w) then interleaved-pair rotary from the table
// row r % L ([L, hd/2, 2] cos/sin). q heads at columns [0, Hq*hd), k heads at [koff, koff + Hk*hd)
// (grouped-query layouts have Hk < Hq). Head dims up to 128 (lanes past hd/2 idle).
template <bool F16>
__global__ __launch_bounds__(64) void qk_norm_rope_kernel(uint16_t* __restrict__ qkv, int ld, int Hq, int koff,
                                                          int hd, const float* __restrict__ wq,
                                                          const float* __restrict__ wk,
                                                          const float* __restrict__ cs, int L, float eps) {
    const int r = blockIdx.x;
    const int which = blockIdx.y >= Hq;  // 0: q, 1: k
    const int h = blockIdx.y - which * Hq;
    const int l = threadIdx.x, np = hd >> 1;
    uint32_t* p = reinterpret_cast<uint32_t*>(qkv + (size_t)r * ld + (which ? koff : 0) + h * hd) + l;
    float x0 = 0.f, x1 = 0.f;
    if (l < np) unpack_act2<F16>(*p, x0, x1);
    float ss = x0 * x0 + x1 * x1;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
    if (l >= np) return;
    const float inv = rsqrtf(ss / (float)hd + eps);
    const float* w = which ? wk : wq;
    const float y0 = x0 * inv * w[2 * l], y1 = x1 * inv * w[2 * l + 1];
    const float2 c = reinterpret_cast<const float2*>(cs)[(size_t)(r % L) * np + l];
    *p = pack_act2<F16>(y0 * c.x - y1 * c.y, y1 * c.x + y0 * c.y);
}

extern "C" int mxk_qk_norm_rope(uint16_t* qkv, int ld, int rows, int D, int H, int head_dim, const float* wq,
                                const float* wk, const float* cs, int L, float eps, hipStream_t st) {
    if (rows == 0) return 0;
    if (head_dim != 128 || D != H * head_dim || (ld & 1)) return (int)hipErrorInvalidValue;
    dim3 grid(rows, 2 * H);
    MX_ACT_DISPATCH((qk_norm_rope_kernel<F16><<<grid, 64, 0, st>>>(qkv, ld, H, D, head_dim, wq, wk, cs, L, eps)));
    return (int)hipGetLastError();
}

// grouped-query variant: Hq query heads at column 0, Hk key heads at column koff, even head dim <= 128
extern "C" int mxk_qk_norm_rope_gqa(uint16_t* qkv, int ld, int rows, int Hq, int Hk, int head_dim, int koff,
                                    const float* wq, const float* wk, const float* cs, int L, float eps,
                                    hipStream_t st) {
    if (rows == 0) return 0;
    if (head_dim > 128 || (head_dim & 1) || (ld & 1) || (koff & 1) || koff < Hq * head_dim) return (int)hipErrorInvalidValue;
    dim3 grid(rows, Hq + Hk);
    MX_ACT_DISPATCH((qk_norm_rope_kernel<F16><<<grid, 64, 0, st>>>(qkv, ld, Hq, koff, head_dim, wq, wk, cs, L, eps)));
    return (int)hipGetLastError();
}
