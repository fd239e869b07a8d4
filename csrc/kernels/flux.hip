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

template <bool F16>
__global__ __launch_bounds__(64) void qk_norm_rope_kernel(uint16_t* __restrict__ qkv, int ld, int D,
                                                          const float* __restrict__ wq,
                                                          const float* __restrict__ wk,
                                                          const float* __restrict__ cs,  // [L, 64, 2]
                                                          int L, int H, float eps) {
    constexpr int HD = 128;
    const int r = blockIdx.x;
    const int which = blockIdx.y >= H;  // 0: q, 1: k
    const int h = blockIdx.y - which * H;
    const int l = threadIdx.x;
    uint32_t* p = reinterpret_cast<uint32_t*>(qkv + (size_t)r * ld + which * D + h * HD) + l;
    float x0, x1;
    unpack_act2<F16>(*p, x0, x1);
    float ss = x0 * x0 + x1 * x1;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
    const float inv = rsqrtf(ss * (1.f / HD) + eps);
    const float* w = which ? wk : wq;
    const float y0 = x0 * inv * w[2 * l], y1 = x1 * inv * w[2 * l + 1];
    const float2 c = reinterpret_cast<const float2*>(cs)[(size_t)(r % L) * 64 + l];
    *p = pack_act2<F16>(y0 * c.x - y1 * c.y, y1 * c.x + y0 * c.y);
}

extern "C" int mxk_qk_norm_rope(uint16_t* qkv, int ld, int rows, int D, int H, int head_dim, const float* wq,
                                const float* wk, const float* cs, int L, float eps, hipStream_t st) {
    if (rows == 0) return 0;
    if (head_dim != 128 || D != H * head_dim || (ld & 1)) return (int)hipErrorInvalidValue;
    dim3 grid(rows, 2 * H);
    MX_ACT_DISPATCH((qk_norm_rope_kernel<F16><<<grid, 64, 0, st>>>(qkv, ld, D, wq, wk, cs, L, H, eps)));
    return (int)hipGetLastError();
}
