// norm.hip — RMSNorm / LayerNorm / activation-quantisation kernels (K6, K7 of SURVEY §2.6).
//
// The LLM keeps its residual stream in fp32 (as ggml does). Each norm kernel reads that stream once
// and writes the GEMM-ready operand directly:
//   * bf16 rows for the MFMA dequant-GEMM path (M > 8), and/or
//   * q8 blocks (int8 x32 + float2{d, d*sum}) for the int8 dot-product GEMV path (M <= 8) — the same
//     activation quantisation llama.cpp's MMVQ uses (ggml q8_1), so decode numerics match the
//     reference engine (grpc-server.cpp:2002 -> llama_decode -> mmvq).
// One 256-thread workgroup per row; float4 loads; the sum of squares never leaves registers/LDS.
#include "mx_common.h"

template <bool WANT_BF16, bool WANT_Q8, bool HAS_RES, bool F16>
__global__ __launch_bounds__(256) void rmsnorm_kernel(const float* __restrict__ x, int ldx,
                                                      const bf16_t* __restrict__ res, int ldr,
                                                      float* __restrict__ xout, const float* __restrict__ w,
                                                      bf16_t* __restrict__ ob, int ldo, int8_t* __restrict__ oq,
                                                      float2* __restrict__ ods, int H, float eps) {
    __shared__ float red[4];
    const int row = blockIdx.x;
    const float* xr = x + (size_t)row * ldx;
    float4 v[8];  // up to H = 8192
    const int nv = H / 1024;  // float4 chunks per thread (H multiple of 1024 handled by main path)
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        if (i < nv) {
            const int c = (i * 256 + threadIdx.x) * 4;
            v[i] = *(const float4*)(xr + c);
            if (HAS_RES) {
                const bf16_t* rr = res + (size_t)row * ldr + c;
                uint2 r = *(const uint2*)rr;
                v[i].x += __uint_as_float(r.x << 16);
                v[i].y += __uint_as_float(r.x & 0xFFFF0000u);
                v[i].z += __uint_as_float(r.y << 16);
                v[i].w += __uint_as_float(r.y & 0xFFFF0000u);
                *(float4*)(xout + (size_t)row * ldx + c) = v[i];
            }
            ss += v[i].x * v[i].x + v[i].y * v[i].y + v[i].z * v[i].z + v[i].w * v[i].w;
        }
    }
    ss = block_sum<256>(ss, red);
    const float rs = rsqrtf(ss / (float)H + eps);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        if (i < nv) {
            const int c = (i * 256 + threadIdx.x) * 4;
            float4 g = *(const float4*)(w + c);
            float a0 = v[i].x * rs * g.x, a1 = v[i].y * rs * g.y, a2 = v[i].z * rs * g.z, a3 = v[i].w * rs * g.w;
            if (WANT_BF16) {
                uint2 p;
                p.x = pack_act2<F16>(a0, a1);
                p.y = pack_act2<F16>(a2, a3);
                *(uint2*)(ob + (size_t)row * ldo + c) = p;
            }
            if (WANT_Q8) {
                // 32-element block = 8 consecutive threads
                float am = fmaxf(fmaxf(fabsf(a0), fabsf(a1)), fmaxf(fabsf(a2), fabsf(a3)));
                am = group_max<8>(am);
                const float d = am / 127.f;
                const float id = d > 0.f ? 1.f / d : 0.f;
                int q0 = __float2int_rn(a0 * id), q1 = __float2int_rn(a1 * id), q2 = __float2int_rn(a2 * id),
                    q3 = __float2int_rn(a3 * id);
                int s = group_sum<8>((float)(q0 + q1 + q2 + q3));
                uint32_t pk = (uint32_t)(q0 & 0xFF) | ((uint32_t)(q1 & 0xFF) << 8) | ((uint32_t)(q2 & 0xFF) << 16) |
                              ((uint32_t)(q3 & 0xFF) << 24);
                *(uint32_t*)(oq + (size_t)row * H + c) = pk;
                if ((threadIdx.x & 7) == 0) ods[(size_t)row * (H / 32) + c / 32] = make_float2(d, d * (float)s);
            }
        }
    }
}

// generic (any H multiple of 32) slow path: one thread per element pair, used for odd model sizes.
template <bool WANT_BF16, bool WANT_Q8, bool F16>
__global__ __launch_bounds__(256) void rmsnorm_generic_kernel(const float* __restrict__ x, int ldx,
                                                              const float* __restrict__ w, bf16_t* __restrict__ ob,
                                                              int ldo, int8_t* __restrict__ oq,
                                                              float2* __restrict__ ods, int H, float eps) {
    __shared__ float red[4];
    const int row = blockIdx.x;
    const float* xr = x + (size_t)row * ldx;
    float ss = 0.f;
    for (int c = threadIdx.x; c < H; c += 256) ss += xr[c] * xr[c];
    ss = block_sum<256>(ss, red);
    const float rs = rsqrtf(ss / (float)H + eps);
    // q8 blocks: each wave handles blocks of 32 with 32 lanes active per half
    for (int b = threadIdx.x / 32; b < (H + 31) / 32; b += 8) {
        const int c = b * 32 + (threadIdx.x & 31);
        float a = c < H ? xr[c] * rs * w[c] : 0.f;
        if (WANT_BF16 && c < H) ob[(size_t)row * ldo + c] = f32_to_act<F16>(a);
        if (WANT_Q8) {
            float am = group_max<32>(fabsf(a));
            float d = am / 127.f;
            float id = d > 0.f ? 1.f / d : 0.f;
            int q = __float2int_rn(a * id);
            float s = group_sum<32>((float)q);
            if (c < H) oq[(size_t)row * H + c] = (int8_t)q;
            if ((threadIdx.x & 31) == 0) ods[(size_t)row * (H / 32) + b] = make_float2(d, d * s);
        }
    }
}

extern "C" int mxk_rmsnorm(const float* x, int ldx, const bf16_t* res, int ldr, float* xout, const float* w,
                           bf16_t* ob, int ldo, int8_t* oq, float2* ods, int rows, int H, float eps,
                           hipStream_t st) {
    if (rows <= 0) return 0;
    const bool wb = ob != nullptr, wq = oq != nullptr, hr = res != nullptr;
    if (H % 1024 == 0 && H <= 8192) {
#define RMS_L(B, Q, R) \
    rmsnorm_kernel<B, Q, R, F16><<<rows, 256, 0, st>>>(x, ldx, res, ldr, xout, w, ob, ldo, oq, ods, H, eps)
        MX_ACT_DISPATCH({
            if (hr) {
                if (wb && wq) RMS_L(true, true, true);
                else if (wb) RMS_L(true, false, true);
                else RMS_L(false, true, true);
            } else {
                if (wb && wq) RMS_L(true, true, false);
                else if (wb) RMS_L(true, false, false);
                else RMS_L(false, true, false);
            }
        });
#undef RMS_L
    } else {
        if (hr) return (int)hipErrorInvalidValue;  // residual fusion only on the fast path
        MX_ACT_DISPATCH({
            if (wb && wq)
                rmsnorm_generic_kernel<true, true, F16><<<rows, 256, 0, st>>>(x, ldx, w, ob, ldo, oq, ods, H, eps);
            else if (wb)
                rmsnorm_generic_kernel<true, false, F16><<<rows, 256, 0, st>>>(x, ldx, w, ob, ldo, oq, ods, H, eps);
            else
                rmsnorm_generic_kernel<false, true, F16><<<rows, 256, 0, st>>>(x, ldx, w, ob, ldo, oq, ods, H, eps);
        });
    }
    MXK_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------------------------
// h += y / rms(y) * w — Gemma 2/3 post-attention / post-FFN norm fused into the residual add.
// One 256-thread workgroup per row, float4 over H (H % 4 == 0); y is re-read from L2 for the add.
__global__ __launch_bounds__(256) void rmsnorm_add_kernel(const float* __restrict__ y, int ldy,
                                                          const float* __restrict__ w, float* __restrict__ h,
                                                          int ldh, int H, float eps) {
    __shared__ float red[4];
    const float* yr = y + (size_t)blockIdx.x * ldy;
    float* hr = h + (size_t)blockIdx.x * ldh;
    float ss = 0.f;
    for (int c = threadIdx.x * 4; c < H; c += 1024) {
        const float4 v = *(const float4*)(yr + c);
        ss += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
    }
    ss = block_sum<256>(ss, red);
    const float rs = rsqrtf(ss / (float)H + eps);
    for (int c = threadIdx.x * 4; c < H; c += 1024) {
        const float4 v = *(const float4*)(yr + c);
        const float4 g = *(const float4*)(w + c);
        float4 o = *(const float4*)(hr + c);
        o.x += v.x * rs * g.x;
        o.y += v.y * rs * g.y;
        o.z += v.z * rs * g.z;
        o.w += v.w * rs * g.w;
        *(float4*)(hr + c) = o;
    }
}

extern "C" int mxk_rmsnorm_add(const float* y, int ldy, const float* w, float* h, int ldh, int rows, int H, float eps,
                               hipStream_t st) {
    if (rows <= 0) return 0;
    if ((H & 3) || (ldy & 3) || (ldh & 3)) return (int)hipErrorInvalidValue;
    rmsnorm_add_kernel<<<rows, 256, 0, st>>>(y, ldy, w, h, ldh, H, eps);
    MXK_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------------------------
// quantise bf16 rows to q8 blocks (for the GEMV path after attention / SwiGLU). One wave per
// 64 x 32-element block group: lane l handles 8 elements; 4 lanes per block.
template <bool F16>
__global__ __launch_bounds__(256) void quant_q8_kernel(const bf16_t* __restrict__ x, int ldx, int8_t* __restrict__ oq,
                                                       float2* __restrict__ ods, int K) {
    const int row = blockIdx.y;
    const int e0 = (blockIdx.x * 256 + threadIdx.x) * 8;
    if (e0 >= K) return;  // K multiple of 32 -> whole 4-lane groups exit together
    uint4 raw = *(const uint4*)(x + (size_t)row * ldx + e0);
    float a[8];
    unpack_act2<F16>(raw.x, a[0], a[1]);
    unpack_act2<F16>(raw.y, a[2], a[3]);
    unpack_act2<F16>(raw.z, a[4], a[5]);
    unpack_act2<F16>(raw.w, a[6], a[7]);
    float am = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) am = fmaxf(am, fabsf(a[i]));
    am = group_max<4>(am);
    const float d = am / 127.f, id = d > 0.f ? 1.f / d : 0.f;
    int q[8], s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) { q[i] = __float2int_rn(a[i] * id); s += q[i]; }
    float sf = group_sum<4>((float)s);
    uint2 pk;
    pk.x = (q[0] & 0xFF) | ((q[1] & 0xFF) << 8) | ((q[2] & 0xFF) << 16) | ((uint32_t)(q[3] & 0xFF) << 24);
    pk.y = (q[4] & 0xFF) | ((q[5] & 0xFF) << 8) | ((q[6] & 0xFF) << 16) | ((uint32_t)(q[7] & 0xFF) << 24);
    *(uint2*)(oq + (size_t)row * K + e0) = pk;
    if ((threadIdx.x & 3) == 0) ods[(size_t)row * (K / 32) + e0 / 32] = make_float2(d, d * sf);
}

extern "C" int mxk_quant_q8(const bf16_t* x, int ldx, int8_t* oq, float2* ods, int rows, int K, hipStream_t st) {
    if (rows <= 0) return 0;
    if (K % 32) return (int)hipErrorInvalidValue;
    dim3 grid((K / 8 + 255) / 256, rows);
    MX_ACT_DISPATCH(quant_q8_kernel<F16><<<grid, 256, 0, st>>>(x, ldx, oq, ods, K));
    MXK_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------------------------
// LayerNorm (BERT / Whisper / CLIP): bf16 or fp32 in, bf16 out, fp32 gamma/beta. Optional fused
// residual add (x + r) written back to `xsum` (fp32) when non-null.
template <bool F16>
__global__ __launch_bounds__(256) void layernorm_kernel(const float* __restrict__ x, int ldx,
                                                        const float* __restrict__ r, int ldr,
                                                        float* __restrict__ xsum, const float* __restrict__ g,
                                                        const float* __restrict__ b, bf16_t* __restrict__ ob,
                                                        float* __restrict__ of, int ldo, int H, float eps) {
    __shared__ float red[4];
    const int row = blockIdx.x;
    float s = 0.f, ss = 0.f;
    for (int c = threadIdx.x; c < H; c += 256) {
        float v = x[(size_t)row * ldx + c];
        if (r) v += r[(size_t)row * ldr + c];
        s += v;
        ss += v * v;
    }
    s = block_sum<256>(s, red);
    ss = block_sum<256>(ss, red);
    const float mean = s / H;
    const float var = fmaxf(ss / H - mean * mean, 0.f);
    const float rs = rsqrtf(var + eps);
    for (int c = threadIdx.x; c < H; c += 256) {
        float v = x[(size_t)row * ldx + c];
        if (r) v += r[(size_t)row * ldr + c];
        if (xsum) xsum[(size_t)row * ldx + c] = v;
        float y = (v - mean) * rs * (g ? g[c] : 1.f) + (b ? b[c] : 0.f);
        if (ob) ob[(size_t)row * ldo + c] = f32_to_act<F16>(y);
        if (of) of[(size_t)row * ldo + c] = y;
    }
}

extern "C" int mxk_layernorm(const float* x, int ldx, const float* r, int ldr, float* xsum, const float* g,
                             const float* b, bf16_t* ob, float* of, int ldo, int rows, int H, float eps,
                             hipStream_t st) {
    if (rows <= 0) return 0;
    MX_ACT_DISPATCH(layernorm_kernel<F16><<<rows, 256, 0, st>>>(x, ldx, r, ldr, xsum, g, b, ob, of, ldo, H, eps));
    MXK_CHECK_LAUNCH();
}

// GroupNorm (+ optional SiLU) over NHWC fp32 activations, used by the SD UNet/VAE and Whisper-free
// paths. One workgroup per (sample, group). x: [N, HW, C]; groups split C.
template <bool SILU>
__global__ __launch_bounds__(256) void groupnorm_nhwc_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                             const float* __restrict__ g,
                                                             const float* __restrict__ b, int HW, int C, int G,
                                                             float eps) {
    __shared__ float red[4];
    const int n = blockIdx.x / G, gi = blockIdx.x % G;
    const int cg = C / G;
    const float* xb = x + (size_t)n * HW * C + gi * cg;
    float s = 0.f, ss = 0.f;
    const int total = HW * cg;
    for (int i = threadIdx.x; i < total; i += 256) {
        const int p = i / cg, c = i % cg;
        float v = xb[(size_t)p * C + c];
        s += v;
        ss += v * v;
    }
    s = block_sum<256>(s, red);
    ss = block_sum<256>(ss, red);
    const float mean = s / total, var = fmaxf(ss / total - mean * mean, 0.f), rs = rsqrtf(var + eps);
    float* yb = y + (size_t)n * HW * C + gi * cg;
    for (int i = threadIdx.x; i < total; i += 256) {
        const int p = i / cg, c = i % cg;
        float v = (xb[(size_t)p * C + c] - mean) * rs * g[gi * cg + c] + b[gi * cg + c];
        if (SILU) v = silu_f(v);
        yb[(size_t)p * C + c] = v;
    }
}

extern "C" int mxk_groupnorm_nhwc(const float* x, float* y, const float* g, const float* b, int N, int HW, int C,
                                  int G, float eps, int silu, hipStream_t st) {
    if (C % G) return (int)hipErrorInvalidValue;
    if (silu) groupnorm_nhwc_kernel<true><<<N * G, 256, 0, st>>>(x, y, g, b, HW, C, G, eps);
    else groupnorm_nhwc_kernel<false><<<N * G, 256, 0, st>>>(x, y, g, b, HW, C, G, eps);
    MXK_CHECK_LAUNCH();
}
