// mx_common.h — shared device helpers for the localai_tfp_amd CDNA4 (gfx950) kernels.
//
// Conventions used by every kernel in this directory:
//   * wave64 only: every lane index is `threadIdx.x & 63`, every reduction is over 64 lanes.
//   * activations in HBM are bf16 (uint16_t bit patterns) or fp32; accumulation is always fp32.
//   * every launcher is `extern "C" int mxk_*(..., hipStream_t)` and returns the hipError_t of the
//     launch so the Python side can raise loudly; launchers never allocate or synchronise, so all of
//     them are safe inside hipGraph stream capture.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint16_t bf16_t;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4v __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

#define MX_DEV __device__ __forceinline__
#define MX_LDS __attribute__((address_space(3)))

// LDS-DMA (global_load_lds) issued from inline asm. hipcc's waitcnt pass counts a compiler-visible LDS-DMA as an
// LGKM event that completes out of order with ds_read, so in any loop that has one it waits lgkmcnt(0) before
// every use of an LDS read — a k-step's fragment reads can then never run ahead of its MFMAs
// (profiles/r6_lgkm_lds_dma.md). Issued from asm the DMA is invisible to that pass: the kernel waits for the DMA
// itself (an explicit `s_waitcnt vmcnt(N)` before the barrier that publishes the slot) and the compiler keeps
// counted lgkmcnt waits for its own ds_reads. M0 = the wave-uniform LDS destination (lane l writes M0 + 16 l).
MX_DEV void mx_lds_dma16(const void* g, const MX_LDS void* lds) {
    const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)lds);
    asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "{m0}"(m0) : "memory");
}
MX_DEV void mx_lds_dma4(const void* g, const MX_LDS void* lds) {
    const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)lds);
    asm volatile("s_nop 0\n\tglobal_load_lds_dword %0, off" ::"v"(g), "{m0}"(m0) : "memory");
}

MX_DEV float bf16_to_f32(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

// round-to-nearest-even; NaN stays NaN (the plain cast lowers to v_cvt_pk_bf16_f32 on gfx950).
MX_DEV bf16_t f32_to_bf16(float f) {
    __bf16 b = (__bf16)f;
    return __builtin_bit_cast(bf16_t, b);
}

MX_DEV uint32_t pack_bf16x2(float lo, float hi) {
    bf16x2v v = {(__bf16)lo, (__bf16)hi};
    return __builtin_bit_cast(uint32_t, v);
}

MX_DEV float half_to_f32(uint16_t h) { return (float)__builtin_bit_cast(_Float16, h); }

// ---- 16-bit activation format -------------------------------------------------------------------
// GEMM operands produced by norms / attention / SwiGLU are either bf16 or f16 ("act16"). f16 lets
// the quantised-weight GEMM dequantise with packed f16 math (2 values per VALU op, see qgemm16.hip)
// and keeps 3 more mantissa bits than bf16 (llama.cpp's GPU GEMMs also run dequantised weights in
// f16). The format is a library-wide mode (mxk_set_act_f16); kernels are templated on it.
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
extern int g_mx_act_f16;  // host-side mode, read by launchers (defined in elementwise.hip)

template <bool F16>
MX_DEV uint16_t f32_to_act(float f) {
    if constexpr (F16) return __builtin_bit_cast(uint16_t, (_Float16)f);
    else return f32_to_bf16(f);
}
template <bool F16>
MX_DEV float act_to_f32(uint16_t v) {
    if constexpr (F16) return half_to_f32(v);
    else return bf16_to_f32(v);
}
template <bool F16>
MX_DEV uint32_t pack_act2(float lo, float hi) {
    if constexpr (F16) {
        f16x2 v = {(_Float16)lo, (_Float16)hi};
        return __builtin_bit_cast(uint32_t, v);
    } else {
        return pack_bf16x2(lo, hi);
    }
}
// unpack 2 activations from one dword
template <bool F16>
MX_DEV void unpack_act2(uint32_t w, float& lo, float& hi) {
    if constexpr (F16) {
        f16x2 v = __builtin_bit_cast(f16x2, w);
        lo = (float)v[0];
        hi = (float)v[1];
    } else {
        lo = __uint_as_float(w << 16);
        hi = __uint_as_float(w & 0xFFFF0000u);
    }
}
// dispatch helper: MX_ACT_DISPATCH(expr) instantiates `expr` with a constexpr bool F16.
#define MX_ACT_DISPATCH(...)                     \
    do {                                         \
        if (g_mx_act_f16) {                      \
            constexpr bool F16 = true;           \
            __VA_ARGS__;                         \
        } else {                                 \
            constexpr bool F16 = false;          \
            __VA_ARGS__;                         \
        }                                        \
    } while (0)

MX_DEV float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
MX_DEV float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}
// sum over groups of `W` consecutive lanes (W power of two <= 64)
template <int W>
MX_DEV float group_sum(float v) {
#pragma unroll
    for (int o = W / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
template <int W>
MX_DEV float group_max(float v) {
#pragma unroll
    for (int o = W / 2; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}
MX_DEV int wave_sum_i(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// block-wide sum for blockDim.x == NT (multiple of 64); `red` must hold NT/64 floats.
template <int NT>
MX_DEV float block_sum(float v, float* red) {
    v = wave_sum(v);
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    if (l == 0) red[w] = v;
    __syncthreads();
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < NT / 64; ++i) t += red[i];
    __syncthreads();
    return t;
}
template <int NT>
MX_DEV float block_max(float v, float* red) {
    v = wave_max(v);
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    if (l == 0) red[w] = v;
    __syncthreads();
    float t = -INFINITY;
#pragma unroll
    for (int i = 0; i < NT / 64; ++i) t = fmaxf(t, red[i]);
    __syncthreads();
    return t;
}

MX_DEV float silu_f(float x) { return x / (1.f + __expf(-x)); }
MX_DEV float gelu_tanh_f(float x) {
    const float k0 = 0.7978845608028654f, k1 = 0.044715f;
    return 0.5f * x * (1.f + tanhf(k0 * (x + k1 * x * x * x)));
}
MX_DEV float gelu_erf_f(float x) { return 0.5f * x * (1.f + erff(x * 0.7071067811865476f)); }
// ---- fp8 (OCP e4m3, gfx950 hardware conversions) paged-KV helpers: K/V are stored unscaled and
// saturated to +-448 (the e4m3 max finite); loads widen 8 fp8 -> 8 fp32 with two cvt_pk per word.
MX_DEV uint8_t f32_to_fp8(float x) {
    x = fminf(fmaxf(x, -448.f), 448.f);
    return (uint8_t)(__builtin_amdgcn_cvt_pk_fp8_f32(x, 0.f, 0, false) & 0xFF);
}
template <bool KV8> struct KVVec { using T = u32x4; };  // 8 elements per lane-load: 16 B bf16
template <> struct KVVec<true> { using T = u32x2; };    //                           8 B fp8
template <bool KV8, typename V>
MX_DEV void kv_unpack8(const V& w, float (&f)[8]) {
    if constexpr (KV8) {
        const f32x2 a = __builtin_amdgcn_cvt_pk_f32_fp8((int)w[0], false), b = __builtin_amdgcn_cvt_pk_f32_fp8((int)w[0], true);
        const f32x2 c = __builtin_amdgcn_cvt_pk_f32_fp8((int)w[1], false), d = __builtin_amdgcn_cvt_pk_f32_fp8((int)w[1], true);
        f[0] = a.x; f[1] = a.y; f[2] = b.x; f[3] = b.y; f[4] = c.x; f[5] = c.y; f[6] = d.x; f[7] = d.y;
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            f[2 * j] = __uint_as_float(w[j] << 16);
            f[2 * j + 1] = __uint_as_float(w[j] & 0xFFFF0000u);
        }
    }
}
// 8 fp8 -> 8 bf16 (exact: e4m3 values are representable in bf16)
MX_DEV uint4 fp8x8_to_bf16x8(uint2 w) {
    float f[8];
    kv_unpack8<true>(u32x2{w.x, w.y}, f);
    uint32_t o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = (__float_as_uint(f[2 * j]) >> 16) | (__float_as_uint(f[2 * j + 1]) & 0xFFFF0000u);
    return make_uint4(o[0], o[1], o[2], o[3]);
}

// gate activation of the fused gated-FFN epilogues: EPI 3 = SwiGLU (silu), EPI 4 = GeGLU (gelu tanh)
template <int EPI>
MX_DEV float glu_gate_f(float g) {
    if constexpr (EPI == 4) return gelu_tanh_f(g);
    else return silu_f(g);
}

#define MXK_CHECK_LAUNCH() return (int)hipGetLastError()

// ---- GGML block formats (byte layouts identical to GGUF on disk) ----
// Q4_K: 256 elements, 144 B: half d, half dmin, u8 scales[12], u8 qs[128]
// Q6_K: repacked at load time to a 16B-aligned 208 B block + a separate fp16 d plane (see quant.py)
// Q8_0: repacked to an int8 plane [N][K] + fp16 d plane [N][K/32]
enum MxQuantType : int {
    MXQ_Q2_K = 10,
    MXQ_Q3_K = 11,
    MXQ_Q4_K = 12,
    MXQ_Q6_K = 14,
    MXQ_Q8_0 = 8,
    MXQ_Q5_K = 13,
    MXQ_Q4_0 = 2,
    // this framework's t32-only layouts of the 32-weight "scale (+ offset)" formats (ops/quant.py to_mxf):
    // w = s * code + m per 32 weights, s / m f16; 4-bit (Q4_0 / Q4_1) or 5-bit (Q5_0 / Q5_1) codes
    MXQ_MX4F = 240,
    MXQ_MX5F = 241,
};

// 4 bits (n & 15) -> bit 0 of each byte of a word (bit i -> byte i)
MX_DEV uint32_t mx_spread4(uint32_t n) { return ((n & 15u) * 0x00204081u) & 0x01010101u; }

// Q4_K 6-bit packed (scale, min) for sub-block j (0..7) out of the 12 scale bytes.
MX_DEV void q4k_scale_min(const uint8_t* q, int j, int& sc, int& m) {
    if (j < 4) {
        sc = q[j] & 63;
        m = q[j + 4] & 63;
    } else {
        sc = (q[j + 4] & 0xF) | ((q[j - 4] >> 6) << 4);
        m = (q[j + 4] >> 4) | ((q[j] >> 6) << 4);
    }
}

// Same decode from the three 32-bit words of the scale array (no byte-addressed loads).
MX_DEV void q4k_scale_min_w(uint32_t w0, uint32_t w1, uint32_t w2, int j, int& sc, int& m) {
    auto byte = [&](int i) -> int {
        uint32_t w = i < 4 ? w0 : (i < 8 ? w1 : w2);
        return (w >> (8 * (i & 3))) & 0xFF;
    };
    if (j < 4) {
        sc = byte(j) & 63;
        m = byte(j + 4) & 63;
    } else {
        sc = (byte(j + 4) & 0xF) | ((byte(j - 4) >> 6) << 4);
        m = (byte(j + 4) >> 4) | ((byte(j) >> 6) << 4);
    }
}

// sign-extend four packed 6-bit unsigned values (0..63, stored one per byte) after subtracting 32.
MX_DEV uint32_t q6_bias_bytes(uint32_t q) {
    uint32_t t = q ^ 0x20202020u;          // flips bit5: (q-32) in 6-bit two's complement
    uint32_t s = t & 0x20202020u;          // sign bits
    return t | (s << 1) | (s << 2);        // extend to bits 6,7
}
