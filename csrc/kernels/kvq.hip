// kvq.hip — quantise staged K / V rows into a block-quantised paged KV cache (kvq.h layout).
//
// The RoPE / KV-append writers (rope_kv.hip, the batch-1 qmv1 epilogue) write a quantised cache's new rows as bf16
// into a per-step staging buffer [T, Hkv, D] (identity slots, block size 1); this kernel then quantises each 32-element
// block with llama.cpp's reference quantisers (quantize_row_q8_0/q4_0/q4_1/q5_0/q5_1_ref; iq4_nl as ggml-cuda's
// cpy_blck_f32_iq4_nl: nearest codebook entry at d = vmax / -127, then the weighted least-squares refit of d) and
// stores the row at its paged slot. One thread per (token, head, K|V, block).
#include "kvq.h"

namespace {

MX_DEV int iq4nl_best(float x) {
    const float* v = kvq_iq4nl_values;
    if (x <= v[0]) return 0;
    if (x >= v[15]) return 15;
    int lo = 0, hi = 15;
    while (hi - lo > 1) {
        const int mid = (lo + hi) / 2;
        if (x < v[mid]) hi = mid;
        else lo = mid;
    }
    return x - v[hi - 1] < v[hi] - x ? hi - 1 : hi;
}

MX_DEV uint16_t f32_to_half_bits(float x) { return __builtin_bit_cast(uint16_t, (_Float16)x); }

template <int KVF, int D>
__global__ __launch_bounds__(256) void kvq_append_kernel(const bf16_t* __restrict__ ks, const bf16_t* __restrict__ vs,
                                                         const int* __restrict__ slots, int T, int Hkv, int bs,
                                                         uint8_t* __restrict__ kc, uint8_t* __restrict__ vc) {
    using Q = KVQ<KVF, D>;
    constexpr int NB = D / 32;
    const int id = blockIdx.x * 256 + threadIdx.x;
    const int total = T * Hkv * 2 * NB;
    if (id >= total) return;
    const int b = id % NB;
    const int which = (id / NB) & 1;
    const int th = id / (2 * NB);  // t * Hkv + h
    const int t = th / Hkv, h = th % Hkv;
    const int slot = slots[t];
    if (slot < 0) return;
    const bf16_t* src = (which ? vs : ks) + (size_t)th * D + 32 * b;
    float x[32];
#pragma unroll
    for (int i = 0; i < 32; i += 8) {
        const uint4 w = *(const uint4*)(src + i);
        const uint32_t ww[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            x[i + 2 * j] = bf16_to_f32((bf16_t)(ww[j] & 0xFFFF));
            x[i + 2 * j + 1] = bf16_to_f32((bf16_t)(ww[j] >> 16));
        }
    }
    uint8_t* row = (which ? vc : kc) + ((((size_t)(slot / bs) * Hkv + h) * bs + slot % bs) * Q::ROWB);
    uint8_t* codes = row + (Q::Q8 ? 32 * b : 16 * b);
    uint8_t* hbp = row + Q::CB + 4 * b;
    uint8_t* sc = row + Q::CB + Q::HBB + (Q::MIN ? 4 : 2) * b;
    float amax = 0.f, vmax = 0.f, mn = x[0], mx = x[0];
#pragma unroll
    for (int i = 0; i < 32; ++i) {
        if (fabsf(x[i]) > amax) {
            amax = fabsf(x[i]);
            vmax = x[i];
        }
        mn = fminf(mn, x[i]);
        mx = fmaxf(mx, x[i]);
    }
    int q[32];
    float d = 0.f, m = 0.f;
    if constexpr (KVF == KVF_Q8_0) {
        d = amax / 127.f;
        const float id_ = d ? 1.f / d : 0.f;
#pragma unroll
        for (int i = 0; i < 32; ++i) q[i] = (int)roundf(x[i] * id_);
    } else if constexpr (KVF == KVF_Q4_0 || KVF == KVF_Q5_0) {
        constexpr float NEG = KVF == KVF_Q4_0 ? -8.f : -16.f, OFF = KVF == KVF_Q4_0 ? 8.5f : 16.5f;
        constexpr int QMAX = KVF == KVF_Q4_0 ? 15 : 31;
        d = vmax / NEG;
        const float id_ = d ? 1.f / d : 0.f;
#pragma unroll
        for (int i = 0; i < 32; ++i) q[i] = min(QMAX, (int)(int8_t)(x[i] * id_ + OFF));
    } else if constexpr (KVF == KVF_Q4_1 || KVF == KVF_Q5_1) {
        constexpr int QMAX = KVF == KVF_Q4_1 ? 15 : 31;
        d = (mx - mn) / (float)QMAX;
        m = mn;
        const float id_ = d ? 1.f / d : 0.f;
#pragma unroll
        for (int i = 0; i < 32; ++i) q[i] = min(QMAX, (int)(int8_t)((x[i] - mn) * id_ + 0.5f));
    } else {  // iq4_nl
        d = vmax / kvq_iq4nl_values[0];
        const float id_ = d ? 1.f / d : 0.f;
        float sqx = 0.f, sq2 = 0.f;
#pragma unroll
        for (int i = 0; i < 32; ++i) {
            q[i] = iq4nl_best(x[i] * id_);
            const float v = kvq_iq4nl_values[q[i]], w = x[i] * x[i];
            sqx += w * v * x[i];
            sq2 += w * v * v;
        }
        d = sq2 > 0.f ? sqx / sq2 : d;
    }
    if constexpr (Q::Q8) {
#pragma unroll
        for (int i = 0; i < 32; i += 4)
            *(uint32_t*)(codes + i) = (uint32_t)(q[i] & 0xFF) | ((uint32_t)(q[i + 1] & 0xFF) << 8) |
                                      ((uint32_t)(q[i + 2] & 0xFF) << 16) | ((uint32_t)(q[i + 3] & 0xFF) << 24);
    } else {
#pragma unroll
        for (int i = 0; i < 32; i += 8) {
            uint32_t w = 0;
#pragma unroll
            for (int j = 0; j < 8; ++j) w |= (uint32_t)(q[i + j] & 0xF) << (4 * j);
            *(uint32_t*)(codes + i / 2) = w;
        }
    }
    if constexpr (Q::HB) {
        uint32_t hb = 0;
#pragma unroll
        for (int i = 0; i < 32; ++i) hb |= (uint32_t)((q[i] >> 4) & 1) << i;
        *(uint32_t*)hbp = hb;
    }
    if constexpr (Q::MIN) *(uint32_t*)sc = (uint32_t)f32_to_half_bits(d) | ((uint32_t)f32_to_half_bits(m) << 16);
    else *(uint16_t*)sc = f32_to_half_bits(d);
}

template <int KVF>
int launch_kvq_append(const bf16_t* ks, const bf16_t* vs, const int* slots, int T, int Hkv, int D, int bs, uint8_t* kc,
                      uint8_t* vc, hipStream_t st) {
    const int total = T * Hkv * 2 * (D / 32);
    const dim3 grid((total + 255) / 256);
    if (D == 128) kvq_append_kernel<KVF, 128><<<grid, 256, 0, st>>>(ks, vs, slots, T, Hkv, bs, kc, vc);
    else if (D == 64) kvq_append_kernel<KVF, 64><<<grid, 256, 0, st>>>(ks, vs, slots, T, Hkv, bs, kc, vc);
    else if (D == 256) kvq_append_kernel<KVF, 256><<<grid, 256, 0, st>>>(ks, vs, slots, T, Hkv, bs, kc, vc);
    else return (int)hipErrorInvalidValue;
    MXK_CHECK_LAUNCH();
}

}  // namespace

// staged bf16 rows ks / vs [T, Hkv, D] -> quantised cache rows at slots[t] (negative: skip); kvf 2..7 (kvq.h)
extern "C" int mxk_kvq_append(int kvf, const bf16_t* ks, const bf16_t* vs, const int* slots, int T, int Hkv, int D,
                              int bs, uint8_t* kc, uint8_t* vc, hipStream_t st) {
    if (T <= 0) return 0;
    switch (kvf) {
        case KVF_Q8_0: return launch_kvq_append<KVF_Q8_0>(ks, vs, slots, T, Hkv, D, bs, kc, vc, st);
        case KVF_Q4_0: return launch_kvq_append<KVF_Q4_0>(ks, vs, slots, T, Hkv, D, bs, kc, vc, st);
        case KVF_Q4_1: return launch_kvq_append<KVF_Q4_1>(ks, vs, slots, T, Hkv, D, bs, kc, vc, st);
        case KVF_Q5_0: return launch_kvq_append<KVF_Q5_0>(ks, vs, slots, T, Hkv, D, bs, kc, vc, st);
        case KVF_Q5_1: return launch_kvq_append<KVF_Q5_1>(ks, vs, slots, T, Hkv, D, bs, kc, vc, st);
        case KVF_IQ4_NL: return launch_kvq_append<KVF_IQ4_NL>(ks, vs, slots, T, Hkv, D, bs, kc, vc, st);
    }
    return (int)hipErrorInvalidValue;
}

// a quantised cache's rows -> bf16 [n, D] (tests / the CPU-visible oracle): rows = row indices (block * Hkv + h) * bs
// + off of the cache viewed as [rows, ROWB]
template <int KVF, int D>
__global__ __launch_bounds__(256) void kvq_dequant_rows_kernel(const uint8_t* __restrict__ c, const int* __restrict__ rows,
                                                               int n, bf16_t* __restrict__ out) {
    const int id = blockIdx.x * 256 + threadIdx.x;
    if (id >= n * (D / 8)) return;
    const int r = id / (D / 8), e = (id % (D / 8)) * 8;
    const KVQRaw w = kvq_load<KVF, D>(c, (size_t)rows[r] * D + e);
    *(uint4*)(out + (size_t)r * D + e) = kvq_to_bf16x8<KVF>(w);
}

extern "C" int mxk_kvq_dequant_rows(int kvf, const uint8_t* c, const int* rows, int n, int D, bf16_t* out,
                                    hipStream_t st) {
    if (n <= 0) return 0;
    if (D != 64 && D != 128 && D != 256) return (int)hipErrorInvalidValue;
    const dim3 grid((n * (D / 8) + 255) / 256);
#define KDQ(F_)                                                                                              \
    {                                                                                                        \
        if (D == 128) kvq_dequant_rows_kernel<F_, 128><<<grid, 256, 0, st>>>(c, rows, n, out);               \
        else if (D == 64) kvq_dequant_rows_kernel<F_, 64><<<grid, 256, 0, st>>>(c, rows, n, out);            \
        else kvq_dequant_rows_kernel<F_, 256><<<grid, 256, 0, st>>>(c, rows, n, out);                        \
        MXK_CHECK_LAUNCH();                                                                                  \
    }
    switch (kvf) {
        case KVF_Q8_0: KDQ(KVF_Q8_0)
        case KVF_Q4_0: KDQ(KVF_Q4_0)
        case KVF_Q4_1: KDQ(KVF_Q4_1)
        case KVF_Q5_0: KDQ(KVF_Q5_0)
        case KVF_Q5_1: KDQ(KVF_Q5_1)
        case KVF_IQ4_NL: KDQ(KVF_IQ4_NL)
    }
#undef KDQ
    return (int)hipErrorInvalidValue;
}
