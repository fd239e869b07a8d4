// kvq.h — block-quantised paged KV cache rows (llama.cpp `cache_type_k / cache_type_v`: q8_0, q4_0, q4_1, q5_0,
// q5_1, iq4_nl; grpc-server.cpp:2338-2341) as the attention kernels read them.
//
// One cache row = one (token, KV head) vector of D elements, stored as its D / 32 blocks with llama.cpp's per-block
// numerics and byte counts (q8_0 34, q4_0 18, q4_1 20, q5_0 22, q5_1 24, iq4_nl 18 bytes per 32 elements), laid out
// for 8-element lane loads: [codes][5-bit high bits][block scales]
//   codes  q8_0: int8 per element; 4-bit formats: element 2j in the low nibble of byte j, 2j + 1 in the high one
//   hb     q5_*: bit e of byte e / 8 = the fifth bit of element e
//   scales f16 d per block (q8_0, q4_0, q5_0, iq4_nl) or f16 {d, m} pairs (q4_1, q5_1)
// Element values: q8_0 d q; q4_0 d (q - 8); q4_1 d q + m; q5_0 d (q - 16); q5_1 d q + m; iq4_nl d kvalues[q].
#pragma once
#include "mx_common.h"

enum { KVF_BF16 = 0, KVF_FP8 = 1, KVF_Q8_0 = 2, KVF_Q4_0 = 3, KVF_Q4_1 = 4, KVF_Q5_0 = 5, KVF_Q5_1 = 6, KVF_IQ4_NL = 7 };

__device__ __constant__ static const float kvq_iq4nl_values[16] = {-127.f, -104.f, -83.f, -65.f, -49.f, -35.f, -22.f,
                                                                   -10.f,  1.f,    13.f,  25.f,  38.f,  53.f,  69.f,
                                                                   89.f,   113.f};

template <int KVF, int D>
struct KVQ {
    static constexpr bool Q8 = KVF == KVF_Q8_0;
    static constexpr bool HB = KVF == KVF_Q5_0 || KVF == KVF_Q5_1;
    static constexpr bool MIN = KVF == KVF_Q4_1 || KVF == KVF_Q5_1;
    static constexpr int CB = Q8 ? D : D / 2;        // code bytes
    static constexpr int HBB = HB ? D / 8 : 0;       // high-bit bytes
    static constexpr int SB = (D / 32) * (MIN ? 4 : 2);
    static constexpr int ROWB = CB + HBB + SB;       // bytes per cache row
};

// the raw bytes of 8 consecutive elements of a row (what a lane keeps in flight)
struct KVQRaw {
    uint2 c;      // codes: 8 bytes (q8_0) or 4 bytes in c.x (4-/5-bit)
    uint32_t s;   // f16 d (| f16 m << 16)
    uint32_t hb;  // high-bit byte (q5_*)
};

// 8 elements starting at element offset eo (= row * D + e, e % 8 == 0) of a cache laid out as rows of ROWB bytes
template <int KVF, int D>
MX_DEV KVQRaw kvq_load(const void* base, size_t eo) {
    using Q = KVQ<KVF, D>;
    const size_t row = eo / D;
    const int e = (int)(eo % D);
    const uint8_t* r = (const uint8_t*)base + row * Q::ROWB;
    KVQRaw o;
    if constexpr (Q::Q8) o.c = *(const uint2*)(r + e);
    else o.c = make_uint2(*(const uint32_t*)(r + e / 2), 0u);
    if constexpr (Q::HB) o.hb = r[Q::CB + e / 8];
    else o.hb = 0;
    if constexpr (Q::MIN) o.s = *(const uint32_t*)(r + Q::CB + Q::HBB + (e / 32) * 4);
    else o.s = *(const uint16_t*)(r + Q::CB + Q::HBB + (e / 32) * 2);
    return o;
}

template <int KVF>
MX_DEV void kvq_dequant(const KVQRaw& w, float (&f)[8]) {
    const float d = half_to_f32((uint16_t)(w.s & 0xFFFF));
    const float m = half_to_f32((uint16_t)(w.s >> 16));
    if constexpr (KVF == KVF_Q8_0) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint32_t word = i < 4 ? w.c.x : w.c.y;
            f[i] = d * (float)(int8_t)((word >> (8 * (i & 3))) & 0xFF);
        }
    } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            int q = (int)((w.c.x >> (4 * i)) & 0xF);
            if constexpr (KVF == KVF_Q5_0 || KVF == KVF_Q5_1) q |= (int)((w.hb >> i) & 1u) << 4;
            if constexpr (KVF == KVF_Q4_0) f[i] = d * (float)(q - 8);
            else if constexpr (KVF == KVF_Q5_0) f[i] = d * (float)(q - 16);
            else if constexpr (KVF == KVF_IQ4_NL) f[i] = d * kvq_iq4nl_values[q];
            else f[i] = fmaf(d, (float)q, m);  // q4_1 / q5_1
        }
    }
}

template <int KVF>
MX_DEV uint4 kvq_to_bf16x8(const KVQRaw& w) {
    float f[8];
    kvq_dequant<KVF>(w, f);
    return make_uint4(pack_bf16x2(f[0], f[1]), pack_bf16x2(f[2], f[3]), pack_bf16x2(f[4], f[5]), pack_bf16x2(f[6], f[7]));
}
