// qdeq16.h — packed-f16 dequantisation of GGML weight blocks into MFMA B fragments, shared by
// qgemm16.hip (16x16x32 tiles) and qgemm32.hip (32x32x16 tiles). See qgemm16.hip for the scheme.
#pragma once
#include "mx_common.h"

enum { E16_F32 = 0, E16_ACT = 1, E16_ADD_F32 = 2, E16_SWIGLU = 3, E16_GEGLU = 4 };

static constexpr uint32_t MAGIC = 0x64646464u;
static constexpr uint32_t SEL_LO = 0x04010400u;  // bytes (t0, 0x64, t1, 0x64)
static constexpr uint32_t SEL_HI = 0x04030402u;  // bytes (t2, 0x64, t3, 0x64)

// 4 codes (one per byte of t, each < 1024) -> two f16x2 holding (1024 + code)
MX_DEV void magic4(uint32_t t, f16x2& p0, f16x2& p1) {
    p0 = __builtin_bit_cast(f16x2, __builtin_amdgcn_perm(MAGIC, t, SEL_LO));
    p1 = __builtin_bit_cast(f16x2, __builtin_amdgcn_perm(MAGIC, t, SEL_HI));
}

template <int QT>
struct W16;

// ---- Q4_K: 144 B block {f16 d, f16 dmin, 12 B scales, 128 B nibbles} ----
template <>
struct W16<MXQ_Q4_K> {
    u32x4 h, a, b;
    f16x2 s2[2], m2[2];
    MX_DEV void load(const uint8_t* W, const uint16_t*, int n, int kb, int nblk, int g) {
        const uint8_t* blk = W + ((size_t)n * nblk + kb) * 144;
        h = __builtin_nontemporal_load((const u32x4*)blk);
        a = __builtin_nontemporal_load((const u32x4*)(blk + 16 + 32 * g));
        b = __builtin_nontemporal_load((const u32x4*)(blk + 32 + 32 * g));
    }
    MX_DEV void zero() { h = a = b = (u32x4){0, 0, 0, 0}; }
    MX_DEV void prep(int g) {
        const float d = half_to_f32(h[0] & 0xFFFF), dm = half_to_f32(h[0] >> 16);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            int sc, mn;
            q4k_scale_min_w(h[1], h[2], h[3], 2 * g + i, sc, mn);
            const _Float16 s = (_Float16)(d * (float)sc), m = (_Float16)(-dm * (float)mn);
            s2[i] = (f16x2){s, s};
            m2[i] = (f16x2){m, m};
        }
    }
    MX_DEV uint32_t q(int i) const { return i < 4 ? a[i] : b[i - 4]; }
    template <int KS>
    MX_DEV f16x8 frag() const {
        constexpr int hi = KS >> 2;
        const uint32_t t0 = (q(2 * (KS & 3)) >> (4 * hi)) & 0x0F0F0F0Fu;
        const uint32_t t1 = (q(2 * (KS & 3) + 1) >> (4 * hi)) & 0x0F0F0F0Fu;
        const f16x2 k1024 = {(_Float16)1024.f, (_Float16)1024.f};
        f16x2 p[4];
        magic4(t0, p[0], p[1]);
        magic4(t1, p[2], p[3]);
        f16x8 r;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const f16x2 v = (p[i] - k1024) * s2[hi] + m2[hi];
            r[2 * i] = v[0];
            r[2 * i + 1] = v[1];
        }
        return r;
    }
};

// ---- Q6_K (repacked 208 B: 128 B low nibbles, 64 B high bits, 16 B int8 scales; d plane) ----
template <>
struct W16<MXQ_Q6_K> {
    u32x4 l0, l1, hh;
    uint32_t sc;
    uint16_t d;
    f16x2 s2[4];
    MX_DEV void load(const uint8_t* W, const uint16_t* D, int n, int kb, int nblk, int g) {
        const uint8_t* blk = W + ((size_t)n * nblk + kb) * 208;
        l0 = __builtin_nontemporal_load((const u32x4*)(blk + 32 * g));
        l1 = __builtin_nontemporal_load((const u32x4*)(blk + 16 + 32 * g));
        hh = __builtin_nontemporal_load((const u32x4*)(blk + 128 + 16 * g));
        sc = *(const uint32_t*)(blk + 192 + 4 * g);
        d = D[(size_t)n * nblk + kb];
    }
    MX_DEV void zero() {
        l0 = l1 = hh = (u32x4){0, 0, 0, 0};
        sc = 0;
        d = 0;
    }
    MX_DEV void prep(int) {
        const float df = half_to_f32(d);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const _Float16 s = (_Float16)(df * (float)(int8_t)((sc >> (8 * i)) & 0xFF));
            s2[i] = (f16x2){s, s};
        }
    }
    MX_DEV uint32_t ql(int i) const { return i < 4 ? l0[i] : l1[i - 4]; }
    template <int KS>
    MX_DEV f16x8 frag() const {
        constexpr int hi = KS >> 2, qsh = 2 * (KS >> 1);
        uint32_t t0 = (ql(2 * (KS & 3)) >> (4 * hi)) & 0x0F0F0F0Fu;
        uint32_t t1 = (ql(2 * (KS & 3) + 1) >> (4 * hi)) & 0x0F0F0F0Fu;
        t0 |= ((hh[2 * (KS & 1)] >> qsh) & 0x03030303u) << 4;
        t1 |= ((hh[2 * (KS & 1) + 1] >> qsh) & 0x03030303u) << 4;
        const f16x2 k = {(_Float16)1056.f, (_Float16)1056.f};  // 1024 magic + 32 code offset
        f16x2 p[4];
        magic4(t0, p[0], p[1]);
        magic4(t1, p[2], p[3]);
        f16x8 r;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const f16x2 v = (p[i] - k) * s2[KS >> 1];
            r[2 * i] = v[0];
            r[2 * i + 1] = v[1];
        }
        return r;
    }
};

// ---- Q8_0 (repacked: int8 plane [N][K] + f16 d plane [N][K/32]) ----
template <>
struct W16<MXQ_Q8_0> {
    u32x4 w[4];
    uint32_t dd;
    f16x2 s2[2];
    MX_DEV void load(const uint8_t* W, const uint16_t* D, int n, int kb, int nblk, int g) {
        const uint8_t* p = W + (size_t)n * nblk * 256 + (size_t)kb * 256 + 64 * g;
#pragma unroll
        for (int i = 0; i < 4; ++i) w[i] = __builtin_nontemporal_load((const u32x4*)(p + 16 * i));
        dd = *(const uint32_t*)(D + (size_t)n * nblk * 8 + kb * 8 + 2 * g);
    }
    MX_DEV void zero() {
#pragma unroll
        for (int i = 0; i < 4; ++i) w[i] = (u32x4){0, 0, 0, 0};
        dd = 0;
    }
    MX_DEV void prep(int) {
        const f16x2 v = __builtin_bit_cast(f16x2, dd);
        s2[0] = (f16x2){v[0], v[0]};
        s2[1] = (f16x2){v[1], v[1]};
    }
    MX_DEV uint32_t word(int i) const { return w[i >> 2][i & 3]; }
    template <int KS>
    MX_DEV f16x8 frag() const {
        const uint32_t t0 = word(2 * KS) ^ 0x80808080u, t1 = word(2 * KS + 1) ^ 0x80808080u;  // int8 -> u8 + 128
        const f16x2 k = {(_Float16)1152.f, (_Float16)1152.f};
        f16x2 p[4];
        magic4(t0, p[0], p[1]);
        magic4(t1, p[2], p[3]);
        f16x8 r;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const f16x2 v = (p[i] - k) * s2[KS >> 2];
            r[2 * i] = v[0];
            r[2 * i + 1] = v[1];
        }
        return r;
    }
};

