// qmm2_fmt.h — the t32 quantised-weight formats as seen by the MFMA GEMMs (qmm2.hip, qmm3.hip): per format the
// unit / header / quant byte geometry of one 32-column group x 256-k super-block (Q2F) and the per-lane register
// decoder that turns LDS-staged bytes into 32x32x16 MFMA B fragments (Q2B: load_hdr, load_q, prep<JQ>,
// frag<JQ, S>). Lane mapping: col = lane & 31, h = lane >> 5 (k 8h .. 8h + 7 of a 16-k step).
#pragma once
#include "qdeq16.h"

namespace {

// Q2_ASM_DMA: issue the ring's LDS-DMA from inline asm (mx_common.h mx_lds_dma16), so the compiler's lgkmcnt
// waits for the fragment reads are counted instead of lgkmcnt(0) (the explicit vmcnt waits below cover the DMA)
#ifndef Q2_ASM_DMA
#define Q2_ASM_DMA 1
#endif
MX_DEV void q2_dma(const void* g, MX_LDS void* lds, int sz) {
#if Q2_ASM_DMA
    if (sz == 16) mx_lds_dma16(g, lds);
    else mx_lds_dma4(g, lds);
#else
    if (sz == 16) __builtin_amdgcn_global_load_lds(g, lds, 16, 0, 0);
    else __builtin_amdgcn_global_load_lds(g, lds, 4, 0, 0);
#endif
}

template <int N_>
MX_DEV void q2_wait_barrier() {
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N_) : "memory");
}

template <int QT>
struct Q2F;
// Q4_K t32 unit (per 32-column group, per super-block): [hdr 32 x 16 B][quarter jq: chunk0, chunk1 (32 x 16 B)]
// QB: quant bytes staged per group per k-tile (source unit offset qoff(JQ)); HB: header bytes per group per
// super-block (staged with the super-block's first k-tile); QI / HI: LDS-DMA instructions for each.
template <>
struct Q2F<MXQ_Q4_K> {
    static constexpr int UNIT = 4608, HB = 512, QB = 1024, QI = 1, HI = 1;
    static constexpr int qoff(int jq) { return 512 + jq * 1024; }
};
// Q5_K t32 unit: [hdr 32 x 16 B][qs as Q4_K: quarter jq = chunk0, chunk1][qh: 2 chunks x 32 x 16 B]; the header
// slot holds hdr + qh (the fifth bit of all four k-tiles, staged once per super-block: qoff(4) = 4608)
template <>
struct Q2F<MXQ_Q5_K> {
    static constexpr int UNIT = 5632, HB = 1536, QB = 1024, QI = 1, HI = 2;
    static constexpr int qoff(int jq) { return 512 + jq * 1024; }
    static constexpr int QH = 4608;  // unit offset of the qh chunks
};
// Q6_K t32 unit: [sc 32 x 16 B][d 32 x 4 B][quarter jq: ql0, ql1, qh (32 x 16 B)]
template <>
struct Q2F<MXQ_Q6_K> {
    static constexpr int UNIT = 6784, HB = 640, QB = 1536, QI = 2, HI = 2;
    static constexpr int qoff(int jq) { return 640 + jq * 1536; }
};
// Q3_K t32 unit: [hdr 32 x 16 B {scales[12], d}][hmask: 2 chunks x 32 x 16 B][qs half n: 2 chunks x 32 x 16 B];
// k-tiles 2n, 2n+1 use qs half n (the 2-bit fields 0-1 / 2-3) -> header slot = hdr + hmask (1.5 KB)
template <>
struct Q2F<MXQ_Q3_K> {
    static constexpr int UNIT = 3584, HB = 1536, QB = 1024, QI = 1, HI = 2;
    static constexpr int qoff(int jq) { return 1536 + (jq >> 1) * 1024; }
};
// Q2_K t32 unit: [sc 32 x 16 B][dd 32 x 4 B {d, dmin}][qs half n: 2 chunks x 32 x 16 B]
template <>
struct Q2F<MXQ_Q2_K> {
    static constexpr int UNIT = 2688, HB = 640, QB = 1024, QI = 1, HI = 2;
    static constexpr int qoff(int jq) { return 640 + (jq >> 1) * 1024; }
};

// MX4F / MX5F t32 unit (Q4_0 / Q4_1 / Q5_0 / Q5_1 carried exactly at 4 / 5 bits): [hdr: 2 halves x 32 x 16 B {f16 s[4],
// m[4]}, k-tiles 0-1 read half 0, 2-3 half 1][k-tile jq: 2 x (32 x 16 B codes) (+ MX5F: 32 x 8 B high bits)]
template <>
struct Q2F<MXQ_MX4F> {
    static constexpr int UNIT = 5120, HB = 1024, QB = 1024, QI = 1, HI = 1;
    static constexpr int qoff(int jq) { return 1024 + jq * 1024; }
};
template <>
struct Q2F<MXQ_MX5F> {
    static constexpr int UNIT = 6144, HB = 1024, QB = 1280, QI = 2, HI = 1;
    static constexpr int qoff(int jq) { return 1024 + jq * 1280; }
};
// Q8_0 t32 unit per 64-k tile: [d: 32 x {f16 d0, f16 d1}][4 k-steps x (32 x 16 B int8 codes)] (2176 B); a "super-block"
// here is 4 such tiles, and each tile's scales travel with its codes (no header)
template <>
struct Q2F<MXQ_Q8_0> {
    static constexpr int UNIT = 4 * 2176, HB = 0, QB = 2176, QI = 3, HI = 0;
    static constexpr int qoff(int jq) { return jq * 2176; }
};

template <int QT>
struct Q2B;

template <>
struct Q2B<MXQ_Q4_K> {
    u32x4 hd;
    u32x2 v0, v1;
    f16x2 sm[2];  // per sub-block of the k-tile: (scale, -dmin * min) as exact f16 products
    MX_DEV void load_hdr(const char* hb, int col, int) { hd = *(const u32x4*)(hb + col * 16); }
    MX_DEV void load_q(const char* qb, int col, int h) {
        v0 = *(const u32x2*)(qb + col * 16 + 8 * h);
        v1 = *(const u32x2*)(qb + 512 + col * 16 + 8 * h);
    }
    template <int JQ>
    MX_DEV void prep() {
        const uint32_t w0 = hd[0];  // scalar first: clang bit-casts the whole vector for bit_cast(T, v[i])
        const f16x2 dd = __builtin_bit_cast(f16x2, w0);
        const f16x2 dn = {dd[0], -dd[1]};
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            int sc, mn;
            q4k_scale_min_w(hd[1], hd[2], hd[3], 2 * JQ + i, sc, mn);
            // d * sc is exact in f32 (11 x 6 bits), so the f16 product rounds exactly like the f32 path
            const f16x2 q = {(_Float16)sc, (_Float16)mn};
            sm[i] = dn * q;
        }
    }
    template <int JQ, int S>
    MX_DEV f16x8 frag() const {
        const u32x2 src = (S & 1) ? v1 : v0;
        constexpr int sh = 4 * (S >> 1);
        const uint32_t t0 = (src[0] >> sh) & 0x0F0F0F0Fu, t1 = (src[1] >> sh) & 0x0F0F0F0Fu;
        const f16x2 k = {(_Float16)1024.f, (_Float16)1024.f};
        const f16x2 s2 = {sm[S >> 1][0], sm[S >> 1][0]}, m2 = {sm[S >> 1][1], sm[S >> 1][1]};
        f16x2 p[4];
        magic4(t0, p[0], p[1]);
        magic4(t1, p[2], p[3]);
        f16x8 r;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const f16x2 v = (p[i] - k) * s2 + m2;
            r[2 * i] = v[0];
            r[2 * i + 1] = v[1];
        }
        return r;
    }
};

// Q5_K: Q4_K's nibbles plus the fifth bit: qh byte l (l = 16 (S & 1) + 8 h + i, this lane's k) bit 2 JQ + (S >> 1)
template <>
struct Q2B<MXQ_Q5_K> {
    u32x4 hd;
    u32x2 qh0, qh1;  // qh bytes 8 h .. 8 h + 7 of chunks 0 / 1
    u32x2 v0, v1;
    f16x2 sm[2];
    MX_DEV void load_hdr(const char* hb, int col, int h) {
        hd = *(const u32x4*)(hb + col * 16);
        qh0 = *(const u32x2*)(hb + 512 + col * 16 + 8 * h);
        qh1 = *(const u32x2*)(hb + 1024 + col * 16 + 8 * h);
    }
    MX_DEV void load_q(const char* qb, int col, int h) {
        v0 = *(const u32x2*)(qb + col * 16 + 8 * h);
        v1 = *(const u32x2*)(qb + 512 + col * 16 + 8 * h);
    }
    template <int JQ>
    MX_DEV void prep() {
        const uint32_t w0 = hd[0];
        const f16x2 dd = __builtin_bit_cast(f16x2, w0);
        const f16x2 dn = {dd[0], -dd[1]};
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            int sc, mn;
            q4k_scale_min_w(hd[1], hd[2], hd[3], 2 * JQ + i, sc, mn);
            const f16x2 q = {(_Float16)sc, (_Float16)mn};
            sm[i] = dn * q;  // exact f16 products (11 x 6 bits)
        }
    }
    template <int JQ, int S>
    MX_DEV f16x8 frag() const {
        const u32x2 src = (S & 1) ? v1 : v0;
        const u32x2 qh = (S & 1) ? qh1 : qh0;
        constexpr int sh = 4 * (S >> 1), hb = 2 * JQ + (S >> 1);
        const uint32_t t0 = ((src[0] >> sh) & 0x0F0F0F0Fu) | (((qh[0] >> hb) & 0x01010101u) << 4);
        const uint32_t t1 = ((src[1] >> sh) & 0x0F0F0F0Fu) | (((qh[1] >> hb) & 0x01010101u) << 4);
        const f16x2 k = {(_Float16)1024.f, (_Float16)1024.f};
        const f16x2 s2 = {sm[S >> 1][0], sm[S >> 1][0]}, m2 = {sm[S >> 1][1], sm[S >> 1][1]};
        f16x2 p[4];
        magic4(t0, p[0], p[1]);
        magic4(t1, p[2], p[3]);
        f16x8 r;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const f16x2 v = (p[i] - k) * s2 + m2;
            r[2 * i] = v[0];
            r[2 * i + 1] = v[1];
        }
        return r;
    }
};

template <>
struct Q2B<MXQ_Q6_K> {
    u32x4 sc;   // 16 int8 sub-block scales (one per 16 k)
    uint32_t dw;
    u32x2 v0, v1, vh;
    f16x2 s2[4];
    MX_DEV void load_hdr(const char* hb, int col, int) {
        sc = *(const u32x4*)(hb + col * 16);
        dw = *(const uint32_t*)(hb + 512 + col * 4);
    }
    MX_DEV void load_q(const char* qb, int col, int h) {
        v0 = *(const u32x2*)(qb + col * 16 + 8 * h);
        v1 = *(const u32x2*)(qb + 512 + col * 16 + 8 * h);
        vh = *(const u32x2*)(qb + 1024 + col * 16 + 8 * h);
    }
    template <int JQ>
    MX_DEV void prep() {
        const _Float16 d = __builtin_bit_cast(f16x2, dw)[0];
        const uint32_t w = sc[JQ];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int v = (int)(int8_t)((w >> (8 * i)) & 0xFF);
            const _Float16 s = d * (_Float16)v;  // 11 x 8 bits: exact product, one f16 rounding
            s2[i] = (f16x2){s, s};
        }
    }
    template <int JQ, int S>
    MX_DEV f16x8 frag() const {
        const u32x2 src = (S & 1) ? v1 : v0;
        constexpr int sh = 4 * (S >> 1), qsh = 2 * S;
        const uint32_t t0 = ((src[0] >> sh) & 0x0F0F0F0Fu) | (((vh[0] >> qsh) & 0x03030303u) << 4);
        const uint32_t t1 = ((src[1] >> sh) & 0x0F0F0F0Fu) | (((vh[1] >> qsh) & 0x03030303u) << 4);
        const f16x2 k = {(_Float16)1056.f, (_Float16)1056.f};  // 1024 magic + 32 code offset
        f16x2 p[4];
        magic4(t0, p[0], p[1]);
        magic4(t1, p[2], p[3]);
        f16x8 r;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const f16x2 v = (p[i] - k) * s2[S];
            r[2 * i] = v[0];
            r[2 * i + 1] = v[1];
        }
        return r;
    }
};

// Q3_K: code c = 2-bit field | hmask bit << 2 in [0, 7], weight = d * (sc - 32) * (c - 4). k-tile JQ: qs half
// n = JQ >> 1, 2-bit fields j = 2 (JQ & 1) + (S >> 1); k-step S uses sub-block scale 4 JQ + S.
template <>
struct Q2B<MXQ_Q3_K> {
    u32x4 hd;           // scales[12] (3 words) + d
    u32x2 hm0, hm1;     // hmask bytes 8 h .. 8 h + 7 of chunks 0 / 1 (this lane's k)
    u32x2 v0, v1;
    f16x2 s2[4];
    MX_DEV void load_hdr(const char* hb, int col, int h) {
        hd = *(const u32x4*)(hb + col * 16);
        hm0 = *(const u32x2*)(hb + 512 + col * 16 + 8 * h);
        hm1 = *(const u32x2*)(hb + 1024 + col * 16 + 8 * h);
    }
    MX_DEV void load_q(const char* qb, int col, int h) {
        v0 = *(const u32x2*)(qb + col * 16 + 8 * h);
        v1 = *(const u32x2*)(qb + 512 + col * 16 + 8 * h);
    }
    template <int JQ>
    MX_DEV void prep() {
        // 16 6-bit scales from 12 bytes (ggml kmask unpack): word JQ of the unpacked array = scales 4 JQ .. 4 JQ + 3
        constexpr uint32_t km1 = 0x03030303u, km2 = 0x0F0F0F0Fu;
        uint32_t w;
        if constexpr (JQ == 0) w = (hd[0] & km2) | ((hd[2] & km1) << 4);
        else if constexpr (JQ == 1) w = (hd[1] & km2) | (((hd[2] >> 2) & km1) << 4);
        else if constexpr (JQ == 2) w = ((hd[0] >> 4) & km2) | (((hd[2] >> 4) & km1) << 4);
        else w = ((hd[1] >> 4) & km2) | (((hd[2] >> 6) & km1) << 4);
        const uint32_t w3 = hd[3];  // scalar first (see Q4_K prep)
        const _Float16 d = __builtin_bit_cast(f16x2, w3)[0];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int v = (int)((w >> (8 * i)) & 0xFF) - 32;
            const _Float16 sv = d * (_Float16)v;  // 11 x 6 bits: exact product, one f16 rounding
            s2[i] = (f16x2){sv, sv};
        }
    }
    template <int JQ, int S>
    MX_DEV f16x8 frag() const {
        const u32x2 src = (S & 1) ? v1 : v0;
        const u32x2 hm = (S & 1) ? hm1 : hm0;
        constexpr int j = 2 * (JQ & 1) + (S >> 1), hb = 4 * (JQ >> 1) + j;
        const uint32_t t0 = ((src[0] >> (2 * j)) & 0x03030303u) | (((hm[0] >> hb) & 0x01010101u) << 2);
        const uint32_t t1 = ((src[1] >> (2 * j)) & 0x03030303u) | (((hm[1] >> hb) & 0x01010101u) << 2);
        const f16x2 k = {(_Float16)1028.f, (_Float16)1028.f};  // 1024 magic + 4 code offset
        f16x2 p[4];
        magic4(t0, p[0], p[1]);
        magic4(t1, p[2], p[3]);
        f16x8 r;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const f16x2 v = (p[i] - k) * s2[S];
            r[2 * i] = v[0];
            r[2 * i + 1] = v[1];
        }
        return r;
    }
};

// Q2_K: weight = d * (sc & 15) * q - dmin * (sc >> 4), q the 2-bit field j = 2 (JQ & 1) + (S >> 1) of qs half
// JQ >> 1; k-step S uses sub-block byte 4 JQ + S.
template <>
struct Q2B<MXQ_Q2_K> {
    u32x4 sc;
    uint32_t dw;
    u32x2 v0, v1;
    f16x2 sm[4];
    MX_DEV void load_hdr(const char* hb, int col, int) {
        sc = *(const u32x4*)(hb + col * 16);
        dw = *(const uint32_t*)(hb + 512 + col * 4);
    }
    MX_DEV void load_q(const char* qb, int col, int h) {
        v0 = *(const u32x2*)(qb + col * 16 + 8 * h);
        v1 = *(const u32x2*)(qb + 512 + col * 16 + 8 * h);
    }
    template <int JQ>
    MX_DEV void prep() {
        const f16x2 dd = __builtin_bit_cast(f16x2, dw);
        const f16x2 dn = {dd[0], -dd[1]};
        const uint32_t w = sc[JQ];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t b = (w >> (8 * i)) & 0xFF;
            const f16x2 q = {(_Float16)(int)(b & 15), (_Float16)(int)(b >> 4)};
            sm[i] = dn * q;  // exact f16 products (11 x 4 bits)
        }
    }
    template <int JQ, int S>
    MX_DEV f16x8 frag() const {
        const u32x2 src = (S & 1) ? v1 : v0;
        constexpr int j = 2 * (JQ & 1) + (S >> 1);
        const uint32_t t0 = (src[0] >> (2 * j)) & 0x03030303u, t1 = (src[1] >> (2 * j)) & 0x03030303u;
        const f16x2 k = {(_Float16)1024.f, (_Float16)1024.f};
        const f16x2 s2 = {sm[S][0], sm[S][0]}, m2 = {sm[S][1], sm[S][1]};
        f16x2 p[4];
        magic4(t0, p[0], p[1]);
        magic4(t1, p[2], p[3]);
        f16x8 r;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const f16x2 v = (p[i] - k) * s2 + m2;
            r[2 * i] = v[0];
            r[2 * i + 1] = v[1];
        }
        return r;
    }
};

// MX4F / MX5F: weight = s * code + m per 32 (f16 s, m); code = nibble (| bit 4 from the k-tile's high-bit word)
template <bool FIVE>
struct Q2BMX {
    u32x4 h0, h1;        // header halves (k-tiles 0-1 / 2-3): {s[4], m[4]} of the half's 4 blocks of 32
    u32x2 v0, v1;
    uint32_t vh0, vh1;   // high-bit words of this lane's k, pre-shifted by 8 h
    f16x2 s2[2], m2[2];
    MX_DEV void load_hdr(const char* hb, int col, int) {
        h0 = *(const u32x4*)(hb + col * 16);
        h1 = *(const u32x4*)(hb + 512 + col * 16);
    }
    MX_DEV void load_q(const char* qb, int col, int h) {
        v0 = *(const u32x2*)(qb + col * 16 + 8 * h);
        v1 = *(const u32x2*)(qb + 512 + col * 16 + 8 * h);
        if constexpr (FIVE) {
            const u32x2 w = *(const u32x2*)(qb + 1024 + col * 8);
            vh0 = w[0] >> (8 * h);
            vh1 = w[1] >> (8 * h);
        }
    }
    template <int JQ>
    MX_DEV void prep() {
        // blocks 2 (JQ & 1), + 1 of the half: word JQ & 1 of the scale pairs, word 2 + (JQ & 1) of the offsets
        const u32x4 hh = (JQ >> 1) ? h1 : h0;
        const uint32_t sw = hh[JQ & 1], mw = hh[2 + (JQ & 1)];
        const f16x2 sv = __builtin_bit_cast(f16x2, sw), mv = __builtin_bit_cast(f16x2, mw);
        s2[0] = (f16x2){sv[0], sv[0]};
        s2[1] = (f16x2){sv[1], sv[1]};
        m2[0] = (f16x2){mv[0], mv[0]};
        m2[1] = (f16x2){mv[1], mv[1]};
    }
    template <int JQ, int S>
    MX_DEV f16x8 frag() const {
        const u32x2 src = (S & 1) ? v1 : v0;
        constexpr int sh = 4 * (S >> 1);
        uint32_t t0 = (src[0] >> sh) & 0x0F0F0F0Fu, t1 = (src[1] >> sh) & 0x0F0F0F0Fu;
        if constexpr (FIVE) {
            const uint32_t hw = ((S >> 1) ? vh1 : vh0) >> (16 * (S & 1));
            t0 |= mx_spread4(hw) << 4;
            t1 |= mx_spread4(hw >> 4) << 4;
        }
        const f16x2 k = {(_Float16)1024.f, (_Float16)1024.f};
        f16x2 p[4];
        magic4(t0, p[0], p[1]);
        magic4(t1, p[2], p[3]);
        f16x8 r;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const f16x2 v = (p[i] - k) * s2[S >> 1] + m2[S >> 1];
            r[2 * i] = v[0];
            r[2 * i + 1] = v[1];
        }
        return r;
    }
};
template <>
struct Q2B<MXQ_MX4F> : Q2BMX<false> {};
template <>
struct Q2B<MXQ_MX5F> : Q2BMX<true> {};

// Q8_0: weight = d * int8 code per 32; k-step S of a tile reads codes chunk S, block S >> 1's scale
template <>
struct Q2B<MXQ_Q8_0> {
    u32x2 qv[4];
    uint32_t dw;
    f16x2 s2[2];
    MX_DEV void load_hdr(const char*, int, int) {}
    MX_DEV void load_q(const char* qb, int col, int h) {
        dw = *(const uint32_t*)(qb + col * 4);
#pragma unroll
        for (int s = 0; s < 4; ++s) qv[s] = *(const u32x2*)(qb + 128 + (s * 32 + col) * 16 + 8 * h);
    }
    template <int JQ>
    MX_DEV void prep() {
        const f16x2 dd = __builtin_bit_cast(f16x2, dw);
        s2[0] = (f16x2){dd[0], dd[0]};
        s2[1] = (f16x2){dd[1], dd[1]};
    }
    template <int JQ, int S>
    MX_DEV f16x8 frag() const {
        const uint32_t t0 = qv[S][0] ^ 0x80808080u, t1 = qv[S][1] ^ 0x80808080u;  // int8 -> u8 + 128
        const f16x2 k = {(_Float16)1152.f, (_Float16)1152.f};                     // 1024 magic + 128
        f16x2 p[4];
        magic4(t0, p[0], p[1]);
        magic4(t1, p[2], p[3]);
        f16x8 r;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const f16x2 v = (p[i] - k) * s2[S >> 1];
            r[2 * i] = v[0];
            r[2 * i + 1] = v[1];
        }
        return r;
    }
};

// LDS-DMA of one 32-column group's weight bytes for k-tile JQ of a super-block (unit `u`): the tile's quant bytes
// (F::QB: whole 1 KB pieces plus one partial piece, F::QI instructions) into `qd` and, with the super-block's first
// tile, its header (F::HB bytes in the format's layout, F::HI instructions) into `hd`.
template <int QT, int JQ>
MX_DEV void q2_stage_weights(const uint8_t* u, char* qd, char* hd, int lane) {
    using F = Q2F<QT>;
    const uint8_t* qs = u + F::qoff(JQ);
    constexpr int NF = F::QB / 1024, REM = F::QB % 1024;
    static_assert(NF + (REM ? 1 : 0) == F::QI && REM % 16 == 0, "quant piece count");
#pragma unroll
    for (int i = 0; i < NF; ++i)
        q2_dma((const void*)(qs + i * 1024 + lane * 16), (MX_LDS void*)(qd + i * 1024), 16);
    if constexpr (REM > 0) {
        if (lane < REM / 16)
            q2_dma((const void*)(qs + NF * 1024 + lane * 16), (MX_LDS void*)(qd + NF * 1024), 16);
    }
    if constexpr (JQ == 0) {
        if constexpr (QT == MXQ_Q3_K) {  // hdr (512 B) + hmask (1 KB): one full and one half instruction
            q2_dma((const void*)(u + lane * 16), (MX_LDS void*)(hd), 16);
            if (lane < 32)
                q2_dma((const void*)(u + 1024 + lane * 16), (MX_LDS void*)(hd + 1024), 16);
        } else if constexpr (QT == MXQ_MX4F || QT == MXQ_MX5F) {  // both header halves (1 KB)
            q2_dma((const void*)(u + lane * 16), (MX_LDS void*)(hd), 16);
        } else if constexpr (F::HB > 0) {
            if (lane < 32) q2_dma((const void*)(u + lane * 16), (MX_LDS void*)(hd), 16);
            if constexpr (QT == MXQ_Q6_K || QT == MXQ_Q2_K) {  // + the 32 x 4 B d (/ dmin) words
                if (lane < 32)
                    q2_dma((const void*)(u + 512 + lane * 4), (MX_LDS void*)(hd + 512), 4);
            }
            if constexpr (QT == MXQ_Q5_K)  // + the qh chunks (fifth bits of the whole super-block)
                q2_dma((const void*)(u + F::QH + lane * 16), (MX_LDS void*)(hd + 512), 16);
        }
    }
}

}  // namespace
