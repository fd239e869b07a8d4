// qmm_fmt.h — the t32 format geometry and B-fragment decoders of qmm.hip (monolithic LDS-DMA ring GEMM):
// the t32 tiled weight layouts, per-wave LDS geometry, the swizzled 16-bit tile addressing, counted-vmcnt
// ring waits and the per-format B-fragment builders (raw block bytes in LDS -> f16x8 MFMA operands).
#pragma once
#include "qdeq16.h"

namespace {

constexpr int QMM_KT = 64;
constexpr int QMM_LDS_BUDGET = 160 * 1024;
constexpr int QMM_MAX_STAGES = 8;

// ---- "t32" tiled weight layout (ops/quant.py: tile32) -------------------------------------------
// Columns are grouped 32 at a time; per (group g, super-block kb) the bytes of the 32 columns are
// stored together, split so that every LDS-DMA wave-instruction of a k-tile reads CONTIGUOUS memory
// (the ggml row-major layout puts each of a wave's 32-64 columns in a different cache line, which
// made the load path, not HBM or the MFMAs, the bottleneck):
//   Q4_K (4608 B / group / kb): [hdr: 32 x 16 B {d, dmin, scales}] [quarter jq: 2 x (32 x 16 B qs)]
//   Q6_K (6784 B / group / kb): [sc: 32 x 16 B] [d: 32 x 4 B] [quarter jq: ql0, ql1, qh (32 x 16 B each)]
//   Q8_0 (2176 B / group / k-tile): [d: 32 x {f16 d0, f16 d1}] [4 x (32 x 16 B qs)]
template <int QT>
struct QmmFmt;
template <>
struct QmmFmt<MXQ_Q4_K> {
    static constexpr int UNIT = 4608, PER_UNIT = 4;       // bytes per group per kb; k-tiles per unit
    static constexpr int QOFF = 512, QSTRIDE = 1024, QB = 1024;
    static constexpr int MOFF = 0, MB = 512, MSTEP = 0;    // header chunks (the same for every k-tile)
    static constexpr int DOFF = 0, DSTRIDE = 0, HAS_D = 0;
};
// MX4F / MX5F (5120 / 6144 B): [hdr: 2 halves x 32 x 16 B {f16 s[4], m[4]}: k-tiles 0-1 read half 0, 2-3 half 1]
// [k-tile jq: 2 x (32 x 16 B) codes (+ MX5F: 32 x 8 B high bits)]
template <>
struct QmmFmt<MXQ_MX4F> {
    static constexpr int UNIT = 5120, PER_UNIT = 4;
    static constexpr int QOFF = 1024, QSTRIDE = 1024, QB = 1024;
    static constexpr int MOFF = 0, MB = 512, MSTEP = 512;  // header half (jq >> 1)
    static constexpr int DOFF = 0, DSTRIDE = 0, HAS_D = 0;
};
template <>
struct QmmFmt<MXQ_MX5F> {
    static constexpr int UNIT = 6144, PER_UNIT = 4;
    static constexpr int QOFF = 1024, QSTRIDE = 1280, QB = 1280;
    static constexpr int MOFF = 0, MB = 512, MSTEP = 512;
    static constexpr int DOFF = 0, DSTRIDE = 0, HAS_D = 0;
};
template <>
struct QmmFmt<MXQ_Q6_K> {
    static constexpr int UNIT = 6784, PER_UNIT = 4;
    static constexpr int QOFF = 640, QSTRIDE = 1536, QB = 1536;
    static constexpr int MOFF = 0, MB = 512, MSTEP = 0;    // int8 scales
    static constexpr int DOFF = 512, DSTRIDE = 0, HAS_D = 1;
};
template <>
struct QmmFmt<MXQ_Q8_0> {
    static constexpr int UNIT = 2176, PER_UNIT = 1;
    static constexpr int QOFF = 128, QSTRIDE = 0, QB = 2048;
    static constexpr int MOFF = 0, MB = 0, MSTEP = 0;
    static constexpr int DOFF = 0, DSTRIDE = 0, HAS_D = 1;
};

template <int QT, int WN>
struct QmmGeom {
    using F = QmmFmt<QT>;
    static constexpr int COLS = 32 * WN;                   // columns per wave (WN groups)
    static constexpr int QCH = F::QB / 16;                 // 16-B chunks per group per k-tile
    static constexpr int QI = (WN * QCH + 63) / 64;        // quant-data wave-instructions
    static constexpr int MI = (WN * F::MB / 16 + 63) / 64; // meta (header / scales) wave-instructions
    static constexpr int DI = F::HAS_D;                    // d-word wave-instructions (WN <= 2)
    static constexpr int NI = QI + MI + DI;
    static constexpr int Q_OFF = 0, M_OFF = QI * 1024, D_OFF = M_OFF + MI * 1024;
    static constexpr int WBYTES = D_OFF + DI * 256;        // per wave per stage
};

// ring depth: as many k-tiles in flight as the LDS holds (memory-level parallelism), capped. OCC = 2 halves
// the budget so two workgroups share a CU (twice the waves to hide dequant / LDS latency, at a shallower ring)
template <int QT, int WM, int WN, int NW, int OCC = 1, int WMW = 1>
struct QmmRing {
    static constexpr int STAGE = 32 * WM * WMW * 128 + NW * QmmGeom<QT, WN>::WBYTES;
    static constexpr int S0 = QMM_LDS_BUDGET / OCC / STAGE;
    static constexpr int STAGES = S0 > QMM_MAX_STAGES ? QMM_MAX_STAGES : S0;
};

MX_DEV int qmm_a_off(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }

template <int N_>
MX_DEV void qmm_wait_barrier() {
    // LDS reads are NOT drained here: every read of the slot about to be refilled has been consumed by
    // its wave before that wave reaches the barrier, and the compiler counts the in-flight ones itself
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N_) : "memory");
}
// wait until at most `ahead` stages (NI LDS-DMA instructions each) are still in flight, then barrier
template <int NI, int A_>
MX_DEV void qmm_wait_ahead(int ahead) {
    if constexpr (A_ <= 0) {
        qmm_wait_barrier<0>();
    } else {
        if (ahead >= A_) qmm_wait_barrier<A_ * NI>();
        else qmm_wait_ahead<NI, A_ - 1>(ahead);
    }
}

// ---- per-format B fragment builders (raw bytes in LDS -> f16x8 for k-step s) ----
// q: this group's quant chunks for the k-tile (32 x 16 B per chunk row), m: its 32 meta chunks,
// d: its 32 d-words; r = column in the group, h = lane half, jq = k-tile within the super-block
template <int QT>
struct QmmB;

template <>
struct QmmB<MXQ_Q4_K> {
    u32x2 v0, v1;
    u32x4 hd;
    f16x2 s2[2], m2[2];
    MX_DEV void load(const char* q, const char* m, const char*, int r, int h, int) {
        hd = *(const u32x4*)(m + r * 16);
        v0 = *(const u32x2*)(q + r * 16 + 8 * h);
        v1 = *(const u32x2*)(q + (32 + r) * 16 + 8 * h);
    }
    MX_DEV void prep(int jq) {
        const float d = half_to_f32(hd[0] & 0xFFFF), dm = half_to_f32(hd[0] >> 16);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            int sc, mn;
            q4k_scale_min_w(hd[1], hd[2], hd[3], 2 * jq + i, sc, mn);
            const _Float16 s = (_Float16)(d * (float)sc), mm = (_Float16)(-dm * (float)mn);
            s2[i] = (f16x2){s, s};
            m2[i] = (f16x2){mm, mm};
        }
    }
    template <int S>
    MX_DEV f16x8 frag() const {
        const u32x2 src = (S & 1) ? v1 : v0;
        constexpr int sh = 4 * (S >> 1);
        const uint32_t t0 = (src[0] >> sh) & 0x0F0F0F0Fu, t1 = (src[1] >> sh) & 0x0F0F0F0Fu;
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

// MX4F / MX5F: the Q4_K fragment with the sub-block (scale, offset) read as f16 pairs from the header half; MX5F
// ORs each code's bit 4 from the k-tile's 64-bit high-bit word (bit u = weight u = 16 S + 8 h + j)
template <bool FIVE>
struct QmmBMX {
    u32x2 v0, v1;
    uint32_t vh0, vh1;  // high-bit words pre-shifted by 8 h
    u32x4 hd;
    f16x2 s2[2], m2[2];
    MX_DEV void load(const char* q, const char* m, const char*, int r, int h, int) {
        hd = *(const u32x4*)(m + r * 16);
        v0 = *(const u32x2*)(q + r * 16 + 8 * h);
        v1 = *(const u32x2*)(q + (32 + r) * 16 + 8 * h);
        if constexpr (FIVE) {
            const u32x2 w = *(const u32x2*)(q + 1024 + r * 8);
            vh0 = w[0] >> (8 * h);
            vh1 = w[1] >> (8 * h);
        }
    }
    MX_DEV void prep(int jq) {
        // entries 2w, 2w+1 of the header half (w = jq & 1). The words go through scalars first: a
        // __builtin_bit_cast of a runtime-indexed ext_vector element reads element 0 (clang, ROCm 7.2)
        const uint32_t sw = (jq & 1) ? hd[1] : hd[0], mw = (jq & 1) ? hd[3] : hd[2];
        const f16x2 s = __builtin_bit_cast(f16x2, sw), mm = __builtin_bit_cast(f16x2, mw);
        s2[0] = (f16x2){s[0], s[0]};
        s2[1] = (f16x2){s[1], s[1]};
        m2[0] = (f16x2){mm[0], mm[0]};
        m2[1] = (f16x2){mm[1], mm[1]};
    }
    template <int S>
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
struct QmmB<MXQ_MX4F> : QmmBMX<false> {};
template <>
struct QmmB<MXQ_MX5F> : QmmBMX<true> {};

template <>
struct QmmB<MXQ_Q6_K> {
    u32x2 v0, v1, vh;
    uint32_t sc, dw;
    f16x2 s2[4];
    MX_DEV void load(const char* q, const char* m, const char* d, int r, int h, int jq) {
        v0 = *(const u32x2*)(q + r * 16 + 8 * h);
        v1 = *(const u32x2*)(q + (32 + r) * 16 + 8 * h);
        vh = *(const u32x2*)(q + (64 + r) * 16 + 8 * h);
        sc = *(const uint32_t*)(m + r * 16 + 4 * jq);
        dw = *(const uint32_t*)(d + r * 4);
    }
    MX_DEV void prep(int) {
        const float df = half_to_f32(dw & 0xFFFF);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const _Float16 s = (_Float16)(df * (float)(int8_t)((sc >> (8 * i)) & 0xFF));
            s2[i] = (f16x2){s, s};
        }
    }
    template <int S>
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

template <>
struct QmmB<MXQ_Q8_0> {
    u32x2 qv[4];
    uint32_t dw;
    f16x2 s2[2];
    MX_DEV void load(const char* q, const char*, const char* d, int r, int h, int) {
#pragma unroll
        for (int s = 0; s < 4; ++s) qv[s] = *(const u32x2*)(q + (s * 32 + r) * 16 + 8 * h);
        dw = *(const uint32_t*)(d + 4 * r);
    }
    MX_DEV void prep(int) {
        const f16x2 dd = __builtin_bit_cast(f16x2, dw);
        s2[0] = (f16x2){dd[0], dd[0]};
        s2[1] = (f16x2){dd[1], dd[1]};
    }
    template <int S>
    MX_DEV f16x8 frag() const {
        const uint32_t t0 = qv[S][0] ^ 0x80808080u, t1 = qv[S][1] ^ 0x80808080u;  // int8 -> u8 + 128
        const f16x2 k = {(_Float16)1152.f, (_Float16)1152.f};
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

}  // namespace
