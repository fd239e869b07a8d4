// qmm8.hip — int8-MFMA GEMM of Q8_K activations with Q4_K / Q6_K weights (t32 tiled layout):
//
//   C[M, N] (+)= A[M, K] · W[N, K]^T
//
// Numerics are llama.cpp's CPU K-quant dot products (ggml vec_dot_q4_K_q8_K / vec_dot_q6_K_q8_K):
// activations are Q8_K blocks (256 int8 codes, one fp32 scale da, int sums of every 16 codes — norm.hip
// q8k_block), weight codes enter the matrix cores as int8, and per 256-k super-block
//   Q4_K:  y += da * (d * Σ_s sc_s · Σ_k qa·q  −  dmin * Σ_s mn_s · Σ_k qa)
//   Q6_K:  y += da * d * (Σ_s sc_s · Σ_k qa·q  −  32 Σ_s sc_s · Σ_k qa)      (q stored unsigned 0..63)
// where every inner Σ_k runs on a `v_mfma_i32_32x32x32_i8` (Q4_K: one 32-element sub-block per
// instruction) or `v_mfma_i32_32x32x16_i8` (Q6_K: 16-element sub-blocks), the integer sub-block scales
// are applied with one `v_mad_i32_i24` per accumulator element, and the min / offset term — an exact
// integer dot of the 16 bsums of a row with the 16 per-column (min | 32·scale) values of a column — is
// ONE f16 MFMA per 32x32 tile per super-block (every operand an integer below 2^11: exact).
//
// Why int8 on the matrix cores: in the serving regime (M = 128..512) a 16-bit GEMM over 4-bit weights is
// bound by the bytes each CU pulls from L2 (≈12 B/clk/CU for LDS-DMA): the activation tile, re-read by
// every column tile, is 3/4 of them. Q8_K activations halve those bytes, halve the LDS traffic of the A
// fragments, and run on the 2x-rate int8 MFMA; the weights are never dequantised to 16 bits.
//
// Structure (mirrors qmm.hip): NW column groups x WMW row waves per workgroup, wave tile 32*WM x 32*WN;
// every operand reaches LDS through `global_load_lds` into an NS-deep ring of 64-k stages advanced with a
// counted `s_waitcnt vmcnt` + raw `s_barrier`; per super-block the weight headers (scales / mins / d)
// ride in the first stage and the activation meta (bsums, da) in the last one (their extra loads are not
// counted: waiting for fewer outstanding loads than exist is always safe). XCD-aware bijective block
// remap; split-K over whole super-blocks (fp32 atomics) for accumulating outputs.
#include "qdeq16.h"

typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
typedef int32_t i32x16 __attribute__((ext_vector_type(16)));

namespace {

constexpr int Q8_KT = 64;
constexpr int Q8_LDS_BUDGET = 160 * 1024;
constexpr int Q8_MAX_STAGES = 8;

// t32 super-block unit per 32-column group: header (per-column scales) + 4 quarters of codes
template <int QT>
struct Q8W;
template <>
struct Q8W<MXQ_Q4_K> {
    static constexpr int UNIT = 4608, HB = 512, QOFF = 512, QB = 1024;  // hdr: 32 x {f16 d, f16 dmin, 12 B scales}
};
template <>
struct Q8W<MXQ_Q5_K> {  // Q4_K + qh (2 chunks x 32 cols x 16 B after the codes: bit 2jq+s of byte b = 5th bit)
    static constexpr int UNIT = 5632, HB = 512, QOFF = 512, QB = 1024;
};
template <>
struct Q8W<MXQ_Q6_K> {
    static constexpr int UNIT = 6784, HB = 640, QOFF = 640, QB = 1536;  // hdr: 32 x 16 int8 scales, 32 x 4 B f16 d
};

template <int QT, int WM, int WN, int NW, int WMW>
struct Q8Geom {
    using F = Q8W<QT>;
    static constexpr int NT = NW * WMW;
    static constexpr int BM = 32 * WM * WMW, NG = NW * WN;
    static constexpr int A_B = BM * 64;                    // codes
    static constexpr int BS_OFF = A_B, DA_OFF = A_B + BM * 32;
    static constexpr int DA_B = (BM < 64 ? 64 : BM) * 4;   // one 4-B LDS-DMA instruction covers 64 rows
    static constexpr int W_OFF = A_B + BM * 32 + DA_B;     // NG x codes, NG x 512 B headers, NG x 128 B d words
    static constexpr int WH_OFF = W_OFF + NG * F::QB;
    static constexpr int WD_OFF = WH_OFF + NG * 512;
    static constexpr int QH_OFF = WD_OFF + (F::HB > 512 ? NG * 128 : 0);  // Q5_K high bits: NG x 1 KB
    static constexpr int STAGE = (QH_OFF + (QT == MXQ_Q5_K ? NG * 1024 : 0) + 15) & ~15;
    static constexpr int AI = BM / 16;                      // A-code wave-instructions per stage
    static constexpr int WA = (AI + NT - 1) / NT;           // per wave (the last ones may issue one less)
    static constexpr int WA0 = AI / NT;
    static constexpr int QCH = F::QB / 16;                  // 16-B code chunks per group
    static constexpr int QI = (WN * QCH + 63) / 64;         // code wave-instructions of a loading wave
    static constexpr int NI = WA + QI;                      // counted per-stage instructions (loading wave)
    static constexpr int NS0 = Q8_LDS_BUDGET / STAGE;
};

template <int N_>
MX_DEV void q8_wait_barrier() {
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N_) : "memory");
}
template <int NI, int A_>
MX_DEV void q8_wait_ahead(int ahead) {
    if constexpr (A_ <= 0) {
        q8_wait_barrier<0>();
    } else {
        if (ahead >= A_) q8_wait_barrier<A_ * NI>();
        else q8_wait_ahead<NI, A_ - 1>(ahead);
    }
}

MX_DEV int q8_chunk(int row, int c) { return c ^ ((row >> 2) & 3); }  // 64-B rows: 4 rows share a bank row

// per-column super-block header, decoded into registers at the first quarter of each super-block
template <int QT>
struct Q8Hdr;
template <>
struct Q8Hdr<MXQ_Q4_K> {
    uint32_t sc0, sc1;  // 8 six-bit sub-block scales, one per byte
    float d, dmin;
    f16x8 mb;            // min-term B fragment: k' = 8h + j -> mn[(8h + j) >> 1]
    MX_DEV void load(const char* hb, const char*, int col, int h) {
        const u32x4 w = *(const u32x4*)(hb + col * 16);
        d = half_to_f32(w[0] & 0xFFFF);
        dmin = half_to_f32(w[0] >> 16);
        int s[8], m[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) q4k_scale_min_w(w[1], w[2], w[3], j, s[j], m[j]);
        sc0 = (uint32_t)s[0] | ((uint32_t)s[1] << 8) | ((uint32_t)s[2] << 16) | ((uint32_t)s[3] << 24);
        sc1 = (uint32_t)s[4] | ((uint32_t)s[5] << 8) | ((uint32_t)s[6] << 16) | ((uint32_t)s[7] << 24);
#pragma unroll
        for (int j = 0; j < 8; ++j) mb[j] = (_Float16)(float)(h ? m[4 + (j >> 1)] : m[j >> 1]);
    }
    MX_DEV int sc(int sb) const {  // sub-block scale (0..7)
        return (int)(((sb < 4 ? sc0 : sc1) >> (8 * (sb & 3))) & 0xFF);
    }
};
template <>
struct Q8Hdr<MXQ_Q5_K> : Q8Hdr<MXQ_Q4_K> {
    u32x4 qh;  // this lane's 16 high-bit bytes (chunk h of its column)
};
template <>
struct Q8Hdr<MXQ_Q6_K> {
    u32x4 sc;  // 16 int8 sub-block scales
    float d;
    f16x8 mb;  // offset-term B fragment: k' = 8h + j -> 32 * sc[8h + j]
    MX_DEV void load(const char* hb, const char* db, int col, int h) {
        sc = *(const u32x4*)(hb + col * 16);
        d = half_to_f32(*(const uint16_t*)(db + col * 4));
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int k = 8 * h + j;
            mb[j] = (_Float16)(32.f * (float)(int8_t)((sc[k >> 2] >> (8 * (k & 3))) & 0xFF));
        }
    }
    MX_DEV int sc16(int sb) const {  // 16-element sub-block scale (0..15), signed
        return (int)(int8_t)((sc[sb >> 2] >> (8 * (sb & 3))) & 0xFF);
    }
};

}  // namespace

template <int QT, int WM, int WN, int NW, int WMW, int OCC, int EPI>
__global__ __launch_bounds__(64 * NW * WMW) __attribute__((amdgpu_waves_per_eu(OCC * NW * WMW / 4, OCC * NW * WMW / 4))) void
qmm8_kernel(const int8_t* __restrict__ A, int lda, const float* __restrict__ AD, const _Float16* __restrict__ AS,
            const uint8_t* __restrict__ W, int M, int N, int K, int n_mt, int splits, int sb_per_split,
            void* __restrict__ Cv, int ldc) {
    using G = Q8Geom<QT, WM, WN, NW, WMW>;
    using F = Q8W<QT>;
    constexpr int BM = G::BM, NT = G::NT, STAGE = G::STAGE;
    constexpr int NS = (G::NS0 / OCC) > Q8_MAX_STAGES ? Q8_MAX_STAGES : (G::NS0 / OCC);
    static_assert(NS >= 3, "ring depth");
    static_assert(G::WA >= 1, "A tile split");
    static_assert((NS - 2) * (G::NI + 4) <= 63, "vmcnt range");
    static_assert(WN <= 2, "header instruction covers two groups");
    extern __shared__ __attribute__((aligned(16))) char smem[];

    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int h = lane >> 5, col = lane & 31;
    const int cg = wave % NW, mw = wave / NW;

    const int nwg = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    const int mt = lid % n_mt;
    const int rest = lid / n_mt;
    const int split = rest % splits;
    const int ct = rest / splits;

    const int m_base = mt * BM;
    const int g_wave = ct * G::NG + cg * WN;  // first 32-column group of this wave
    const int nsb = K / 256;
    const int sb0 = split * sb_per_split;
    const int sb1 = min(sb0 + sb_per_split, nsb);
    if (sb0 >= sb1) return;
    const int kt0 = sb0 * 4, kt1 = sb1 * 4;
    const int ngrp = N >> 5;
    const size_t gstride = (size_t)nsb * F::UNIT;

    // ---- per-lane LDS-DMA sources ----
    uint32_t aoff[G::WA];
    const bool a_extra = G::WA != G::WA0 && wave < G::AI % NT;  // issues WA (else WA0) A instructions
#pragma unroll
    for (int i = 0; i < G::WA; ++i) {
        const int j = wave + i * NT;
        const int r = j * 16 + (lane >> 2);
        const int c = q8_chunk(r, lane & 3);
        aoff[i] = (uint32_t)(min(m_base + r, M - 1) * lda + c * 16);
    }
    const uint8_t* qsrc[G::QI];
    bool qact[G::QI];
#pragma unroll
    for (int ci = 0; ci < G::QI; ++ci) {
        const int q = ci * 64 + lane;
        const int t = q / G::QCH, jc = q % G::QCH;
        qact[ci] = q < WN * G::QCH;
        const int g = min(g_wave + (qact[ci] ? t : 0), ngrp - 1);
        qsrc[ci] = W + (size_t)g * gstride + F::QOFF + jc * 16;
    }
    const int hg = min(g_wave + (lane >> 5), ngrp - 1);
    const uint8_t* hsrc = W + (size_t)hg * gstride + (lane & 31) * 16;
    const uint8_t* dsrc = W + (size_t)hg * gstride + 512 + (lane & 31) * 4;  // Q6_K d words
    const bool hact = lane < 32 * WN;
    const int nk16 = K / 16;

    // stage issue: A codes (all waves), weight codes (+ headers at quarter 0) by the mw == 0 wave of each
    // column group, activation meta at quarter 3 (bsums: 32 rows per instruction; da: 64 rows)
    auto issue = [&](int kt, int slot, auto jq_c) {
        constexpr int jq = decltype(jq_c)::value;  // == kt & 3
        char* sb = smem + slot * STAGE;
        const int8_t* ak = A + (size_t)kt * Q8_KT;
#pragma unroll
        for (int i = 0; i < G::WA; ++i)
            if (i < G::WA0 || a_extra)
                __builtin_amdgcn_global_load_lds((const void*)(ak + aoff[i]),
                                                 (MX_LDS void*)(sb + (wave + i * NT) * 1024), 16, 0, 0);
        if (mw == 0) {
            const size_t unit = (size_t)(kt >> 2) * F::UNIT;
#pragma unroll
            for (int ci = 0; ci < G::QI; ++ci)
                if (qact[ci])
                    __builtin_amdgcn_global_load_lds((const void*)(qsrc[ci] + unit + jq * F::QB),
                                                     (MX_LDS void*)(sb + G::W_OFF + cg * WN * F::QB + ci * 1024), 16, 0, 0);
            if (jq == 0 && hact) {
                __builtin_amdgcn_global_load_lds((const void*)(hsrc + unit),
                                                 (MX_LDS void*)(sb + G::WH_OFF + cg * WN * 512), 16, 0, 0);
                if constexpr (QT == MXQ_Q6_K)
                    __builtin_amdgcn_global_load_lds((const void*)(dsrc + unit),
                                                     (MX_LDS void*)(sb + G::WD_OFF + cg * WN * 128), 4, 0, 0);
            }
            if constexpr (QT == MXQ_Q5_K) {
                if (jq == 0) {
#pragma unroll
                    for (int t = 0; t < WN; ++t) {
                        const int g = min(g_wave + t, ngrp - 1);
                        __builtin_amdgcn_global_load_lds((const void*)(W + (size_t)g * gstride + unit + 4608 + lane * 16),
                                                         (MX_LDS void*)(sb + G::QH_OFF + (cg * WN + t) * 1024), 16, 0, 0);
                    }
                }
            }
        }
        if constexpr (jq == 3) {
            const int sbk = kt >> 2;
            for (int j = wave; j < BM / 32; j += NT) {  // bsums: row = 32 j + lane / 2, 16 B half lane % 2
                const int r = min(m_base + j * 32 + (lane >> 1), M - 1);
                __builtin_amdgcn_global_load_lds((const void*)(AS + (size_t)r * nk16 + sbk * 16 + (lane & 1) * 8),
                                                 (MX_LDS void*)(sb + G::BS_OFF + j * 1024), 16, 0, 0);
            }
            for (int j = wave; j < (BM + 63) / 64; j += NT) {
                const int r = min(m_base + j * 64 + lane, M - 1);
                __builtin_amdgcn_global_load_lds((const void*)(AD + (size_t)r * nsb + sbk),
                                                 (MX_LDS void*)(sb + G::DA_OFF + j * 256), 4, 0, 0);
            }
        }
    };

    f32x16 acc[WM][WN];
    i32x16 J[WM][WN];
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
        for (int t = 0; t < WN; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                acc[i][t][r] = 0.f;
                J[i][t][r] = 0;
            }
    const i32x16 zero16 = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    const f32x16 zf16 = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    Q8Hdr<QT> hd[WN];
    const int row_w = mw * WM * 32;  // first row of this wave inside the tile

    auto body = [&](const char* sb, auto jq_c) {
        constexpr int JQ = decltype(jq_c)::value;
        const char* wq = sb + G::W_OFF + cg * WN * F::QB;
        if constexpr (JQ == 0) {
#pragma unroll
            for (int t = 0; t < WN; ++t) {
                hd[t].load(sb + G::WH_OFF + (cg * WN + t) * 512, sb + G::WD_OFF + (cg * WN + t) * 128, col, h);
                if constexpr (QT == MXQ_Q5_K) hd[t].qh = *(const u32x4*)(sb + G::QH_OFF + (cg * WN + t) * 1024 + (h * 32 + col) * 16);
            }
        }
        if constexpr (QT == MXQ_Q4_K || QT == MXQ_Q5_K) {
            i32x4 bf[WN][2];
#pragma unroll
            for (int t = 0; t < WN; ++t) {
                const u32x4 raw = *(const u32x4*)(wq + t * F::QB + (h * 32 + col) * 16);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    uint32_t lo = raw[e] & 0x0F0F0F0Fu, hi = (raw[e] >> 4) & 0x0F0F0F0Fu;
                    if constexpr (QT == MXQ_Q5_K) {
                        lo |= ((hd[t].qh[e] >> (2 * JQ)) & 0x01010101u) << 4;
                        hi |= ((hd[t].qh[e] >> (2 * JQ + 1)) & 0x01010101u) << 4;
                    }
                    bf[t][0][e] = (int32_t)lo;
                    bf[t][1][e] = (int32_t)hi;
                }
            }
            i32x4 af[2][WM];
#pragma unroll
            for (int s = 0; s < 2; ++s)
#pragma unroll
                for (int i = 0; i < WM; ++i) {
                    const int r = row_w + i * 32 + col;
                    af[s][i] = *(const i32x4*)(sb + r * 64 + q8_chunk(r, 2 * s + h) * 16);
                }
            // software pipeline: the sub-block scale of MFMA n is applied while MFMA n+1 runs, so only two
            // integer result tiles are ever live (the scheduler otherwise issues every MFMA first and spills)
            constexpr int NIT = 2 * WM * WN;
            i32x16 Ip;
            int scp = 0, ip = 0, tp = 0;
#pragma unroll
            for (int it = 0; it < NIT; ++it) {
                const int s = it / (WM * WN), i = (it / WN) % WM, t = it % WN;
                const i32x16 I = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[s][i], bf[t][s], zero16, 0, 0, 0);
                if (it > 0) {
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        J[ip][tp][r] += __mul24(Ip[r], scp);
                        asm volatile("" : "+v"(J[ip][tp][r]));  // one mad per element: no cross-item add3
                    }
                }
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, 16, 0);
                Ip = I;
                scp = hd[t].sc(2 * JQ + s);
                ip = i;
                tp = t;
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) J[ip][tp][r] += __mul24(Ip[r], scp);
        } else {
            u32x2 bf[WN][4];
#pragma unroll
            for (int t = 0; t < WN; ++t) {
                const char* q = wq + t * F::QB;
                const u32x2 l0 = *(const u32x2*)(q + col * 16 + 8 * h);
                const u32x2 l1 = *(const u32x2*)(q + 512 + col * 16 + 8 * h);
                const u32x2 hh = *(const u32x2*)(q + 1024 + col * 16 + 8 * h);
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                    bf[t][0][e] = (l0[e] & 0x0F0F0F0Fu) | ((hh[e] & 0x03030303u) << 4);
                    bf[t][1][e] = (l1[e] & 0x0F0F0F0Fu) | (((hh[e] >> 2) & 0x03030303u) << 4);
                    bf[t][2][e] = ((l0[e] >> 4) & 0x0F0F0F0Fu) | (((hh[e] >> 4) & 0x03030303u) << 4);
                    bf[t][3][e] = ((l1[e] >> 4) & 0x0F0F0F0Fu) | (((hh[e] >> 6) & 0x03030303u) << 4);
                }
            }
            long af[4][WM];
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int i = 0; i < WM; ++i) {
                    const int r = row_w + i * 32 + col;
                    af[u][i] = *(const long*)(sb + r * 64 + q8_chunk(r, u) * 16 + 8 * h);
                }
            constexpr int NIT = 4 * WM * WN;
            i32x16 Ip;
            int scp = 0, ip = 0, tp = 0;
#pragma unroll
            for (int it = 0; it < NIT; ++it) {
                const int u = it / (WM * WN), i = (it / WN) % WM, t = it % WN;
                const i32x16 I = __builtin_amdgcn_mfma_i32_32x32x16_i8(af[u][i], __builtin_bit_cast(long, bf[t][u]),
                                                                       zero16, 0, 0, 0);
                if (it > 0) {
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        J[ip][tp][r] += __mul24(Ip[r], scp);
                        asm volatile("" : "+v"(J[ip][tp][r]));  // one mad per element: no cross-item add3
                    }
                }
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, 16, 0);
                Ip = I;
                scp = hd[t].sc16(4 * JQ + u);
                ip = i;
                tp = t;
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) J[ip][tp][r] += __mul24(Ip[r], scp);
        }
        if constexpr (JQ == 3) {
            // super-block epilogue: exact integer min / offset term on the matrix cores, then scale
#pragma unroll
            for (int i = 0; i < WM; ++i) {
                const int r0 = row_w + i * 32;
                const f16x8 ab = *(const f16x8*)(sb + G::BS_OFF + (r0 + col) * 32 + 16 * h);
                f32x4 dav[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) dav[q] = *(const f32x4*)(sb + G::DA_OFF + (r0 + 8 * q + 4 * h) * 4);
#pragma unroll
                for (int t = 0; t < WN; ++t) {
                    const f32x16 Mi = __builtin_amdgcn_mfma_f32_32x32x16_f16(ab, hd[t].mb, zf16, 0, 0, 0);
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const float da = dav[r >> 2][r & 3];
                        if constexpr (QT == MXQ_Q4_K || QT == MXQ_Q5_K) {
                            const float v = fmaf((float)J[i][t][r], hd[t].d, -hd[t].dmin * Mi[r]);
                            acc[i][t][r] = fmaf(v, da, acc[i][t][r]);
                        } else {
                            acc[i][t][r] = fmaf(((float)J[i][t][r] - Mi[r]) * hd[t].d, da, acc[i][t][r]);
                        }
                        J[i][t][r] = 0;
                    }
                }
            }
        }
    };

    // ---- ring: NS-1 stages in flight; tile kt waited for at the top of its own iteration ----
    // counted per-stage instructions of this wave: WA0 (+1) A pieces, + QI weight pieces on mw == 0
    using C0 = std::integral_constant<int, 0>;
    using C1 = std::integral_constant<int, 1>;
    using C2 = std::integral_constant<int, 2>;
    using C3 = std::integral_constant<int, 3>;
    auto issue_any = [&](int kt, int slot) {
        switch (kt & 3) {
            case 0: issue(kt, slot, C0{}); break;
            case 1: issue(kt, slot, C1{}); break;
            case 2: issue(kt, slot, C2{}); break;
            default: issue(kt, slot, C3{}); break;
        }
    };
    for (int s = 0; s < NS - 1; ++s)
        if (kt0 + s < kt1) issue_any(kt0 + s, s);
    int slot = 0;
    auto step = [&](int kt, auto jq_c) {
        constexpr int JQ = decltype(jq_c)::value;
        const int k = kt + JQ;
        const int ahead = min(kt1 - 1, k + NS - 2) - k;
        if (mw == 0) {
            if (a_extra) q8_wait_ahead<G::WA0 + 1 + G::QI, NS - 2>(ahead);
            else q8_wait_ahead<G::WA0 + G::QI, NS - 2>(ahead);
        } else {
            if (a_extra) q8_wait_ahead<G::WA0 + 1, NS - 2>(ahead);
            else q8_wait_ahead<G::WA0, NS - 2>(ahead);
        }
        if (k + NS - 1 < kt1) {
            int ns = slot + NS - 1;
            if (ns >= NS) ns -= NS;
            issue(k + NS - 1, ns, std::integral_constant<int, (JQ + NS - 1) & 3>{});
        }
        body(smem + slot * STAGE, jq_c);
        if (++slot == NS) slot = 0;
    };
    for (int kt = kt0; kt < kt1; kt += 4) {
        step(kt, C0{});
        step(kt, C1{});
        step(kt, C2{});
        step(kt, C3{});
    }

    // ---- epilogue: 32x32 C/D layout: col = lane & 31, row = 8*(r>>2) + 4*(lane>>5) + (r&3) ----
    const int m_wave = m_base + row_w;
#pragma unroll
    for (int t = 0; t < WN; ++t) {
        const int nt = (g_wave + t) * 32;
        const int n = nt + col;
        if constexpr (EPI == E16_SWIGLU || EPI == E16_GEGLU) {
#pragma unroll
            for (int i = 0; i < WM; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const float v = acc[i][t][r];
                    const float up = __shfl_xor(v, 16);
                    const int m = m_wave + i * 32 + 8 * (r >> 2) + 4 * h + (r & 3);
                    if (col < 16 && n < N && m < M)
                        ((uint16_t*)Cv)[(size_t)m * ldc + (nt >> 1) + col] = f32_to_act<true>(glu_gate_f<EPI>(v) * up);
                }
            continue;
        }
        if (n >= N) continue;
#pragma unroll
        for (int i = 0; i < WM; ++i) {
            const int m0 = m_wave + i * 32 + 4 * h;
            float* cf = ((float*)Cv) + (size_t)m0 * ldc + n;
            uint16_t* ch = ((uint16_t*)Cv) + (size_t)m0 * ldc + n;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int dr = 8 * (r >> 2) + (r & 3);
                if (m0 + dr >= M) continue;
                const float v = acc[i][t][r];
                if constexpr (EPI == E16_F32) cf[(size_t)dr * ldc] = v;
                else if constexpr (EPI == E16_ACT) ch[(size_t)dr * ldc] = f32_to_act<true>(v);
                else if (splits == 1) cf[(size_t)dr * ldc] += v;
                else atomicAdd(cf + (size_t)dr * ldc, v);
            }
        }
    }
}

template <int QT, int WM, int WN, int NW, int WMW, int OCC, int EPI>
static int launch_qmm8(const int8_t* A, int lda, const float* AD, const _Float16* AS, const uint8_t* W, int M, int N,
                       int K, int splits, void* C, int ldc, hipStream_t st) {
    using G = Q8Geom<QT, WM, WN, NW, WMW>;
    constexpr int NS = (G::NS0 / OCC) > Q8_MAX_STAGES ? Q8_MAX_STAGES : (G::NS0 / OCC);
    constexpr int BN = 32 * G::NG;
    const int nsb = K / 256;
    splits = max(1, min(splits, nsb));
    const int sps = (nsb + splits - 1) / splits;
    splits = (nsb + sps - 1) / sps;
    const int n_ct = (N + BN - 1) / BN, n_mt = (M + G::BM - 1) / G::BM;
    const long nwg = (long)n_ct * splits * n_mt;
    if (nwg <= 0 || nwg > 0x7fffffff) return (int)hipErrorInvalidValue;
    constexpr size_t lds = (size_t)NS * G::STAGE;
    static_assert(lds * OCC <= 160 * 1024, "LDS");
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)qmm8_kernel<QT, WM, WN, NW, WMW, OCC, EPI>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        attr_set = true;
    }
    qmm8_kernel<QT, WM, WN, NW, WMW, OCC, EPI><<<dim3((unsigned)nwg), 64 * NW * WMW, lds, st>>>(
        A, lda, AD, AS, W, M, N, K, n_mt, splits, sps, C, ldc);
    MXK_CHECK_LAUNCH();
}

template <int QT, int EPI>
static int dispatch_qmm8(int wm, int wn, int nw, int wmw, int occ, const int8_t* A, int lda, const float* AD,
                         const _Float16* AS, const uint8_t* W, int M, int N, int K, int splits, void* C, int ldc,
                         hipStream_t st) {
#define Q8_CASE(WM_, WN_, NW_, WMW_, OCC_)                                                                  \
    if (wm == WM_ && wn == WN_ && nw == NW_ && wmw == WMW_ && occ == OCC_)                                  \
        return launch_qmm8<QT, WM_, WN_, NW_, WMW_, OCC_, EPI>(A, lda, AD, AS, W, M, N, K, splits, C, ldc, st);
    // two 32x32 tiles per wave (the integer scale pipeline needs ~170 VGPRs: two waves per SIMD)
    Q8_CASE(2, 1, 4, 1, 1) Q8_CASE(2, 1, 4, 2, 1) Q8_CASE(2, 1, 4, 1, 2) Q8_CASE(1, 2, 4, 2, 1)
    Q8_CASE(2, 1, 8, 1, 1) Q8_CASE(1, 2, 2, 2, 1) Q8_CASE(1, 2, 4, 1, 2)
#undef Q8_CASE
    return (int)hipErrorInvalidValue;
}

// A: Q8_K activations (int8 [M][lda], lda % 16 == 0, 16-B aligned), AD fp32 [M][K/256], AS f16 [M][K/16];
// W: t32 Q4_K / Q6_K (N % 32 == 0, K % 256 == 0). epi as qmm.hip (0 fp32, 1 act16 (f16), 2 fp32 accumulate —
// split-K via atomics when splits > 1 —, 3/4 SwiGLU/GeGLU over 16-row interleaved gate|up -> f16 [M, N/2]).
// Tile: 32*wm*wmw rows x 32*wn*nw columns, nw*wmw waves; occ 2 = half-LDS ring (two workgroups per CU).
extern "C" int mxk_qmm8(int qtype, int epi, int wm, int wn, int nw, int wmw, int occ, const int8_t* A, int lda,
                        const float* AD, const _Float16* AS, const uint8_t* W, int M, int N, int K, int splits, void* C,
                        int ldc, hipStream_t st) {
    if (M <= 0) return 0;
    if (K % 256 || (lda & 15) || ((uintptr_t)A & 15) || ((uintptr_t)W & 15) || ((uintptr_t)AS & 15) || (N & 31))
        return (int)hipErrorInvalidValue;
    if (epi != E16_ADD_F32 && splits != 1) return (int)hipErrorInvalidValue;
#define Q8_EPI(QT_)                                                                                              \
    switch (epi) {                                                                                               \
        case E16_F32: return dispatch_qmm8<QT_, E16_F32>(wm, wn, nw, wmw, occ, A, lda, AD, AS, W, M, N, K, splits, C, ldc, st); \
        case E16_ACT: return dispatch_qmm8<QT_, E16_ACT>(wm, wn, nw, wmw, occ, A, lda, AD, AS, W, M, N, K, splits, C, ldc, st); \
        case E16_ADD_F32: return dispatch_qmm8<QT_, E16_ADD_F32>(wm, wn, nw, wmw, occ, A, lda, AD, AS, W, M, N, K, splits, C, ldc, st); \
        case E16_SWIGLU: return dispatch_qmm8<QT_, E16_SWIGLU>(wm, wn, nw, wmw, occ, A, lda, AD, AS, W, M, N, K, splits, C, ldc, st); \
        case E16_GEGLU: return dispatch_qmm8<QT_, E16_GEGLU>(wm, wn, nw, wmw, occ, A, lda, AD, AS, W, M, N, K, splits, C, ldc, st); \
    }
    switch (qtype) {
        case MXQ_Q4_K: Q8_EPI(MXQ_Q4_K) break;
        case MXQ_Q5_K: Q8_EPI(MXQ_Q5_K) break;
        case MXQ_Q6_K: Q8_EPI(MXQ_Q6_K) break;
    }
#undef Q8_EPI
    return (int)hipErrorInvalidValue;
}
