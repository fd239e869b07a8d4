// qmm3_impl.h — kernel templates of qmm3.hip (see there), shared by the per-format translation units.
#pragma once
#include "qmm2_fmt.h"

namespace {

constexpr int Q3_NR = 3;  // A / raw-quant ring slots (64-k tiles)

template <int QT, int WM>
struct Q3Geom {
    using F = Q2F<QT>;
    static constexpr int WN = 2;                      // column groups per consumer wave
    static constexpr int BM = 64 * WM;                // 2 consumer rows of 32 WM
    static constexpr int A_BYTES = BM * 128;          // one 64-k tile of A, f16
    static constexpr int QSZ = 4 * F::QB;             // raw quant bytes of the 4 groups, one tile
    static constexpr int B16 = 16 * 1024;             // f16 B tile: [k-step 4][group 4][lane 64][16 B]
    static constexpr int HSZ = 4 * F::HB;             // one super-block header slot (4 groups)
    static constexpr int OFF_Q = Q3_NR * A_BYTES;
    static constexpr int OFF_B = OFF_Q + Q3_NR * QSZ;
    static constexpr int OFF_H = OFF_B + 2 * B16;
    static constexpr int LDS = OFF_H + 2 * HSZ;
    static constexpr int WA = BM / 32;                // A LDS-DMA instructions per producer per tile
    template <int JQ, int DBG = 0>
    static constexpr int cnt() {
        return ((DBG & 4) ? 0 : WA) + ((DBG & 8) ? 0 : F::QI + (JQ == 0 ? F::HI : 0));
    }
};

// DBG (isolation builds, tools/prof_qmm.py --q3dbg): 1 consumers skip the MFMAs, 2 producers skip the dequant,
// 4 producers skip the A DMA, 8 producers skip the weight DMA, 16 consumers skip the fragment reads (MFMAs on
// register-resident operands)
template <int QT, int WM, int EPI, int DBG = 0>
__global__ __launch_bounds__(512) void qmm3_kernel(const uint16_t* __restrict__ A, int lda, const uint8_t* __restrict__ W,
                                                   int M, int N, int K, int n_mt, int splits, int sbps,
                                                   void* __restrict__ Cv, int ldc) {
    using G = Q3Geom<QT, WM>;
    using F = Q2F<QT>;
    constexpr int BM = G::BM, WA = G::WA, WN = G::WN, A_BYTES = G::A_BYTES;
    static_assert(G::LDS <= 160 * 1024, "LDS");
    static_assert(G::template cnt<0>() <= 63, "vmcnt range");
    extern __shared__ __attribute__((aligned(16))) char smem[];

    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int h = lane >> 5, col = lane & 31;

    // XCD-aware bijective remap (as qmm2): the row tiles and splits of one column panel share an XCD's L2
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    const int mt = lid % n_mt;
    const int rest = lid / n_mt;
    const int split = rest % splits;
    const int ct = rest / splits;
    const int nsb = K >> 8;
    const int sb0 = split * sbps, sb1 = min(sb0 + sbps, nsb);
    if (sb0 >= sb1) return;  // whole workgroup: no barrier is left waiting
    const int m_base = mt * BM;
    const int T = 4 * (sb1 - sb0);  // 64-k tiles of this split

    if (wave < 4) {
        // ================= producer: LDS-DMA of every operand + dequant of group p =================
        const int p = wave;
        const int g = min(ct * 4 + p, (N >> 5) - 1);  // groups past N decode the last (never stored)
        const uint8_t* wg = W + (size_t)g * ((size_t)nsb * F::UNIT);
        uint32_t aoff[WA];
#pragma unroll
        for (int i = 0; i < WA; ++i) {  // 8-row block j = p WA + i: lane -> (k-step, row, half ^ parity)
            const int j = p * WA + i;
            const int s = lane >> 4, rr = (lane >> 1) & 7, hh = (lane & 1) ^ (j & 1);
            const int row = min(m_base + 8 * j + rr, M - 1);
            aoff[i] = (uint32_t)(row * lda + 16 * s + 8 * hh);
        }
        // DMA of tile t (ring slot t % 3; header slot = super-block parity)
        auto issue = [&](int t, int slot, auto jq_c) {
            constexpr int JQ = decltype(jq_c)::value;
            const int sb = sb0 + (t >> 2);
            char* as = smem + slot * A_BYTES;
            const uint16_t* ak = A + (size_t)(sb * 4 + JQ) * 64;
            if constexpr (!(DBG & 4)) {
#pragma unroll
                for (int i = 0; i < WA; ++i)
                    q2_dma((const void*)(ak + aoff[i]), (MX_LDS void*)(as + (p * WA + i) * 1024), 16);
            }
            if constexpr (DBG & 8) return;
            const uint8_t* u = wg + (size_t)sb * F::UNIT;
            q2_stage_weights<QT, JQ>(u, smem + G::OFF_Q + slot * G::QSZ + p * F::QB,
                                     smem + G::OFF_H + ((t >> 2) & 1) * G::HSZ + p * F::HB, lane);
        };
        // dequant of tile t (its bytes landed) into f16 B buffer t & 1
        Q2B<QT> bq;
        auto dequant = [&](int t, int slot, auto jq_c) {
            constexpr int JQ = decltype(jq_c)::value;
            if constexpr (DBG & 2) return;
            if constexpr (JQ == 0) bq.load_hdr(smem + G::OFF_H + ((t >> 2) & 1) * G::HSZ + p * F::HB, col, h);
            bq.load_q(smem + G::OFF_Q + slot * G::QSZ + p * F::QB, col, h);
            bq.template prep<JQ>();
            char* bd = smem + G::OFF_B + (t & 1) * G::B16 + p * 1024 + lane * 16;
            *(f16x8*)(bd + 0 * 4096) = bq.template frag<JQ, 0>();
            *(f16x8*)(bd + 1 * 4096) = bq.template frag<JQ, 1>();
            *(f16x8*)(bd + 2 * 4096) = bq.template frag<JQ, 2>();
            *(f16x8*)(bd + 3 * 4096) = bq.template frag<JQ, 3>();
        };
        using I0 = std::integral_constant<int, 0>;
        using I1 = std::integral_constant<int, 1>;
        using I2 = std::integral_constant<int, 2>;
        using I3 = std::integral_constant<int, 3>;
        issue(0, 0, I0{});
        issue(1, 1, I1{});
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G::template cnt<1, DBG>()) : "memory");
        dequant(0, 0, I0{});
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // B(-1): tile 0 published
        int s0 = 0;  // ring slot of tile t
        // period t (JQ = t & 3): DMA t + 2, dequant t + 1, barrier
        auto period = [&](int t, auto jq_c) {
            constexpr int JQ = decltype(jq_c)::value;
            constexpr int J1 = (JQ + 1) & 3, J2 = (JQ + 2) & 3;
            const int s1 = s0 == Q3_NR - 1 ? 0 : s0 + 1;
            const int s2 = s1 == Q3_NR - 1 ? 0 : s1 + 1;
            if (t + 2 < T) {
                issue(t + 2, s2, std::integral_constant<int, J2>{});
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G::template cnt<J2, DBG>()) : "memory");
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            if (t + 1 < T) dequant(t + 1, s1, std::integral_constant<int, J1>{});
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // B(t)
            s0 = s1;
        };
        for (int t = 0; t < T; t += 4) {
            period(t, I0{});
            period(t + 1, I1{});
            period(t + 2, I2{});
            period(t + 3, I3{});
        }
        return;
    }

    // ================= consumer: fragment reads + MFMA =================
    const int cw = wave - 4;
    const int mw = cw >> 1, nw = cw & 1;
    const int rb = col >> 3;
    const uint32_t a_rd = (uint32_t)(mw * WM * 4096 + rb * 1024 + (col & 7) * 32 + ((h ^ (rb & 1)) << 4));
    const uint32_t b_rd = (uint32_t)(G::OFF_B + nw * WN * 1024 + lane * 16);
    f32x16 acc[WM][WN];
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
        for (int j = 0; j < WN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    f16x8 fa[2][WM], fb[2][WN];
    if constexpr (DBG & 16) {  // register-resident operands: any finite values
#pragma unroll
        for (int b = 0; b < 2; ++b) {
#pragma unroll
            for (int i = 0; i < WM; ++i)
#pragma unroll
                for (int e = 0; e < 8; ++e) fa[b][i][e] = (_Float16)(0.001f * (float)(lane + e + i));
#pragma unroll
            for (int j = 0; j < WN; ++j)
#pragma unroll
                for (int e = 0; e < 8; ++e) fb[b][j][e] = (_Float16)(0.002f * (float)(lane - e + j));
        }
    }
    auto rd = [&](int buf, int slot, int tb, int S) {  // fragments of k-step S of the tile in (slot, B buffer tb)
        if constexpr (DBG & 16) {
            if (S == 0 && buf == 0 && slot < 0) {
#pragma unroll
                for (int i = 0; i < WM; ++i) fa[buf][i] = *(const f16x8*)(smem + a_rd + i * 4096);
            }
            return;
        }
#pragma unroll
        for (int i = 0; i < WM; ++i) fa[buf][i] = *(const f16x8*)(smem + slot * A_BYTES + a_rd + i * 4096 + S * 256);
#pragma unroll
        for (int j = 0; j < WN; ++j) fb[buf][j] = *(const f16x8*)(smem + b_rd + tb * G::B16 + S * 4096 + j * 1024);
    };
    auto mma = [&](int buf) {
#pragma unroll
        for (int j = 0; j < WN; ++j)
#pragma unroll
            for (int i = 0; i < WM; ++i) {
                if constexpr (DBG & 1) asm volatile("" ::"v"(fa[buf][i]), "v"(fb[buf][j]));
                else acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[buf][i], fb[buf][j], acc[i][j], 0, 0, 0);
            }
    };
    asm volatile("s_barrier" ::: "memory");  // B(-1)
    int slot = 0;
    rd(0, 0, 0, 0);
    // sched_barrier fences: the reads of k-step S + 1 are issued BEFORE k-step S's MFMAs (left alone, the
    // scheduler sinks them between the MFMAs into the same registers and every k-step waits on lgkmcnt)
    for (int t = 0; t < T; ++t) {
        const int tb = t & 1;
        rd(1, slot, tb, 1);
        __builtin_amdgcn_sched_barrier(0);
        mma(0);
        __builtin_amdgcn_sched_barrier(0);
        rd(0, slot, tb, 2);
        __builtin_amdgcn_sched_barrier(0);
        mma(1);
        __builtin_amdgcn_sched_barrier(0);
        rd(1, slot, tb, 3);
        __builtin_amdgcn_sched_barrier(0);
        mma(0);
        __builtin_amdgcn_sched_barrier(0);
        // every read of tile t has returned (fa/fb[1] hold k-step 3): the producers may refill its slots
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // B(t)
        __builtin_amdgcn_sched_barrier(0);
        slot = slot == Q3_NR - 1 ? 0 : slot + 1;
        if (t + 1 < T) rd(0, slot, tb ^ 1, 0);
        __builtin_amdgcn_sched_barrier(0);
        mma(1);  // k-step 3 of tile t, over the latency of tile t + 1's first reads
        __builtin_amdgcn_sched_barrier(0);
    }

    // ---- epilogue: 32x32 C/D layout: col = lane & 31, row = 8*(r>>2) + 4*(lane>>5) + (r&3) ----
    const int mb = m_base + mw * WM * 32;
#pragma unroll
    for (int j = 0; j < WN; ++j) {
        const int nt = (ct * 4 + nw * WN + j) * 32;
        const int n = nt + col;
        if (nt >= N) break;
        if constexpr (EPI == E16_SWIGLU || EPI == E16_GEGLU) {
#pragma unroll
            for (int i = 0; i < WM; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const float v = acc[i][j][r];
                    const float up = __shfl_xor(v, 16);
                    const int m = mb + i * 32 + 8 * (r >> 2) + 4 * h + (r & 3);
                    if (col < 16 && m < M)
                        ((uint16_t*)Cv)[(size_t)m * ldc + (nt >> 1) + col] = f32_to_act<true>(glu_gate_f<EPI>(v) * up);
                }
            continue;
        }
#pragma unroll
        for (int i = 0; i < WM; ++i) {
            const int m0 = mb + i * 32 + 4 * h;
            if (mb + i * 32 >= M) break;
            float* cf = ((float*)Cv) + (size_t)m0 * ldc + n;
            uint16_t* ch = ((uint16_t*)Cv) + (size_t)m0 * ldc + n;
            auto roff = [&](int r) { return (size_t)(8 * (r >> 2) + (r & 3)) * ldc; };
            if (mb + i * 32 + 32 <= M) {
                if constexpr (EPI == E16_ADD_F32) {
                    if (splits == 1) {
                        float old[16];
#pragma unroll
                        for (int r = 0; r < 16; ++r) old[r] = cf[roff(r)];
#pragma unroll
                        for (int r = 0; r < 16; ++r) cf[roff(r)] = old[r] + acc[i][j][r];
                    } else {
#pragma unroll
                        for (int r = 0; r < 16; ++r) atomicAdd(cf + roff(r), acc[i][j][r]);
                    }
                } else {
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        if constexpr (EPI == E16_F32) cf[roff(r)] = acc[i][j][r];
                        else ch[roff(r)] = f32_to_act<true>(acc[i][j][r]);
                    }
                }
                continue;
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                if (m0 + 8 * (r >> 2) + (r & 3) >= M) continue;
                const float v = acc[i][j][r];
                if constexpr (EPI == E16_F32) cf[roff(r)] = v;
                else if constexpr (EPI == E16_ACT) ch[roff(r)] = f32_to_act<true>(v);
                else if (splits == 1) cf[roff(r)] += v;
                else atomicAdd(cf + roff(r), v);
            }
        }
    }
}

template <int QT, int WM, int EPI>
static int launch_qmm3(const uint16_t* A, int lda, const uint8_t* W, int M, int N, int K, int splits, void* C, int ldc,
                       hipStream_t st) {
    using G = Q3Geom<QT, WM>;
    const int nsb = K >> 8;
    splits = max(1, min(splits, nsb));
    const int sbps = (nsb + splits - 1) / splits;
    splits = (nsb + sbps - 1) / sbps;  // no empty splits
    const int n_ct = (N + 127) / 128, n_mt = (M + G::BM - 1) / G::BM;
    const long nwg = (long)n_ct * splits * n_mt;
    if (nwg <= 0 || nwg > 0x7fffffff) return (int)hipErrorInvalidValue;
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)qmm3_kernel<QT, WM, EPI>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  G::LDS);
        attr_set = true;
    }
    qmm3_kernel<QT, WM, EPI><<<dim3((unsigned)nwg), 512, G::LDS, st>>>(A, lda, W, M, N, K, n_mt, splits, sbps, C, ldc);
    MXK_CHECK_LAUNCH();
}

template <int QT, int EPI>
static int dispatch_qmm3(int wm, const uint16_t* A, int lda, const uint8_t* W, int M, int N, int K, int splits, void* C,
                         int ldc, hipStream_t st) {
    if (wm == 1) return launch_qmm3<QT, 1, EPI>(A, lda, W, M, N, K, splits, C, ldc, st);
    if (wm == 2) return launch_qmm3<QT, 2, EPI>(A, lda, W, M, N, K, splits, C, ldc, st);
    if (wm == 4) return launch_qmm3<QT, 4, EPI>(A, lda, W, M, N, K, splits, C, ldc, st);
    if (wm == 3) return launch_qmm3<QT, 3, EPI>(A, lda, W, M, N, K, splits, C, ldc, st);  // 192-row tiles
    return (int)hipErrorInvalidValue;
}

template <int DBG>
static int launch_q3dbg(int wm, const uint16_t* A, int lda, const uint8_t* W, int M, int N, int K, void* C, int ldc,
                        hipStream_t st) {
    constexpr int QT = MXQ_Q4_K, EPI = E16_SWIGLU;
    auto go = [&](auto kern, int bm, int lds) {
        (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        const int n_ct = (N + 127) / 128, n_mt = (M + bm - 1) / bm;
        kern<<<dim3(n_ct * n_mt), 512, lds, st>>>(A, lda, W, M, N, K, n_mt, 1, K >> 8, C, ldc);
        return (int)hipGetLastError();
    };
    if (wm == 4) return go(qmm3_kernel<QT, 4, EPI, DBG>, 256, Q3Geom<QT, 4>::LDS);
    if (wm == 2) return go(qmm3_kernel<QT, 2, EPI, DBG>, 128, Q3Geom<QT, 2>::LDS);
    return (int)hipErrorInvalidValue;
}


// all epilogues of one block format (each format's instances live in their own translation unit, qmm3_q*.hip)
template <int QT>
static int qmm3_run(int epi, int wm, const uint16_t* A, int lda, const uint8_t* W, int M, int N, int K, int splits, void* C, int ldc, hipStream_t st) {
    switch (epi) {
        case E16_F32: return dispatch_qmm3<QT, E16_F32>(wm, A, lda, W, M, N, K, splits, C, ldc, st);
        case E16_ACT: return dispatch_qmm3<QT, E16_ACT>(wm, A, lda, W, M, N, K, splits, C, ldc, st);
        case E16_ADD_F32: return dispatch_qmm3<QT, E16_ADD_F32>(wm, A, lda, W, M, N, K, splits, C, ldc, st);
        case E16_SWIGLU: return dispatch_qmm3<QT, E16_SWIGLU>(wm, A, lda, W, M, N, K, splits, C, ldc, st);
        case E16_GEGLU: return dispatch_qmm3<QT, E16_GEGLU>(wm, A, lda, W, M, N, K, splits, C, ldc, st);
    }
    return (int)hipErrorInvalidValue;
}

}  // namespace

int qmm3_run_q4k(int epi, int wm, const uint16_t* A, int lda, const uint8_t* W, int M, int N, int K, int splits, void* C, int ldc, hipStream_t st);
int qmm3_run_q5k(int epi, int wm, const uint16_t* A, int lda, const uint8_t* W, int M, int N, int K, int splits, void* C, int ldc, hipStream_t st);
int qmm3_run_q6k(int epi, int wm, const uint16_t* A, int lda, const uint8_t* W, int M, int N, int K, int splits, void* C, int ldc, hipStream_t st);
int qmm3_run_q3k(int epi, int wm, const uint16_t* A, int lda, const uint8_t* W, int M, int N, int K, int splits, void* C, int ldc, hipStream_t st);
int qmm3_run_q2k(int epi, int wm, const uint16_t* A, int lda, const uint8_t* W, int M, int N, int K, int splits, void* C, int ldc, hipStream_t st);
int qmm3_run_q80(int epi, int wm, const uint16_t* A, int lda, const uint8_t* W, int M, int N, int K, int splits, void* C, int ldc, hipStream_t st);
int qmm3_run_mx4(int epi, int wm, const uint16_t* A, int lda, const uint8_t* W, int M, int N, int K, int splits, void* C, int ldc, hipStream_t st);
int qmm3_run_mx5(int epi, int wm, const uint16_t* A, int lda, const uint8_t* W, int M, int N, int K, int splits, void* C, int ldc, hipStream_t st);
int qmm3_dbg_q4k(int dbg, int wm, const uint16_t* A, int lda, const uint8_t* W, int M, int N, int K, void* C, int ldc, hipStream_t st);
