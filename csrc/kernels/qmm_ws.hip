// qmm_ws.hip — warp-specialised quantised-weight GEMM (see the block comment below); shares the t32 formats
// and fragment builders of qmm.hip through qmm_fmt.h.
#include "qmm_fmt.h"

// =====================================================================================================
// qmm_ws — warp-specialised variant for the serving regime (M ~ 64..512: continuous-batching steps).
//
// Why: the monolithic qmm_kernel above runs dequant VALU, LDS reads and MFMAs in the same wave, so at
// these M the ~8 VALU per MFMA (nibble dequant + Q4_K scale decode + address arithmetic) and their
// dependency stalls serialise with the matrix pipe: profiles/r3_pmc_qmm_gate_up_m256.md shows MFMA issue
// at ~31 % of the kernel time. A CDNA4 SIMD runs a MFMA-only wave and a VALU-only wave side by side
// (MI355X_MICROARCH "Wave scheduling"), so here the roles are split:
//   * 4 PRODUCER waves (one per SIMD): issue every LDS-DMA (A rows + raw quantised weight bytes, t32
//     layout, NS-deep ring), then dequantise the raw bytes of a k-tile ONCE into an f16 B tile in LDS
//     (the same swizzled [n][64 k] layout as the A tile, so both operands are plain ds_read_b128);
//   * 4 CONSUMER waves (one per SIMD, CM x CN grid, wave tile 32WM x 32WN): LDS reads + MFMAs only.
// One s_barrier per k-tile. Producers run LEAD k-tiles ahead of the consumers (NB = LEAD + 1 B16 buffers);
// with LEAD = 2 the consumers also prefetch the next tile's first fragments before the barrier, so the
// matrix pipe sees no per-tile bubble.
// =====================================================================================================
// AD > 0: the consumer waves read their A fragments straight from global memory (L2-resident rows) into an
// AD-deep register ring instead of an LDS tile: the LDS then holds only the raw weight ring + the B16 tiles,
// so far more bytes are in flight per CU, and the A operand never crosses the LDS port.
template <int QT, int CM, int WM, int WN, int GP, int LEAD, int AD = 0>
struct QwsCfg {
    static constexpr int CN = 4 / CM;
    static constexpr int BM = 32 * WM * CM, BN = 32 * WN * CN;
    using G = QmmGeom<QT, GP>;
    static constexpr int A_BYTES = AD ? 0 : BM * 128;
    static constexpr int STAGE = A_BYTES + 4 * G::WBYTES;
    static constexpr int NB = LEAD + 1;
    static constexpr int B16 = BN * 128;
    static constexpr int S0 = (QMM_LDS_BUDGET - NB * B16) / STAGE;
    static constexpr int SCAP = AD ? 10 : 6;
    static constexpr int NS = S0 > SCAP ? SCAP : S0;
    static constexpr int WA = AD ? 0 : BM / 32;  // A-tile LDS-DMA instructions per producer wave (8 rows x 128 B each)
    static constexpr int NI = WA + G::NI;
    static constexpr bool OK =
        BN == 128 * GP && CM * CN == 4 && NS >= 2 + LEAD && (NS - 2) * NI <= 63 && (AD ? AD * 4 * WM <= 48 : WA >= 1);
};

// wait (no barrier) until at most `ahead` k-tiles (NI LDS-DMA instructions each) of this wave are in flight
template <int NI, int A_>
MX_DEV void qws_wait(int ahead) {
    if constexpr (A_ <= 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
        if (ahead >= A_) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(A_ * NI) : "memory");
        else qws_wait<NI, A_ - 1>(ahead);
    }
}

MX_DEV void qws_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
MX_DEV void qws_barrier(int dbg) {
    if (dbg & 32) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // timing experiment only: no barrier
    else qws_barrier();
}

template <int QT, int CM, int WM, int WN, int GP, int LEAD, int AD, int EPI>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) void
qmm_ws_kernel(const uint16_t* __restrict__ A, int lda, const uint8_t* __restrict__ W, int M, int N, int K, int n_mt,
              int splits, int kt_per_split, void* __restrict__ Cv, int ldc, int dbg) {
    using C = QwsCfg<QT, CM, WM, WN, GP, LEAD, AD>;
    using G = typename C::G;
    using F = QmmFmt<QT>;
    constexpr int NS = C::NS, NB = C::NB, WA = C::WA, NI = C::NI;
    static_assert(C::OK, "qmm_ws configuration");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* const b16 = smem + NS * C::STAGE;

    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int h = lane >> 5, col = lane & 31;

    // XCD-aware bijective remap (as qmm_kernel): the row tiles sharing a weight column panel run on one XCD
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    const int mt = lid % n_mt;
    const int rest = lid / n_mt;
    const int split = rest % splits;
    const int ct = rest / splits;
    const int m_base = mt * C::BM, n_base = ct * C::BN;
    const int nkt = K / QMM_KT;
    const int kt0 = split * kt_per_split;
    const int kt1 = min(kt0 + kt_per_split, nkt);
    if (kt0 >= kt1) return;  // uniform over the workgroup

    if (wave >= 4) {
        // ------------------------------------ producer ------------------------------------
        const int p = wave - 4;
        const int n_p = n_base + p * GP * 32;
        const int ngrp = N >> 5;
        const size_t gstride = (size_t)(nkt / F::PER_UNIT) * F::UNIT;
        uint32_t aoff[WA > 0 ? WA : 1];
#pragma unroll
        for (int i = 0; i < WA; ++i) {
            const int r = (p * WA + i) * 8 + (lane >> 3);
            const int c = (lane & 7) ^ ((r >> 1) & 7);
            aoff[i] = (uint32_t)(min(m_base + r, M - 1) * lda + c * 8);
        }
        const uint8_t* qsrc[G::QI];
        bool qact[G::QI];
#pragma unroll
        for (int ci = 0; ci < G::QI; ++ci) {
            const int q = ci * 64 + lane;
            const int t = q / G::QCH, j = q % G::QCH;
            qact[ci] = q < GP * G::QCH;
            const int g = min((n_p >> 5) + (qact[ci] ? t : 0), ngrp - 1);
            qsrc[ci] = W + (size_t)g * gstride + F::QOFF + j * 16;
        }
        const int mg = min((n_p >> 5) + (lane >> 5), ngrp - 1);
        const uint8_t* msrc = W + (size_t)mg * gstride + F::MOFF + (lane & 31) * 16;
        const uint8_t* dsrc = W + (size_t)mg * gstride + F::DOFF + (lane & 31) * 4;
        const bool mact = lane < 32 * GP;

        auto issue = [&](int kt) {
            char* sb = smem + ((kt - kt0) % NS) * C::STAGE;
            const uint16_t* ak = A + (size_t)kt * QMM_KT;
            if (!(dbg & 4))
#pragma unroll
            for (int i = 0; i < WA; ++i)
                __builtin_amdgcn_global_load_lds((const void*)(ak + aoff[i]), (MX_LDS void*)(sb + (p * WA + i) * 1024), 16,
                                                 0, 0);
            if (dbg & 8) return;
            char* wb = sb + C::A_BYTES + p * G::WBYTES;
            const size_t unit = (size_t)(kt / F::PER_UNIT) * F::UNIT;
            const int jq = kt % F::PER_UNIT;
#pragma unroll
            for (int ci = 0; ci < G::QI; ++ci)
                if (qact[ci])
                    __builtin_amdgcn_global_load_lds((const void*)(qsrc[ci] + unit + jq * F::QSTRIDE),
                                                     (MX_LDS void*)(wb + G::Q_OFF + ci * 1024), 16, 0, 0);
            if constexpr (G::MI > 0) {
                if (mact)
                    __builtin_amdgcn_global_load_lds((const void*)(msrc + unit + (jq >> 1) * F::MSTEP),
                                                     (MX_LDS void*)(wb + G::M_OFF), 16, 0, 0);
            }
            if constexpr (G::DI > 0) {
                if (mact)
                    __builtin_amdgcn_global_load_lds((const void*)(dsrc + unit), (MX_LDS void*)(wb + G::D_OFF), 4, 0, 0);
            }
        };
        // raw bytes of k-tile kt (landed) -> f16 B tile buffer (kt - kt0) % NB, rows n = p*GP*32 + g*32 + col
        auto dequant = [&](int kt) {
            if (dbg & 2) return;
            const char* wl = smem + ((kt - kt0) % NS) * C::STAGE + C::A_BYTES + p * G::WBYTES;
            char* dst = b16 + ((kt - kt0) % NB) * C::B16;
            const int jq = kt % F::PER_UNIT;
#pragma unroll
            for (int g = 0; g < GP; ++g) {
                QmmB<QT> b;
                b.load(wl + G::Q_OFF + g * F::QB, wl + G::M_OFF + g * 512, wl + G::D_OFF + g * 128, col, h, jq);
                b.prep(jq);
                const int n = (p * GP + g) * 32 + col;
                *(f16x8*)(dst + qmm_a_off(n, h)) = b.template frag<0>();
                *(f16x8*)(dst + qmm_a_off(n, 2 + h)) = b.template frag<1>();
                *(f16x8*)(dst + qmm_a_off(n, 4 + h)) = b.template frag<2>();
                *(f16x8*)(dst + qmm_a_off(n, 6 + h)) = b.template frag<3>();
            }
        };
        // prologue: NS-1 tiles in flight; the first LEAD tiles dequantised before barrier #0
        const int last_pro = min(kt1 - 1, kt0 + NS - 2);
        for (int kt = kt0; kt <= last_pro; ++kt) issue(kt);
#pragma unroll
        for (int j = 0; j < LEAD; ++j)
            if (kt0 + j < kt1) {
                qws_wait<NI, NS - 2>(last_pro - (kt0 + j));
                dequant(kt0 + j);
            }
        qws_barrier();
        const int pend = AD > 0 ? kt0 + (kt1 - kt0 + AD - 1) / AD * AD : kt1;
        for (int t = kt0; t < pend; ++t) {
            const int tt = t + LEAD;
            if (tt < kt1) {
                // issued so far: tiles up to min(kt1 - 1, t + NS - 2)
                qws_wait<NI, NS - 2 - LEAD>(min(kt1 - 1, t + NS - 2) - tt);
                dequant(tt);
            }
            // the slot of tile t - 1 is free: every consumer finished it before barrier #t
            if (t + NS - 1 < kt1) issue(t + NS - 1);
            qws_barrier(dbg);
        }
        return;
    }

    // ------------------------------------ consumer ------------------------------------
    const int cm = wave % CM, cn = wave / CM;
    f32x16 acc[WM][WN];
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
        for (int j = 0; j < WN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    if constexpr (AD > 0) {
        // A fragments from global memory: lane (col, h) of row block i, k-step s reads the 16 B at
        // row m_base + (cm WM + i) 32 + col, k = 64 kt + 16 s + 8 h (the 32x32x16 A-operand layout)
        const uint16_t* arow[WM];
#pragma unroll
        for (int i = 0; i < WM; ++i)
            arow[i] = A + (size_t)min(m_base + (cm * WM + i) * 32 + col, M - 1) * lda + 8 * h;
        f16x8 abuf[AD][4][WM];
        auto aload = [&](int kt, f16x8 (&dst)[4][WM]) {
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
                for (int i = 0; i < WM; ++i) dst[s][i] = *(const f16x8*)(arow[i] + (size_t)kt * QMM_KT + 16 * s);
        };
        f16x8 bb[2][WN];
        auto rdb = [&](int kt, int s, f16x8 (&b)[WN]) {
            const char* sb = b16 + ((kt - kt0) % NB) * C::B16;
            if (dbg & 16) return;
#pragma unroll
            for (int j = 0; j < WN; ++j) b[j] = *(const f16x8*)(sb + qmm_a_off((cn * WN + j) * 32 + col, 2 * s + h));
        };
        // prefetches past kt1 re-read the last tile (unconditional loads keep the compiler's vmcnt counting exact);
        // the loop runs a multiple of AD tiles, MFMAs only on live ones, one barrier per tile as the producers do
#pragma unroll
        for (int d = 0; d < AD; ++d) aload(min(kt0 + d, kt1 - 1), abuf[d]);
        qws_barrier();
        if constexpr (LEAD >= 2) rdb(kt0, 0, bb[0]);
        const int kend = kt0 + (kt1 - kt0 + AD - 1) / AD * AD;
        for (int tb = kt0; tb < kend; tb += AD) {
#pragma unroll
            for (int d = 0; d < AD; ++d) {
                const int t = tb + d;
                const bool live = t < kt1;
                if constexpr (LEAD < 2) rdb(t, 0, bb[0]);
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    const int cur = s & 1;
                    if (s < 3) rdb(t, s + 1, bb[cur ^ 1]);
                    else if constexpr (LEAD >= 2) rdb(t + 1, 0, bb[0]);
                    if (live && !(dbg & 1))
#pragma unroll
                        for (int i = 0; i < WM; ++i)
#pragma unroll
                            for (int j = 0; j < WN; ++j)
                                acc[i][j] =
                                    __builtin_amdgcn_mfma_f32_32x32x16_f16(abuf[d][s][i], bb[cur][j], acc[i][j], 0, 0, 0);
                }
                aload(min(t + AD, kt1 - 1), abuf[d]);
                qws_barrier(dbg);
            }
        }
    } else {
    f16x8 ar[2][WM], br[2][WN];
    auto rd = [&](int kt, int s, f16x8 (&a)[WM], f16x8 (&b)[WN]) {
        const char* sa = smem + ((kt - kt0) % NS) * C::STAGE;
        const char* sb = b16 + ((kt - kt0) % NB) * C::B16;
#pragma unroll
        for (int i = 0; i < WM; ++i) a[i] = *(const f16x8*)(sa + qmm_a_off((cm * WM + i) * 32 + col, 2 * s + h));
#pragma unroll
        for (int j = 0; j < WN; ++j) b[j] = *(const f16x8*)(sb + qmm_a_off((cn * WN + j) * 32 + col, 2 * s + h));
    };
    qws_barrier();
    if constexpr (LEAD >= 2) rd(kt0, 0, ar[0], br[0]);
    for (int t = kt0; t < kt1; ++t) {
        if constexpr (LEAD < 2) rd(t, 0, ar[0], br[0]);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int cur = s & 1;
            if (s < 3) rd(t, s + 1, ar[cur ^ 1], br[cur ^ 1]);
            else if constexpr (LEAD >= 2) rd(t + 1, 0, ar[0], br[0]);  // published at barrier #t (a stale slot past kt1: unused)
            if (!(dbg & 1))
#pragma unroll
            for (int i = 0; i < WM; ++i)
#pragma unroll
                for (int j = 0; j < WN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ar[cur][i], br[cur][j], acc[i][j], 0, 0, 0);
        }
        qws_barrier();
    }
    }

    // ---- epilogue (32x32 C/D layout: col = lane & 31, row = 8*(r>>2) + 4*(lane>>5) + (r&3)) ----
    const int m_wave = m_base + cm * WM * 32;
#pragma unroll
    for (int j = 0; j < WN; ++j) {
        const int nt = n_base + (cn * WN + j) * 32;
        const int n = nt + col;
        if constexpr (EPI == E16_SWIGLU || EPI == E16_GEGLU) {
#pragma unroll
            for (int i = 0; i < WM; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const float v = acc[i][j][r];
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
            auto roff = [&](int r) { return (size_t)(8 * (r >> 2) + (r & 3)) * ldc; };
            if (m_wave + i * 32 + 32 <= M) {
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

static int g_qws_dbg = 0;  // isolation experiments (tools/tune_qmm_ws.py --dbg): 1 no MFMA, 2 no dequant, 4 no A loads,
                           // 8 no W loads, 16 no B16 reads (register-A consumers), 32 no per-tile barrier
extern "C" int mxk_qmm_ws_dbg(int v) {
    g_qws_dbg = v;
    return 0;
}

template <int QT, int CM, int WM, int WN, int GP, int LEAD, int AD, int EPI>
static int launch_qmm_ws(const uint16_t* A, int lda, const uint8_t* W, int M, int N, int K, int splits, void* C, int ldc,
                         hipStream_t st) {
    using Cf = QwsCfg<QT, CM, WM, WN, GP, LEAD, AD>;
    if constexpr (!Cf::OK) {
        return (int)hipErrorInvalidValue;  // this format's stage does not fit the ring at this tile
    } else {
        constexpr size_t lds = (size_t)Cf::NS * Cf::STAGE + (size_t)Cf::NB * Cf::B16;
        static_assert(lds <= 160 * 1024, "LDS");
        const int nkt = K / QMM_KT;
        splits = max(1, min(splits, nkt));
        const int ktps = (nkt + splits - 1) / splits;
        splits = (nkt + ktps - 1) / ktps;
        const int n_ct = (N + Cf::BN - 1) / Cf::BN, n_mt = (M + Cf::BM - 1) / Cf::BM;
        const long nwg = (long)n_ct * splits * n_mt;
        if (nwg <= 0 || nwg > 0x7fffffff) return (int)hipErrorInvalidValue;
        static bool attr_set = false;
        if (!attr_set) {
            (void)hipFuncSetAttribute((const void*)qmm_ws_kernel<QT, CM, WM, WN, GP, LEAD, AD, EPI>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            attr_set = true;
        }
        qmm_ws_kernel<QT, CM, WM, WN, GP, LEAD, AD, EPI><<<dim3((unsigned)nwg), 512, lds, st>>>(A, lda, W, M, N, K, n_mt, splits,
                                                                                          ktps, C, ldc, g_qws_dbg);
        MXK_CHECK_LAUNCH();
    }
}

// cfg packs (AD, CM, WM, WN, GP, LEAD) as decimal digits AD*100000 + CM*10000 + WM*1000 + WN*100 + GP*10 + LEAD
template <int QT, int EPI>
static int dispatch_qmm_ws(int cfg, const uint16_t* A, int lda, const uint8_t* W, int M, int N, int K, int splits, void* C,
                           int ldc, hipStream_t st) {
#define QWS_CASE(CM_, WM_, WN_, GP_, L_) QWS_CASE_A(0, CM_, WM_, WN_, GP_, L_)
#define QWS_CASE_A(AD_, CM_, WM_, WN_, GP_, L_)                                                         \
    if (cfg == AD_ * 100000 + CM_ * 10000 + WM_ * 1000 + WN_ * 100 + GP_ * 10 + L_)                      \
        return launch_qmm_ws<QT, CM_, WM_, WN_, GP_, L_, AD_, EPI>(A, lda, W, M, N, K, splits, C, ldc, st);
    // BM x BN: 128x128 (2x2 waves of 64x64), 256x128 (2x2 of 128x64), 128x256 (2x2 of 64x128),
    // 64x128 (1x4 of 64x32), 64x256 (1x4 of 64x64), 128x128 (4x1 of 32x128)
    QWS_CASE(2, 2, 2, 1, 1) QWS_CASE(2, 2, 2, 1, 2) QWS_CASE(2, 4, 2, 1, 1) QWS_CASE(2, 2, 4, 2, 1)
    QWS_CASE(1, 2, 1, 1, 1) QWS_CASE(1, 2, 1, 1, 2) QWS_CASE(1, 2, 2, 2, 1) QWS_CASE(4, 1, 4, 1, 1)
    QWS_CASE(4, 1, 4, 1, 2)
    // A fragments in a register ring (AD tiles deep): 128x128 (4x1 of 32x128), 256x128 (4x1 of 64x128),
    // 128x256 (4x1 of 32x256), 128x128 (2x2 of 64x64)
    QWS_CASE_A(4, 4, 1, 4, 1, 2) QWS_CASE_A(2, 4, 2, 4, 1, 2) QWS_CASE_A(2, 4, 1, 8, 2, 1) QWS_CASE_A(4, 2, 2, 2, 1, 2)
#undef QWS_CASE_A
#undef QWS_CASE
    return (int)hipErrorInvalidValue;
}

extern "C" int mxk_qmm_ws(int qtype, int epi, int cfg, const uint16_t* A, int lda, const uint8_t* W, int M, int N, int K,
                          int splits, void* C, int ldc, hipStream_t st) {
    if (M <= 0) return 0;
    if (K % 256 || (lda & 7) || ((uintptr_t)A & 15) || ((uintptr_t)W & 15)) return (int)hipErrorInvalidValue;
    if (epi != E16_ADD_F32 && splits != 1) return (int)hipErrorInvalidValue;
    if (N & 31) return (int)hipErrorInvalidValue;
#define QWS_EPI(QT_)                                                                                               \
    switch (epi) {                                                                                                 \
        case E16_F32: return dispatch_qmm_ws<QT_, E16_F32>(cfg, A, lda, W, M, N, K, splits, C, ldc, st);           \
        case E16_ACT: return dispatch_qmm_ws<QT_, E16_ACT>(cfg, A, lda, W, M, N, K, splits, C, ldc, st);           \
        case E16_ADD_F32: return dispatch_qmm_ws<QT_, E16_ADD_F32>(cfg, A, lda, W, M, N, K, splits, C, ldc, st);   \
        case E16_SWIGLU: return dispatch_qmm_ws<QT_, E16_SWIGLU>(cfg, A, lda, W, M, N, K, splits, C, ldc, st);     \
        case E16_GEGLU: return dispatch_qmm_ws<QT_, E16_GEGLU>(cfg, A, lda, W, M, N, K, splits, C, ldc, st);       \
    }
    switch (qtype) {
        case MXQ_Q4_K: QWS_EPI(MXQ_Q4_K) break;
        case MXQ_Q6_K: QWS_EPI(MXQ_Q6_K) break;
        case MXQ_Q8_0: QWS_EPI(MXQ_Q8_0) break;
        case MXQ_MX4F: QWS_EPI(MXQ_MX4F) break;
        case MXQ_MX5F: QWS_EPI(MXQ_MX5F) break;
    }
#undef QWS_EPI
    return (int)hipErrorInvalidValue;
}
