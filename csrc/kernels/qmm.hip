// qmm.hip — quantised-weight GEMM for the M >= 64 regime (mixed continuous-batching steps, prefill):
//
//   C[M, N] (+)= A[M, K] · W[N, K]^T,   A f16 (act16 mode f16), W in Q4_K / Q6_K(repacked) / Q8_0(repacked)
//
// Replaces the dense-f16-weight-copy + hipBLASLt path for large M: the weights stay in their GGUF
// block format in HBM (3.5x fewer bytes than f16) and are dequantised on the fly into MFMA operands.
//
// Structure (one 256-thread workgroup = 4 waves; BM = 32*WM rows x BN = 128*WN columns):
//   * every operand reaches the CU through `global_load_lds` (LDS-DMA, no VGPR staging) into an
//     NSTAGE-deep ring of KT = 64-wide k-tiles, so NSTAGE-1 tiles of weights are in flight per
//     workgroup (the memory-level parallelism a weight-streaming GEMM needs at 1 workgroup per CU);
//   * the ring is advanced with a COUNTED `s_waitcnt vmcnt(N)` + raw `s_barrier` (never vmcnt(0) in
//     the loop: every load in this kernel is an LDS-DMA, so the count is exact);
//   * the A tile (BM x 64 f16) is shared by the 4 waves (XOR-swizzled 128-B rows, conflict-free
//     ds_read_b128 fragment reads); the 4 waves split N, so each weight is dequantised exactly once
//     per workgroup, by the wave that owns its column, straight from the raw block bytes in LDS into
//     a 32x32x16 f16 MFMA B fragment (packed-f16 magic-number dequantisation, qdeq16.h);
//   * k order inside a tile is the natural one for all three block formats: MFMA k-step s, lane half h,
//     element j <-> k = 16 s + 8 h + j, which for Q4_K/Q6_K is low nibbles (s < 2) / high nibbles
//     (s >= 2) of the same 32 bytes, so one 8-byte LDS read feeds two k-steps;
//   * the block index -> (column tile, split, row tile) map is XCD-aware (bijective remap; the row
//     tiles that share a column panel of W run on one XCD and re-read it from that XCD's L2).
// Split-K over K (fp32 atomics) only for accumulating outputs; otherwise a plain store / RMW add.
#include "qmm_fmt.h"


// KS waves share each of the NW column groups and split every k-tile's four k-steps between them
// (wave kh runs k-steps kh, kh+KS, ...; fp32 partials summed through LDS before the epilogue): at small M
// a workgroup of 4 waves leaves one wave per SIMD, whose dequant VALU, LDS-read latency and MFMAs then
// serialise (measured: loads alone took half the kernel time); KS = 2 puts two waves on every SIMD
// without dequantising any weight twice.
// WMW waves split the BM rows of each column group (wave tile 32*WM x 32*WN): with WMW = 1 every wave
// re-reads the whole A tile from LDS for its 32*WN columns, and at WN = 1 those A-fragment reads alone
// saturate the CU's LDS port (64 KB of reads per 64-k tile against 512 MFMA cycles); squarer wave tiles
// (64x64, 128x64) halve that traffic at the price of dequantising each weight fragment WMW times.
template <int QT, int WM, int WN, int NW, int KS, int OCC, int EPI, int WMW>
// The ring takes the whole LDS (1/OCC of it), so a CU holds OCC workgroups: tell the scheduler that
// OCC*NW*KS/4 waves per SIMD is the occupancy (it otherwise sinks the LDS reads next to their MFMAs to save
// registers nobody can use).
__global__ __launch_bounds__(64 * NW * KS * WMW) __attribute__((amdgpu_waves_per_eu(OCC * NW * KS * WMW / 4, OCC * NW * KS * WMW / 4))) void
qmm_kernel(const uint16_t* __restrict__ A, int lda, const uint8_t* __restrict__ W, const uint16_t* __restrict__ WD,
           int M, int N, int K, int n_ct, int n_mt, int splits, int kt_per_split, void* __restrict__ Cv, int ldc) {
    using G = QmmGeom<QT, WN>;
    using F = QmmFmt<QT>;
    constexpr int BM = 32 * WM * WMW, COLS = G::COLS;
    constexpr int A_BYTES = BM * 128;
    constexpr int STAGE = A_BYTES + NW * G::WBYTES;
    constexpr int NS = QmmRing<QT, WM, WN, NW, OCC, WMW>::STAGES;
    static_assert(STAGE == QmmRing<QT, WM, WN, NW, OCC, WMW>::STAGE && NS >= 3, "ring");
    static_assert(KS == 1 || NW * WMW * WM * WN * 16 * 64 * 4 <= NS * STAGE, "k-split partials fit in the ring");
    constexpr int NT = NW * KS * WMW;  // waves
    constexpr int WA = BM / 8 / NT;   // A-tile LDS-DMA instructions per wave (8 rows x 128 B each)
    static_assert(WA >= 1 && WA * 8 * NT == BM, "A tile split");
    static_assert(KS == 1 || KS == 2, "k-step split");
    static_assert((NS - 2) * (WA + G::NI) <= 63, "vmcnt range");
    static_assert(WN <= 2, "one d / meta instruction covers at most 2 groups");
    extern __shared__ __attribute__((aligned(16))) char smem[];

    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int h = lane >> 5, col = lane & 31;
    const int cg = wave % NW, mw = (wave / NW) % WMW, kh = wave / (NW * WMW);  // column group, row slice, k-step phase

    // XCD-aware bijective remap of the 1-D grid: consecutive logical ids share an XCD
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    const int mt = lid % n_mt;
    const int rest = lid / n_mt;
    const int split = rest % splits;
    const int ct = rest / splits;
    (void)n_ct;

    const int m_base = mt * BM;
    const int n_wave = ct * NW * COLS + cg * COLS;
    const int nkt = K / QMM_KT;
    const int kt0 = split * kt_per_split;
    const int kt1 = min(kt0 + kt_per_split, nkt);
    if (kt0 >= kt1) return;
    const int ngrp = N >> 5;
    const size_t gstride = (size_t)(nkt / F::PER_UNIT) * F::UNIT;  // bytes per 32-column group

    // ---- per-lane LDS-DMA source offsets (k-tile independent parts) ----
    uint32_t aoff[WA];
#pragma unroll
    for (int i = 0; i < WA; ++i) {
        const int r = (wave * WA + i) * 8 + (lane >> 3);
        const int c = (lane & 7) ^ ((r >> 1) & 7);
        aoff[i] = (uint32_t)(min(m_base + r, M - 1) * lda + c * 8);
    }
    // quant chunk slot q = ci*64 + lane -> group t = q / QCH, chunk j = q % QCH (contiguous per group)
    const uint8_t* qsrc[G::QI];
    bool qact[G::QI];
#pragma unroll
    for (int ci = 0; ci < G::QI; ++ci) {
        const int q = ci * 64 + lane;
        const int t = q / G::QCH, j = q % G::QCH;
        qact[ci] = q < WN * G::QCH;
        const int g = min((n_wave >> 5) + (qact[ci] ? t : 0), ngrp - 1);  // groups past N: re-read the last
        qsrc[ci] = W + (size_t)g * gstride + F::QOFF + j * 16;
    }
    // meta / d slots: lane -> group t = lane / 32, column r = lane % 32
    const int mg = min((n_wave >> 5) + (lane >> 5), ngrp - 1);
    const uint8_t* msrc = W + (size_t)mg * gstride + F::MOFF + (lane & 31) * 16;
    const uint8_t* dsrc = W + (size_t)mg * gstride + F::DOFF + (lane & 31) * 4;
    const bool mact = lane < 32 * WN;

    // every wave streams its share of the A rows; the (kh, mw) == 0 wave of a column group its weight bytes
    auto issue = [&](int kt, int slot, auto wl_c) {
        char* sb = smem + slot * STAGE;
        const uint16_t* ak = A + (size_t)kt * QMM_KT;
#pragma unroll
        for (int i = 0; i < WA; ++i)
            __builtin_amdgcn_global_load_lds((const void*)(ak + aoff[i]),
                                             (MX_LDS void*)(sb + (wave * WA + i) * 1024), 16, 0, 0);
        if constexpr (decltype(wl_c)::value) {
            char* wb = sb + A_BYTES + cg * G::WBYTES;
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
        }
    };

    f32x16 acc[WM][WN];
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
        for (int t = 0; t < WN; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][t][r] = 0.f;

    // Register-level software pipeline, one k-step deep: the A fragments of the wave's next k-step
    // (across the tile boundary too: tile kt+1 is waited for at the top of tile kt) are read while the
    // MFMAs of the current one run, and the raw weight bytes of tile kt+1 while tile kt computes. The
    // scale prep (VALU) of a tile runs at the start of its compute, when its raw bytes have landed.
    f16x8 ar[2][WM];
    QmmB<QT> bw[WN], bn[WN];
    auto load_a = [&](const char* sb, int s, f16x8 (&dst)[WM]) {
#pragma unroll
        for (int i = 0; i < WM; ++i) dst[i] = *(const f16x8*)(sb + qmm_a_off((mw * WM + i) * 32 + col, 2 * s + h));
    };
    auto load_b = [&](const char* sb, QmmB<QT> (&dst)[WN], int jq) {
        const char* wl = sb + A_BYTES + cg * G::WBYTES;
#pragma unroll
        for (int t = 0; t < WN; ++t)
            dst[t].load(wl + G::Q_OFF + t * F::QB, wl + G::M_OFF + t * 512, wl + G::D_OFF + t * 128, col, h, jq);
    };

    auto mainloop = [&](auto kh_c, auto wl_c) {
        constexpr int KH = decltype(kh_c)::value;
        constexpr bool WLOAD = decltype(wl_c)::value;
        constexpr int NI = WA + (WLOAD ? G::NI : 0);  // LDS-DMA wave-instructions per stage of this wave
        using WLc = std::integral_constant<bool, WLOAD>;
        // prologue: NSTAGE-1 tiles in flight; wait for the first
#pragma unroll
        for (int s = 0; s < NS - 1; ++s)
            if (kt0 + s < kt1) issue(kt0 + s, s, WLc{});
        qmm_wait_ahead<NI, NS - 2>(min(kt1 - 1, kt0 + NS - 2) - kt0);
        load_b(smem, bw, kt0 & 3);
        load_a(smem, KH, ar[0]);
        f16x8 bcur[WN];
#pragma unroll
        for (int t = 0; t < WN; ++t) {
            bw[t].prep(kt0 & 3);
            bcur[t] = bw[t].template frag<KH>();
        }

        int slot = 0;
        for (int kt = kt0; kt < kt1; ++kt) {
            int nslot = slot + 1;
            if (nslot == NS) nslot = 0;
            const char* sb = smem + slot * STAGE;
            const char* nb = smem + nslot * STAGE;
            if (kt + 1 < kt1) {
                // tile kt+1 landed (at most min(kt1-1, kt+NS-2) - (kt+1) tiles still in flight behind it);
                // every wave is past tile kt-1 (all its reads consumed), so that slot takes tile kt+NS-1
                qmm_wait_ahead<NI, NS - 3>(min(kt1 - 1, kt + NS - 2) - (kt + 1));
                if (kt + NS - 1 < kt1) {
                    int ns = slot + NS - 1;
                    if (ns >= NS) ns -= NS;
                    issue(kt + NS - 1, ns, WLc{});
                }
            }
            // next-tile reads are unconditional (on the last tile they read a stale slot and are
            // discarded): one straight-line body keeps the compiler's LDS counter exact across the edge
            load_b(nb, bn, (kt + 1) & 3);
            // Each k-step region: issue the A reads of the wave's next k-step, then run this k-step's
            // MFMAs with the B fragment dequantised in the PREVIOUS region, interleaved (sched_group_barrier:
            // one MFMA, then a slice of VALU) with the dequant of the next k-step's fragment — on the last
            // k-step the next tile's scale prep + first fragment — so the VALU issue hides under the
            // matrix pipe instead of serialising in front of it.
#define QMM_KSTEP(J)                                                                                       \
    {                                                                                                      \
        constexpr int S = KH + KS * (J), CUR = (J) & 1;                                                    \
        constexpr bool LAST = S + KS >= 4;                                                                 \
        load_a(LAST ? nb : sb, LAST ? KH : S + KS, ar[CUR ^ 1]);                                           \
        __builtin_amdgcn_sched_barrier(0);                                                                 \
        f16x8 bnx[WN];                                                                                     \
        if constexpr (LAST) {                                                                              \
            _Pragma("unroll") for (int t = 0; t < WN; ++t) {                                               \
                bn[t].prep((kt + 1) & 3);                                                                  \
                bnx[t] = bn[t].template frag<KH>();                                                        \
            }                                                                                              \
        } else {                                                                                           \
            _Pragma("unroll") for (int t = 0; t < WN; ++t) bnx[t] = bw[t].template frag<(LAST ? KH : S + KS)>(); \
        }                                                                                                  \
        _Pragma("unroll") for (int i = 0; i < WM; ++i)                                                     \
            _Pragma("unroll") for (int t = 0; t < WN; ++t) acc[i][t] =                                     \
                __builtin_amdgcn_mfma_f32_32x32x16_f16(ar[CUR][i], bcur[t], acc[i][t], 0, 0, 0);           \
        _Pragma("unroll") for (int i = 0; i < WM * WN; ++i) {                                              \
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                                             \
            __builtin_amdgcn_sched_group_barrier(0x002, (LAST ? 40 : 16) * WN / (WM * WN) + 1, 0);         \
        }                                                                                                  \
        __builtin_amdgcn_sched_barrier(0);                                                                 \
        _Pragma("unroll") for (int t = 0; t < WN; ++t) bcur[t] = bnx[t];                                   \
    }
            QMM_KSTEP(0) QMM_KSTEP(1)
            if constexpr (KS == 1) { QMM_KSTEP(2) QMM_KSTEP(3) }
#undef QMM_KSTEP
            // an even number of k-steps per tile: the next tile's first A fragments are in ar[0] and its
            // first B fragment in bcur
#pragma unroll
            for (int t = 0; t < WN; ++t) bw[t] = bn[t];
            slot = nslot;
        }
    };
    using T_ = std::integral_constant<bool, true>;
    using F_ = std::integral_constant<bool, false>;
    if constexpr (KS == 1) {
        if (WMW == 1 || mw == 0) mainloop(std::integral_constant<int, 0>{}, T_{});
        else mainloop(std::integral_constant<int, 0>{}, F_{});
    } else {
        if (kh == 0) {
            if (WMW == 1 || mw == 0) mainloop(std::integral_constant<int, 0>{}, T_{});
            else mainloop(std::integral_constant<int, 0>{}, F_{});
        } else {
            mainloop(std::integral_constant<int, 1>{}, F_{});
        }
        // sum the two k-step phases: kh = 1 waves park their partials in the (drained) ring
        __syncthreads();
        float* red = (float*)smem + (size_t)(cg * WMW + mw) * (WM * WN * 16 * 64) + lane;
        if (kh == 1) {
#pragma unroll
            for (int i = 0; i < WM; ++i)
#pragma unroll
                for (int t = 0; t < WN; ++t)
#pragma unroll
                    for (int r = 0; r < 16; ++r) red[((i * WN + t) * 16 + r) * 64] = acc[i][t][r];
        }
        __syncthreads();
        if (kh == 1) return;
#pragma unroll
        for (int i = 0; i < WM; ++i)
#pragma unroll
            for (int t = 0; t < WN; ++t)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[i][t][r] += red[((i * WN + t) * 16 + r) * 64];
    }

    // ---- epilogue: 32x32 C/D layout: col = lane & 31, row = 8*(r>>2) + 4*(lane>>5) + (r&3) ----
    const int m_wave = m_base + mw * WM * 32;
#pragma unroll
    for (int t = 0; t < WN; ++t) {
        const int nt = n_wave + 32 * t;
        const int n = nt + col;
        if constexpr (EPI == E16_SWIGLU || EPI == E16_GEGLU) {
            // W rows interleaved in 16-row groups: tile columns 0..15 gate, 16..31 up of the same features
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
            auto roff = [&](int r) { return (size_t)(8 * (r >> 2) + (r & 3)) * ldc; };
            if (m_wave + i * 32 + 32 <= M) {
                // full tile: branch-free, so the RMW loads issue back to back and wait once
                if constexpr (EPI == E16_ADD_F32) {
                    if (splits == 1) {
                        float old[16];
#pragma unroll
                        for (int r = 0; r < 16; ++r) old[r] = cf[roff(r)];
#pragma unroll
                        for (int r = 0; r < 16; ++r) cf[roff(r)] = old[r] + acc[i][t][r];
                    } else {
#pragma unroll
                        for (int r = 0; r < 16; ++r) atomicAdd(cf + roff(r), acc[i][t][r]);
                    }
                } else {
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        if constexpr (EPI == E16_F32) cf[roff(r)] = acc[i][t][r];
                        else ch[roff(r)] = f32_to_act<true>(acc[i][t][r]);
                    }
                }
                continue;
            }
            // partial tile (rows past M): clamp the RMW loads so they still issue together
            float old[16];
            if constexpr (EPI == E16_ADD_F32) {
                if (splits == 1) {
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int rr = min(m0 + 8 * (r >> 2) + (r & 3), M - 1) - m0;
                        old[r] = cf[(size_t)rr * ldc];
                    }
                }
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                if (m0 + 8 * (r >> 2) + (r & 3) >= M) continue;
                const float v = acc[i][t][r];
                if constexpr (EPI == E16_F32) cf[roff(r)] = v;
                else if constexpr (EPI == E16_ACT) ch[roff(r)] = f32_to_act<true>(v);
                else if (splits == 1) cf[roff(r)] = old[r] + v;  // sole owner of the tile: plain RMW
                else atomicAdd(cf + roff(r), v);
            }
        }
    }
}

template <int QT, int WM, int WN, int NW, int KS, int OCC, int EPI, int WMW>
static int launch_qmm(const uint16_t* A, int lda, const uint8_t* W, const uint16_t* WD, int M, int N, int K,
                      int splits, void* C, int ldc, hipStream_t st) {
    using G = QmmGeom<QT, WN>;
    constexpr int BM = 32 * WM * WMW, BN = NW * G::COLS;
    constexpr int STAGE = BM * 128 + NW * G::WBYTES;
    constexpr int NS = QmmRing<QT, WM, WN, NW, OCC, WMW>::STAGES;
    if constexpr (NS < 3 || (KS > 1 && NW * WMW * WM * WN * 16 * 64 * 4 > NS * STAGE)) {
        return (int)hipErrorInvalidValue;  // this format's stage does not fit OCC rings of >= 3 k-tiles
    } else {
    constexpr size_t lds = (size_t)NS * STAGE;
    static_assert(lds * OCC <= 160 * 1024, "LDS");
    const int nkt = K / QMM_KT;
    splits = max(1, min(splits, nkt));
    const int ktps = (nkt + splits - 1) / splits;
    splits = (nkt + ktps - 1) / ktps;  // no empty splits
    const int n_ct = (N + BN - 1) / BN, n_mt = (M + BM - 1) / BM;
    const long nwg = (long)n_ct * splits * n_mt;
    if (nwg <= 0 || nwg > 0x7fffffff) return (int)hipErrorInvalidValue;
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)qmm_kernel<QT, WM, WN, NW, KS, OCC, EPI, WMW>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        attr_set = true;
    }
    qmm_kernel<QT, WM, WN, NW, KS, OCC, EPI, WMW><<<dim3((unsigned)nwg), 64 * NW * KS * WMW, lds, st>>>(
        A, lda, W, WD, M, N, K, n_ct, n_mt, splits, ktps, C, ldc);
    MXK_CHECK_LAUNCH();
    }
}

template <int QT, int EPI>
static int dispatch_qmm(int wm, int wn, int nw, int ks, const uint16_t* A, int lda, const uint8_t* W, const uint16_t* WD,
                        int M, int N, int K, int splits, void* C, int ldc, hipStream_t st) {
    const int occ = 1 + ((ks >> 4) & 1);
    const int wmw = 1 + ((ks >> 5) & 3);
    ks &= 15;
#define QMM_CASE(WM_, WN_, NW_, KS_, OCC_, WMW_)                                                              \
    if (wm == WM_ && wn == WN_ && nw == NW_ && ks == KS_ && occ == OCC_ && wmw == WMW_)                       \
        return launch_qmm<QT, WM_, WN_, NW_, KS_, OCC_, EPI, WMW_>(A, lda, W, WD, M, N, K, splits, C, ldc, st);
    QMM_CASE(1, 1, 4, 1, 1, 1) QMM_CASE(2, 1, 4, 1, 1, 1) QMM_CASE(4, 1, 4, 1, 1, 1) QMM_CASE(1, 2, 4, 1, 1, 1)
    QMM_CASE(2, 2, 4, 1, 1, 1) QMM_CASE(4, 2, 4, 1, 1, 1) QMM_CASE(2, 1, 8, 1, 1, 1) QMM_CASE(4, 1, 8, 1, 1, 1)
    QMM_CASE(2, 2, 8, 1, 1, 1) QMM_CASE(4, 2, 8, 1, 1, 1) QMM_CASE(2, 1, 4, 2, 1, 1) QMM_CASE(4, 1, 4, 2, 1, 1)
    QMM_CASE(2, 2, 4, 2, 1, 1)
    // two workgroups per CU (half-LDS ring)
    QMM_CASE(2, 1, 4, 1, 2, 1) QMM_CASE(4, 1, 4, 1, 2, 1) QMM_CASE(2, 2, 4, 1, 2, 1) QMM_CASE(2, 1, 4, 2, 2, 1)
    // row-split wave grids (WMW waves along M): 64x64 / 128x64 / 64x32 / 128x32 wave tiles
    QMM_CASE(2, 2, 2, 1, 1, 2) QMM_CASE(4, 2, 2, 1, 1, 2) QMM_CASE(2, 2, 2, 2, 1, 2) QMM_CASE(2, 1, 4, 1, 1, 2)
    QMM_CASE(4, 1, 4, 1, 1, 2) QMM_CASE(2, 2, 4, 1, 1, 2) QMM_CASE(4, 2, 4, 1, 1, 2) QMM_CASE(1, 2, 4, 1, 1, 2)
    QMM_CASE(2, 2, 2, 1, 2, 2) QMM_CASE(1, 2, 2, 1, 1, 4) QMM_CASE(2, 2, 2, 1, 1, 4)
#undef QMM_CASE
    return (int)hipErrorInvalidValue;
}

// A must be f16 (act16 mode f16), 16-B aligned rows (lda % 8 == 0); K % 256 == 0; W in the t32 tiled
// layout (N % 32 == 0; WD unused). epi: 0 fp32 store, 1 act16 store, 2 fp32 accumulate (split-K via
// atomics when splits > 1), 3/4 SwiGLU/GeGLU over 16-row interleaved gate/up -> act16 [M, N/2].
// (wm, wn, nw, ks): 32*wm-row x 32*wn*nw-column tiles, nw*ks waves (ks waves per column group split the
// k-steps; nw*ks = 8 -> 2 waves per SIMD, whose dequant / LDS phases overlap each other's MFMAs).
// ks | 16: the half-LDS ring variant, two workgroups resident per CU.
extern "C" int mxk_qmm(int qtype, int epi, int wm, int wn, int nw, int ks, const uint16_t* A, int lda, const uint8_t* W,
                       const uint16_t* WD, int M, int N, int K, int splits, void* C, int ldc, hipStream_t st) {
    if (M <= 0) return 0;
    if (K % 256 || (lda & 7) || ((uintptr_t)A & 15) || ((uintptr_t)W & 15)) return (int)hipErrorInvalidValue;
    if (epi != E16_ADD_F32 && splits != 1) return (int)hipErrorInvalidValue;
    if (N & 31) return (int)hipErrorInvalidValue;
#define QMM_EPI(QT_)                                                                                                \
    switch (epi) {                                                                                                  \
        case E16_F32: return dispatch_qmm<QT_, E16_F32>(wm, wn, nw, ks, A, lda, W, WD, M, N, K, splits, C, ldc, st);         \
        case E16_ACT: return dispatch_qmm<QT_, E16_ACT>(wm, wn, nw, ks, A, lda, W, WD, M, N, K, splits, C, ldc, st);         \
        case E16_ADD_F32: return dispatch_qmm<QT_, E16_ADD_F32>(wm, wn, nw, ks, A, lda, W, WD, M, N, K, splits, C, ldc, st); \
        case E16_SWIGLU: return dispatch_qmm<QT_, E16_SWIGLU>(wm, wn, nw, ks, A, lda, W, WD, M, N, K, splits, C, ldc, st);   \
        case E16_GEGLU: return dispatch_qmm<QT_, E16_GEGLU>(wm, wn, nw, ks, A, lda, W, WD, M, N, K, splits, C, ldc, st);     \
    }
    switch (qtype) {
        case MXQ_Q4_K: QMM_EPI(MXQ_Q4_K) break;
        case MXQ_Q6_K: QMM_EPI(MXQ_Q6_K) break;
        case MXQ_Q8_0: QMM_EPI(MXQ_Q8_0) break;
        case MXQ_MX4F: QMM_EPI(MXQ_MX4F) break;
        case MXQ_MX5F: QMM_EPI(MXQ_MX5F) break;
    }
#undef QMM_EPI
    return (int)hipErrorInvalidValue;
}

