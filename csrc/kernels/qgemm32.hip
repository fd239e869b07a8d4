// qgemm32.hip — quantised-weight GEMM on 32x32x16 f16 MFMA tiles for decode / mixed batches
// (M ~ 64..256), the shape class that dominates continuous-batching decode steps.
//
//   C[M, N] (+)= A[M, K] · W[N, K]^T,   A f16 (act16 mode), W in Q4_K / Q6_K(repacked) / Q8_0(repacked)
//
// Why 32x32 tiles: with 16x16x32 tiles (qgemm16.hip) one dequantised B fragment (8 weights per lane,
// ~16 packed-f16 VALU ops) feeds WM 16-cycle MFMAs, and at WM = 4 the dequantisation VALU plus the
// MFMA-held issue slots exceed the MFMA time (VALU-bound). A 32x32x16 MFMA consumes the same
// 8 weights per lane for twice the FLOPs (32 cycles), so one fragment feeds WM x 32 cycles of matrix
// work and the dequantisation hides in the free issue slots; the A operand is read from LDS at half
// the bytes per FLOP.
//
// Virtual-k: lane group h = lane >> 5 owns elements [128h, 128h + 128) of every 256-element
// super-block (two "quarters" 2h, 2h+1 in the qgemm16 layouts, so the W16 decoders are reused);
// MFMA k-step ks (0..15) consumes elements 128h + 8ks + j on both operands. A k-block's A tile
// (BM x 256 f16) is staged once per workgroup into an XOR-swizzled LDS image (16-B chunk c of row r at
// chunk c ^ (r & 7): the 8 rows a ds_read_b128 lane group touches hit distinct banks) and shared by
// the 4 waves, which split N (32 columns each). Split-K over grid.y accumulates with fp32 atomics.
#include "qdeq16.h"

MX_DEV int a32_lds_off(int r, int c) { return r * 512 + ((c ^ (r & 15)) << 4); }

template <int QT, int WM, int WN, int EPI>
__global__ __launch_bounds__(256, 1) __attribute__((amdgpu_waves_per_eu(1, 1))) void qgemm32_kernel(const uint16_t* __restrict__ A, int lda,
                                                          const uint8_t* __restrict__ W,
                                                          const uint16_t* __restrict__ WD, int M, int N, int K,
                                                          int kb_per_split, void* __restrict__ Cv, int ldc) {
    constexpr int BM = WM * 32;
    constexpr int A_BYTES = BM * 512;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int h = lane >> 5, col = lane & 31;
    const int nblk = K >> 8;
    const int n_base = (blockIdx.x * 4 + wave) * 32 * WN;
    const int m_base = blockIdx.z * BM;
    const int kb0 = blockIdx.y * kb_per_split;
    const int kb1 = min(kb0 + kb_per_split, nblk);
    if (kb0 >= kb1) return;

    f32x16 acc[WM][WN];
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
        for (int t = 0; t < WN; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][t][r] = 0.f;

    // A staging: global -> LDS directly (global_load_lds, 16 B per lane). The LDS image is lane-linear
    // per wave-instruction, so the XOR swizzle is applied to the SOURCE address: LDS chunk p (row
    // p / 32, physical chunk p % 32) receives logical chunk (p % 32) ^ (row & 7).
    constexpr int G_PER_WAVE = BM / 8;  // 1 KB wave-instructions per wave per k-block
    uint32_t aoff[G_PER_WAVE];          // per-lane source element offsets (k-block 0), computed once
#pragma unroll
    for (int j = 0; j < G_PER_WAVE; ++j) {
        const int p = (wave * G_PER_WAVE + j) * 64 + lane;
        const int r = p >> 5, c = (p & 31) ^ (r & 15);
        const int m = min(m_base + r, M - 1);  // rows past M compute garbage that is never stored
        aoff[j] = (uint32_t)(m * lda + c * 8);
    }
    auto stage_a = [&](int kb, int buf) {
        char* base = smem + buf * A_BYTES + wave * G_PER_WAVE * 1024;
        const uint16_t* ak = A + (size_t)kb * 256;
#pragma unroll
        for (int j = 0; j < G_PER_WAVE; ++j)
            __builtin_amdgcn_global_load_lds((const void*)(ak + aoff[j]),
                                             (__attribute__((address_space(3))) void*)(base + j * 1024), 16, 0, 0);
    };
    constexpr int WPF = 1;
    W16<QT> w0[WN][2], w1[WN][2];
    auto load_w = [&](W16<QT>(&f)[WN][2], int kb) {
#pragma unroll
        for (int t = 0; t < WN; ++t) {
            const int n = n_base + 32 * t + col;
            if (n < N) {
                f[t][0].load(W, WD, n, kb, nblk, 2 * h);
                f[t][1].load(W, WD, n, kb, nblk, 2 * h + 1);
            } else {
                f[t][0].zero();
                f[t][1].zero();
            }
        }
    };

    // k-block body; the two W register sets swap roles statically (loop unrolled by 2) so no
    // register copy ties the next block's loads to the middle of this block's compute.
    auto body = [&](W16<QT>(&cur)[WN][2], W16<QT>(&nxt)[WN][2], int kb, int buf) {
        if (kb + 1 < kb1) stage_a(kb + 1, buf ^ 1);
        if (kb + WPF < kb1) load_w(nxt, kb + WPF);  // W register ring: WPF blocks ahead
#pragma unroll
        for (int t = 0; t < WN; ++t) {
            cur[t][0].prep(2 * h);
            cur[t][1].prep(2 * h + 1);
        }
        const char* abuf = smem + buf * A_BYTES;
        // Software pipeline over the 16 k-steps: step ks issues the LDS reads of A(ks+1) and the
        // dequantisation of B(ks+1) between its own WM x WN MFMAs (sched_group_barrier pins the
        // interleave; left alone the scheduler sinks the reads next to their use and every MFMA
        // waits a full LDS latency).
        f16x8 a0[WM], a1[WM], b0[WN], b1[WN];
#pragma unroll
        for (int i = 0; i < WM; ++i) a0[i] = *(const f16x8*)(abuf + a32_lds_off(i * 32 + col, 16 * h));
#pragma unroll
        for (int t = 0; t < WN; ++t) b0[t] = cur[t][0].template frag<0>();
#define Q32_KSTEP(KS, AC, BC, AN, BN)                                                                      \
    {                                                                                                      \
        if constexpr ((KS) < 15) {                                                                         \
            _Pragma("unroll") for (int i = 0; i < WM; ++i) AN[i] =                                         \
                *(const f16x8*)(abuf + a32_lds_off(i * 32 + col, 16 * h + (KS) + 1));                     \
            _Pragma("unroll") for (int t = 0; t < WN; ++t) BN[t] =                                         \
                cur[t][((KS) + 1) >> 3].template frag<((KS) + 1) & 7>();                                   \
        }                                                                                                  \
        _Pragma("unroll") for (int i = 0; i < WM; ++i)                                                     \
            _Pragma("unroll") for (int t = 0; t < WN; ++t) acc[i][t] =                                     \
                __builtin_amdgcn_mfma_f32_32x32x16_f16(AC[i], BC[t], acc[i][t], 0, 0, 0);                  \
        if constexpr ((KS) < 15) __builtin_amdgcn_sched_group_barrier(0x100, WM, 0);                      \
        _Pragma("unroll") for (int i = 0; i < WM * WN; ++i) {                                              \
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                                             \
            if constexpr ((KS) < 15)                                                                       \
                __builtin_amdgcn_sched_group_barrier(0x002, (16 * WN + WM * WN - 1) / (WM * WN), 0);       \
        }                                                                                                  \
    }
        Q32_KSTEP(0, a0, b0, a1, b1) Q32_KSTEP(1, a1, b1, a0, b0) Q32_KSTEP(2, a0, b0, a1, b1)
        Q32_KSTEP(3, a1, b1, a0, b0) Q32_KSTEP(4, a0, b0, a1, b1) Q32_KSTEP(5, a1, b1, a0, b0)
        Q32_KSTEP(6, a0, b0, a1, b1) Q32_KSTEP(7, a1, b1, a0, b0) Q32_KSTEP(8, a0, b0, a1, b1)
        Q32_KSTEP(9, a1, b1, a0, b0) Q32_KSTEP(10, a0, b0, a1, b1) Q32_KSTEP(11, a1, b1, a0, b0)
        Q32_KSTEP(12, a0, b0, a1, b1) Q32_KSTEP(13, a1, b1, a0, b0) Q32_KSTEP(14, a0, b0, a1, b1)
        Q32_KSTEP(15, a1, b1, a0, b0)
#undef Q32_KSTEP
        __syncthreads();  // drains the k+1 global_load_lds / W loads (vmcnt(0)) and orders LDS reuse
    };
    stage_a(kb0, 0);
    load_w(w0, kb0);
    __syncthreads();
    int buf = 0;
    for (int kb = kb0; kb < kb1; ++kb) {
        body(w0, w1, kb, buf);
        // keep the register hand-over after the block's MFMAs: hoisted, it would wait (vmcnt) for the
        // next block's loads in the middle of this block's compute
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int t = 0; t < WN; ++t) {
            w0[t][0] = w1[t][0];
            w0[t][1] = w1[t][1];
        }
        buf ^= 1;
    }

    // epilogue: 32x32 C/D layout: col = lane & 31, row = 8*(r>>2) + 4*(lane>>5) + (r&3)
#pragma unroll
    for (int t = 0; t < WN; ++t) {
        const int nt = n_base + 32 * t;
        const int n = nt + col;
        if constexpr (EPI == E16_SWIGLU || EPI == E16_GEGLU) {
            // W rows interleaved in 16-row groups: tile columns 0..15 gate, 16..31 up of the same features
#pragma unroll
            for (int i = 0; i < WM; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const float v = acc[i][t][r];
                    const float up = __shfl_xor(v, 16);
                    const int m = m_base + i * 32 + 8 * (r >> 2) + 4 * h + (r & 3);
                    if (col < 16 && n < N && m < M)
                        ((uint16_t*)Cv)[(size_t)m * ldc + (nt >> 1) + col] = f32_to_act<true>(glu_gate_f<EPI>(v) * up);
                }
            continue;
        }
        if (n >= N) continue;
#pragma unroll
        for (int i = 0; i < WM; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m_base + i * 32 + 8 * (r >> 2) + 4 * h + (r & 3);
                if (m >= M) continue;
                const float v = acc[i][t][r];
                if constexpr (EPI == E16_F32) ((float*)Cv)[(size_t)m * ldc + n] = v;
                else if constexpr (EPI == E16_ACT) ((uint16_t*)Cv)[(size_t)m * ldc + n] = f32_to_act<true>(v);
                else atomicAdd(((float*)Cv) + (size_t)m * ldc + n, v);
            }
    }
}

template <int QT, int WM, int WN, int EPI>
static int launch32(const uint16_t* A, int lda, const uint8_t* W, const uint16_t* WD, int M, int N, int K, int splits,
                    void* C, int ldc, hipStream_t st) {
    const int nblk = K / 256;
    const int kbs = (nblk + splits - 1) / splits;
    dim3 grid((N + 128 * WN - 1) / (128 * WN), splits, (M + WM * 32 - 1) / (WM * 32));
    const size_t lds = 2 * WM * 32 * 512;
    if constexpr (QT != MXQ_Q4_K && WM * WN > 4) return (int)hipErrorInvalidValue;  // register-bound
    else qgemm32_kernel<QT, WM, WN, EPI><<<grid, 256, lds, st>>>(A, lda, W, WD, M, N, K, kbs, C, ldc);
    MXK_CHECK_LAUNCH();
}

template <int QT, int EPI>
static int dispatch32(int wm, int wn, const uint16_t* A, int lda, const uint8_t* W, const uint16_t* WD, int M,
                      int N, int K, int splits, void* C, int ldc, hipStream_t st) {
    if (QT != MXQ_Q4_K && wm * wn > 4) wn = 1;  // Q6_K / Q8_0 fragments need more registers (spills)
#define Q32_CASE(WM_, WN_) \
    if (wm == WM_ && wn == WN_) return launch32<QT, WM_, WN_, EPI>(A, lda, W, WD, M, N, K, splits, C, ldc, st);
    Q32_CASE(1, 1) Q32_CASE(2, 1) Q32_CASE(4, 1) Q32_CASE(1, 2) Q32_CASE(2, 2) Q32_CASE(4, 2)
#undef Q32_CASE
    return (int)hipErrorInvalidValue;
}

// A must be f16 (act16 mode f16). epi as mxk_qgemm16: 0 fp32 store, 1 act16 store, 2 fp32 atomic
// accumulate (split-K allowed), 3 SwiGLU over 16-row interleaved gate/up -> act16.
extern "C" int mxk_qgemm32(int qtype, int epi, int wm, int wn, const uint16_t* A, int lda, const uint8_t* W,
                           const uint16_t* WD, int M, int N, int K, int splits, void* C, int ldc, hipStream_t st) {
    if (M <= 0) return 0;
    if (K % 256 || (lda & 7)) return (int)hipErrorInvalidValue;
    if (epi != E16_ADD_F32 && splits != 1) return (int)hipErrorInvalidValue;
    if ((epi == E16_SWIGLU || epi == E16_GEGLU) && (N & 31)) return (int)hipErrorInvalidValue;
#define Q32_EPI(QT_)                                                                                       \
    switch (epi) {                                                                                         \
        case E16_F32: return dispatch32<QT_, E16_F32>(wm, wn, A, lda, W, WD, M, N, K, splits, C, ldc, st);         \
        case E16_ACT: return dispatch32<QT_, E16_ACT>(wm, wn, A, lda, W, WD, M, N, K, splits, C, ldc, st);         \
        case E16_ADD_F32: return dispatch32<QT_, E16_ADD_F32>(wm, wn, A, lda, W, WD, M, N, K, splits, C, ldc, st); \
        case E16_SWIGLU: return dispatch32<QT_, E16_SWIGLU>(wm, wn, A, lda, W, WD, M, N, K, splits, C, ldc, st);   \
        case E16_GEGLU: return dispatch32<QT_, E16_GEGLU>(wm, wn, A, lda, W, WD, M, N, K, splits, C, ldc, st);     \
    }
    switch (qtype) {
        case MXQ_Q4_K: Q32_EPI(MXQ_Q4_K) break;
        case MXQ_Q6_K: Q32_EPI(MXQ_Q6_K) break;
        case MXQ_Q8_0: Q32_EPI(MXQ_Q8_0) break;
    }
#undef Q32_EPI
    return (int)hipErrorInvalidValue;
}
