// qgemm16.hip — quantised-weight GEMM for decode-sized batches (16 < M <= ~256) with f16 operands.
//
//   C[M, N] (+)= A[M, K] · W[N, K]^T,   A f16 (act16 mode), W in Q4_K / Q6_K(repacked) / Q8_0(repacked)
//
// Why a second MFMA kernel: at decode batch sizes the bf16 variant (qgemm.hip) is VALU-bound on
// dequantisation (~3.8 VALU per weight; 489 VALU vs 128 MFMA per k-block at WM=8, WN=2, 328 VGPRs).
// Here every weight is dequantised with PACKED f16 math:
//   * the 4/6/8-bit codes are placed into f16 mantissas with one v_perm_b32 per 2 weights
//     (bit pattern 0x6400|q == 1024 + q exactly: the "magic number" conversion),
//   * v_pk_add_f16 removes the 1024 (+ the Q6_K/Q8_0 code offset) exactly,
//   * v_pk_fma_f16 / v_pk_mul_f16 applies the super-block scale and min,
// i.e. 1.5-2 VALU per weight, and f16 (11-bit mantissa) is a closer dequantised value than bf16.
// MFMA: v_mfma_f32_16x16x32_f16 (same rate as bf16). A tile staged once per workgroup into the
// same XOR-swizzled LDS image as qgemm.hip (conflict-free ds_read_b128); W fragments are loaded
// straight to registers one k-block ahead. The virtual-k relabelling is the one of qgemm.hip (lane
// group g owns elements [64g, 64g+64) of each 256-element super-block; MFMA k-step ks consumes
// 64g + 8ks + j on both operands), so the reduction over k is unchanged.
// Split-K over the grid's y dimension (fp32 atomics into a zeroed C) fills the 256 CUs when N is
// small; the 4 waves of a workgroup split N.
#include "mx_common.h"

#include "qdeq16.h"

MX_DEV int a16_lds_off(int r, int c) {
    const int rr = r & 15;
    return r * 512 + ((c ^ (rr ^ ((rr + 4) & 8))) << 4);
}

// Grouped mode (GR, mixture-of-experts): rows of A are token-expert pairs sorted by expert
// (moe.hip moe_sort); expert e owns sorted rows [off[e], off[e+1]) and weight rows [e*N, (e+1)*N)
// of one stacked [E*N, K] matrix. blockIdx.z walks a compacted tile list: tile_start[e] is the
// prefix sum of ceil(rows_e / BM) (computed on the device by moe_sort for this BM), so a launch
// sized for the worst case (ceil(P/BM) + E tiles) needs no host round-trip and stays inside a
// captured hipGraph; surplus workgroups exit at once. `a_rows` (optional) gathers A rows through
// an index (pair -> token row), so the router's input is never copied per expert.
struct MoeGroups {
    const int* a_rows;      // [P] A row of sorted pair p, or null (A already in sorted order)
    const int* off;         // [E+1] sorted-row offsets per expert
    const int* tile_start;  // [E+1] tile prefix sums for this BM
    int E;
};

template <int QT, int WM, int WN, int EPI, bool GR = false>
__global__ __launch_bounds__(256, (WM >= 8 ? 1 : 2)) void qgemm16_kernel(const uint16_t* __restrict__ A, int lda,
                                                         const uint8_t* __restrict__ W,
                                                         const uint16_t* __restrict__ WD, int M, int N, int K,
                                                         int kb_per_split, void* __restrict__ Cv, int ldc,
                                                         MoeGroups grp = {}) {
    constexpr int BM = WM * 16;
    constexpr int A_BYTES = BM * 512;
    constexpr int A_PASSES = BM * 32 / 256;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int g = lane >> 4, col = lane & 15;
    const int nblk = K >> 8;
    const int n_base = (blockIdx.x * 4 + wave) * (WN * 16);
    int m_base = blockIdx.z * BM;
    int m_end = M, n_row0 = 0;
    if constexpr (GR) {
        const int z = blockIdx.z;
        if (z >= grp.tile_start[grp.E]) return;
        int lo = 0, hi = grp.E;  // largest e with tile_start[e] <= z (empty experts have equal starts)
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (grp.tile_start[mid] <= z) lo = mid;
            else hi = mid;
        }
        m_base = grp.off[lo] + (z - grp.tile_start[lo]) * BM;
        m_end = grp.off[lo + 1];
        n_row0 = lo * N;
    }
    const int kb0 = blockIdx.y * kb_per_split;
    const int kb1 = min(kb0 + kb_per_split, nblk);
    if (kb0 >= kb1) return;

    f32x4 acc[WM][WN];
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
        for (int t = 0; t < WN; ++t) acc[i][t] = (f32x4){0.f, 0.f, 0.f, 0.f};

    u32x4 areg[A_PASSES];
    auto load_a = [&](int kb) {
#pragma unroll
        for (int p = 0; p < A_PASSES; ++p) {
            const int id = p * 256 + threadIdx.x;
            const int r = id >> 5, c = id & 31;
            const int m = m_base + r;
            const int ar = (GR && grp.a_rows) ? (m < m_end ? grp.a_rows[m] : 0) : m;
            if (m < m_end) areg[p] = *(const u32x4*)(A + (size_t)ar * lda + (size_t)kb * 256 + c * 8);
            else areg[p] = (u32x4){0, 0, 0, 0};
        }
    };
    auto store_a = [&](int buf) {
#pragma unroll
        for (int p = 0; p < A_PASSES; ++p) {
            const int id = p * 256 + threadIdx.x;
            *(u32x4*)(smem + buf * A_BYTES + a16_lds_off(id >> 5, id & 31)) = areg[p];
        }
    };
    W16<QT> wf[WN], wn[WN];
    auto load_w = [&](W16<QT>(&f)[WN], int kb) {
#pragma unroll
        for (int t = 0; t < WN; ++t) {
            const int n = n_base + t * 16 + col;
            if (n < N) f[t].load(W, WD, n_row0 + n, kb, nblk, g);
            else f[t].zero();
        }
    };

    load_a(kb0);
    load_w(wf, kb0);
    store_a(0);
    __syncthreads();
    int buf = 0;
    for (int kb = kb0; kb < kb1; ++kb) {
        const bool more = kb + 1 < kb1;
        if (more) {
            load_a(kb + 1);
            load_w(wn, kb + 1);
        }
#pragma unroll
        for (int t = 0; t < WN; ++t) wf[t].prep(g);
        const char* abuf = smem + buf * A_BYTES;
#define Q16_KSTEP(KS)                                                                                    \
    {                                                                                                    \
        f16x8 bfr[WN];                                                                                   \
        _Pragma("unroll") for (int t = 0; t < WN; ++t) bfr[t] = wf[t].template frag<KS>();              \
        _Pragma("unroll") for (int i = 0; i < WM; ++i) {                                                 \
            const f16x8 af = *(const f16x8*)(abuf + a16_lds_off(i * 16 + col, 8 * g + KS));             \
            _Pragma("unroll") for (int t = 0; t < WN; ++t) acc[i][t] =                                   \
                __builtin_amdgcn_mfma_f32_16x16x32_f16(af, bfr[t], acc[i][t], 0, 0, 0);                  \
        }                                                                                                \
    }
        Q16_KSTEP(0) Q16_KSTEP(1) Q16_KSTEP(2) Q16_KSTEP(3) Q16_KSTEP(4) Q16_KSTEP(5) Q16_KSTEP(6) Q16_KSTEP(7)
#undef Q16_KSTEP
        if (more) {
            store_a(buf ^ 1);
#pragma unroll
            for (int t = 0; t < WN; ++t) wf[t] = wn[t];
        }
        __syncthreads();
        buf ^= 1;
    }

    // epilogue: C/D layout col = lane&15, row = 4*(lane>>4) + e
#pragma unroll
    for (int i = 0; i < WM; ++i) {
#pragma unroll
        for (int t = 0; t < WN; ++t) {
            if constexpr (EPI == E16_SWIGLU || EPI == E16_GEGLU) {
                if (t & 1) continue;
                const int feat = (n_base >> 1) + (t >> 1) * 16 + col;
                if (n_base + t * 16 + col >= N) continue;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int m = m_base + i * 16 + 4 * g + e;
                    if (m < m_end) {
                        const float gv = acc[i][t][e], uv = acc[i][t + 1][e];
                        ((uint16_t*)Cv)[(size_t)m * ldc + feat] = f32_to_act<true>(glu_gate_f<EPI>(gv) * uv);
                    }
                }
            } else {
                const int n = n_base + t * 16 + col;
                if (n >= N) continue;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int m = m_base + i * 16 + 4 * g + e;
                    if (m >= m_end) continue;
                    const float v = acc[i][t][e];
                    if constexpr (EPI == E16_F32) ((float*)Cv)[(size_t)m * ldc + n] = v;
                    else if constexpr (EPI == E16_ACT) ((uint16_t*)Cv)[(size_t)m * ldc + n] = f32_to_act<true>(v);
                    else atomicAdd(((float*)Cv) + (size_t)m * ldc + n, v);
                }
            }
        }
    }
}

template <int QT, int WM, int WN, int EPI>
static int launch16(const uint16_t* A, int lda, const uint8_t* W, const uint16_t* WD, int M, int N, int K, int splits,
                    void* C, int ldc, hipStream_t st) {
    const int nblk = K / 256;
    const int kbs = (nblk + splits - 1) / splits;
    dim3 grid((N + 64 * WN - 1) / (64 * WN), splits, (M + WM * 16 - 1) / (WM * 16));
    const size_t lds = 2 * WM * 16 * 512;
    qgemm16_kernel<QT, WM, WN, EPI><<<grid, 256, lds, st>>>(A, lda, W, WD, M, N, K, kbs, C, ldc);
    MXK_CHECK_LAUNCH();
}

template <int QT, int EPI>
static int dispatch16(int wm, int wn, const uint16_t* A, int lda, const uint8_t* W, const uint16_t* WD, int M, int N,
                      int K, int splits, void* C, int ldc, hipStream_t st) {
    if (QT == MXQ_Q8_0 && wn > 2) wn = 2;
#define Q16_CASE(WM_, WN_) \
    if (wm == WM_ && wn == WN_) return launch16<QT, WM_, WN_, EPI>(A, lda, W, WD, M, N, K, splits, C, ldc, st);
    Q16_CASE(1, 2) Q16_CASE(2, 2) Q16_CASE(4, 2) Q16_CASE(8, 2) Q16_CASE(4, 4) Q16_CASE(2, 4) Q16_CASE(4, 1)
    Q16_CASE(8, 1)
#undef Q16_CASE
    return (int)hipErrorInvalidValue;
}

// A must be f16 (act16 mode). epi: 0 fp32 store, 1 act16 store, 2 fp32 atomic accumulate,
// 3 SwiGLU (16-row interleaved gate/up) -> act16. splits > 1 only with epi 2 (or 0 into a zeroed C,
// which the host maps to 2).
extern "C" int mxk_qgemm16(int qtype, int epi, int wm, int wn, const uint16_t* A, int lda, const uint8_t* W,
                           const uint16_t* WD, int M, int N, int K, int splits, void* C, int ldc, hipStream_t st) {
    if (M <= 0) return 0;
    if (K % 256) return (int)hipErrorInvalidValue;
    if ((epi == E16_SWIGLU || epi == E16_GEGLU || epi == E16_ACT || epi == E16_F32) && splits != 1) return (int)hipErrorInvalidValue;
    if ((epi == E16_SWIGLU || epi == E16_GEGLU) && (wn & 1)) return (int)hipErrorInvalidValue;
#define Q16_EPI(QT_)                                                                                          \
    switch (epi) {                                                                                            \
        case E16_F32: return dispatch16<QT_, E16_F32>(wm, wn, A, lda, W, WD, M, N, K, splits, C, ldc, st);         \
        case E16_ACT: return dispatch16<QT_, E16_ACT>(wm, wn, A, lda, W, WD, M, N, K, splits, C, ldc, st);         \
        case E16_ADD_F32: return dispatch16<QT_, E16_ADD_F32>(wm, wn, A, lda, W, WD, M, N, K, splits, C, ldc, st); \
        case E16_SWIGLU: return dispatch16<QT_, E16_SWIGLU>(wm, wn, A, lda, W, WD, M, N, K, splits, C, ldc, st);   \
        case E16_GEGLU: return dispatch16<QT_, E16_GEGLU>(wm, wn, A, lda, W, WD, M, N, K, splits, C, ldc, st);     \
    }
    switch (qtype) {
        case MXQ_Q4_K: Q16_EPI(MXQ_Q4_K) break;
        case MXQ_Q6_K: Q16_EPI(MXQ_Q6_K) break;
        case MXQ_Q8_0: Q16_EPI(MXQ_Q8_0) break;
    }
#undef Q16_EPI
    return (int)hipErrorInvalidValue;
}

// ---------------------------------------------------------------------------------------------
// Grouped (MoE) entry: P sorted token-expert rows, per-expert N x K weights stacked in W.
// epi: E16_SWIGLU (gate|up interleaved per expert, act16 out [P, N/2]) or E16_F32 / E16_ACT.
template <int QT, int EPI>
static int launch16g(int wm, const uint16_t* A, int lda, const int* a_rows, const uint8_t* W, const uint16_t* WD,
                     const int* off, const int* tile_start, int E, int P, int N, int K, void* C, int ldc,
                     hipStream_t st) {
    const int BM = wm * 16;
    const int max_tiles = (P + BM - 1) / BM + (E < P ? E : P);
    dim3 grid((N + 127) / 128, 1, max_tiles);
    MoeGroups g{a_rows, off, tile_start, E};
    const size_t lds = 2 * BM * 512;
#define Q16G(WM_)                                                                                     \
    if (wm == WM_) {                                                                                  \
        qgemm16_kernel<QT, WM_, 2, EPI, true><<<grid, 256, lds, st>>>(A, lda, W, WD, P, N, K, K / 256, C, ldc, g); \
        MXK_CHECK_LAUNCH();                                                                           \
    }
    Q16G(1) Q16G(2) Q16G(4)
#undef Q16G
    return (int)hipErrorInvalidValue;
}

extern "C" int mxk_moe_qgemm16(int qtype, int epi, int wm, const uint16_t* A, int lda, const int* a_rows,
                               const uint8_t* W, const uint16_t* WD, const int* off, const int* tile_start, int E,
                               int P, int N, int K, void* C, int ldc, hipStream_t st) {
    if (P <= 0) return 0;
    if (K % 256 || N % 32) return (int)hipErrorInvalidValue;
#define Q16G_EPI(QT_)                                                                                               \
    switch (epi) {                                                                                                  \
        case E16_F32: return launch16g<QT_, E16_F32>(wm, A, lda, a_rows, W, WD, off, tile_start, E, P, N, K, C, ldc, st); \
        case E16_ACT: return launch16g<QT_, E16_ACT>(wm, A, lda, a_rows, W, WD, off, tile_start, E, P, N, K, C, ldc, st); \
        case E16_SWIGLU:                                                                                            \
            return launch16g<QT_, E16_SWIGLU>(wm, A, lda, a_rows, W, WD, off, tile_start, E, P, N, K, C, ldc, st);  \
        case E16_GEGLU:                                                                                             \
            return launch16g<QT_, E16_GEGLU>(wm, A, lda, a_rows, W, WD, off, tile_start, E, P, N, K, C, ldc, st);   \
    }
    switch (qtype) {
        case MXQ_Q4_K: Q16G_EPI(MXQ_Q4_K) break;
        case MXQ_Q6_K: Q16G_EPI(MXQ_Q6_K) break;
        case MXQ_Q8_0: Q16G_EPI(MXQ_Q8_0) break;
    }
#undef Q16G_EPI
    return (int)hipErrorInvalidValue;
}
