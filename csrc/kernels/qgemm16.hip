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

enum { E16_F32 = 0, E16_ACT = 1, E16_ADD_F32 = 2, E16_SWIGLU = 3 };

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

MX_DEV int a16_lds_off(int r, int c) {
    const int rr = r & 15;
    return r * 512 + ((c ^ (rr ^ ((rr + 4) & 8))) << 4);
}

template <int QT, int WM, int WN, int EPI>
__global__ __launch_bounds__(256, (WM >= 8 ? 1 : 2)) void qgemm16_kernel(const uint16_t* __restrict__ A, int lda,
                                                         const uint8_t* __restrict__ W,
                                                         const uint16_t* __restrict__ WD, int M, int N, int K,
                                                         int kb_per_split, void* __restrict__ Cv, int ldc) {
    constexpr int BM = WM * 16;
    constexpr int A_BYTES = BM * 512;
    constexpr int A_PASSES = BM * 32 / 256;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int g = lane >> 4, col = lane & 15;
    const int nblk = K >> 8;
    const int n_base = (blockIdx.x * 4 + wave) * (WN * 16);
    const int m_base = blockIdx.z * BM;
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
            if (m < M) areg[p] = *(const u32x4*)(A + (size_t)m * lda + (size_t)kb * 256 + c * 8);
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
            if (n < N) f[t].load(W, WD, n, kb, nblk, g);
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
            if constexpr (EPI == E16_SWIGLU) {
                if (t & 1) continue;
                const int feat = (n_base >> 1) + (t >> 1) * 16 + col;
                if (n_base + t * 16 + col >= N) continue;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int m = m_base + i * 16 + 4 * g + e;
                    if (m < M) {
                        const float gv = acc[i][t][e], uv = acc[i][t + 1][e];
                        ((uint16_t*)Cv)[(size_t)m * ldc + feat] = f32_to_act<true>(silu_f(gv) * uv);
                    }
                }
            } else {
                const int n = n_base + t * 16 + col;
                if (n >= N) continue;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int m = m_base + i * 16 + 4 * g + e;
                    if (m >= M) continue;
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
    if ((epi == E16_SWIGLU || epi == E16_ACT || epi == E16_F32) && splits != 1) return (int)hipErrorInvalidValue;
    if (epi == E16_SWIGLU && (wn & 1)) return (int)hipErrorInvalidValue;
#define Q16_EPI(QT_)                                                                                          \
    switch (epi) {                                                                                            \
        case E16_F32: return dispatch16<QT_, E16_F32>(wm, wn, A, lda, W, WD, M, N, K, splits, C, ldc, st);         \
        case E16_ACT: return dispatch16<QT_, E16_ACT>(wm, wn, A, lda, W, WD, M, N, K, splits, C, ldc, st);         \
        case E16_ADD_F32: return dispatch16<QT_, E16_ADD_F32>(wm, wn, A, lda, W, WD, M, N, K, splits, C, ldc, st); \
        case E16_SWIGLU: return dispatch16<QT_, E16_SWIGLU>(wm, wn, A, lda, W, WD, M, N, K, splits, C, ldc, st);   \
    }
    switch (qtype) {
        case MXQ_Q4_K: Q16_EPI(MXQ_Q4_K) break;
        case MXQ_Q6_K: Q16_EPI(MXQ_Q6_K) break;
        case MXQ_Q8_0: Q16_EPI(MXQ_Q8_0) break;
    }
#undef Q16_EPI
    return (int)hipErrorInvalidValue;
}
