// qgemm.hip — quantised-weight matmuls for GGUF K-quants on CDNA4 (K1/K2 of SURVEY §2.6).
//
//   C[M, N] (+)= A[M, K] · W[N, K]^T,   W in Q4_K / Q6_K(repacked) / Q8_0(repacked)
//
// Two kernels, picked by the host on M (see ops/linear.py):
//   * qgemv_dot4  (M <= 4): decode GEMV. Activations are pre-quantised to q8 blocks (int8 x 32 +
//     {d, d*sum}) by the producing norm kernel, weights stay packed; the inner product is
//     v_dot4_i32_i8 on raw nibbles — the integer form llama.cpp's MMVQ uses, so decode numerics
//     match the reference engine. HBM-bound: each weight byte is read exactly once.
//   * qgemm_mfma  (M > 4): each wave dequantises its weight fragment straight into bf16 MFMA
//     B-operands (no LDS round trip for W), the activation tile is staged once per workgroup into an
//     XOR-swizzled LDS image (conflict-free ds_read_b128), and v_mfma_f32_16x16x32_bf16 accumulates.
//     Lane group g (lane>>4) owns the 64 contiguous elements [64g, 64g+64) of every 256-element
//     super-block; MFMA k-step ks consumes elements 64g+8ks+j. The A image is read with the same
//     permutation, so the sum over k is unchanged (a virtual-k relabelling, not a transpose).
// Epilogues fuse what follows each projection in a Llama block: fp32 store (QKV -> RoPE), fp32
// accumulate into the residual stream (o_proj / down_proj, split-K via atomics), and SwiGLU
// (gate/up rows interleaved in 16-row groups at load time -> silu(g)*u written as bf16).
#include "mx_common.h"

enum { EPI_F32 = 0, EPI_BF16 = 1, EPI_ADD_F32 = 2, EPI_SWIGLU = 3, EPI_GEGLU = 4 };

// ---------------------------------------------------------------------------------------------
// Per-lane weight fragment: the 64 elements [64g, 64g+64) of super-block `kb` of row `n`.
template <int QT>
struct WFrag;

template <>
struct WFrag<MXQ_Q4_K> {
    u32x4 h, a, b;  // header (d, dmin, scales[12]) + 32 bytes of qs
    MX_DEV void load(const uint8_t* W, const uint16_t*, int n, int kb, int nblk, int g) {
        const uint8_t* blk = W + ((size_t)n * nblk + kb) * 144;
        h = __builtin_nontemporal_load((const u32x4*)blk);
        a = __builtin_nontemporal_load((const u32x4*)(blk + 16 + 32 * g));
        b = __builtin_nontemporal_load((const u32x4*)(blk + 32 + 32 * g));
    }
    MX_DEV void zero() { h = a = b = (u32x4){0, 0, 0, 0}; }
    MX_DEV uint32_t q(int i) const { return i < 4 ? a[i] : b[i - 4]; }
};

template <>
struct WFrag<MXQ_Q6_K> {
    u32x4 l0, l1, hh;  // 32 B low nibbles, 16 B high bits
    uint32_t sc;       // 4 int8 scales
    uint16_t d;
    MX_DEV void load(const uint8_t* W, const uint16_t* D, int n, int kb, int nblk, int g) {
        const uint8_t* blk = W + ((size_t)n * nblk + kb) * 208;
        l0 = __builtin_nontemporal_load((const u32x4*)(blk + 32 * g));
        l1 = __builtin_nontemporal_load((const u32x4*)(blk + 16 + 32 * g));
        hh = __builtin_nontemporal_load((const u32x4*)(blk + 128 + 16 * g));
        sc = *(const uint32_t*)(blk + 192 + 4 * g);
        d = D[(size_t)n * nblk + kb];
    }
    MX_DEV void zero() { l0 = l1 = hh = (u32x4){0, 0, 0, 0}; sc = 0; d = 0; }
    MX_DEV uint32_t ql(int i) const { return i < 4 ? l0[i] : l1[i - 4]; }
};

template <>
struct WFrag<MXQ_Q8_0> {
    u32x4 w[4];  // 64 int8
    uint32_t d;  // two fp16 scales (blocks 2g, 2g+1)
    MX_DEV void load(const uint8_t* W, const uint16_t* D, int n, int kb, int nblk, int g) {
        const uint8_t* p = W + (size_t)n * nblk * 256 + (size_t)kb * 256 + 64 * g;
#pragma unroll
        for (int i = 0; i < 4; ++i) w[i] = __builtin_nontemporal_load((const u32x4*)(p + 16 * i));
        d = *(const uint32_t*)(D + (size_t)n * nblk * 8 + kb * 8 + 2 * g);
    }
    MX_DEV void zero() {
#pragma unroll
        for (int i = 0; i < 4; ++i) w[i] = (u32x4){0, 0, 0, 0};
        d = 0;
    }
    MX_DEV uint32_t word(int i) const { return w[i >> 2][i & 3]; }
};

// ---------------------------------------------------------------------------------------------
// Dequantisation to bf16 MFMA B-fragments (MFMA path)
template <int QT>
struct Deq;

template <int KS, class D, class F>
MX_DEV bf16x8 to_bf16x8(const D& d, const F& f) {
    float v[8];
    d.template vals<KS>(f, v);
    bf16x8 r;
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = (__bf16)v[j];
    return r;
}

template <>
struct Deq<MXQ_Q4_K> {
    float s[2], m[2];
    MX_DEV void prep(const WFrag<MXQ_Q4_K>& f, int g) {
        const float d = half_to_f32(f.h[0] & 0xFFFF), dm = half_to_f32(f.h[0] >> 16);
        int sc, mn;
        q4k_scale_min_w(f.h[1], f.h[2], f.h[3], 2 * g, sc, mn);
        s[0] = d * sc; m[0] = dm * mn;
        q4k_scale_min_w(f.h[1], f.h[2], f.h[3], 2 * g + 1, sc, mn);
        s[1] = d * sc; m[1] = dm * mn;
    }
    template <int KS>
    MX_DEV void vals(const WFrag<MXQ_Q4_K>& f, float (&v)[8]) const {
        constexpr int hi = KS >> 2;
        uint32_t w0 = f.q(2 * (KS & 3)), w1 = f.q(2 * (KS & 3) + 1);
        w0 = (w0 >> (4 * hi)) & 0x0F0F0F0Fu;
        w1 = (w1 >> (4 * hi)) & 0x0F0F0F0Fu;
        const float sc = s[hi], mn = -m[hi];
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = fmaf(sc, (float)((w0 >> (8 * j)) & 0xFF), mn);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[4 + j] = fmaf(sc, (float)((w1 >> (8 * j)) & 0xFF), mn);
    }
    template <int KS>
    MX_DEV bf16x8 frag(const WFrag<MXQ_Q4_K>& f) const { return to_bf16x8<KS>(*this, f); }
};

template <>
struct Deq<MXQ_Q6_K> {
    float s[4];
    MX_DEV void prep(const WFrag<MXQ_Q6_K>& f, int) {
        const float d = half_to_f32(f.d);
#pragma unroll
        for (int i = 0; i < 4; ++i) s[i] = d * (float)(int8_t)((f.sc >> (8 * i)) & 0xFF);
    }
    template <int KS>
    MX_DEV void vals(const WFrag<MXQ_Q6_K>& f, float (&v)[8]) const {
        constexpr int hi = KS >> 2, qsh = 2 * (KS >> 1);
        uint32_t w0 = (f.ql(2 * (KS & 3)) >> (4 * hi)) & 0x0F0F0F0Fu;
        uint32_t w1 = (f.ql(2 * (KS & 3) + 1) >> (4 * hi)) & 0x0F0F0F0Fu;
        w0 |= ((f.hh[2 * (KS & 1)] >> qsh) & 0x03030303u) << 4;
        w1 |= ((f.hh[2 * (KS & 1) + 1] >> qsh) & 0x03030303u) << 4;
        const float sc = s[KS >> 1], off = -32.f * sc;
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = fmaf(sc, (float)((w0 >> (8 * j)) & 0xFF), off);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[4 + j] = fmaf(sc, (float)((w1 >> (8 * j)) & 0xFF), off);
    }
    template <int KS>
    MX_DEV bf16x8 frag(const WFrag<MXQ_Q6_K>& f) const { return to_bf16x8<KS>(*this, f); }
};

template <>
struct Deq<MXQ_Q8_0> {
    float s[2];
    MX_DEV void prep(const WFrag<MXQ_Q8_0>& f, int) {
        s[0] = half_to_f32(f.d & 0xFFFF);
        s[1] = half_to_f32(f.d >> 16);
    }
    template <int KS>
    MX_DEV void vals(const WFrag<MXQ_Q8_0>& f, float (&v)[8]) const {
        const uint32_t w0 = f.word(2 * KS), w1 = f.word(2 * KS + 1);
        const float sc = s[KS >> 2];
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = sc * (float)(int8_t)((w0 >> (8 * j)) & 0xFF);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[4 + j] = sc * (float)(int8_t)((w1 >> (8 * j)) & 0xFF);
    }
    template <int KS>
    MX_DEV bf16x8 frag(const WFrag<MXQ_Q8_0>& f) const { return to_bf16x8<KS>(*this, f); }
};

// LDS image of the activation tile: row r (0..BM-1) holds the 256 k of one super-block as 32
// 16-byte chunks; chunk c is stored at slot c ^ f(r&15), f(r) = r ^ ((r+4)&8). With the MFMA
// A-operand read pattern (row = lane&15, chunk = 8*(lane>>4)+ks) every ds_read_b128 lane group
// hits 16 distinct 16-byte slots of the 256-byte bank row: conflict-free (verified exhaustively in
// tests/test_kernels_cpu.py::test_lds_swizzle_conflict_free).
MX_DEV int a_lds_off(int r, int c) {
    const int rr = r & 15;
    return r * 512 + ((c ^ (rr ^ ((rr + 4) & 8))) << 4);
}

template <int QT, int WM, int WN, int EPI>
__global__ __launch_bounds__(256) void qgemm_mfma_kernel(const bf16_t* __restrict__ A, int lda,
                                                         const uint8_t* __restrict__ W,
                                                         const uint16_t* __restrict__ WD, int M, int N, int K,
                                                         int kb_per_split, void* __restrict__ Cv, int ldc) {
    constexpr int BM = WM * 16;
    constexpr int A_BYTES = BM * 512;
    constexpr int A_PASSES = BM * 32 / 256;  // 16-byte chunks per thread per stage
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

    // --- stage helpers for A ---
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
            *(u32x4*)(smem + buf * A_BYTES + a_lds_off(id >> 5, id & 31)) = areg[p];
        }
    };

    WFrag<QT> wf[WN], wn[WN];
    auto load_w = [&](WFrag<QT>(&f)[WN], int kb) {
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
        Deq<QT> dq[WN];
#pragma unroll
        for (int t = 0; t < WN; ++t) dq[t].prep(wf[t], g);
        const char* abuf = smem + buf * A_BYTES;
#define QG_KSTEP(KS)                                                                           \
    {                                                                                          \
        bf16x8 bfr[WN];                                                                        \
        _Pragma("unroll") for (int t = 0; t < WN; ++t) bfr[t] = dq[t].template frag<KS>(wf[t]); \
        _Pragma("unroll") for (int i = 0; i < WM; ++i) {                                       \
            const bf16x8 af = *(const bf16x8*)(abuf + a_lds_off(i * 16 + col, 8 * g + KS));    \
            _Pragma("unroll") for (int t = 0; t < WN; ++t) acc[i][t] =                         \
                __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr[t], acc[i][t], 0, 0, 0);       \
        }                                                                                      \
    }
        QG_KSTEP(0) QG_KSTEP(1) QG_KSTEP(2) QG_KSTEP(3) QG_KSTEP(4) QG_KSTEP(5) QG_KSTEP(6) QG_KSTEP(7)
#undef QG_KSTEP
        if (more) {
            store_a(buf ^ 1);
#pragma unroll
            for (int t = 0; t < WN; ++t) wf[t] = wn[t];
        }
        __syncthreads();
        buf ^= 1;
    }

    // --- epilogue: C/D layout col = lane&15, row = 4*(lane>>4) + i ---
#pragma unroll
    for (int i = 0; i < WM; ++i) {
#pragma unroll
        for (int t = 0; t < WN; ++t) {
            if constexpr (EPI == EPI_SWIGLU || EPI == EPI_GEGLU) {
                if (t & 1) continue;
                const int feat = (n_base >> 1) + (t >> 1) * 16 + col;
                if (n_base + t * 16 + col >= N) continue;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int m = m_base + i * 16 + 4 * g + e;
                    if (m < M) {
                        const float gv = acc[i][t][e], uv = acc[i][t + 1][e];
                        ((bf16_t*)Cv)[(size_t)m * ldc + feat] = f32_to_bf16(glu_gate_f<EPI>(gv) * uv);
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
                    if constexpr (EPI == EPI_F32) ((float*)Cv)[(size_t)m * ldc + n] = v;
                    else if constexpr (EPI == EPI_BF16) ((bf16_t*)Cv)[(size_t)m * ldc + n] = f32_to_bf16(v);
                    else atomicAdd(((float*)Cv) + (size_t)m * ldc + n, v);
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------
// GEMV with int8 dot products (decode, M <= 4). Each wave owns two weight rows; 4 lanes per
// super-block, 16 super-blocks per pass. Activations: xq [M][K] int8 + xds [M][K/32] float2{d,d*sum}.
template <int QT>
struct Dot;

template <>
struct Dot<MXQ_Q4_K> {
    // returns the fp32 contribution of this lane's 64 elements against one activation row
    MX_DEV static float run(const WFrag<MXQ_Q4_K>& f, int g, const int8_t* xq, const float2* xds) {
        const u32x4 x0 = *(const u32x4*)(xq), x1 = *(const u32x4*)(xq + 16);
        const u32x4 x2 = *(const u32x4*)(xq + 32), x3 = *(const u32x4*)(xq + 48);
        const float4 ds = *(const float4*)xds;  // {d_lo, s_lo, d_hi, s_hi}
        int il = 0, ih = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint32_t w = f.q(i);
            const uint32_t xl = i < 4 ? x0[i] : x1[i - 4];
            const uint32_t xh = i < 4 ? x2[i] : x3[i - 4];
            il = __builtin_amdgcn_sdot4((int)(w & 0x0F0F0F0Fu), (int)xl, il, false);
            ih = __builtin_amdgcn_sdot4((int)((w >> 4) & 0x0F0F0F0Fu), (int)xh, ih, false);
        }
        const float d = half_to_f32(f.h[0] & 0xFFFF), dm = half_to_f32(f.h[0] >> 16);
        int sc0, m0, sc1, m1;
        q4k_scale_min_w(f.h[1], f.h[2], f.h[3], 2 * g, sc0, m0);
        q4k_scale_min_w(f.h[1], f.h[2], f.h[3], 2 * g + 1, sc1, m1);
        return d * (sc0 * ds.x * (float)il + sc1 * ds.z * (float)ih) - dm * (m0 * ds.y + m1 * ds.w);
    }
};

template <>
struct Dot<MXQ_Q6_K> {
    MX_DEV static float run(const WFrag<MXQ_Q6_K>& f, int, const int8_t* xq, const float2* xds) {
        const u32x4 x0 = *(const u32x4*)(xq), x1 = *(const u32x4*)(xq + 16);
        const u32x4 x2 = *(const u32x4*)(xq + 32), x3 = *(const u32x4*)(xq + 48);
        const float4 ds = *(const float4*)xds;
        int is[4] = {0, 0, 0, 0};
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint32_t l = f.ql(i), h = f.hh[i & 3];
            uint32_t qlo = (l & 0x0F0F0F0Fu) | (((h >> (2 * (i >> 2))) & 0x03030303u) << 4);
            uint32_t qhi = ((l >> 4) & 0x0F0F0F0Fu) | (((h >> (2 * (2 + (i >> 2)))) & 0x03030303u) << 4);
            const uint32_t xl = i < 4 ? x0[i] : x1[i - 4];
            const uint32_t xh = i < 4 ? x2[i] : x3[i - 4];
            is[i >> 2] = __builtin_amdgcn_sdot4((int)q6_bias_bytes(qlo), (int)xl, is[i >> 2], false);
            is[2 + (i >> 2)] = __builtin_amdgcn_sdot4((int)q6_bias_bytes(qhi), (int)xh, is[2 + (i >> 2)], false);
        }
        const float d = half_to_f32(f.d);
        float s[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) s[i] = (float)(int8_t)((f.sc >> (8 * i)) & 0xFF);
        return d * (ds.x * (s[0] * is[0] + s[1] * is[1]) + ds.z * (s[2] * is[2] + s[3] * is[3]));
    }
};

template <>
struct Dot<MXQ_Q8_0> {
    MX_DEV static float run(const WFrag<MXQ_Q8_0>& f, int, const int8_t* xq, const float2* xds) {
        const float4 ds = *(const float4*)xds;
        int i0 = 0, i1 = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const u32x4 x = *(const u32x4*)(xq + 16 * q);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (q < 2) i0 = __builtin_amdgcn_sdot4((int)f.w[q][j], (int)x[j], i0, false);
                else i1 = __builtin_amdgcn_sdot4((int)f.w[q][j], (int)x[j], i1, false);
            }
        }
        return half_to_f32(f.d & 0xFFFF) * ds.x * (float)i0 + half_to_f32(f.d >> 16) * ds.z * (float)i1;
    }
};

template <int QT, int MM, int EPI, bool F16>
__global__ __launch_bounds__(256) void qgemv_dot4_kernel(const int8_t* __restrict__ xq,
                                                         const float2* __restrict__ xds,
                                                         const uint8_t* __restrict__ W,
                                                         const uint16_t* __restrict__ WD, int M, int N, int K,
                                                         void* __restrict__ Cv, int ldc) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int slot = blockIdx.x * 4 + wave;  // each slot produces 2 rows (or 1 SwiGLU feature)
    int r0, r1;
    if constexpr (EPI == EPI_SWIGLU || EPI == EPI_GEGLU) {
        r0 = 32 * (slot >> 4) + (slot & 15);
        r1 = r0 + 16;
    } else {
        r0 = 2 * slot;
        r1 = r0 + 1;
    }
    if (r0 >= N) return;
    const bool v1 = r1 < N;
    const int nblk = K >> 8;
    const int q = lane & 3;
    float acc0[MM], acc1[MM];
#pragma unroll
    for (int m = 0; m < MM; ++m) acc0[m] = acc1[m] = 0.f;
    for (int bi = lane >> 2; bi < nblk; bi += 16) {
        WFrag<QT> f0, f1;
        f0.load(W, WD, r0, bi, nblk, q);
        if (v1) f1.load(W, WD, r1, bi, nblk, q);
        else f1.zero();
#pragma unroll
        for (int m = 0; m < MM; ++m) {
            if (m < M) {
                const int8_t* xr = xq + (size_t)m * K + bi * 256 + 64 * q;
                const float2* dr = xds + (size_t)m * (K / 32) + bi * 8 + 2 * q;
                acc0[m] += Dot<QT>::run(f0, q, xr, dr);
                acc1[m] += Dot<QT>::run(f1, q, xr, dr);
            }
        }
    }
#pragma unroll
    for (int m = 0; m < MM; ++m) {
        if (m >= M) break;
        const float a0 = wave_sum(acc0[m]);
        const float a1 = wave_sum(acc1[m]);
        if (lane == 0) {
            if constexpr (EPI == EPI_SWIGLU || EPI == EPI_GEGLU) {
                ((bf16_t*)Cv)[(size_t)m * ldc + slot] = f32_to_act<F16>(glu_gate_f<EPI>(a0) * a1);
            } else if constexpr (EPI == EPI_F32) {
                ((float*)Cv)[(size_t)m * ldc + r0] = a0;
                if (v1) ((float*)Cv)[(size_t)m * ldc + r1] = a1;
            } else if constexpr (EPI == EPI_BF16) {
                ((bf16_t*)Cv)[(size_t)m * ldc + r0] = f32_to_act<F16>(a0);
                if (v1) ((bf16_t*)Cv)[(size_t)m * ldc + r1] = f32_to_act<F16>(a1);
            } else {
                ((float*)Cv)[(size_t)m * ldc + r0] += a0;
                if (v1) ((float*)Cv)[(size_t)m * ldc + r1] += a1;
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------
// dequantise whole rows to bf16 (embedding lookup K9, and the optional bf16 weight cache used by
// large-M prefill through hipBLASLt). rows[i] selects the source row (nullptr -> identity).
template <int QT, bool F16>
__global__ __launch_bounds__(256) void dequant_rows_kernel(const uint8_t* __restrict__ W,
                                                           const uint16_t* __restrict__ WD,
                                                           const int* __restrict__ rows, int K,
                                                           bf16_t* __restrict__ ob, float* __restrict__ of,
                                                           int ldo) {
    const int orow = blockIdx.y;
    const int n = rows ? rows[orow] : orow;
    const int nblk = K >> 8;
    // one wave per super-block, lane: g = lane>>4 (64-element quarter), c = lane&15 selects 4 elems
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int kb = blockIdx.x * 4 + wave;
    if (kb >= nblk) return;
    const int g = lane >> 4, c = lane & 15;
    WFrag<QT> f;
    f.load(W, WD, n, kb, nblk, g);
    Deq<QT> dq;
    dq.prep(f, g);
    // lane writes elements 64g + 4c .. +3  => k-step ks = c>>1, j in (c&1)*4 .. +3
    float v[8];
    switch (c >> 1) {
        case 0: dq.template vals<0>(f, v); break;
        case 1: dq.template vals<1>(f, v); break;
        case 2: dq.template vals<2>(f, v); break;
        case 3: dq.template vals<3>(f, v); break;
        case 4: dq.template vals<4>(f, v); break;
        case 5: dq.template vals<5>(f, v); break;
        case 6: dq.template vals<6>(f, v); break;
        default: dq.template vals<7>(f, v); break;
    }
    const int e0 = kb * 256 + 64 * g + 4 * c;
    const int jo = (c & 1) * 4;
    if (ob) {
        uint2 p;
        p.x = pack_act2<F16>(v[jo], v[jo + 1]);
        p.y = pack_act2<F16>(v[jo + 2], v[jo + 3]);
        *(uint2*)(ob + (size_t)orow * ldo + e0) = p;
    }
    if (of) *(float4*)(of + (size_t)orow * ldo + e0) = make_float4(v[jo], v[jo + 1], v[jo + 2], v[jo + 3]);
}

// ---------------------------------------------------------------------------------------------
// launchers
template <int QT, int WM, int WN, int EPI>
static int launch_mfma(const bf16_t* A, int lda, const uint8_t* W, const uint16_t* WD, int M, int N, int K,
                       int splits, void* C, int ldc, hipStream_t st) {
    const int nblk = K / 256;
    const int kbs = (nblk + splits - 1) / splits;
    dim3 grid((N + 64 * WN - 1) / (64 * WN), splits, (M + WM * 16 - 1) / (WM * 16));
    const size_t lds = 2 * WM * 16 * 512;
    qgemm_mfma_kernel<QT, WM, WN, EPI><<<grid, 256, lds, st>>>(A, lda, W, WD, M, N, K, kbs, C, ldc);
    MXK_CHECK_LAUNCH();
}

template <int QT, int EPI>
static int dispatch_mfma(int wm, int wn, const bf16_t* A, int lda, const uint8_t* W, const uint16_t* WD, int M,
                         int N, int K, int splits, void* C, int ldc, hipStream_t st) {
    if (QT == MXQ_Q8_0 && wn > 2) wn = 2;  // 64 B/lane fragments: WN=4 would spill
#define QG_CASE(WM_, WN_) \
    if (wm == WM_ && wn == WN_) return launch_mfma<QT, WM_, WN_, EPI>(A, lda, W, WD, M, N, K, splits, C, ldc, st);
    QG_CASE(1, 2) QG_CASE(1, 4) QG_CASE(2, 2) QG_CASE(2, 4) QG_CASE(4, 2) QG_CASE(4, 4) QG_CASE(8, 2)
#undef QG_CASE
    return (int)hipErrorInvalidValue;
}

extern "C" int mxk_qgemm_mfma(int qtype, int epi, int wm, int wn, const bf16_t* A, int lda, const uint8_t* W,
                              const uint16_t* WD, int M, int N, int K, int splits, void* C, int ldc,
                              hipStream_t st) {
    if (M <= 0) return 0;
    if (K % 256) return (int)hipErrorInvalidValue;
    if ((epi == EPI_SWIGLU || epi == EPI_GEGLU || epi == EPI_BF16 || epi == EPI_F32) && splits != 1) return (int)hipErrorInvalidValue;
    if ((epi == EPI_SWIGLU || epi == EPI_GEGLU) && (wn & 1)) return (int)hipErrorInvalidValue;
#define QG_EPI(QT_)                                                                                     \
    switch (epi) {                                                                                      \
        case EPI_F32: return dispatch_mfma<QT_, EPI_F32>(wm, wn, A, lda, W, WD, M, N, K, splits, C, ldc, st);   \
        case EPI_BF16: return dispatch_mfma<QT_, EPI_BF16>(wm, wn, A, lda, W, WD, M, N, K, splits, C, ldc, st); \
        case EPI_ADD_F32:                                                                               \
            return dispatch_mfma<QT_, EPI_ADD_F32>(wm, wn, A, lda, W, WD, M, N, K, splits, C, ldc, st);        \
        case EPI_SWIGLU:                                                                                \
            return dispatch_mfma<QT_, EPI_SWIGLU>(wm, wn, A, lda, W, WD, M, N, K, splits, C, ldc, st);         \
        case EPI_GEGLU:                                                                                 \
            return dispatch_mfma<QT_, EPI_GEGLU>(wm, wn, A, lda, W, WD, M, N, K, splits, C, ldc, st);          \
    }
    switch (qtype) {
        case MXQ_Q4_K: QG_EPI(MXQ_Q4_K) break;
        case MXQ_Q6_K: QG_EPI(MXQ_Q6_K) break;
        case MXQ_Q8_0: QG_EPI(MXQ_Q8_0) break;
    }
#undef QG_EPI
    return (int)hipErrorInvalidValue;
}

template <int QT, int MM, int EPI>
static int launch_gemv(const int8_t* xq, const float2* xds, const uint8_t* W, const uint16_t* WD, int M, int N,
                       int K, void* C, int ldc, hipStream_t st) {
    const int slots = (EPI == EPI_SWIGLU || EPI == EPI_GEGLU) ? N / 2 : (N + 1) / 2;
    dim3 grid((slots + 3) / 4);
    MX_ACT_DISPATCH(qgemv_dot4_kernel<QT, MM, EPI, F16><<<grid, 256, 0, st>>>(xq, xds, W, WD, M, N, K, C, ldc));
    MXK_CHECK_LAUNCH();
}

extern "C" int mxk_qgemv(int qtype, int epi, const int8_t* xq, const float2* xds, const uint8_t* W,
                         const uint16_t* WD, int M, int N, int K, void* C, int ldc, hipStream_t st) {
    if (M <= 0) return 0;
    if (M > 4 || K % 256) return (int)hipErrorInvalidValue;
    if ((epi == EPI_SWIGLU || epi == EPI_GEGLU) && (N % 32)) return (int)hipErrorInvalidValue;
#define GV_M(QT_, EPI_)                                                                 \
    if (M == 1) return launch_gemv<QT_, 1, EPI_>(xq, xds, W, WD, M, N, K, C, ldc, st);  \
    if (M == 2) return launch_gemv<QT_, 2, EPI_>(xq, xds, W, WD, M, N, K, C, ldc, st);  \
    return launch_gemv<QT_, 4, EPI_>(xq, xds, W, WD, M, N, K, C, ldc, st);
#define GV_EPI(QT_)                                   \
    switch (epi) {                                    \
        case EPI_F32: { GV_M(QT_, EPI_F32) }          \
        case EPI_BF16: { GV_M(QT_, EPI_BF16) }        \
        case EPI_ADD_F32: { GV_M(QT_, EPI_ADD_F32) }  \
        case EPI_SWIGLU: { GV_M(QT_, EPI_SWIGLU) }    \
        case EPI_GEGLU: { GV_M(QT_, EPI_GEGLU) }      \
    }
    switch (qtype) {
        case MXQ_Q4_K: GV_EPI(MXQ_Q4_K) break;
        case MXQ_Q6_K: GV_EPI(MXQ_Q6_K) break;
        case MXQ_Q8_0: GV_EPI(MXQ_Q8_0) break;
    }
#undef GV_EPI
#undef GV_M
    return (int)hipErrorInvalidValue;
}

extern "C" int mxk_dequant_rows(int qtype, const uint8_t* W, const uint16_t* WD, const int* rows, int nrows, int K,
                                bf16_t* ob, float* of, int ldo, hipStream_t st) {
    if (nrows <= 0) return 0;
    if (K % 256) return (int)hipErrorInvalidValue;
    dim3 grid((K / 256 + 3) / 4, nrows);
    int rc = 0;
    MX_ACT_DISPATCH({
        switch (qtype) {
            case MXQ_Q4_K: dequant_rows_kernel<MXQ_Q4_K, F16><<<grid, 256, 0, st>>>(W, WD, rows, K, ob, of, ldo); break;
            case MXQ_Q6_K: dequant_rows_kernel<MXQ_Q6_K, F16><<<grid, 256, 0, st>>>(W, WD, rows, K, ob, of, ldo); break;
            case MXQ_Q8_0: dequant_rows_kernel<MXQ_Q8_0, F16><<<grid, 256, 0, st>>>(W, WD, rows, K, ob, of, ldo); break;
            default: rc = (int)hipErrorInvalidValue;
        }
    });
    if (rc) return rc;
    MXK_CHECK_LAUNCH();
}
