// qmv.hip — decode GEMV (M <= 4 rows) and row dequantisation for weights in the "t32" tiled layout
// (see qmm.hip / ops/quant.py tile32):
//
//   C[M, N] (+)= X[M, K] · W[N, K]^T   with X as q8 activations (int8 [M][K] + float2 {d, d*sum} per 32)
//
// One workgroup (8 waves) owns one 32-column group and splits its K range over the waves; lane
// (r = lane & 31, h = lane >> 5) owns column r and half h of every 64-element quarter, so each wave's
// weight loads are 1 KB contiguous wave-instructions (the tiled layout's point), all issued before
// the int8 dot products (sdot4) consume them. Partial sums meet in LDS; the epilogue (fp32 store /
// act16 store / fp32 accumulate / SwiGLU|GeGLU over the 16+16 interleaved gate|up rows) is fused.
#include "qdeq16.h"

namespace {
constexpr int QMV_WAVES = 8;
int g_qmv1_on = 1;  // mxk_qmv1_enable: the batch-1 fast-prologue kernel (A/B switch)

// per-lane weight state for one unit (Q4_K/Q6_K: one 256-element super-block; Q8_0: one 64-k tile)
template <int QT>
struct TUnit;

template <>
struct TUnit<MXQ_Q4_K> {
    static constexpr int BYTES = 4608, ELEMS = 256;
    u32x4 hd, q[4];
    MX_DEV void load(const uint8_t* u, int r, int h) {
        hd = *(const u32x4*)(u + r * 16);
#pragma unroll
        for (int jq = 0; jq < 4; ++jq) q[jq] = __builtin_nontemporal_load((const u32x4*)(u + 512 + jq * 1024 + h * 512 + r * 16));
    }
    // this lane's contribution against activation row x (k offset of the unit already applied)
    MX_DEV float dot(const int8_t* x, const float2* ds, int h) const {
        const float d = half_to_f32(hd[0] & 0xFFFF), dm = half_to_f32(hd[0] >> 16);
        float acc = 0.f, mins = 0.f;
#pragma unroll
        for (int jq = 0; jq < 4; ++jq) {
            const u32x4 xl = *(const u32x4*)(x + 64 * jq + 16 * h);
            const u32x4 xh = *(const u32x4*)(x + 64 * jq + 32 + 16 * h);
            int il = 0, ih = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                il = __builtin_amdgcn_sdot4((int)(q[jq][i] & 0x0F0F0F0Fu), (int)xl[i], il, false);
                ih = __builtin_amdgcn_sdot4((int)((q[jq][i] >> 4) & 0x0F0F0F0Fu), (int)xh[i], ih, false);
            }
            int sc0, m0, sc1, m1;
            q4k_scale_min_w(hd[1], hd[2], hd[3], 2 * jq, sc0, m0);
            q4k_scale_min_w(hd[1], hd[2], hd[3], 2 * jq + 1, sc1, m1);
            const float2 dl = ds[2 * jq], dh = ds[2 * jq + 1];
            acc += (float)sc0 * dl.x * (float)il + (float)sc1 * dh.x * (float)ih;
            mins += (float)m0 * dl.y + (float)m1 * dh.y;  // {d, d*sum} covers the whole 32-block
        }
        return d * acc - (h == 0 ? dm * mins : 0.f);
    }
};

// Q5_K: the Q4_K unit plus one high bit per code: qh (32 B per column, bit 2jq / 2jq+1 of byte b = code b of
// quarter jq's low / high half), stored after the codes as 2 chunks x 32 columns x 16 B.
template <>
struct TUnit<MXQ_Q5_K> {
    static constexpr int BYTES = 5632, ELEMS = 256;
    u32x4 hd, q[4], qh;
    MX_DEV void load(const uint8_t* u, int r, int h) {
        hd = *(const u32x4*)(u + r * 16);
#pragma unroll
        for (int jq = 0; jq < 4; ++jq) q[jq] = __builtin_nontemporal_load((const u32x4*)(u + 512 + jq * 1024 + h * 512 + r * 16));
        qh = __builtin_nontemporal_load((const u32x4*)(u + 4608 + h * 512 + r * 16));
    }
    MX_DEV float dot(const int8_t* x, const float2* ds, int h) const {
        const float d = half_to_f32(hd[0] & 0xFFFF), dm = half_to_f32(hd[0] >> 16);
        float acc = 0.f, mins = 0.f;
#pragma unroll
        for (int jq = 0; jq < 4; ++jq) {
            const u32x4 xl = *(const u32x4*)(x + 64 * jq + 16 * h);
            const u32x4 xh = *(const u32x4*)(x + 64 * jq + 32 + 16 * h);
            int il = 0, ih = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint32_t lo = (q[jq][i] & 0x0F0F0F0Fu) | (((qh[i] >> (2 * jq)) & 0x01010101u) << 4);
                const uint32_t hi = ((q[jq][i] >> 4) & 0x0F0F0F0Fu) | (((qh[i] >> (2 * jq + 1)) & 0x01010101u) << 4);
                il = __builtin_amdgcn_sdot4((int)lo, (int)xl[i], il, false);
                ih = __builtin_amdgcn_sdot4((int)hi, (int)xh[i], ih, false);
            }
            int sc0, m0, sc1, m1;
            q4k_scale_min_w(hd[1], hd[2], hd[3], 2 * jq, sc0, m0);
            q4k_scale_min_w(hd[1], hd[2], hd[3], 2 * jq + 1, sc1, m1);
            const float2 dl = ds[2 * jq], dh = ds[2 * jq + 1];
            acc += (float)sc0 * dl.x * (float)il + (float)sc1 * dh.x * (float)ih;
            mins += (float)m0 * dl.y + (float)m1 * dh.y;
        }
        return d * acc - (h == 0 ? dm * mins : 0.f);
    }
};

// MX4F / MX5F (t32 unit of 256 weights): [hdr: 2 halves x 32 columns x 16 B {f16 s[4], f16 m[4]}]
// [k-tile jq: 2 x (32 x 16 B) codes in the Q4_K nibble order (+ MX5F: 32 x 8 B high bits)]. The high bits of
// k-tile jq are one little-endian 64-bit word per column: bit u = bit 4 of weight 64 jq + u.
template <bool FIVE>
struct TUnitMX {
    static constexpr int KTB = FIVE ? 1280 : 1024, BYTES = 1024 + 4 * KTB, ELEMS = 256;
    u32x4 h0, h1, q[4];
    u32x2 qh[4];
    MX_DEV void load(const uint8_t* u, int r, int h) {
        h0 = *(const u32x4*)(u + r * 16);
        h1 = *(const u32x4*)(u + 512 + r * 16);
#pragma unroll
        for (int jq = 0; jq < 4; ++jq) {
            q[jq] = __builtin_nontemporal_load((const u32x4*)(u + 1024 + jq * KTB + h * 512 + r * 16));
            if constexpr (FIVE) qh[jq] = __builtin_nontemporal_load((const u32x2*)(u + 1024 + jq * KTB + 1024 + r * 8));
        }
    }
    MX_DEV static float hf(uint32_t w, int hi) { return half_to_f32(hi ? (w >> 16) : (w & 0xFFFF)); }
    MX_DEV float dot(const int8_t* x, const float2* ds, int h) const {
        float acc = 0.f, mins = 0.f;
#pragma unroll
        for (int jq = 0; jq < 4; ++jq) {
            const u32x4 xl = *(const u32x4*)(x + 64 * jq + 16 * h);
            const u32x4 xh = *(const u32x4*)(x + 64 * jq + 32 + 16 * h);
            int il = 0, ih = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                uint32_t lo = q[jq][i] & 0x0F0F0F0Fu, hi = (q[jq][i] >> 4) & 0x0F0F0F0Fu;
                if constexpr (FIVE) {
                    // weights 16 h + 4 i .. +3 (low nibbles) / 32 + 16 h + 4 i .. +3 (high nibbles) of the k-tile
                    const uint32_t wl = qh[jq][0], wh = qh[jq][1];
                    lo |= mx_spread4(wl >> (16 * h + 4 * i)) << 4;
                    hi |= mx_spread4(wh >> (16 * h + 4 * i)) << 4;
                }
                il = __builtin_amdgcn_sdot4((int)lo, (int)xl[i], il, false);
                ih = __builtin_amdgcn_sdot4((int)hi, (int)xh[i], ih, false);
            }
            const u32x4& hd = jq < 2 ? h0 : h1;
            const int i0 = 2 * (jq & 1);  // sub-blocks 2 jq, 2 jq + 1 = entries i0, i0 + 1 of the half
            const float s0 = hf(hd[0 + (i0 >> 1)], 0), s1 = hf(hd[0 + (i0 >> 1)], 1);
            const float m0 = hf(hd[2 + (i0 >> 1)], 0), m1 = hf(hd[2 + (i0 >> 1)], 1);
            const float2 dl = ds[2 * jq], dh = ds[2 * jq + 1];
            acc += s0 * dl.x * (float)il + s1 * dh.x * (float)ih;
            mins += m0 * dl.y + m1 * dh.y;  // {d, d*sum} covers the whole 32-block
        }
        return acc + (h == 0 ? mins : 0.f);
    }
};
template <>
struct TUnit<MXQ_MX4F> : TUnitMX<false> {};
template <>
struct TUnit<MXQ_MX5F> : TUnitMX<true> {};

template <>
struct TUnit<MXQ_Q6_K> {
    static constexpr int BYTES = 6784, ELEMS = 256;
    u32x4 sc, ql[4], qh[4];
    uint32_t dw;
    MX_DEV void load(const uint8_t* u, int r, int h) {
        sc = *(const u32x4*)(u + r * 16);
        dw = *(const uint32_t*)(u + 512 + r * 4);
#pragma unroll
        for (int jq = 0; jq < 4; ++jq) {
            const uint8_t* p = u + 640 + jq * 1536;
            ql[jq] = __builtin_nontemporal_load((const u32x4*)(p + h * 512 + r * 16));
            qh[jq] = __builtin_nontemporal_load((const u32x4*)(p + 1024 + r * 16));
        }
    }
    MX_DEV float dot(const int8_t* x, const float2* ds, int h) const {
        const float d = half_to_f32(dw & 0xFFFF);
        float acc = 0.f;
#pragma unroll
        for (int jq = 0; jq < 4; ++jq) {
            const u32x4 xl = *(const u32x4*)(x + 64 * jq + 16 * h);
            const u32x4 xh = *(const u32x4*)(x + 64 * jq + 32 + 16 * h);
            // the 6-bit codes (0..63) are non-negative int8 as they are: sum(q x) by sdot4 directly, and the -32
            // offset as -32 sum(x) (one more sdot4 against 0x01 per word) instead of re-biasing every code byte
            int il = 0, ih = 0, sl = 0, sh = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint32_t lo = (ql[jq][i] & 0x0F0F0F0Fu) | (((qh[jq][i] >> (2 * h)) & 0x03030303u) << 4);
                const uint32_t hi = ((ql[jq][i] >> 4) & 0x0F0F0F0Fu) | (((qh[jq][i] >> (2 * (2 + h))) & 0x03030303u) << 4);
                il = __builtin_amdgcn_sdot4((int)lo, (int)xl[i], il, false);
                ih = __builtin_amdgcn_sdot4((int)hi, (int)xh[i], ih, false);
                sl = __builtin_amdgcn_sdot4(0x01010101, (int)xl[i], sl, false);
                sh = __builtin_amdgcn_sdot4(0x01010101, (int)xh[i], sh, false);
            }
            il -= 32 * sl;
            ih -= 32 * sh;
            const int s_lo = (int8_t)((sc[jq] >> (8 * h)) & 0xFF), s_hi = (int8_t)((sc[jq] >> (8 * (2 + h))) & 0xFF);
            acc += (float)s_lo * ds[2 * jq].x * (float)il + (float)s_hi * ds[2 * jq + 1].x * (float)ih;
        }
        return d * acc;
    }
};

// Q3_K t32 unit (3584 B): [hdr 32 x 16 B {scales[12], d}][hmask: 2 chunks x 32 x 16 B][qs half n = 0, 1: 2 chunks x
// 32 x 16 B]. Lane half h takes bytes 16 h .. 16 h + 15 of every 32-byte run, i.e. elements 128 n + 32 j + 16 h + i:
// 16 consecutive activations per (n, j), one q8 block half, sub-block scale 8 n + 2 j + h.
template <>
struct TUnit<MXQ_Q3_K> {
    static constexpr int BYTES = 3584, ELEMS = 256;
    u32x4 hd, hm, q[2];
    MX_DEV void load(const uint8_t* u, int r, int h) {
        hd = *(const u32x4*)(u + r * 16);
        hm = __builtin_nontemporal_load((const u32x4*)(u + 512 + h * 512 + r * 16));
#pragma unroll
        for (int n = 0; n < 2; ++n) q[n] = __builtin_nontemporal_load((const u32x4*)(u + 1536 + n * 1024 + h * 512 + r * 16));
    }
    MX_DEV float dot(const int8_t* x, const float2* ds, int h) const {
        constexpr uint32_t km1 = 0x03030303u, km2 = 0x0F0F0F0Fu;
        const uint32_t sw[4] = {(hd[0] & km2) | ((hd[2] & km1) << 4), (hd[1] & km2) | (((hd[2] >> 2) & km1) << 4),
                                ((hd[0] >> 4) & km2) | (((hd[2] >> 4) & km1) << 4),
                                ((hd[1] >> 4) & km2) | (((hd[2] >> 6) & km1) << 4)};
        const float d = half_to_f32(hd[3] & 0xFFFF);
        float acc = 0.f;
#pragma unroll
        for (int n = 0; n < 2; ++n) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const u32x4 xv = *(const u32x4*)(x + 128 * n + 32 * j + 16 * h);
                // 3-bit codes 0..7 straight into sdot4 (non-negative int8); the -4 offset as -4 sum(x) by one more
                // sdot4 against 0x01 per word instead of sign-extending every code byte
                int is = 0, sx = 0;
#pragma unroll
                for (int w = 0; w < 4; ++w) {
                    const uint32_t c = ((q[n][w] >> (2 * j)) & 0x03030303u) | (((hm[w] >> (4 * n + j)) & 0x01010101u) << 2);
                    is = __builtin_amdgcn_sdot4((int)c, (int)xv[w], is, false);
                    sx = __builtin_amdgcn_sdot4(0x01010101, (int)xv[w], sx, false);
                }
                is -= 4 * sx;
                const int isx = 8 * n + 2 * j + h;
                const int sc = (int)((sw[isx >> 2] >> (8 * (isx & 3))) & 0xFF) - 32;
                acc += (float)sc * ds[4 * n + j].x * (float)is;
            }
        }
        return d * acc;
    }
};

// Q2_K t32 unit (2688 B): [sc 32 x 16 B][dd 32 x 4 B {d, dmin}][qs half n: 2 chunks x 32 x 16 B]; the lane split is
// Q3_K's. The min term needs the 16-element activation sums: one sdot4 against ones per word.
template <>
struct TUnit<MXQ_Q2_K> {
    static constexpr int BYTES = 2688, ELEMS = 256;
    u32x4 sc, q[2];
    uint32_t dw;
    MX_DEV void load(const uint8_t* u, int r, int h) {
        sc = *(const u32x4*)(u + r * 16);
        dw = *(const uint32_t*)(u + 512 + r * 4);
#pragma unroll
        for (int n = 0; n < 2; ++n) q[n] = __builtin_nontemporal_load((const u32x4*)(u + 640 + n * 1024 + h * 512 + r * 16));
    }
    MX_DEV float dot(const int8_t* x, const float2* ds, int h) const {
        float acc = 0.f, mins = 0.f;
#pragma unroll
        for (int n = 0; n < 2; ++n) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const u32x4 xv = *(const u32x4*)(x + 128 * n + 32 * j + 16 * h);
                int is = 0, xs = 0;
#pragma unroll
                for (int w = 0; w < 4; ++w) {
                    is = __builtin_amdgcn_sdot4((int)((q[n][w] >> (2 * j)) & 0x03030303u), (int)xv[w], is, false);
                    xs = __builtin_amdgcn_sdot4(0x01010101, (int)xv[w], xs, false);
                }
                const int isx = 8 * n + 2 * j + h;
                const uint32_t b = (sc[isx >> 2] >> (8 * (isx & 3))) & 0xFF;
                const float dx = ds[4 * n + j].x;
                acc += (float)(b & 15) * dx * (float)is;
                mins += (float)(b >> 4) * dx * (float)xs;
            }
        }
        return half_to_f32(dw & 0xFFFF) * acc - half_to_f32(dw >> 16) * mins;
    }
};

template <>
struct TUnit<MXQ_Q8_0> {
    static constexpr int BYTES = 2176, ELEMS = 64;
    uint32_t dw;
    u32x4 q0, q1;
    MX_DEV void load(const uint8_t* u, int r, int h) {
        dw = *(const uint32_t*)(u + r * 4);
        q0 = __builtin_nontemporal_load((const u32x4*)(u + 128 + (2 * h) * 512 + r * 16));
        q1 = __builtin_nontemporal_load((const u32x4*)(u + 128 + (2 * h + 1) * 512 + r * 16));
    }
    MX_DEV float dot(const int8_t* x, const float2* ds, int h) const {
        const u32x4 x0 = *(const u32x4*)(x + 32 * h), x1 = *(const u32x4*)(x + 32 * h + 16);
        int s = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            s = __builtin_amdgcn_sdot4((int)q0[i], (int)x0[i], s, false);
            s = __builtin_amdgcn_sdot4((int)q1[i], (int)x1[i], s, false);
        }
        const float d = half_to_f32(h ? (dw >> 16) : (dw & 0xFFFF));
        return d * ds[h].x * (float)s;
    }
};

}  // namespace

// Activation source of the GEMV: SRC_Q8 = q8 rows prepared by a separate kernel (quant_q8 / rmsnorm);
// SRC_ACT = 16-bit rows quantised in the prologue; SRC_NORM = fp32 residual rows RMS-normalised (weight nw)
// and quantised in the prologue. The fused sources remove the rmsnorm / quant_q8 launch in front of every
// decode GEMV (at batch 1 those tiny kernels cost as much as the weight streaming): each workgroup
// quantises only its own K slice into LDS (the norm's sum of squares still spans the whole row, read
// from L2 — every workgroup of the launch reads the same row).
enum { SRC_Q8 = 0, SRC_ACT = 1, SRC_NORM = 2 };

template <int QT, int MM, int EPI, bool F16, int SRC>
__global__ __launch_bounds__(64 * QMV_WAVES) void qmv_kernel(const int8_t* __restrict__ xq,
                                                             const float2* __restrict__ xds,
                                                             const uint8_t* __restrict__ W, int M, int N, int K,
                                                             void* __restrict__ Cv, int ldc,
                                                             const void* __restrict__ xsrc, int ldx,
                                                             const float* __restrict__ nw, float eps) {
    using U = TUnit<QT>;
    __shared__ float red[QMV_WAVES][MM][32];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int r = lane & 31, h = lane >> 5;
    const int g = blockIdx.x;
    const int nunit = K / U::ELEMS;
    // K split over gridDim.y workgroups (fp32 atomic accumulate epilogue)
    const int per = (nunit + gridDim.y - 1) / gridDim.y;
    const int u0 = blockIdx.y * per, u1 = min(nunit, u0 + per);
    const uint8_t* wg = W + (size_t)g * nunit * U::BYTES;
    int ldq = K, ubase = 0;
    // the wave's first two units are in flight before the activation prologue runs (HBM latency overlaps
    // the norm / quantisation; at batch 1 the whole weight stream is usually these two loads per wave)
    U a, b;
    int u = u0 + wave;
    if (u < u1) a.load(wg + (size_t)u * U::BYTES, r, h);
    if (u + QMV_WAVES < u1) b.load(wg + (size_t)(u + QMV_WAVES) * U::BYTES, r, h);
    float rsv[MM];
#pragma unroll
    for (int m = 0; m < MM; ++m) rsv[m] = 1.f;
    if constexpr (SRC != SRC_Q8) {
        extern __shared__ __attribute__((aligned(16))) char qmv_smem[];
        const int SL = per * U::ELEMS;  // slice capacity per row (dynamic LDS: MM x (SL + SL/32 x 8) bytes)
        int8_t* sq = (int8_t*)qmv_smem;
        float2* sd = (float2*)(qmv_smem + MM * SL);
        const int k0 = u0 * U::ELEMS, klen = max(0, u1 - u0) * U::ELEMS;
        __shared__ float nred[MM][QMV_WAVES];
        for (int m = 0; m < M; ++m) {
            if constexpr (SRC == SRC_NORM) {
                // sum of squares over the whole row (every workgroup reads the same row from L2); the slice
                // below is quantised without 1/rms — q8 codes are scale invariant, the GEMV result is
                // multiplied by 1/rms at the end — so the two passes do not wait on each other
                const float* xr = (const float*)xsrc + (size_t)m * ldx;
                float ss = 0.f;
                for (int c = threadIdx.x * 4; c < K; c += 64 * QMV_WAVES * 4) {
                    const float4 v = *(const float4*)(xr + c);
                    ss += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
                }
                ss = wave_sum(ss);
                if (lane == 0) nred[m][wave] = ss;
            }
            // 8 consecutive elements per lane, 4 lanes per 32-element q8 block (klen % 256 == 0, so the
            // 4-lane groups enter and leave the loop together)
            for (int e = threadIdx.x * 8; e < klen; e += 64 * QMV_WAVES * 8) {
                float a8[8];
                if constexpr (SRC == SRC_NORM) {
                    const float* xr = (const float*)xsrc + (size_t)m * ldx + k0 + e;
                    const float4 v0 = *(const float4*)xr, v1 = *(const float4*)(xr + 4);
                    const float4 w0 = *(const float4*)(nw + k0 + e), w1 = *(const float4*)(nw + k0 + e + 4);
                    a8[0] = v0.x * w0.x; a8[1] = v0.y * w0.y; a8[2] = v0.z * w0.z; a8[3] = v0.w * w0.w;
                    a8[4] = v1.x * w1.x; a8[5] = v1.y * w1.y; a8[6] = v1.z * w1.z; a8[7] = v1.w * w1.w;
                } else {
                    const uint4 raw = *(const uint4*)((const bf16_t*)xsrc + (size_t)m * ldx + k0 + e);
                    unpack_act2<F16>(raw.x, a8[0], a8[1]);
                    unpack_act2<F16>(raw.y, a8[2], a8[3]);
                    unpack_act2<F16>(raw.z, a8[4], a8[5]);
                    unpack_act2<F16>(raw.w, a8[6], a8[7]);
                }
                float am = 0.f;
#pragma unroll
                for (int i = 0; i < 8; ++i) am = fmaxf(am, fabsf(a8[i]));
                am = group_max<4>(am);
                const float d = am / 127.f, id = d > 0.f ? 1.f / d : 0.f;
                int q[8], sum = 0;
#pragma unroll
                for (int i = 0; i < 8; ++i) { q[i] = __float2int_rn(a8[i] * id); sum += q[i]; }
                const float sf = group_sum<4>((float)sum);
                uint2 pk;
                pk.x = (q[0] & 0xFF) | ((q[1] & 0xFF) << 8) | ((q[2] & 0xFF) << 16) | ((uint32_t)(q[3] & 0xFF) << 24);
                pk.y = (q[4] & 0xFF) | ((q[5] & 0xFF) << 8) | ((q[6] & 0xFF) << 16) | ((uint32_t)(q[7] & 0xFF) << 24);
                *(uint2*)(sq + m * SL + e) = pk;
                if ((threadIdx.x & 3) == 0) sd[m * (SL / 32) + e / 32] = make_float2(d, d * sf);
            }
        }
        __syncthreads();
        if constexpr (SRC == SRC_NORM) {
#pragma unroll
            for (int m = 0; m < MM; ++m) {
                if (m < M) {
                    float t = 0.f;
#pragma unroll
                    for (int w = 0; w < QMV_WAVES; ++w) t += nred[m][w];
                    rsv[m] = rsqrtf(t / (float)K + eps);
                }
            }
        }
        xq = sq;
        xds = sd;
        ldq = SL;
        ubase = u0;
    }
    float acc[MM];
#pragma unroll
    for (int m = 0; m < MM; ++m) acc[m] = 0.f;
    // two units in flight per wave: both loads issue before either dot product
    while (u < u1) {
        const int ul = u - ubase;
        const bool hb = u + QMV_WAVES < u1;
#pragma unroll
        for (int m = 0; m < MM; ++m) {
            if (m < M) {
                const int8_t* x = xq + (size_t)m * ldq;
                const float2* ds = xds + (size_t)m * (ldq / 32);
                acc[m] += a.dot(x + (size_t)ul * U::ELEMS, ds + ul * (U::ELEMS / 32), h);
                if (hb) acc[m] += b.dot(x + (size_t)(ul + QMV_WAVES) * U::ELEMS, ds + (ul + QMV_WAVES) * (U::ELEMS / 32), h);
            }
        }
        u += 2 * QMV_WAVES;
        if (u < u1) a.load(wg + (size_t)u * U::BYTES, r, h);
        if (u + QMV_WAVES < u1) b.load(wg + (size_t)(u + QMV_WAVES) * U::BYTES, r, h);
    }
#pragma unroll
    for (int m = 0; m < MM; ++m) acc[m] *= rsv[m];
#pragma unroll
    for (int m = 0; m < MM; ++m) {
        const float v = acc[m] + __shfl_xor(acc[m], 32);
        if (h == 0) red[wave][m][r] = v;
    }
    __syncthreads();
    if (wave != 0) return;
#pragma unroll
    for (int m = 0; m < MM; ++m) {
        if (m >= M) break;
        float v = 0.f;
        if (h == 0) {
#pragma unroll
            for (int w = 0; w < QMV_WAVES; ++w) v += red[w][m][r];
        }
        const int n = g * 32 + r;
        if constexpr (EPI == E16_SWIGLU || EPI == E16_GEGLU) {
            const float up = __shfl_down(v, 16);
            if (h == 0 && r < 16) ((uint16_t*)Cv)[(size_t)m * ldc + g * 16 + r] = f32_to_act<F16>(glu_gate_f<EPI>(v) * up);
        } else if (h == 0) {
            if constexpr (EPI == E16_F32) ((float*)Cv)[(size_t)m * ldc + n] = v;
            else if constexpr (EPI == E16_ACT) ((uint16_t*)Cv)[(size_t)m * ldc + n] = f32_to_act<F16>(v);
            else if (gridDim.y > 1) atomicAdd(((float*)Cv) + (size_t)m * ldc + n, v);
            else ((float*)Cv)[(size_t)m * ldc + n] += v;
        }
    }
}

// Batch-1 GEMV with the activation prologue fused (SRC_ACT / SRC_NORM) for at most two units per wave (K slices
// of <= 4096): straight-line code with no unit loop, and the workgroup's activation slice is read BEFORE the
// weights are requested — loads complete in issue order for s_waitcnt, so qmv_kernel's prologue (issued after
// the weights) waited for the wave's whole weight stream before it could start the norm / quantisation.
// SRC_NORM runs unsplit (ks = 1, K = 4096): the slice is the whole row and the norm's sum of squares comes
// from the same registers.
// EPI_ROPEKV: the qkv projection's epilogue does the RoPE (adjacent-pair rotation over the whole head) and the
// paged KV append itself — q rows go to `qo` (bf16), k / v rows into the caches at slots[0] — so no separate
// rope_kv launch runs at batch 1. Column c of this launch is column n_off + c of the fused q|k|v row.
constexpr int EPI_ROPEKV = 5;
struct QRope {
    const int* pos;
    const int* slots;
    const float* inv_freq;
    const float* bias;  // this part's bias (nullptr: none)
    float attn_factor;
    int Hq, Hkv, D, n_off, block_size;
    bf16_t* qo;
    bf16_t* kc;
    bf16_t* vc;
};

// NU: weight units per wave (2: K slices <= 16 units, e.g. K = 4096; 4: <= 32 units, the 8192-wide rows of 70B-class
// models). The activation slice is read in NU / 2 passes of 8 elements per thread (4096 per pass).
// Split K (gridDim.y > 1) with an epilogue that needs whole sums (RoPE / KV append, SwiGLU, 16-bit store): the
// workgroups' partial column sums meet in the fp32 workspace `skw` and the last workgroup of each column group
// (ticket `skc[g]`) runs the epilogue on the total, then re-zeroes its workspace columns and ticket (graph replays
// start clean). Lets the narrow batch-1 projections (qkv parts of 1024-6144 columns: 32-192 column groups) use
// every CU. SRC_NORM then reads the whole row once more for the norm's sum of squares.
template <int QT, int EPI, bool F16, int SRC, int NU = 2>
__global__ __launch_bounds__(64 * QMV_WAVES) void qmv1_kernel(const uint8_t* __restrict__ W, int N, int K,
                                                              void* __restrict__ Cv, const void* __restrict__ xsrc,
                                                              const float* __restrict__ nw, float eps, QRope rp,
                                                              float* __restrict__ skw, unsigned* __restrict__ skc) {
    using U = TUnit<QT>;
    constexpr int NT = 64 * QMV_WAVES;
    constexpr int NP = NU / 2;  // activation passes of 8 elements per thread
    static_assert(SRC == SRC_ACT || SRC == SRC_NORM, "fused prologue only");
    static_assert(NU == 2 || NU == 4, "units per wave");
    __shared__ float red[QMV_WAVES][32];
    __shared__ float nred[QMV_WAVES];
    extern __shared__ __attribute__((aligned(16))) char qmv1_smem[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int r = lane & 31, h = lane >> 5;
    const int g = blockIdx.x;
    const int nunit = K / U::ELEMS;  // SRC_NORM: K == 4096 NU (checked by the launcher)
    const int per = (nunit + gridDim.y - 1) / gridDim.y;
    const int u0 = blockIdx.y * per, u1 = min(nunit, u0 + per);
    const int k0 = u0 * U::ELEMS, klen = max(0, u1 - u0) * U::ELEMS;
    const uint8_t* wg = W + (size_t)g * nunit * U::BYTES;
    // 1. this workgroup's slice of the activation row (8 elements per thread per pass; SRC_NORM: the whole row,
    //    ks = 1) and, for the norm, its weights
    float a8[NP][8], w8[NP][8];
#pragma unroll
    for (int ps = 0; ps < NP; ++ps) {
        const int er = 8 * threadIdx.x + 8 * NT * ps, e = k0 + min(er, max(klen - 8, 0));  // clamped: a valid address
        if constexpr (SRC == SRC_NORM) {
            const float* xr = (const float*)xsrc + e;
            const float4 v0 = *(const float4*)xr, v1 = *(const float4*)(xr + 4);
            const float4 n0 = *(const float4*)(nw + e), n1 = *(const float4*)(nw + e + 4);
            a8[ps][0] = v0.x; a8[ps][1] = v0.y; a8[ps][2] = v0.z; a8[ps][3] = v0.w;
            a8[ps][4] = v1.x; a8[ps][5] = v1.y; a8[ps][6] = v1.z; a8[ps][7] = v1.w;
            w8[ps][0] = n0.x; w8[ps][1] = n0.y; w8[ps][2] = n0.z; w8[ps][3] = n0.w;
            w8[ps][4] = n1.x; w8[ps][5] = n1.y; w8[ps][6] = n1.z; w8[ps][7] = n1.w;
        } else {
            const uint4 raw = *(const uint4*)((const bf16_t*)xsrc + e);
            unpack_act2<F16>(raw.x, a8[ps][0], a8[ps][1]);
            unpack_act2<F16>(raw.y, a8[ps][2], a8[ps][3]);
            unpack_act2<F16>(raw.z, a8[ps][4], a8[ps][5]);
            unpack_act2<F16>(raw.w, a8[ps][6], a8[ps][7]);
        }
    }
    asm volatile("" ::: "memory");  // the row reads stay ahead of the weight requests
    // 2. this wave's (at most) NU weight units: u0 + wave + 8 j
    U un[NU];
    bool hv[NU];
    const int u = u0 + wave;
#pragma unroll
    for (int j = 0; j < NU; ++j) {
        hv[j] = u + QMV_WAVES * j < u1;
        if (hv[j]) un[j].load(wg + (size_t)(u + QMV_WAVES * j) * U::BYTES, r, h);
    }
    // 3. norm + quantisation of the slice into LDS while the weights stream
    int8_t* sq = (int8_t*)qmv1_smem;
    float2* sd = (float2*)(qmv1_smem + klen);
    float rs = 1.f;
    if constexpr (SRC == SRC_NORM) {
        float ss = 0.f;
        if (gridDim.y == 1) {  // the slice is the whole row
#pragma unroll
            for (int ps = 0; ps < NP; ++ps)
#pragma unroll
                for (int j = 0; j < 8; ++j) ss += a8[ps][j] * a8[ps][j];
        } else {
            for (int e = 8 * threadIdx.x; e < K; e += 8 * NT) {
                const float4 v0 = *(const float4*)((const float*)xsrc + e), v1 = *(const float4*)((const float*)xsrc + e + 4);
                ss += v0.x * v0.x + v0.y * v0.y + v0.z * v0.z + v0.w * v0.w + v1.x * v1.x + v1.y * v1.y + v1.z * v1.z +
                      v1.w * v1.w;
            }
        }
        ss = wave_sum(ss);
        if (lane == 0) nred[wave] = ss;
    }
#pragma unroll
    for (int ps = 0; ps < NP; ++ps) {
        const int er = 8 * threadIdx.x + 8 * NT * ps;
        if (er < klen) {  // whole 4-lane groups (klen % 256 == 0)
            float v8[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v8[j] = SRC == SRC_NORM ? a8[ps][j] * w8[ps][j] : a8[ps][j];
            float am = 0.f;
#pragma unroll
            for (int j = 0; j < 8; ++j) am = fmaxf(am, fabsf(v8[j]));
            am = group_max<4>(am);
            const float d = am / 127.f, id = d > 0.f ? 1.f / d : 0.f;
            int q[8], sum = 0;
#pragma unroll
            for (int j = 0; j < 8; ++j) { q[j] = __float2int_rn(v8[j] * id); sum += q[j]; }
            const float sf = group_sum<4>((float)sum);
            uint2 pk;
            pk.x = (q[0] & 0xFF) | ((q[1] & 0xFF) << 8) | ((q[2] & 0xFF) << 16) | ((uint32_t)(q[3] & 0xFF) << 24);
            pk.y = (q[4] & 0xFF) | ((q[5] & 0xFF) << 8) | ((q[6] & 0xFF) << 16) | ((uint32_t)(q[7] & 0xFF) << 24);
            *(uint2*)(sq + er) = pk;
            if ((threadIdx.x & 3) == 0) sd[er / 32] = make_float2(d, d * sf);
        }
    }
    __syncthreads();
    if constexpr (SRC == SRC_NORM) {
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < QMV_WAVES; ++w) t += nred[w];
        rs = rsqrtf(t / (float)K + eps);
    }
    // 4. dot products
    float acc = 0.f;
    const int ul = u - u0;
#pragma unroll
    for (int j = 0; j < NU; ++j) {
        const int uj = ul + QMV_WAVES * j;
        if (hv[j]) acc += un[j].dot(sq + (size_t)uj * U::ELEMS, sd + uj * (U::ELEMS / 32), h);
    }
    acc *= rs;
    {
        const float v = acc + __shfl_xor(acc, 32);
        if (h == 0) red[wave][r] = v;
    }
    __syncthreads();
    if (wave != 0) return;
    float v = 0.f;
    if (h == 0) {
#pragma unroll
        for (int w = 0; w < QMV_WAVES; ++w) v += red[w][r];
    }
    const int n = g * 32 + r;
    if (EPI != E16_ADD_F32 && gridDim.y > 1) {
        // hand-off without agent fences (each is an L2 write-back / invalidate, ~3.5 us): the partials are agent-scope
        // atomics, completed (vmcnt) before the ticket; the last workgroup reads them with agent-scope (sc1) loads
        if (h == 0) atomicAdd(skw + n, v);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        unsigned last = 0;
        if (lane == 0) last = __hip_atomic_fetch_add(skc + g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.y - 1;
        last = __shfl(last, 0);
        if (!last) return;
        if (h == 0) {
            v = __hip_atomic_load(skw + n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            atomicExch(skw + n, 0.f);
        }
        if (lane == 0) atomicExch(skc + g, 0u);
    }
    if constexpr (EPI == EPI_ROPEKV) {
        if (rp.bias) v += rp.bias[n];
        const float partner = __shfl_xor(v, 1);  // the other element of this adjacent rotation pair
        const int c = rp.n_off + n, hh = c / rp.D, d = c - hh * rp.D;
        if (h == 0) {
            float y = v;
            if (hh < rp.Hq + rp.Hkv) {
                float sv, cv;
                sincosf((float)rp.pos[0] * rp.inv_freq[d >> 1], &sv, &cv);
                cv *= rp.attn_factor;
                sv *= rp.attn_factor;
                y = (d & 1) ? partner * sv + v * cv : v * cv - partner * sv;
            }
            const uint16_t yb = (uint16_t)(pack_bf16x2(y, 0.f) & 0xFFFF);
            if (hh < rp.Hq) {
                rp.qo[(size_t)hh * rp.D + d] = yb;
            } else {
                const int slot = rp.slots[0];
                if (slot >= 0) {
                    const bool isk = hh < rp.Hq + rp.Hkv;
                    const int kvh = hh - rp.Hq - (isk ? 0 : rp.Hkv);
                    const size_t e = (((size_t)(slot / rp.block_size) * rp.Hkv + kvh) * rp.block_size +
                                      slot % rp.block_size) * rp.D + d;
                    (isk ? rp.kc : rp.vc)[e] = yb;
                }
            }
        }
    } else if constexpr (EPI == E16_SWIGLU || EPI == E16_GEGLU) {
        const float up = __shfl_down(v, 16);
        if (h == 0 && r < 16) ((uint16_t*)Cv)[g * 16 + r] = f32_to_act<F16>(glu_gate_f<EPI>(v) * up);
    } else if (h == 0) {
        if constexpr (EPI == E16_F32) ((float*)Cv)[n] = v;
        else if constexpr (EPI == E16_ACT) ((uint16_t*)Cv)[n] = f32_to_act<F16>(v);
        else if (gridDim.y > 1) atomicAdd(((float*)Cv) + n, v);
        else ((float*)Cv)[n] += v;
    }
}

// ---- dequantise whole rows (output features) of a t32 weight: embedding gather / debugging ----
template <int QT, bool F16>
__global__ __launch_bounds__(256) void dequant_t32_kernel(const uint8_t* __restrict__ W, const int* __restrict__ rows,
                                                          int K, uint16_t* __restrict__ ob, float* __restrict__ of,
                                                          int ldo) {
    const int orow = blockIdx.y;
    const int n = rows ? rows[orow] : orow;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int chunk = blockIdx.x * 4 + wave;  // 256 elements per wave
    if (chunk * 256 >= K) return;
    const int g = n >> 5, r = n & 31;
    const int e = 4 * lane;  // this lane's 4 consecutive elements of the chunk
    float v[4];
    if constexpr (QT == MXQ_Q8_0) {
        const int kt = chunk * 4 + (e >> 6), u = e & 63;
        const uint8_t* base = W + ((size_t)g * (K / 64) + kt) * 2176;
        const uint32_t dw = *(const uint32_t*)(base + r * 4);
        const float d = half_to_f32(u < 32 ? (dw & 0xFFFF) : (dw >> 16));
        const uint32_t qq = *(const uint32_t*)(base + 128 + (u >> 4) * 512 + r * 16 + (u & 15));
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = d * (float)(int8_t)((qq >> (8 * i)) & 0xFF);
    } else if constexpr (QT == MXQ_Q4_K || QT == MXQ_Q5_K) {
        constexpr int UB = QT == MXQ_Q4_K ? 4608 : 5632;
        const uint8_t* base = W + ((size_t)g * (K / 256) + chunk) * UB;
        const u32x4 hd = *(const u32x4*)(base + r * 16);
        const int jq = e >> 6, u = e & 63, b = u & 31;
        const uint32_t qq = *(const uint32_t*)(base + 512 + jq * 1024 + (b >> 4) * 512 + r * 16 + (b & 15));
        int sc, mn;
        q4k_scale_min_w(hd[1], hd[2], hd[3], 2 * jq + (u >> 5), sc, mn);
        const float d = half_to_f32(hd[0] & 0xFFFF) * (float)sc, m = half_to_f32(hd[0] >> 16) * (float)mn;
        const int sh = (u >> 5) * 4;
        uint32_t hb = 0;
        if constexpr (QT == MXQ_Q5_K) hb = *(const uint32_t*)(base + 4608 + (b >> 4) * 512 + r * 16 + (b & 15));
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            int qv = (int)((qq >> (8 * i + sh)) & 0xF);
            if constexpr (QT == MXQ_Q5_K) qv |= (int)(((hb >> (8 * i + 2 * jq + (u >> 5))) & 1) << 4);
            v[i] = d * (float)qv - m;
        }
    } else if constexpr (QT == MXQ_MX4F || QT == MXQ_MX5F) {
        constexpr int KTB = QT == MXQ_MX5F ? 1280 : 1024;
        const uint8_t* base = W + ((size_t)g * (K / 256) + chunk) * (1024 + 4 * KTB);
        const int jq = e >> 6, u = e & 63, b = u & 31, sb = 2 * jq + (u >> 5);
        const uint8_t* kt = base + 1024 + jq * KTB;
        const uint32_t qq = *(const uint32_t*)(kt + (b >> 4) * 512 + r * 16 + (b & 15));
        const uint32_t hw = *(const uint32_t*)(base + (sb >> 2) * 512 + r * 16 + 4 * ((sb & 3) >> 1));
        const uint32_t mw = *(const uint32_t*)(base + (sb >> 2) * 512 + r * 16 + 8 + 4 * ((sb & 3) >> 1));
        const float s = half_to_f32((sb & 1) ? (hw >> 16) : (hw & 0xFFFF));
        const float m = half_to_f32((sb & 1) ? (mw >> 16) : (mw & 0xFFFF));
        const int sh = (u >> 5) * 4;
        uint32_t hb = 0;
        if constexpr (QT == MXQ_MX5F) hb = *(const uint32_t*)(kt + 1024 + r * 8 + (u >> 5) * 4) >> (u & 31);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            int qv = (int)((qq >> (8 * i + sh)) & 0xF);
            if constexpr (QT == MXQ_MX5F) qv |= (int)((hb >> i) & 1) << 4;
            v[i] = s * (float)qv + m;
        }
    } else if constexpr (QT == MXQ_Q3_K || QT == MXQ_Q2_K) {
        // element e = 128 n + 32 j + 16 half + i (4 consecutive i per lane)
        constexpr int UB = QT == MXQ_Q3_K ? 3584 : 2688, QO = QT == MXQ_Q3_K ? 1536 : 640;
        const uint8_t* base = W + ((size_t)g * (K / 256) + chunk) * UB;
        const int n = e >> 7, j = (e >> 5) & 3, half = (e >> 4) & 1, i0 = e & 15;
        const uint32_t qq = *(const uint32_t*)(base + QO + n * 1024 + half * 512 + r * 16 + i0) >> (2 * j);
        const int isx = 8 * n + 2 * j + half;
        if constexpr (QT == MXQ_Q3_K) {
            const uint32_t hm = *(const uint32_t*)(base + 512 + half * 512 + r * 16 + i0) >> (4 * n + j);
            const uint8_t* sc = base + r * 16;
            const int lo = (isx < 8 ? sc[isx] : sc[isx - 8] >> 4) & 15;
            const int hi = (sc[8 + (isx & 3)] >> (2 * (isx >> 2))) & 3;
            const float d = half_to_f32(*(const uint16_t*)(base + r * 16 + 12)) * (float)((lo | (hi << 4)) - 32);
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = d * (float)((int)(((qq >> (8 * i)) & 3) | (((hm >> (8 * i)) & 1) << 2)) - 4);
        } else {
            const uint32_t b = base[r * 16 + isx], dw = *(const uint32_t*)(base + 512 + r * 4);
            const float d = half_to_f32(dw & 0xFFFF) * (float)(b & 15), m = half_to_f32(dw >> 16) * (float)(b >> 4);
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = d * (float)((qq >> (8 * i)) & 3) - m;
        }
    } else {
        const uint8_t* base = W + ((size_t)g * (K / 256) + chunk) * 6784;
        const int jq = e >> 6, u = e & 63, b = u & 31, s16 = u >> 4;
        const uint8_t* p = base + 640 + jq * 1536;
        const uint32_t ql = *(const uint32_t*)(p + (b >> 4) * 512 + r * 16 + (b & 15));
        const uint32_t qh = *(const uint32_t*)(p + 1024 + r * 16 + (u & 15));
        const float d = half_to_f32(*(const uint32_t*)(base + 512 + r * 4) & 0xFFFF) *
                        (float)(int8_t)base[r * 16 + 4 * jq + s16];
        const int sh = (u >> 5) * 4;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int q = (int)((ql >> (8 * i + sh)) & 0xF) | (int)(((qh >> (8 * i + 2 * s16)) & 0x3) << 4);
            v[i] = d * (float)(q - 32);
        }
    }
    const int k0 = chunk * 256 + e;
    if (ob) {
        uint2 p;
        p.x = pack_act2<F16>(v[0], v[1]);
        p.y = pack_act2<F16>(v[2], v[3]);
        *(uint2*)(ob + (size_t)orow * ldo + k0) = p;
    }
    if (of) *(float4*)(of + (size_t)orow * ldo + k0) = make_float4(v[0], v[1], v[2], v[3]);
}

template <int QT, int MM, int EPI>
static int launch_qmv(const int8_t* xq, const float2* xds, const uint8_t* W, int M, int N, int K, int ks, void* C,
                      int ldc, hipStream_t st, int src = SRC_Q8, const void* xsrc = nullptr, int ldx = 0,
                      const float* nw = nullptr, float eps = 0.f) {
    if (src == SRC_Q8) {
        MX_ACT_DISPATCH(qmv_kernel<QT, MM, EPI, F16, SRC_Q8><<<dim3(N / 32, ks), 64 * QMV_WAVES, 0, st>>>(
            xq, xds, W, M, N, K, C, ldc, nullptr, 0, nullptr, 0.f));
    } else {
        const int per = (K / TUnit<QT>::ELEMS + ks - 1) / ks;
        const size_t sl = (size_t)per * TUnit<QT>::ELEMS;
        const size_t lds = MM * (sl + sl / 32 * sizeof(float2));
        if (lds > 64 * 1024) return (int)hipErrorInvalidValue;
        // qmv1: batch 1, at most four units per wave; the norm needs the whole row in one workgroup (ks = 1)
        if (MM == 1 && M == 1 && per <= 4 * QMV_WAVES && g_qmv1_on &&
            (src == SRC_ACT || ((K == 4096 || K == 8192) && ks == 1 && per == K / TUnit<QT>::ELEMS))) {
            const bool four = per > 2 * QMV_WAVES;
            if (src == SRC_ACT) {
                if (four)
                    MX_ACT_DISPATCH(qmv1_kernel<QT, EPI, F16, SRC_ACT, 4><<<dim3(N / 32, ks), 64 * QMV_WAVES, lds, st>>>(
                        W, N, K, C, xsrc, nullptr, 0.f, QRope{}, nullptr, nullptr));
                else
                    MX_ACT_DISPATCH(qmv1_kernel<QT, EPI, F16, SRC_ACT><<<dim3(N / 32, ks), 64 * QMV_WAVES, lds, st>>>(
                        W, N, K, C, xsrc, nullptr, 0.f, QRope{}, nullptr, nullptr));
            } else {
                if (four)
                    MX_ACT_DISPATCH(qmv1_kernel<QT, EPI, F16, SRC_NORM, 4><<<dim3(N / 32, ks), 64 * QMV_WAVES, lds, st>>>(
                        W, N, K, C, xsrc, nw, eps, QRope{}, nullptr, nullptr));
                else
                    MX_ACT_DISPATCH(qmv1_kernel<QT, EPI, F16, SRC_NORM><<<dim3(N / 32, ks), 64 * QMV_WAVES, lds, st>>>(
                        W, N, K, C, xsrc, nw, eps, QRope{}, nullptr, nullptr));
            }
            MXK_CHECK_LAUNCH();
        }
        if (src == SRC_ACT) {
            MX_ACT_DISPATCH(qmv_kernel<QT, MM, EPI, F16, SRC_ACT><<<dim3(N / 32, ks), 64 * QMV_WAVES, lds, st>>>(
                nullptr, nullptr, W, M, N, K, C, ldc, xsrc, ldx, nullptr, 0.f));
        } else {
            MX_ACT_DISPATCH(qmv_kernel<QT, MM, EPI, F16, SRC_NORM><<<dim3(N / 32, ks), 64 * QMV_WAVES, lds, st>>>(
                nullptr, nullptr, W, M, N, K, C, ldc, xsrc, ldx, nw, eps));
        }
    }
    MXK_CHECK_LAUNCH();
}

// X as q8 (int8 [M][K] + float2 [M][K/32]); W t32-tiled; M <= 4; N % 32 == 0; K % 256 == 0.
// epi: 0 fp32 store, 1 act16 store, 2 fp32 accumulate, 3/4 SwiGLU/GeGLU (act16 [M, N/2]).
// ks > 1 splits K over workgroups and needs epi 2 (fp32 atomics).
extern "C" int mxk_qmv(int qtype, int epi, const int8_t* xq, const float2* xds, const uint8_t* W, int M, int N,
                       int K, int ks, void* C, int ldc, hipStream_t st) {
    if (M <= 0) return 0;
    if (M > 4 || K % 256 || N % 32 || ks < 1 || (ks > 1 && epi != E16_ADD_F32)) return (int)hipErrorInvalidValue;
#define QMV_M(QT_, EPI_)                                                                \
    if (M == 1) return launch_qmv<QT_, 1, EPI_>(xq, xds, W, M, N, K, ks, C, ldc, st);   \
    if (M == 2) return launch_qmv<QT_, 2, EPI_>(xq, xds, W, M, N, K, ks, C, ldc, st);   \
    return launch_qmv<QT_, 4, EPI_>(xq, xds, W, M, N, K, ks, C, ldc, st);
#define QMV_EPI(QT_)                                    \
    switch (epi) {                                      \
        case E16_F32: { QMV_M(QT_, E16_F32) }           \
        case E16_ACT: { QMV_M(QT_, E16_ACT) }           \
        case E16_ADD_F32: { QMV_M(QT_, E16_ADD_F32) }   \
        case E16_SWIGLU: { QMV_M(QT_, E16_SWIGLU) }     \
        case E16_GEGLU: { QMV_M(QT_, E16_GEGLU) }       \
    }
    switch (qtype) {
        case MXQ_Q4_K: QMV_EPI(MXQ_Q4_K) break;
        case MXQ_Q5_K: QMV_EPI(MXQ_Q5_K) break;
        case MXQ_Q6_K: QMV_EPI(MXQ_Q6_K) break;
        case MXQ_Q8_0: QMV_EPI(MXQ_Q8_0) break;
        case MXQ_MX4F: QMV_EPI(MXQ_MX4F) break;
        case MXQ_MX5F: QMV_EPI(MXQ_MX5F) break;
        case MXQ_Q3_K: QMV_EPI(MXQ_Q3_K) break;
        case MXQ_Q2_K: QMV_EPI(MXQ_Q2_K) break;
    }
#undef QMV_EPI
#undef QMV_M
    return (int)hipErrorInvalidValue;
}

// The same GEMV with the activation quantisation (and optionally the RMSNorm in front of it) fused into
// the prologue: src 1 = x 16-bit [M, K] (row stride ldx); src 2 = x fp32 residual [M, K], y = x / rms(x) * nw.
extern "C" int mxk_qmv_x(int qtype, int epi, int src, const void* x, int ldx, const float* nw, float eps,
                         const uint8_t* W, int M, int N, int K, int ks, void* C, int ldc, hipStream_t st) {
    if (M <= 0) return 0;
    if (M > 4 || K % 256 || N % 32 || ks < 1 || (ks > 1 && epi != E16_ADD_F32) || (src != SRC_ACT && src != SRC_NORM) ||
        (src == SRC_NORM && !nw) || ((uintptr_t)x & 15) || (ldx % 8))
        return (int)hipErrorInvalidValue;
#define QMVX_M(QT_, EPI_)                                                                                   \
    if (M == 1) return launch_qmv<QT_, 1, EPI_>(nullptr, nullptr, W, M, N, K, ks, C, ldc, st, src, x, ldx, nw, eps); \
    if (M == 2) return launch_qmv<QT_, 2, EPI_>(nullptr, nullptr, W, M, N, K, ks, C, ldc, st, src, x, ldx, nw, eps); \
    return launch_qmv<QT_, 4, EPI_>(nullptr, nullptr, W, M, N, K, ks, C, ldc, st, src, x, ldx, nw, eps);
#define QMVX_EPI(QT_)                                   \
    switch (epi) {                                      \
        case E16_F32: { QMVX_M(QT_, E16_F32) }          \
        case E16_ACT: { QMVX_M(QT_, E16_ACT) }          \
        case E16_ADD_F32: { QMVX_M(QT_, E16_ADD_F32) }  \
        case E16_SWIGLU: { QMVX_M(QT_, E16_SWIGLU) }    \
        case E16_GEGLU: { QMVX_M(QT_, E16_GEGLU) }      \
    }
    switch (qtype) {
        case MXQ_Q4_K: QMVX_EPI(MXQ_Q4_K) break;
        case MXQ_Q5_K: QMVX_EPI(MXQ_Q5_K) break;
        case MXQ_Q6_K: QMVX_EPI(MXQ_Q6_K) break;
        case MXQ_Q8_0: QMVX_EPI(MXQ_Q8_0) break;
        case MXQ_MX4F: QMVX_EPI(MXQ_MX4F) break;
        case MXQ_MX5F: QMVX_EPI(MXQ_MX5F) break;
        case MXQ_Q3_K: QMVX_EPI(MXQ_Q3_K) break;
        case MXQ_Q2_K: QMVX_EPI(MXQ_Q2_K) break;
    }
#undef QMVX_EPI
#undef QMVX_M
    return (int)hipErrorInvalidValue;
}

// Batch-1 qkv GEMV with the input RMSNorm fused in front and RoPE + paged KV append fused behind (EPI_ROPEKV):
// x fp32 [1, K] residual row (K = 4096, or 8192: 70B-class hidden size, four units per wave), W one t32 part (q, k, v or a fused run of them) whose columns start at column
// n_off of the q|k|v row; rotation over whole heads of D (adjacent pairs, rot_dim == D), bf16 q and caches.
extern "C" int mxk_qmv1_rope(int qtype, const float* x, const float* nw, float eps, const uint8_t* W, int N, int K,
                             int n_off, const int* pos, const int* slots, const float* inv_freq, const float* bias,
                             float attn_factor, int Hq, int Hkv, int D, bf16_t* qo, bf16_t* kc, bf16_t* vc,
                             int block_size, int ks, float* skw, unsigned* skc, hipStream_t st) {
    // ks > 1: split K over ks workgroups per column group (skw: >= N zeroed floats, skc: >= N / 32 zeroed tickets)
    if (ks < 1 || (ks > 1 && (!skw || !skc)) || (K / 256) % ks) return (int)hipErrorInvalidValue;
    if ((K != 4096 && K != 8192) || N % 32 || (D != 64 && D != 128) || n_off % 32 || ((uintptr_t)x & 15))
        return (int)hipErrorInvalidValue;
    const QRope rp{pos, slots, inv_freq, bias, attn_factor, Hq, Hkv, D, n_off, block_size, qo, kc, vc};
    const size_t lds = (size_t)K + K / 32 * sizeof(float2);
#define QR1(QT_)                                                                                                     \
    if (K == 8192)                                                                                                   \
        qmv1_kernel<QT_, EPI_ROPEKV, true, SRC_NORM, 4><<<dim3(N / 32, ks), 64 * QMV_WAVES, lds, st>>>(W, N, K, nullptr, x, \
                                                                                                    nw, eps, rp, skw, skc); \
    else                                                                                                             \
        qmv1_kernel<QT_, EPI_ROPEKV, true, SRC_NORM><<<dim3(N / 32, ks), 64 * QMV_WAVES, lds, st>>>(W, N, K, nullptr, x, nw, \
                                                                                                 eps, rp, skw, skc)
    switch (qtype) {
        case MXQ_Q4_K: QR1(MXQ_Q4_K); break;
        case MXQ_Q5_K: QR1(MXQ_Q5_K); break;
        case MXQ_Q6_K: QR1(MXQ_Q6_K); break;
        case MXQ_Q3_K: QR1(MXQ_Q3_K); break;
        case MXQ_Q2_K: QR1(MXQ_Q2_K); break;
        default: return (int)hipErrorInvalidValue;
    }
#undef QR1
    MXK_CHECK_LAUNCH();
}

extern "C" int mxk_qmv1_enable(int on) {
    g_qmv1_on = on;
    return 0;
}

// Grouped (mixture-of-experts) decode GEMV on t32 expert stacks: one workgroup per (32-column group g of one expert's
// N, token-expert pair p). Pair p multiplies activation row p / xdiv (xdiv = k: the token's normed hidden state for
// gate|up; 1: the pair's own gate|up activations for the down projection) by expert ids[p] - e0's columns
// (W = the experts' [N, K] t32 matrices back to back) and writes output row p (pair order, no sort). Pairs routed to
// experts outside [e0, e0 + El) (another rank's, expert parallelism) are skipped: their rows stay as the caller
// initialised them. Every workgroup quantises its whole activation row into LDS (q8 per 32, llama.cpp q8_1
// numerics as qmv), two weight units in flight per wave. Used at decode batch sizes (P = T k pairs <= 64), where a
// 32-row grouped GEMM tile would stream each expert through at most a few busy CUs.
template <int QT, int EPI, bool F16>
__global__ __launch_bounds__(64 * QMV_WAVES) void qmv_moe_kernel(const uint8_t* __restrict__ W, int N, int K,
                                                                 const int* __restrict__ ids, int e0, int El,
                                                                 const bf16_t* __restrict__ x, int ldx, int xdiv,
                                                                 void* __restrict__ Cv, int ldc) {
    using U = TUnit<QT>;
    __shared__ float red[QMV_WAVES][32];
    extern __shared__ __attribute__((aligned(16))) char qmv_smem[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int r = lane & 31, h = lane >> 5;
    const int g = blockIdx.x, p = blockIdx.y;
    const int e = ids[p] - e0;
    if (e < 0 || e >= El) return;
    const int nunit = K / U::ELEMS;
    const uint8_t* wg = W + ((size_t)e * (N >> 5) + g) * ((size_t)nunit * U::BYTES);
    U a, b;
    int u = wave;
    if (u < nunit) a.load(wg + (size_t)u * U::BYTES, r, h);
    if (u + QMV_WAVES < nunit) b.load(wg + (size_t)(u + QMV_WAVES) * U::BYTES, r, h);
    int8_t* sq = (int8_t*)qmv_smem;
    float2* sd = (float2*)(qmv_smem + K);
    const bf16_t* xr = x + (size_t)(p / xdiv) * ldx;
    // 8 consecutive elements per lane, 4 lanes per 32-element block (K % 256 == 0: the 4-lane groups enter and
    // leave the loop together)
    for (int e8 = threadIdx.x * 8; e8 < K; e8 += 64 * QMV_WAVES * 8) {
        float a8[8];
        const uint4 raw = *(const uint4*)(xr + e8);
        unpack_act2<F16>(raw.x, a8[0], a8[1]);
        unpack_act2<F16>(raw.y, a8[2], a8[3]);
        unpack_act2<F16>(raw.z, a8[4], a8[5]);
        unpack_act2<F16>(raw.w, a8[6], a8[7]);
        float am = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) am = fmaxf(am, fabsf(a8[i]));
        am = group_max<4>(am);
        const float d = am / 127.f, id = d > 0.f ? 1.f / d : 0.f;
        int q[8], sum = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) { q[i] = __float2int_rn(a8[i] * id); sum += q[i]; }
        const float sf = group_sum<4>((float)sum);
        uint2 pk;
        pk.x = (q[0] & 0xFF) | ((q[1] & 0xFF) << 8) | ((q[2] & 0xFF) << 16) | ((uint32_t)(q[3] & 0xFF) << 24);
        pk.y = (q[4] & 0xFF) | ((q[5] & 0xFF) << 8) | ((q[6] & 0xFF) << 16) | ((uint32_t)(q[7] & 0xFF) << 24);
        *(uint2*)(sq + e8) = pk;
        if ((threadIdx.x & 3) == 0) sd[e8 / 32] = make_float2(d, d * sf);
    }
    __syncthreads();
    float acc = 0.f;
    while (u < nunit) {
        const bool hb = u + QMV_WAVES < nunit;
        acc += a.dot(sq + (size_t)u * U::ELEMS, sd + u * (U::ELEMS / 32), h);
        if (hb) acc += b.dot(sq + (size_t)(u + QMV_WAVES) * U::ELEMS, sd + (u + QMV_WAVES) * (U::ELEMS / 32), h);
        u += 2 * QMV_WAVES;
        if (u < nunit) a.load(wg + (size_t)u * U::BYTES, r, h);
        if (u + QMV_WAVES < nunit) b.load(wg + (size_t)(u + QMV_WAVES) * U::BYTES, r, h);
    }
    {
        const float v = acc + __shfl_xor(acc, 32);
        if (h == 0) red[wave][r] = v;
    }
    __syncthreads();
    if (wave != 0) return;
    float v = 0.f;
    if (h == 0) {
#pragma unroll
        for (int w = 0; w < QMV_WAVES; ++w) v += red[w][r];
    }
    if constexpr (EPI == E16_SWIGLU || EPI == E16_GEGLU) {
        const float up = __shfl_down(v, 16);
        if (h == 0 && r < 16) ((uint16_t*)Cv)[(size_t)p * ldc + g * 16 + r] = f32_to_act<F16>(glu_gate_f<EPI>(v) * up);
    } else if (h == 0) {
        ((float*)Cv)[(size_t)p * ldc + g * 32 + r] = v;
    }
}

// W t32 expert stack [E_local * N, K]; x 16-bit rows (row p / xdiv for pair p); ids [P]; epi 0 fp32 [P, N] or
// 3 / 4 SwiGLU / GeGLU f16 [P, N / 2]. N % 32 == 0, K % 256 == 0, K <= 16384.
extern "C" int mxk_qmv_moe(int qtype, int epi, const uint8_t* W, int N, int K, const int* ids, int P, int e0, int El,
                           const void* x, int ldx, int xdiv, void* C, int ldc, hipStream_t st) {
    if (P <= 0) return 0;
    if (K % 256 || N % 32 || K > 16384 || xdiv < 1 || ((uintptr_t)x & 15) || (ldx % 8)) return (int)hipErrorInvalidValue;
    const size_t lds = (size_t)K + (size_t)K / 32 * sizeof(float2);
    const dim3 grid(N / 32, P);
#define QMOE(QT_, EPI_)                                                                                         \
    MX_ACT_DISPATCH(qmv_moe_kernel<QT_, EPI_, F16><<<grid, 64 * QMV_WAVES, lds, st>>>(                          \
        W, N, K, ids, e0, El, (const bf16_t*)x, ldx, xdiv, C, ldc));                                            \
    MXK_CHECK_LAUNCH();
#define QMOE_EPI(QT_)                                          \
    switch (epi) {                                             \
        case E16_F32: { QMOE(QT_, E16_F32) }                   \
        case E16_SWIGLU: { QMOE(QT_, E16_SWIGLU) }             \
        case E16_GEGLU: { QMOE(QT_, E16_GEGLU) }               \
    }                                                          \
    break;
    switch (qtype) {
        case MXQ_Q4_K: QMOE_EPI(MXQ_Q4_K)
        case MXQ_Q5_K: QMOE_EPI(MXQ_Q5_K)
        case MXQ_Q6_K: QMOE_EPI(MXQ_Q6_K)
        case MXQ_Q8_0: QMOE_EPI(MXQ_Q8_0)
    }
#undef QMOE_EPI
#undef QMOE
    return (int)hipErrorInvalidValue;
}

// Token-major grouped down projection with the MoE combine fused: one workgroup per (32-column group of H, token t).
// The workgroup quantises the token's k pair rows of the SwiGLU activations (act rows t k .. t k + k - 1, q8 per 32)
// into LDS, then its waves walk the k x (F / 256) weight units of the token's experts (unit i: pair i / nu, unit
// i % nu), each dot product scaled by the pair's routing weight before the cross-wave reduction, and the workgroup
// adds the weighted sum into h[t] — no [P, H] buffer, no combine launch, one writer per output (deterministic).
// Pairs routed outside [e0, e0 + El) (another rank's experts) contribute nothing.
template <int QT, bool F16>
__global__ __launch_bounds__(64 * QMV_WAVES) void qmv_moe_down_kernel(const uint8_t* __restrict__ W, int N, int K,
                                                                      const int* __restrict__ ids,
                                                                      const float* __restrict__ wts, int k, int e0,
                                                                      int El, const bf16_t* __restrict__ act, int lda,
                                                                      float* __restrict__ h, int ldh) {
    using U = TUnit<QT>;
    __shared__ float red[QMV_WAVES][32];
    extern __shared__ __attribute__((aligned(16))) char qmd_smem[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int r = lane & 31, hh = lane >> 5;
    const int g = blockIdx.x, t = blockIdx.y;
    const int nu = K / U::ELEMS, total = k * nu;
    int8_t* sq = (int8_t*)qmd_smem;                      // [k][K]
    float2* sd = (float2*)(qmd_smem + (size_t)k * K);    // [k][K / 32]
    // unit j of this wave: flat index wave + QMV_WAVES j -> (pair, unit); weights requested before the quantisation
    auto unit_ptr = [&](int i, int& pr, int& ok) -> const uint8_t* {
        pr = min(i / nu, k - 1);  // (i >= total: a valid pair index, never used)
        const int e = ids[(size_t)t * k + pr] - e0;
        ok = i < total && e >= 0 && e < El;
        return W + ((size_t)(ok ? e : 0) * (N >> 5) + g) * ((size_t)nu * U::BYTES) + (size_t)(i % nu) * U::BYTES;
    };
    U a, b;
    int pa = 0, pb = 0, oka = 0, okb = 0;
    int i = wave;
    {
        const uint8_t* pa_ = unit_ptr(i, pa, oka);
        if (oka) a.load(pa_, r, hh);
        const uint8_t* pb_ = unit_ptr(i + QMV_WAVES, pb, okb);
        if (okb) b.load(pb_, r, hh);
    }
    for (int e8 = threadIdx.x * 8; e8 < k * K; e8 += 64 * QMV_WAVES * 8) {
        const int j = e8 / K, c = e8 % K;
        float a8[8];
        const uint4 raw = *(const uint4*)(act + ((size_t)t * k + j) * lda + c);
        unpack_act2<F16>(raw.x, a8[0], a8[1]);
        unpack_act2<F16>(raw.y, a8[2], a8[3]);
        unpack_act2<F16>(raw.z, a8[4], a8[5]);
        unpack_act2<F16>(raw.w, a8[6], a8[7]);
        float am = 0.f;
#pragma unroll
        for (int q = 0; q < 8; ++q) am = fmaxf(am, fabsf(a8[q]));
        am = group_max<4>(am);
        const float d = am / 127.f, id = d > 0.f ? 1.f / d : 0.f;
        int q8[8], sum = 0;
#pragma unroll
        for (int q = 0; q < 8; ++q) { q8[q] = __float2int_rn(a8[q] * id); sum += q8[q]; }
        const float sf = group_sum<4>((float)sum);
        uint2 pk;
        pk.x = (q8[0] & 0xFF) | ((q8[1] & 0xFF) << 8) | ((q8[2] & 0xFF) << 16) | ((uint32_t)(q8[3] & 0xFF) << 24);
        pk.y = (q8[4] & 0xFF) | ((q8[5] & 0xFF) << 8) | ((q8[6] & 0xFF) << 16) | ((uint32_t)(q8[7] & 0xFF) << 24);
        *(uint2*)(sq + e8) = pk;
        if ((threadIdx.x & 3) == 0) sd[e8 / 32] = make_float2(d, d * sf);
    }
    __syncthreads();
    float acc = 0.f;
    while (i < total) {
        if (oka) {
            const int u = i % nu;
            acc += wts[(size_t)t * k + pa] * a.dot(sq + (size_t)pa * K + (size_t)u * U::ELEMS,
                                                   sd + (size_t)pa * (K / 32) + u * (U::ELEMS / 32), hh);
        }
        if (okb) {
            const int u = (i + QMV_WAVES) % nu;
            acc += wts[(size_t)t * k + pb] * b.dot(sq + (size_t)pb * K + (size_t)u * U::ELEMS,
                                                   sd + (size_t)pb * (K / 32) + u * (U::ELEMS / 32), hh);
        }
        i += 2 * QMV_WAVES;
        const uint8_t* pa_ = unit_ptr(i, pa, oka);
        if (oka) a.load(pa_, r, hh);
        const uint8_t* pb_ = unit_ptr(i + QMV_WAVES, pb, okb);
        if (okb) b.load(pb_, r, hh);
    }
    {
        const float v = acc + __shfl_xor(acc, 32);
        if (hh == 0) red[wave][r] = v;
    }
    __syncthreads();
    if (wave != 0 || hh != 0) return;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < QMV_WAVES; ++w) v += red[w][r];
    h[(size_t)t * ldh + g * 32 + r] += v;
}

// h [T, N] fp32 += sum_j wts[t, j] * (act[t k + j] . W_{ids[t, j] - e0}^T): W t32 expert stack [El * N, K], act 16-bit
// [T k, K] (the SwiGLU output rows in pair order). N % 32 == 0, K % 256 == 0, k K + k K / 4 <= 64 KB.
extern "C" int mxk_qmv_moe_down(int qtype, const uint8_t* W, int N, int K, const int* ids, const float* wts, int T,
                                int k, int e0, int El, const void* act, int lda, float* h, int ldh, hipStream_t st) {
    if (T <= 0) return 0;
    const size_t lds = (size_t)k * K + (size_t)k * K / 32 * sizeof(float2);
    if (K % 256 || N % 32 || k < 1 || lds > 64 * 1024 || ((uintptr_t)act & 15) || (lda % 8))
        return (int)hipErrorInvalidValue;
    const dim3 grid(N / 32, T);
#define QMD(QT_)                                                                                                  \
    MX_ACT_DISPATCH(qmv_moe_down_kernel<QT_, F16><<<grid, 64 * QMV_WAVES, lds, st>>>(W, N, K, ids, wts, k, e0, El, \
                                                                                     (const bf16_t*)act, lda, h, ldh)); \
    MXK_CHECK_LAUNCH();
    switch (qtype) {
        case MXQ_Q4_K: { QMD(MXQ_Q4_K) }
        case MXQ_Q5_K: { QMD(MXQ_Q5_K) }
        case MXQ_Q6_K: { QMD(MXQ_Q6_K) }
        case MXQ_Q8_0: { QMD(MXQ_Q8_0) }
    }
#undef QMD
    return (int)hipErrorInvalidValue;
}

extern "C" int mxk_dequant_t32(int qtype, const uint8_t* W, const int* rows, int nrows, int K, uint16_t* ob,
                               float* of, int ldo, hipStream_t st) {
    if (nrows <= 0) return 0;
    if (K % 256) return (int)hipErrorInvalidValue;
    dim3 grid((K / 256 + 3) / 4, nrows);
    int rc = 0;
    MX_ACT_DISPATCH({
        switch (qtype) {
            case MXQ_Q4_K: dequant_t32_kernel<MXQ_Q4_K, F16><<<grid, 256, 0, st>>>(W, rows, K, ob, of, ldo); break;
            case MXQ_Q5_K: dequant_t32_kernel<MXQ_Q5_K, F16><<<grid, 256, 0, st>>>(W, rows, K, ob, of, ldo); break;
            case MXQ_Q6_K: dequant_t32_kernel<MXQ_Q6_K, F16><<<grid, 256, 0, st>>>(W, rows, K, ob, of, ldo); break;
            case MXQ_Q8_0: dequant_t32_kernel<MXQ_Q8_0, F16><<<grid, 256, 0, st>>>(W, rows, K, ob, of, ldo); break;
            case MXQ_MX4F: dequant_t32_kernel<MXQ_MX4F, F16><<<grid, 256, 0, st>>>(W, rows, K, ob, of, ldo); break;
            case MXQ_MX5F: dequant_t32_kernel<MXQ_MX5F, F16><<<grid, 256, 0, st>>>(W, rows, K, ob, of, ldo); break;
            case MXQ_Q3_K: dequant_t32_kernel<MXQ_Q3_K, F16><<<grid, 256, 0, st>>>(W, rows, K, ob, of, ldo); break;
            case MXQ_Q2_K: dequant_t32_kernel<MXQ_Q2_K, F16><<<grid, 256, 0, st>>>(W, rows, K, ob, of, ldo); break;
            default: rc = (int)hipErrorInvalidValue;
        }
    });
    if (rc) return rc;
    MXK_CHECK_LAUNCH();
}
