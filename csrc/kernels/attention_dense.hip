// attention_dense.hip — fused MFMA flash attention over dense (non-paged) Q/K/V, for the encoder /
// diffusion / embedding models: BERT & cross-encoders (key padding), Whisper encoder (bidirectional)
// and decoder (causal self-attention, cross-attention to the audio states), UNet / MMDiT attention
// (SURVEY §2.6 K4 for the non-LLM workers).
//
//   O[b, i, h, :] = softmax(scale · Q[b, i, h, :] · K[b, :, h/G, :]^T  (+ masks)) · V[b, :, h/G, :]
//
// Layout: token-major rows with explicit strides (q/k/v/o[(b·S + s)·stride + head·D + d]) so fused
// QKV projections can be consumed in place. 16-bit operands in the library's act16 format (bf16 or
// f16 MFMA), fp32 softmax state, online (flash) softmax in the log2 domain.
// Workgroup: 4 waves x 16 query rows of one head; K/V staged 64 keys at a time into the XOR-swizzled
// LDS images of attention.hip (conflict-free ds_read_b128 for K^T, ds_read_b64_tr_b16 for V).
// Masks: `causal` (key position > query position + (Sk - Sq) dropped) and per-batch key lengths
// `klen` (BERT padding); rows past `qlen[b]` are not written. Optional additive relative-position bias
// `rbias[h][j - i + Sq - 1]` (fp32, T5's bucketed bias table expanded per offset; shared by the batch).
#include "mx_common.h"

#define LOG2E_D 1.4426950408889634f

// K image: row p holds D/8 16-byte chunks; chunk c lives at c ^ f(p) (f < 16: 16 consecutive rows, one chunk
// column, land in 16 different banks). D = 512 uses the D = 128 swizzle (its rows are 4 x as wide, same banking).
template <int D>
MX_DEV int kd_lds_off(int p, int c) {
    const int r = p & 15;
    int f;
    if constexpr (D >= 128) f = r ^ (((r + 4) >> 3) & 1);
    else f = ((r >> 1) & 7) ^ (((r + 4) >> 3) & 1);
    return p * (D * 2) + ((c ^ (f & (D / 8 - 1))) << 4);
}
template <int D>
MX_DEV int vd_lds_off(int p, int nt) {
    int sv;
    if constexpr (D >= 128) sv = (p & 3) | (((p >> 3) & 1) << 2);
    else sv = ((p >> 1) & 1) | (((p >> 3) & 1) << 1);
    return p * (D * 2) + ((nt ^ sv) << 5);
}

template <bool F16>
MX_DEV f32x4 mfma16(const u32x4& a, const u32x4& b, f32x4 c) {
    if constexpr (F16)
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c,
                                                       0, 0, 0);
    else
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b),
                                                        c, 0, 0, 0);
}

template <int D, bool F16>
__global__ __launch_bounds__(256) void attn_dense_kernel(const uint16_t* __restrict__ q, int q_stride,
                                                         const uint16_t* __restrict__ k, int k_stride,
                                                         const uint16_t* __restrict__ v, int v_stride,
                                                         uint16_t* __restrict__ o, int o_stride, int Sq, int Sk,
                                                         int Hq, int Hkv, const int* __restrict__ qlen_b,
                                                         const int* __restrict__ klen_b, int causal, float scale,
                                                         int kv_rows, const float* __restrict__ rbias, int rb_ld) {
    // key tile: 64 keys (D <= 128) or 32 (D = 512: the VAE mid-block's single 512-wide head; K + V tiles 64 KB)
    constexpr int KT = D > 128 ? 32 : 64;
    constexpr int KBYTES = KT * D * 2;
    constexpr int PSTRIDE = (KT + 8) * 2;
    __shared__ __attribute__((aligned(16))) char smem[2 * KBYTES + 4 * 16 * PSTRIDE];
    char* k_lds = smem;
    char* v_lds = smem + KBYTES;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int g = lane >> 4, col = lane & 15;
    const int b = blockIdx.z, h = blockIdx.y;
    const int kvh = h / (Hq / Hkv);
    const int qlen = qlen_b ? qlen_b[b] : Sq;
    const int klen = klen_b ? klen_b[b] : Sk;
    const int row_q0 = blockIdx.x * 64 + wave * 16;
    if (blockIdx.x * 64 >= qlen) return;  // whole workgroup idle (uniform)
    const int shift = Sk - Sq;            // causal: query i sees keys <= i + shift
    int kv_end = klen;
    if (causal) kv_end = min(kv_end, blockIdx.x * 64 + 64 + shift);
    const float qs = scale * LOG2E_D;
    const uint16_t* kb = k + (size_t)b * kv_rows * k_stride + (size_t)kvh * D;
    const uint16_t* vb_ = v + (size_t)b * kv_rows * v_stride + (size_t)kvh * D;

    u32x4 qf[D / 32];
    {
        const int qi = row_q0 + col;
#pragma unroll
        for (int ks = 0; ks < D / 32; ++ks) {
            if (qi < qlen) qf[ks] = *(const u32x4*)(q + ((size_t)b * Sq + qi) * q_stride + (size_t)h * D + 32 * ks + 8 * g);
            else qf[ks] = (u32x4){0, 0, 0, 0};
        }
    }
    f32x4 oacc[D / 16];
#pragma unroll
    for (int i = 0; i < D / 16; ++i) oacc[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
    float mrow[4], lrow[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) { mrow[i] = -INFINITY; lrow[i] = 0.f; }
    char* pw = smem + 2 * KBYTES + wave * 16 * PSTRIDE;

    // K / V tiles software-pipelined one tile deep: the next tile's 16-byte chunks are requested right after
    // this tile is staged in LDS, so their latency hides behind this tile's MFMAs and softmax
    constexpr int CH = KT * D / 8;
    constexpr int NCH = (CH + 255) / 256;  // chunks per thread
    uint4 kr[NCH], vr[NCH];
    auto load_tile = [&](int kt0) {
#pragma unroll
        for (int j = 0; j < NCH; ++j) {
            const int id = threadIdx.x + 256 * j;
            const int p = id / (D / 8), c = id % (D / 8);
            const int pos = kt0 + p;
            kr[j] = make_uint4(0, 0, 0, 0);
            vr[j] = make_uint4(0, 0, 0, 0);
            if (id < CH && pos < kv_end) {
                kr[j] = *(const uint4*)(kb + (size_t)pos * k_stride + c * 8);
                vr[j] = *(const uint4*)(vb_ + (size_t)pos * v_stride + c * 8);
            }
        }
    };
    // (D = 512: a tile is 8 chunks per thread and per operand; prefetching it would spill, so it loads in place)
    constexpr bool PF = D <= 128;
    if (PF && kv_end > 0) load_tile(0);
    for (int kt0 = 0; kt0 < kv_end; kt0 += KT) {
        if constexpr (!PF) load_tile(kt0);
#pragma unroll
        for (int j = 0; j < NCH; ++j) {
            const int id = threadIdx.x + 256 * j;
            if (id >= CH) continue;
            const int p = id / (D / 8), c = id % (D / 8);
            *(uint4*)(k_lds + kd_lds_off<D>(p, c)) = kr[j];
            *(uint4*)(v_lds + vd_lds_off<D>(p, c >> 1) + 16 * (c & 1)) = vr[j];
        }
        if (PF && kt0 + KT < kv_end) load_tile(kt0 + KT);
        __syncthreads();
        constexpr int NT16 = KT / 16;
        f32x4 sacc[NT16];
#pragma unroll
        for (int t = 0; t < NT16; ++t) {
            sacc[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ks = 0; ks < D / 32; ++ks) {
                const u32x4 kf = *(const u32x4*)(k_lds + kd_lds_off<D>(16 * t + col, 4 * ks + g));
                sacc[t] = mfma16<F16>(qf[ks], kf, sacc[t]);
            }
        }
        float rmax[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int qi = row_q0 + 4 * g + i;
            float mx = -INFINITY;
#pragma unroll
            for (int t = 0; t < NT16; ++t) {
                const int kp = kt0 + 16 * t + col;
                float s = sacc[t][i] * qs;
                if (kp >= kv_end || qi >= qlen || (causal && kp > qi + shift)) s = -INFINITY;
                else if (rbias) s += rbias[(size_t)h * rb_ld + (kp - qi + Sq - 1)] * LOG2E_D;
                sacc[t][i] = s;
                mx = fmaxf(mx, s);
            }
            rmax[i] = group_max<16>(mx);
        }
        float alpha[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float mn = fmaxf(mrow[i], rmax[i]);
            alpha[i] = mn == -INFINITY ? 1.f : exp2f(mrow[i] - mn);
            float rs = 0.f;
#pragma unroll
            for (int t = 0; t < NT16; ++t) {
                const float pv = mn == -INFINITY ? 0.f : exp2f(sacc[t][i] - mn);
                sacc[t][i] = pv;
                rs += pv;
            }
            rs = group_sum<16>(rs);
            lrow[i] = lrow[i] * alpha[i] + rs;
            mrow[i] = mn;
        }
#pragma unroll
        for (int nt = 0; nt < D / 16; ++nt)
#pragma unroll
            for (int i = 0; i < 4; ++i) oacc[nt][i] *= alpha[i];
#pragma unroll
        for (int t = 0; t < NT16; ++t)
#pragma unroll
            for (int i = 0; i < 4; ++i)
                *(uint16_t*)(pw + (4 * g + i) * PSTRIDE + (16 * t + col) * 2) = f32_to_act<F16>(sacc[t][i]);
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int ks = 0; ks < KT / 32; ++ks) {
            const u32x4 pa = *(const u32x4*)(pw + col * PSTRIDE + (32 * ks + 8 * g) * 2);
            const int r0 = 32 * ks + 8 * g;
            const int q4 = col >> 2, p4 = col & 3;
#pragma unroll
            for (int nt = 0; nt < D / 16; ++nt) {
                const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                    (MX_LDS s16x4*)(v_lds + vd_lds_off<D>(r0 + q4, nt) + 8 * p4));
                const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                    (MX_LDS s16x4*)(v_lds + vd_lds_off<D>(r0 + 4 + q4, nt) + 8 * p4));
                const u32x2 l2 = __builtin_bit_cast(u32x2, lo), h2 = __builtin_bit_cast(u32x2, hi);
                const u32x4 vv = {l2[0], l2[1], h2[0], h2[1]};
                oacc[nt] = mfma16<F16>(pa, vv, oacc[nt]);
            }
        }
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int qi = row_q0 + 4 * g + i;
        if (qi >= qlen) continue;
        const float inv = lrow[i] > 0.f ? 1.f / lrow[i] : 0.f;
#pragma unroll
        for (int nt = 0; nt < D / 16; ++nt)
            o[((size_t)b * Sq + qi) * o_stride + (size_t)h * D + 16 * nt + col] = f32_to_act<F16>(oacc[nt][i] * inv);
    }
}

// q/k/v/o: 16-bit (act16 mode) token-major with row strides in elements; B batches of Sq queries /
// Sk keys; Hq query heads, Hkv key/value heads (Hq % Hkv == 0); D in {64, 128, 512}. K/V rows of batch b
// start at row b * kv_rows (kv_rows = 0 -> Sk): a fixed-capacity KV cache [B, cap, H*D] is read in
// place with Sk = valid length (causal offset Sk - Sq) or Sk = cap with per-batch klen.
extern "C" int mxk_attn_dense(const uint16_t* q, int q_stride, const uint16_t* k, int k_stride, const uint16_t* v,
                              int v_stride, uint16_t* o, int o_stride, int B, int Sq, int Sk, int Hq, int Hkv, int D,
                              const int* qlen, const int* klen, int causal, float scale, int kv_rows,
                              const float* rbias, int rb_ld, hipStream_t st) {
    if (B <= 0 || Sq <= 0) return 0;
    if (kv_rows <= 0) kv_rows = Sk;
    if (Hq % Hkv || (D != 64 && D != 128 && D != 512)) return (int)hipErrorInvalidValue;
    if ((q_stride | k_stride | v_stride) & 7) return (int)hipErrorInvalidValue;
    dim3 grid((Sq + 63) / 64, Hq, B);
    MX_ACT_DISPATCH({
        if (D == 512)
            attn_dense_kernel<512, F16><<<grid, 256, 0, st>>>(q, q_stride, k, k_stride, v, v_stride, o, o_stride, Sq, Sk,
                                                             Hq, Hkv, qlen, klen, causal, scale, kv_rows, rbias, rb_ld);
        else if (D == 128)
            attn_dense_kernel<128, F16><<<grid, 256, 0, st>>>(q, q_stride, k, k_stride, v, v_stride, o, o_stride, Sq, Sk,
                                                             Hq, Hkv, qlen, klen, causal, scale, kv_rows, rbias, rb_ld);
        else
            attn_dense_kernel<64, F16><<<grid, 256, 0, st>>>(q, q_stride, k, k_stride, v, v_stride, o, o_stride, Sq, Sk,
                                                            Hq, Hkv, qlen, klen, causal, scale, kv_rows, rbias, rb_ld);
    });
    MXK_CHECK_LAUNCH();
}
