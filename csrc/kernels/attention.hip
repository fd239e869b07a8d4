// attention.hip — paged GQA attention for the LLM worker (K4/K5 of SURVEY §2.6).
//
// KV cache layout (written by rope_kv.hip): [num_blocks][Hkv][block_size][D] bf16, or fp8 e4m3
// (KV8: half the bytes per position; widened to fp32 in registers / to bf16 while staging to LDS), or rows of the
// llama.cpp block formats q8_0 / q4_0 / q4_1 / q5_0 / q5_1 / iq4_nl (kvq.h; written by kvq.hip, dequantised to bf16
// in registers like fp8 — the decode-MFMA and prefill kernels take the format as template KVF).
//
// decode  (one query token per sequence): memory-bound split-K over context partitions. A 256-thread
//   workgroup owns (sequence, kv-head, partition); D/8 lanes cover one cached position with 16-byte
//   loads, so a wave streams 64*16 B of K (then V) per step; all G = Hq/Hkv query heads of the kv
//   head are scored from the same K/V bytes (GQA packing: K/V are read once per kv head, not per q
//   head). Online softmax in the log2 domain; partitions merge in attn_decode_reduce.
// prefill (varlen, causal, paged context incl. cached prefix): flash-attention forward on MFMA
//   16x16x32 bf16. A workgroup holds 16 query rows x up to 8 query heads of one kv head (one wave per
//   head) so every K/V tile staged in LDS is reused by all heads of the group. K is stored
//   XOR-swizzled for conflict-free ds_read_b128 B-fragments; V is read with ds_read_b64_tr_b16
//   (hardware transpose) from a region-swizzled image; P goes register -> LDS -> A-fragment.
#include <type_traits>

#include "kvq.h"

#define LOG2E 1.4426950408889634f

// ------------------------------------------------------------------------------------------------
template <int D, int G, bool F16, bool KV8>
__global__ __launch_bounds__(256) void attn_decode_kernel(const bf16_t* __restrict__ q, int q_stride,
                                                          const void* __restrict__ kcv,
                                                          const void* __restrict__ vcv,
                                                          const int* __restrict__ block_tables, int bt_stride,
                                                          const int* __restrict__ seq_lens, int Hkv, int bs,
                                                          float scale, int window, float softcap, int part_size,
                                                          int n_parts, bf16_t* __restrict__ out, int out_stride,
                                                          float2* __restrict__ part_ml, float* __restrict__ part_o) {
    // window > 0: sliding-window attention, keys p >= L - window only (Gemma 2/3 local layers);
    // softcap > 0: scores s -> softcap * tanh(s / softcap) before the softmax (Gemma 2).
    constexpr int LPP = D / 8;        // lanes per position
    constexpr int PPW = 64 / LPP;     // positions per wave step
    constexpr int PPB = 4 * PPW;      // positions per workgroup step
    __shared__ float sm_m[4][G], sm_l[4][G];
    __shared__ float sm_o[4][G][D];
    const int kvh = blockIdx.x, b = blockIdx.y, part = blockIdx.z;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int pg = lane / LPP, dl = lane % LPP;
    const int L = seq_lens[b];
    const int p0 = part * part_size;
    const int p1 = min(L, p0 + part_size);
    const int Hq = Hkv * G;
    // partitions past the end of this sequence do nothing (the reduce kernel reads only the
    // ceil(L / part_size) live ones); graphs launch a fixed partition count for max_model_len.
    if (p0 >= L && part > 0) return;

    float qf[G][8];
    const float qs = scale * LOG2E;
    const float sc_l2 = softcap * LOG2E, sc_inv = softcap > 0.f ? 1.f / (softcap * LOG2E) : 0.f;
    const int p_start = window > 0 ? max(p0, L - window) : p0;
#pragma unroll
    for (int h = 0; h < G; ++h) {
        const uint4 raw = *(const uint4*)(q + (size_t)b * q_stride + (size_t)(kvh * G + h) * D + dl * 8);
        const uint32_t w[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            qf[h][2 * j] = __uint_as_float(w[j] << 16) * qs;
            qf[h][2 * j + 1] = __uint_as_float(w[j] & 0xFFFF0000u) * qs;
        }
    }
    float m[G], l[G], o[G][8];
#pragma unroll
    for (int h = 0; h < G; ++h) {
        m[h] = -INFINITY;
        l[h] = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) o[h][j] = 0.f;
    }
    // The partition's block ids are staged in LDS once (no dependent global load in front of every
    // K/V fetch), and K/V are double-buffered in registers: the loads of step i+1 are in flight
    // while step i is scored, so each lane keeps 2*U 16-byte loads outstanding (memory-level
    // parallelism is what bounds this kernel, not VALU).
    constexpr int MAXB = 256;  // part_size / bs + 1 <= MAXB (host checks)
    __shared__ int sbt[MAXB];
    const int* bt = block_tables + (size_t)b * bt_stride;
    using kvec = typename KVVec<KV8>::T;
    constexpr int ES = KV8 ? 1 : 2;  // bytes per cached element
    const char* kc = (const char*)kcv;
    const char* vc = (const char*)vcv;
    const int blk0 = p0 / bs;
    const int nblk = p1 > p0 ? (p1 - 1) / bs - blk0 + 1 : 0;
    for (int i = threadIdx.x; i < nblk; i += 256) sbt[i] = bt[blk0 + i];
    __syncthreads();
    constexpr int U = 2;
    constexpr int STEP = PPB * U;
    // two register buffers with compile-time names (a runtime buffer index, or arrays passed by
    // reference to helpers, would put them in scratch): the step is a macro over (K, V)
    kvec ka[U], va[U], kb[U], vb[U];
#define DEC_LOAD(K, V, BASE)                                                                  \
    _Pragma("unroll") for (int u = 0; u < U; ++u) {                                           \
        const int p = (BASE) + u * PPB + wave * PPW + pg;                                     \
        if (p < p1) {                                                                         \
            const int blk = sbt[p / bs - blk0], off = p % bs;                                 \
            const size_t eo = (((size_t)blk * Hkv + kvh) * bs + off) * D + dl * 8;            \
            K[u] = __builtin_nontemporal_load((const kvec*)(kc + eo * ES));                   \
            V[u] = __builtin_nontemporal_load((const kvec*)(vc + eo * ES));                   \
        } else {                                                                              \
            K[u] = V[u] = kvec{};                                                             \
        }                                                                                     \
    }
#define DEC_CONSUME(K, V, BASE)                                                               \
    _Pragma("unroll") for (int h = 0; h < G; ++h) {                                           \
        float s[U];                                                                           \
        _Pragma("unroll") for (int u = 0; u < U; ++u) {                                       \
            float acc = 0.f, kf[8];                                                           \
            kv_unpack8<KV8>(K[u], kf);                                                        \
            _Pragma("unroll") for (int j = 0; j < 8; ++j) acc = fmaf(qf[h][j], kf[j], acc);   \
            s[u] = group_sum<LPP>(acc);                                                       \
            if (softcap > 0.f) s[u] = sc_l2 * tanhf(s[u] * sc_inv);                           \
            if ((BASE) + u * PPB + wave * PPW + pg >= p1) s[u] = -INFINITY;                   \
        }                                                                                     \
        float mx = m[h];                                                                      \
        _Pragma("unroll") for (int u = 0; u < U; ++u) mx = fmaxf(mx, s[u]);                  \
        if (mx != -INFINITY) {                                                                \
            const float a = exp2f(m[h] - mx);                                                 \
            l[h] *= a;                                                                        \
            _Pragma("unroll") for (int j = 0; j < 8; ++j) o[h][j] *= a;                       \
            _Pragma("unroll") for (int u = 0; u < U; ++u) {                                   \
                const float pr = exp2f(s[u] - mx);                                            \
                l[h] += pr;                                                                   \
                float vf[8];                                                                  \
                kv_unpack8<KV8>(V[u], vf);                                                    \
                _Pragma("unroll") for (int j = 0; j < 8; ++j) o[h][j] = fmaf(pr, vf[j], o[h][j]); \
            }                                                                                 \
            m[h] = mx;                                                                        \
        }                                                                                     \
    }
    if (p_start < p1) { DEC_LOAD(ka, va, p_start) }
    for (int base = p_start; base < p1; base += 2 * STEP) {
        if (base + STEP < p1) { DEC_LOAD(kb, vb, base + STEP) }
        DEC_CONSUME(ka, va, base)
        if (base + STEP >= p1) break;
        if (base + 2 * STEP < p1) { DEC_LOAD(ka, va, base + 2 * STEP) }
        DEC_CONSUME(kb, vb, base + STEP)
    }
#undef DEC_LOAD
#undef DEC_CONSUME
    // merge the PPW position groups of the wave (xor over lane offsets LPP, 2LPP, ...)
#pragma unroll
    for (int off = LPP; off < 64; off <<= 1) {
#pragma unroll
        for (int h = 0; h < G; ++h) {
            const float m2 = __shfl_xor(m[h], off, 64), l2 = __shfl_xor(l[h], off, 64);
            const float mn = fmaxf(m[h], m2);
            const float a1 = mn == -INFINITY ? 0.f : exp2f(m[h] - mn);
            const float a2 = mn == -INFINITY ? 0.f : exp2f(m2 - mn);
            l[h] = l[h] * a1 + l2 * a2;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float o2 = __shfl_xor(o[h][j], off, 64);
                o[h][j] = o[h][j] * a1 + o2 * a2;
            }
            m[h] = mn;
        }
    }
    if (pg == 0) {
#pragma unroll
        for (int h = 0; h < G; ++h) {
            if (dl == 0) { sm_m[wave][h] = m[h]; sm_l[wave][h] = l[h]; }
#pragma unroll
            for (int j = 0; j < 8; ++j) sm_o[wave][h][dl * 8 + j] = o[h][j];
        }
    }
    __syncthreads();
    // combine the 4 waves: thread -> (h, d)
    for (int idx = threadIdx.x; idx < G * D; idx += 256) {
        const int h = idx / D, d = idx % D;
        float mx = -INFINITY;
#pragma unroll
        for (int w = 0; w < 4; ++w) mx = fmaxf(mx, sm_m[w][h]);
        float ls = 0.f, os = 0.f;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const float a = mx == -INFINITY ? 0.f : exp2f(sm_m[w][h] - mx);
            ls += sm_l[w][h] * a;
            os += sm_o[w][h][d] * a;
        }
        const int hq = kvh * G + h;
        // one partition holds the whole sequence: final output here (attn_decode_reduce skips it)
        if (n_parts == 1 || (part == 0 && L <= part_size)) {
            out[(size_t)b * out_stride + (size_t)hq * D + d] = f32_to_act<F16>(ls > 0.f ? os / ls : 0.f);
        } else {
            const size_t pi = ((size_t)b * Hq + hq) * n_parts + part;
            if (d == 0) part_ml[pi] = make_float2(mx, ls);
            part_o[pi * D + d] = os;
        }
    }
}

constexpr int DEC_RED_MAXP = 512;  // partitions whose merge weights fit the reduce kernel's LDS table

template <bool F16>
__global__ __launch_bounds__(128) void attn_decode_reduce_kernel(const float2* __restrict__ part_ml,
                                                                  const float* __restrict__ part_o, int n_parts,
                                                                  int Hq, int D, const int* __restrict__ seq_lens,
                                                                  int part_size, bf16_t* __restrict__ out,
                                                                  int out_stride) {
    // wave 0 reads the partitions' (m, l) with all its lanes at once and publishes the merge weights through
    // LDS (a serial loop of dependent loads made this launch as long as the attention itself at batch 1);
    // every thread then sums its dims over the partitions with independent loads
    __shared__ float wts[DEC_RED_MAXP];
    __shared__ float s_mx, s_ls;
    const int bh = blockIdx.x;
    const int b = bh / Hq, h = bh % Hq;
    const int np = min(n_parts, (seq_lens[b] + part_size - 1) / part_size);
    if (np <= 1) return;  // the attention workgroup wrote this sequence's output directly
    const size_t pb = (size_t)bh * n_parts;
    if (threadIdx.x < 64) {
        float m = -INFINITY;
        for (int p = threadIdx.x; p < np; p += 64) m = fmaxf(m, part_ml[pb + p].x);
        m = wave_max(m);
        float l = 0.f;
        for (int p = threadIdx.x; p < np; p += 64) {
            const float2 ml = part_ml[pb + p];
            const float a = m == -INFINITY ? 0.f : exp2f(ml.x - m);
            l += ml.y * a;
            if (p < DEC_RED_MAXP) wts[p] = a;
        }
        l = wave_sum(l);
        if (threadIdx.x == 0) { s_mx = m; s_ls = l; }
    }
    __syncthreads();
    const float mx = s_mx, L = s_ls;
    for (int d = threadIdx.x; d < D; d += blockDim.x) {
        float os = 0.f;
        int p = 0;
        for (; p + 4 <= min(np, DEC_RED_MAXP); p += 4) {
            const float o0 = part_o[(pb + p) * D + d], o1 = part_o[(pb + p + 1) * D + d];
            const float o2 = part_o[(pb + p + 2) * D + d], o3 = part_o[(pb + p + 3) * D + d];
            os += o0 * wts[p] + o1 * wts[p + 1] + o2 * wts[p + 2] + o3 * wts[p + 3];
        }
        for (; p < np; ++p) {
            const float a = p < DEC_RED_MAXP ? wts[p] : (mx == -INFINITY ? 0.f : exp2f(part_ml[pb + p].x - mx));
            os += part_o[(pb + p) * D + d] * a;
        }
        out[(size_t)b * out_stride + (size_t)h * D + d] = f32_to_act<F16>(L > 0.f ? os / L : 0.f);
    }
}

template <int D, int G>
static int launch_decode(const bf16_t* q, int q_stride, const void* kc, const void* vc, const int* bt,
                         int bt_stride, const int* seq_lens, int B, int Hkv, int bs, float scale, int window,
                         float softcap, int part_size, int n_parts, bf16_t* out, int out_stride, float2* part_ml,
                         float* part_o, int kv8, hipStream_t st) {
    dim3 grid(Hkv, B, n_parts);
    MX_ACT_DISPATCH({
        if (kv8)
            attn_decode_kernel<D, G, F16, true><<<grid, 256, 0, st>>>(q, q_stride, kc, vc, bt, bt_stride, seq_lens,
                                                                      Hkv, bs, scale, window, softcap, part_size,
                                                                      n_parts, out, out_stride, part_ml, part_o);
        else
            attn_decode_kernel<D, G, F16, false><<<grid, 256, 0, st>>>(q, q_stride, kc, vc, bt, bt_stride, seq_lens,
                                                                       Hkv, bs, scale, window, softcap, part_size,
                                                                       n_parts, out, out_stride, part_ml, part_o);
        if (n_parts > 1)
            attn_decode_reduce_kernel<F16><<<B * Hkv * G, 128, 0, st>>>(part_ml, part_o, n_parts, Hkv * G, D, seq_lens,
                                                                        part_size, out, out_stride);
    });
#undef DQK
    MXK_CHECK_LAUNCH();
}

extern "C" int mxk_attn_decode(const bf16_t* q, int q_stride, const void* kc, const void* vc, const int* bt,
                               int bt_stride, const int* seq_lens, int B, int Hq, int Hkv, int D, int bs,
                               float scale, int window, float softcap, int part_size, int n_parts, bf16_t* out,
                               int out_stride, float2* part_ml, float* part_o, int kv8, hipStream_t st) {
    if (B <= 0) return 0;
    if (Hq % Hkv || kv8 > KVF_FP8) return (int)hipErrorInvalidValue;  // block-quantised caches: the MFMA kernel only
    const int G = Hq / Hkv;
    if (n_parts > 1 && (!part_ml || !part_o)) return (int)hipErrorInvalidValue;
    if (bs <= 0 || part_size / bs + 1 > 256) return (int)hipErrorInvalidValue;  // LDS block-id stage
#define DEC(D_, G_) \
    if (D == D_ && G == G_) return launch_decode<D_, G_>(q, q_stride, kc, vc, bt, bt_stride, seq_lens, B, Hkv, bs, scale, window, softcap, part_size, n_parts, out, out_stride, part_ml, part_o, kv8, st);
    DEC(128, 1) DEC(128, 2) DEC(128, 3) DEC(128, 4) DEC(128, 5) DEC(128, 6) DEC(128, 7) DEC(128, 8)
    DEC(64, 1) DEC(64, 2) DEC(64, 4) DEC(64, 8) DEC(256, 1) DEC(256, 2) DEC(256, 4) DEC(256, 8)
#undef DEC
    return (int)hipErrorInvalidValue;
}

// ------------------------------------------------------------------------------------------------
// prefill: MFMA flash attention over the paged cache.
// K image: row p (64 per tile) holds D/8 16-byte chunks; chunk c lives at slot c ^ fk(p).
template <int D>
MX_DEV int k_lds_off(int p, int c) {
    const int r = p & 15;
    int f;
    if constexpr (D == 128) f = r ^ (((r + 4) >> 3) & 1);
    else f = ((r >> 1) & 7) ^ (((r + 4) >> 3) & 1);
    return p * (D * 2) + ((c ^ (f & (D / 8 - 1))) << 4);
}
// V image: row p holds D/16 32-byte regions (16 dims each); region nt lives at nt ^ sv(p).
template <int D>
MX_DEV int v_lds_off(int p, int nt) {
    int sv;
    if constexpr (D == 128) sv = (p & 3) | (((p >> 3) & 1) << 2);
    else sv = ((p >> 1) & 1) | (((p >> 3) & 1) << 1);
    return p * (D * 2) + ((nt ^ sv) << 5);
}

// ------------------------------------------------------------------------------------------------
// decode on MFMA. The VALU kernel above spends its time on the per-position dot products and the
// 16-lane shuffle reductions (~30% of HBM bandwidth at B=128); here the G query heads of a kv head are
// the rows of a 16x16x32 bf16 MFMA tile, so QK^T and PV run on the matrix cores and the softmax
// reductions happen once per 32-key tile.
//   workgroup = (kv head, sequence, partition), 4 waves; wave w takes the partition's 32-key tiles
//   w, w+4, ...: K fragments come straight from the paged cache into MFMA B operands (16-byte loads,
//   one cached position x 8 dims per lane), V is staged in the wave's LDS slice and read back with
//   the hardware-transposing ds_read_b64_tr_b16 (same V image as the prefill kernel), P goes
//   register -> LDS -> A fragment. The 4 waves' (m, l, O) merge through LDS at the end, in the same
//   partial-result format as attn_decode_kernel (attn_decode_reduce merges partitions).
// Occupancy, not register double buffering, hides HBM latency: ~9.3 KB of LDS per wave lets 4
// workgroups (16 waves) share a CU, each with one tile's 16 KB of K/V loads in flight.
template <int D>
constexpr int dec_wave_lds() { return 32 * D * 2 + 16 * (32 + 8) * 2; }

// NW = 16 (1024 threads, one workgroup per CU): the small-batch form — a 512-key partition per workgroup, so a
// context of <= 512 keys is ONE partition whose workgroup writes the final output (no reduce work for it).
// TS: debug instantiation writing wall-clock stamps of workgroup (0, 0, 0) wave 0 to ts[0..7] (tools/prof_attn_decode.py)
// DPF: the K-prefetch form (below; 2 waves / SIMD for its registers, MX_DECODE_PF=0 selects the 4-wave form)
// 8 cached elements at element offset eo widened to bf16 (fp8 / block-quantised caches)
template <int KVF, int D>
MX_DEV uint4 kv_widen8(const void* base, size_t eo) {
    if constexpr (KVF == KVF_FP8) return fp8x8_to_bf16x8(*(const uint2*)((const uint8_t*)base + eo));
    else return kvq_to_bf16x8<KVF>(kvq_load<KVF, D>(base, eo));
}

template <int D, bool F16, int KVF, int NW = 4, bool TS = false, bool DPF = false>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(
    (KVF != KVF_BF16 || (DPF && !TS && NW <= 8)) ? 2 : 4, (KVF != KVF_BF16 || (DPF && !TS && NW <= 8)) ? 2 : 4))) void attn_decode_mfma_kernel(
    const bf16_t* __restrict__ q, int q_stride, const void* __restrict__ kcv, const void* __restrict__ vcv,
    const int* __restrict__ block_tables, int bt_stride, const int* __restrict__ seq_lens, int Hkv, int G, int bs,
    float scale, int window, float softcap, int part_size, int n_parts, bf16_t* __restrict__ out, int out_stride,
    float2* __restrict__ part_ml, float* __restrict__ part_o, int* __restrict__ part_cnt,
    unsigned long long* __restrict__ ts = nullptr) {
    const bool ts_on = TS && blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0 && threadIdx.x == 0;
#define DEC_TS(k)                                    \
    if constexpr (TS) {                              \
        __builtin_amdgcn_s_waitcnt(0);               \
        if (ts_on) ts[k] = wall_clock64();           \
    }
    DEC_TS(0)
    constexpr int KT = 32;                      // keys per wave tile
    constexpr int VBYTES = KT * D * 2;
    constexpr int PSTRIDE = (KT + 8) * 2;       // bytes per P row (padded)
    constexpr int WB = dec_wave_lds<D>();
    constexpr int NVC = KT * D / 8 / 64;        // 16-byte V chunks per lane per tile
    constexpr bool KV8 = KVF != KVF_BF16;       // a cache widened in registers (fp8 or block-quantised)
    constexpr int ES = KV8 ? 1 : 2;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int MAXB = 256;
    __shared__ int sbt[MAXB];
    const int kvh = blockIdx.x, b = blockIdx.y, part = blockIdx.z;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int g = lane >> 4, col = lane & 15;
    const int p0 = part * part_size;
    const int* bt = block_tables + (size_t)b * bt_stride;
    const int blk0 = p0 / bs;
    // the partition's block-table entries are requested before (not after) the sequence length: the
    // table read does not wait for seq_lens, entries past the context are loaded but never used
    {
        const int nbt = min(part_size / bs + 1, bt_stride - blk0);
        for (int i = threadIdx.x; i < nbt; i += 64 * NW) sbt[i] = bt[blk0 + i];
    }
    const int L = seq_lens[b];
    const int p1 = min(L, p0 + part_size);
    if (p0 >= L && part > 0) return;  // uniform: graphs launch n_parts for max_model_len
    DEC_TS(1)
    const int Hq = Hkv * G;
    const int p_start = window > 0 ? max(p0, L - window) : p0;
    const float qs = scale * LOG2E;
    const float sc_l2 = softcap * LOG2E, sc_inv = softcap > 0.f ? 1.f / (softcap * LOG2E) : 0.f;
    // Q as the A operand: row = head (lane col), k = dims 32 ks + 8 g — requested before the block-table
    // barrier so its latency overlaps the table read
    bf16x8 qf[D / 32];
#pragma unroll
    for (int ks = 0; ks < D / 32; ++ks) {
        if (col < G) qf[ks] = *(const bf16x8*)(q + (size_t)b * q_stride + (size_t)(kvh * G + col) * D + 32 * ks + 8 * g);
        else qf[ks] = (bf16x8){};
    }
    __syncthreads();
    DEC_TS(2)
    f32x4 oacc[D / 16];
#pragma unroll
    for (int i = 0; i < D / 16; ++i) oacc[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
    float mrow[4], lrow[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) { mrow[i] = -INFINITY; lrow[i] = 0.f; }
    char* v_lds = smem + wave * WB;
    char* pw = v_lds + VBYTES;
    const char* kc = (const char*)kcv;
    const char* vc = (const char*)vcv;

    // PF (bf16 caches): the next tile's K fragments are requested while this tile computes. Every K load is then
    // issued unconditionally (keys past the end read a valid row and are zeroed after the load), and V comes
    // through registers (plain loads, stored to the LDS image after QK^T) instead of LDS-DMA: the explicit vmcnt
    // waits below count exactly NK K loads and NVC V loads per tile, which holds only for loads that complete in
    // issue order (LDS-DMA completions are not ordered against plain loads).
    constexpr bool PF = DPF && !KV8 && !TS && NW <= 8;  // (16-wave form: 128 VGPRs, no room for a second K tile)
    constexpr int NK = 2 * (D / 32);
    auto load_k = [&](int kt, bf16x8(&kf_)[2][D / 32]) {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int key = kt + 16 * t + col;
            const bool ok = key < p1;
            const int kk = (PF || ok) ? (ok ? key : kt) : 0;
            const size_t eo = (PF || ok) ? (((size_t)sbt[kk / bs - blk0] * Hkv + kvh) * bs + kk % bs) * D : 0;
#pragma unroll
            for (int ks = 0; ks < D / 32; ++ks) {
                if constexpr (KV8) {
                    kf_[t][ks] = ok ? __builtin_bit_cast(bf16x8, kv_widen8<KVF, D>(kc, eo + 32 * ks + 8 * g))
                                    : (bf16x8){};
                } else if constexpr (PF) {
                    const bf16x8 w = *(const bf16x8*)(kc + (eo + 32 * ks + 8 * g) * ES);
                    kf_[t][ks] = ok ? w : (bf16x8){};
                } else {
                    kf_[t][ks] = ok ? *(const bf16x8*)(kc + (eo + 32 * ks + 8 * g) * ES) : (bf16x8){};
                }
            }
        }
    };
    [[maybe_unused]] bf16x8 knext[2][D / 32];
    if constexpr (PF) {
        if (p_start + wave * KT < p1) load_k(p_start + wave * KT, knext);
    }
    for (int kt0 = p_start + wave * KT; kt0 < p1; kt0 += NW * KT) {
        // ---- the tile's K fragments (PF: requested during the previous tile) and V chunk loads ----
        bf16x8 kf[2][D / 32];
        if constexpr (PF) {
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int ks = 0; ks < D / 32; ++ks) kf[t][ks] = knext[t][ks];
        } else {
            load_k(kt0, kf);
        }
        // V: bf16 caches go HBM -> LDS by DMA (global_load_lds, no VGPR staging): instruction j fills
        // bytes [1024 j, 1024 j + 1024) of the slice linearly by lane, so each lane fetches the chunk
        // that the swizzled V image (v_lds_off) places at its slot; fp8 caches widen in registers.
        [[maybe_unused]] uint4 vv[(KV8 || PF) ? NVC : 1];
#pragma unroll
        for (int j = 0; j < NVC; ++j) {
            int p, c;
            if constexpr (KV8 || PF) {
                const int id = lane + 64 * j;
                p = id / (D / 8);
                c = id % (D / 8);
            } else {
                const int X = 1024 * j + 16 * lane;  // slot in the V image
                p = X / (D * 2);
                const int o = X % (D * 2);
                int sv;
                if constexpr (D == 128) sv = (p & 3) | (((p >> 3) & 1) << 2);
                else sv = ((p >> 1) & 1) | (((p >> 3) & 1) << 1);
                c = 2 * ((o >> 5) ^ sv) + ((o >> 4) & 1);
            }
            const int key = kt0 + p < p1 ? kt0 + p : kt0;  // past the end: a valid row (P = 0 there)
            const size_t eo = (((size_t)sbt[key / bs - blk0] * Hkv + kvh) * bs + key % bs) * D + c * 8;
            if constexpr (KV8) {
                vv[j] = kt0 + p < p1 ? kv_widen8<KVF, D>(vc, eo) : make_uint4(0, 0, 0, 0);
            } else if constexpr (PF) {
                vv[j] = *(const uint4*)(vc + eo * ES);  // rows past the end: a valid row, P = 0 there
            } else {
                __builtin_amdgcn_global_load_lds((const void*)(vc + eo * ES), (MX_LDS void*)(v_lds + 1024 * j), 16, 0, 0);
            }
        }
        [[maybe_unused]] const bool more = kt0 + NW * KT < p1;  // wave-uniform
        if constexpr (PF) {
            __builtin_amdgcn_sched_barrier(0);
            if (more) load_k(kt0 + NW * KT, knext);
            __builtin_amdgcn_sched_barrier(0);
            // this tile's K (issued before its V DMAs and the next tile's K) has landed
            if (more) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NVC + NK) : "memory");
            else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NVC) : "memory");
        }
        // ---- S = Q K^T : 16 head rows x 32 keys ----
        f32x4 sacc[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            sacc[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ks = 0; ks < D / 32; ++ks)
                sacc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qf[ks], kf[t][ks], sacc[t], 0, 0, 0);
        }
        if constexpr (TS) {
            if (kt0 == p_start) DEC_TS(3)  // the K tile has landed (first tile of wave 0)
        }
        if constexpr (KV8 || PF) {  // V -> this wave's LDS slice (the previous tile's reads have returned)
#pragma unroll
            for (int j = 0; j < NVC; ++j) {
                const int id = lane + 64 * j, p = id / (D / 8), c = id % (D / 8);
                *(uint4*)(v_lds + v_lds_off<D>(p, c >> 1) + 16 * (c & 1)) = vv[j];
            }
        }
        // ---- online softmax over the tile (rows 4g+i, keys 16t+col) ----
        float alpha[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            float mx = -INFINITY;
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                float v = sacc[t][i] * qs;
                if (softcap > 0.f) v = sc_l2 * tanhf(v * sc_inv);
                if (kt0 + 16 * t + col >= p1) v = -INFINITY;
                sacc[t][i] = v;
                mx = fmaxf(mx, v);
            }
            mx = group_max<16>(mx);
            const float mn = fmaxf(mrow[i], mx);
            alpha[i] = mn == -INFINITY ? 1.f : exp2f(mrow[i] - mn);
            float rs = 0.f;
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                const float pv = mn == -INFINITY ? 0.f : exp2f(sacc[t][i] - mn);
                sacc[t][i] = pv;
                rs += pv;
            }
            lrow[i] = lrow[i] * alpha[i] + group_sum<16>(rs);
            mrow[i] = mn;
        }
#pragma unroll
        for (int nt = 0; nt < D / 16; ++nt)
#pragma unroll
            for (int i = 0; i < 4; ++i) oacc[nt][i] *= alpha[i];
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int i = 0; i < 4; ++i)
                *(bf16_t*)(pw + (4 * g + i) * PSTRIDE + (16 * t + col) * 2) = f32_to_bf16(sacc[t][i]);
        // the V DMA has landed and the P (and fp8 V) writes are visible (PF: the next tile's K may stay in flight)
        if constexpr (PF) {
            if (more) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(NK) : "memory");
            else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        } else {
            __builtin_amdgcn_s_waitcnt(0);
        }
        __builtin_amdgcn_wave_barrier();
        // ---- O += P V ----
        const bf16x8 pa = *(const bf16x8*)(pw + col * PSTRIDE + 8 * g * 2);
        const int r0 = 8 * g, q4 = col >> 2, p4 = col & 3;
#pragma unroll
        for (int nt = 0; nt < D / 16; ++nt) {
            const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (MX_LDS s16x4*)(v_lds + v_lds_off<D>(r0 + q4, nt) + 8 * p4));
            const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (MX_LDS s16x4*)(v_lds + v_lds_off<D>(r0 + 4 + q4, nt) + 8 * p4));
            const u32x2 l2 = __builtin_bit_cast(u32x2, lo), h2 = __builtin_bit_cast(u32x2, hi);
            const u32x4 w4 = {l2[0], l2[1], h2[0], h2[1]};
            oacc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, __builtin_bit_cast(bf16x8, w4), oacc[nt], 0, 0, 0);
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);  // the transposed reads have returned before V is rewritten
        __builtin_amdgcn_wave_barrier();
    }
    // ---- merge the NW waves: (m, l) per row and O rows through the (now free) LDS slices ----
    DEC_TS(4)
    __syncthreads();
    DEC_TS(5)
    float* wo = (float*)(smem + wave * WB);        // [16 rows][D] fp32 (8 KB for D=128 <= WB)
    float* wml = (float*)(smem + NW * WB) + wave * 32;  // [16 rows] m, [16 rows] l
    // waves past the context's last tile hold nothing (m = -inf, l = 0): neither written nor read
    const int nwa = p1 > p_start ? min(NW, (p1 - p_start + KT - 1) / KT) : 0;
    if (wave < nwa) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int r = 4 * g + i;
            if (r >= G) continue;  // only the G real head rows of the 16-row tile
#pragma unroll
            for (int nt = 0; nt < D / 16; ++nt) wo[r * D + 16 * nt + col] = oacc[nt][i];
            if (col == 0) { wml[r] = mrow[i]; wml[16 + r] = lrow[i]; }
        }
    }
    __syncthreads();
    DEC_TS(6)
    const float* ml = (const float*)(smem + NW * WB);
    // a sequence that fits this one partition: the final output here, no partials (the reduce skips it)
    const bool single = n_parts == 1 || (p0 == 0 && L <= part_size);
    // per head row: the waves' merge weights exp2(m_w - mx) and the row's (mx, l) — once per row in 16-lane
    // groups, not once per output element (the output loop below is then one FMA per wave)
    __shared__ float s_wt[16 * 16];
    __shared__ float2 s_rml[16];
    if (threadIdx.x < G * 16) {  // whole 16-lane groups (G * 16 is a multiple of 16)
        const int h = threadIdx.x >> 4, w = threadIdx.x & 15;
        const float m = w < nwa ? ml[w * 32 + h] : -INFINITY;
        const float mx = group_max<16>(m);
        const float a = (w < nwa && mx != -INFINITY) ? exp2f(m - mx) : 0.f;
        const float ls = group_sum<16>(w < nwa ? ml[w * 32 + 16 + h] * a : 0.f);
        s_wt[threadIdx.x] = a;
        if (w == 0) s_rml[h] = make_float2(mx, ls);
    }
    __syncthreads();
    for (int idx = threadIdx.x; idx < G * D; idx += 64 * NW) {
        const int h = idx / D, d = idx % D;
        const float mx = s_rml[h].x, ls = s_rml[h].y;
        float os = 0.f;
#pragma unroll 4
        for (int w = 0; w < nwa; ++w) os += ((const float*)(smem + w * WB))[h * D + d] * s_wt[h * 16 + w];
        const int hq = kvh * G + h;
        if (single) {
            out[(size_t)b * out_stride + (size_t)hq * D + d] = f32_to_act<F16>(ls > 0.f ? os / ls : 0.f);
        } else {
            const size_t pi = ((size_t)b * Hq + hq) * n_parts + part;
            // sc1 stores (agent-scope relaxed atomics): the fused merge below reads them from another CU / XCD with
            // sc1 loads, so no L2 write-back fence is needed (MI355X_MICROARCH.md inter-workgroup hand-off, row 1)
            if (d == 0)
                __hip_atomic_store((unsigned long long*)(part_ml + pi),
                                   __builtin_bit_cast(unsigned long long, make_float2(mx, ls)), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(part_o + pi * D + d, os, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    DEC_TS(7)
#undef DEC_TS
    if (single || !part_cnt) return;
    // fused split-K merge: the last of the (b, kvh) partition workgroups to finish merges all of them,
    // instead of a separate reduce launch (at batch 1 that launch costs as much as the attention itself).
    // The counter is left at zero for the next launch / graph replay.
    // hand-off without fences: every storing wave waits for its sc1 stores, a barrier, then ONE agent-scope atomic add
    // per workgroup; the workgroup whose add came last reads the partials with sc1 loads (no buffer_wbl2 / buffer_inv:
    // an agent fence costs ~3.5 us per workgroup here and made this merge lose to a separate launch in round 5)
    __shared__ int s_last;
    const int np = min(n_parts, (L + part_size - 1) / part_size);  // partitions that did not return early
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const int old = __hip_atomic_fetch_add(&part_cnt[b * Hkv + kvh], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = old == np - 1;
        if (old == np - 1) __hip_atomic_store(&part_cnt[b * Hkv + kvh], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!s_last) return;
    auto ml_at = [&](size_t i) {
        return __builtin_bit_cast(float2, __hip_atomic_load((unsigned long long*)(part_ml + i), __ATOMIC_RELAXED,
                                                            __HIP_MEMORY_SCOPE_AGENT));
    };
    for (int idx = threadIdx.x; idx < G * D; idx += 64 * NW) {
        const int h = idx / D, d = idx % D, hq = kvh * G + h;
        const size_t pb = ((size_t)b * Hq + hq) * n_parts;
        float mx = -INFINITY;
        for (int p = 0; p < np; ++p) mx = fmaxf(mx, ml_at(pb + p).x);
        float ls = 0.f, os = 0.f;
        for (int p = 0; p < np; ++p) {
            const float2 pm = ml_at(pb + p);
            const float a = mx == -INFINITY ? 0.f : exp2f(pm.x - mx);
            ls += pm.y * a;
            os += __hip_atomic_load(part_o + (pb + p) * D + d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) * a;
        }
        out[(size_t)b * out_stride + (size_t)hq * D + d] = f32_to_act<F16>(ls > 0.f ? os / ls : 0.f);
    }
}

static bool decode_pf() {
    // off by default: at c128 the 2-wave prefetch form measured 1.5 % slower end to end than the 4-wave form
    // (profiles/r5_step_composition.md); MX_DECODE_PF=1 selects it
    static const bool on = getenv("MX_DECODE_PF") && atoi(getenv("MX_DECODE_PF")) != 0;
    return on;
}

template <int D>
static int launch_decode_mfma(const bf16_t* q, int q_stride, const void* kc, const void* vc, const int* bt,
                              int bt_stride, const int* seq_lens, int B, int Hkv, int G, int bs, float scale,
                              int window, float softcap, int part_size, int n_parts, bf16_t* out, int out_stride,
                              float2* part_ml, float* part_o, int* part_cnt, int kv8, hipStream_t st) {
    dim3 grid(Hkv, B, n_parts);
    static_assert(16 * D * 4 <= dec_wave_lds<D>(), "merge buffer");
    // 512-key partitions run 16 waves per workgroup (one 32-key tile each), 256-key ones 8, smaller ones 4
    const bool wide = part_size >= 512 && !kv8 && B < 8;  // (large batches keep 4-wave workgroups)
    const bool mid = !wide && part_size >= 256 && !kv8 && B < 8;
    const int NWs = wide ? 16 : mid ? 8 : 4;
    const size_t lds = NWs * dec_wave_lds<D>() + NWs * 32 * 4;
#define DQK(F_)                                                                                                   \
    attn_decode_mfma_kernel<D, F16, F_><<<grid, 256, lds, st>>>(q, q_stride, kc, vc, bt, bt_stride, seq_lens, Hkv, G, \
                                                               bs, scale, window, softcap, part_size, n_parts, out,   \
                                                               out_stride, part_ml, part_o, part_cnt)
    MX_ACT_DISPATCH({
        if (kv8 == KVF_FP8) DQK(KVF_FP8);
        else if (kv8 == KVF_Q8_0) DQK(KVF_Q8_0);
        else if (kv8 == KVF_Q4_0) DQK(KVF_Q4_0);
        else if (kv8 == KVF_Q4_1) DQK(KVF_Q4_1);
        else if (kv8 == KVF_Q5_0) DQK(KVF_Q5_0);
        else if (kv8 == KVF_Q5_1) DQK(KVF_Q5_1);
        else if (kv8 == KVF_IQ4_NL) DQK(KVF_IQ4_NL);
        else if (wide) {
            static bool attr = false;
            if (!attr) {
                (void)hipFuncSetAttribute((const void*)attn_decode_mfma_kernel<D, F16, KVF_BF16, 16>,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
                attr = true;
            }
            attn_decode_mfma_kernel<D, F16, KVF_BF16, 16><<<grid, 1024, lds, st>>>(
                q, q_stride, kc, vc, bt, bt_stride, seq_lens, Hkv, G, bs, scale, window, softcap, part_size, n_parts,
                out, out_stride, part_ml, part_o, part_cnt);
        } else if (mid) {
            static bool attr8 = false;
            if (!attr8) {
                (void)hipFuncSetAttribute((const void*)attn_decode_mfma_kernel<D, F16, KVF_BF16, 8>,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
                attr8 = true;
            }
            attn_decode_mfma_kernel<D, F16, KVF_BF16, 8><<<grid, 512, lds, st>>>(
                q, q_stride, kc, vc, bt, bt_stride, seq_lens, Hkv, G, bs, scale, window, softcap, part_size, n_parts,
                out, out_stride, part_ml, part_o, part_cnt);
        } else if (decode_pf())
            attn_decode_mfma_kernel<D, F16, KVF_BF16, 4, false, true><<<grid, 256, lds, st>>>(
                q, q_stride, kc, vc, bt, bt_stride, seq_lens, Hkv, G, bs, scale, window, softcap, part_size, n_parts,
                out, out_stride, part_ml, part_o, part_cnt);
        else
            attn_decode_mfma_kernel<D, F16, KVF_BF16><<<grid, 256, lds, st>>>(q, q_stride, kc, vc, bt, bt_stride,
                                                                          seq_lens, Hkv, G, bs, scale, window, softcap,
                                                                          part_size, n_parts, out, out_stride, part_ml,
                                                                          part_o, part_cnt);
        if (n_parts > 1 && !part_cnt)
            attn_decode_reduce_kernel<F16><<<B * Hkv * G, 128, 0, st>>>(part_ml, part_o, n_parts, Hkv * G, D, seq_lens,
                                                                        part_size, out, out_stride);
    });
    MXK_CHECK_LAUNCH();
}

// debug: the 16-wave single-pass decode (bf16 activations and cache, D = 128) with phase stamps of workgroup 0's
// wave 0 in ts[0..7] (s_memrealtime, 100 MHz): entry, past the seq-len check, block table in LDS, first K tile
// landed, tiles done, merge barrier 1, merge barrier 2, output stored
extern "C" int mxk_attn_decode_ts(const bf16_t* q, int q_stride, const void* kc, const void* vc, const int* bt,
                                  int bt_stride, const int* seq_lens, int B, int Hq, int Hkv, int bs, float scale,
                                  int part_size, bf16_t* out, int out_stride, unsigned long long* ts, hipStream_t st) {
    if (Hq % Hkv || Hq / Hkv > 16 || part_size < 512 || bs <= 0 || part_size / bs + 1 > 256)
        return (int)hipErrorInvalidValue;
    const size_t lds = 16 * dec_wave_lds<128>() + 16 * 32 * 4;
    (void)hipFuncSetAttribute((const void*)attn_decode_mfma_kernel<128, false, KVF_BF16, 16, true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attn_decode_mfma_kernel<128, false, KVF_BF16, 16, true><<<dim3(Hkv, B, 1), 1024, lds, st>>>(
        q, q_stride, kc, vc, bt, bt_stride, seq_lens, Hkv, Hq / Hkv, bs, scale, 0, 0.f, part_size, 1, out, out_stride,
        nullptr, nullptr, nullptr, ts);
    MXK_CHECK_LAUNCH();
}

// MFMA decode for D in {64, 128} and up to 16 query heads per kv head; other shapes return
// hipErrorInvalidValue (the caller falls back to mxk_attn_decode). part_cnt: B x Hkv zero-initialised
// counters for the in-kernel partition merge (nullptr: a separate reduce launch).
extern "C" int mxk_attn_decode_mfma(const bf16_t* q, int q_stride, const void* kc, const void* vc, const int* bt,
                                    int bt_stride, const int* seq_lens, int B, int Hq, int Hkv, int D, int bs,
                                    float scale, int window, float softcap, int part_size, int n_parts, bf16_t* out,
                                    int out_stride, float2* part_ml, float* part_o, int kv8, int* part_cnt,
                                    hipStream_t st) {
    if (B <= 0) return 0;
    if (Hq % Hkv || Hq / Hkv > 16) return (int)hipErrorInvalidValue;
    if (n_parts > 1 && (!part_ml || !part_o)) return (int)hipErrorInvalidValue;
    if (bs <= 0 || part_size / bs + 1 > 256) return (int)hipErrorInvalidValue;
    const int G = Hq / Hkv;
    if (D == 128) return launch_decode_mfma<128>(q, q_stride, kc, vc, bt, bt_stride, seq_lens, B, Hkv, G, bs, scale, window, softcap, part_size, n_parts, out, out_stride, part_ml, part_o, part_cnt, kv8, st);
    if (D == 64) return launch_decode_mfma<64>(q, q_stride, kc, vc, bt, bt_stride, seq_lens, B, Hkv, G, bs, scale, window, softcap, part_size, n_parts, out, out_stride, part_ml, part_o, part_cnt, kv8, st);
    return (int)hipErrorInvalidValue;
}

// KSP = 2 (key split, GW = 4 only: 8 waves): two groups of GW waves share the workgroup's 16 query rows x GW heads and take alternate
// 64-key tiles (each group stages its own K / V tile), then merge (m, l, O) through LDS. A short prompt chunk runs
// only ~n_tiles x Hq / GW workgroups (136 for a 270-token chunk of Llama-3-8B, fewer than the CUs), each walking
// its causal key range one tile at a time: the split halves the longest walk.
template <int D, int GW, int VT, bool F16, int KVF, int KSP = 1>
__global__ __launch_bounds__(512) void attn_prefill_kernel(const bf16_t* __restrict__ q,
                                                           const void* __restrict__ kc,
                                                           const void* __restrict__ vc,
                                                           const int* __restrict__ block_tables, int bt_stride,
                                                           const int* __restrict__ tile_seq,
                                                           const int* __restrict__ tile_q0,
                                                           const int* __restrict__ cu_q,
                                                           const int* __restrict__ ctx_lens, int Hq, int Hkv,
                                                           int G, int bs, float scale, int window, float softcap,
                                                           bf16_t* __restrict__ out) {
    static_assert(KSP == 1 || GW == 4, "key split: 2 x 4 waves (the 512-thread launch bound)");
    constexpr int NWG = GW >= 3 ? GW : 4;     // waves per key group
    constexpr int NW = NWG * KSP;             // waves per workgroup
    constexpr int RT = NWG / GW;              // 16-row query tiles per workgroup
    constexpr int KT = 64;                    // keys per tile
    constexpr int KBYTES = KT * D * 2;
    constexpr int PSTRIDE = (KT + 8) * 2;     // bytes per P row (padded)
    constexpr int VTSTRIDE = (KT + 8) * 2;    // VT=1: bytes per transposed V row (one dim)
    constexpr int VBYTES = VT ? D * VTSTRIDE : KBYTES;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int ksp = KSP > 1 ? wave / NWG : 0;  // key group
    char* k_lds = smem + ksp * (KBYTES + VBYTES);
    char* v_lds = k_lds + KBYTES;
    char* p_lds = smem + KSP * (KBYTES + VBYTES);
    constexpr int NT_C = NWG * 64;             // threads staging one group's tile
    const int tid = threadIdx.x - ksp * NT_C;
    const int g = lane >> 4, col = lane & 15;
    const int tile = blockIdx.x;
    const int s = tile_seq[tile], q0 = tile_q0[tile];
    if (s < 0) return;  // padding tile of a graph-captured step (uniform across the workgroup)
    const int hq = blockIdx.y * GW + (wave % GW);
    const int kvh = (blockIdx.y * GW) / G;
    const int rt = KSP > 1 ? 0 : wave / GW;
    const int qbeg = cu_q[s], qlen = cu_q[s + 1] - qbeg;
    const int ctx = ctx_lens[s];
    const int pos_off = ctx - qlen;  // position of query 0
    const int* bt = block_tables + (size_t)s * bt_stride;
    const int row_q0 = q0 + rt * 16;        // first query index of this wave
    const int wg_rows = RT * 16;
    const int kv_end = min(ctx, pos_off + min(qlen, q0 + wg_rows));
    const float qs = scale * LOG2E;
    const float sc_l2 = softcap * LOG2E, sc_inv = softcap > 0.f ? 1.f / (softcap * LOG2E) : 0.f;
    // sliding window: key tiles entirely before the earliest query's window are skipped
    const int kt_begin = window > 0 ? (max(0, pos_off + q0 - window + 1) / 64) * 64 : 0;

    // Q fragments: lane row = col, dims 32ks + 8g
    bf16x8 qf[D / 32];
    {
        const int qi = row_q0 + col;
#pragma unroll
        for (int ks = 0; ks < D / 32; ++ks) {
            if (qi < qlen) qf[ks] = *(const bf16x8*)(q + ((size_t)(qbeg + qi) * Hq + hq) * D + 32 * ks + 8 * g);
            else qf[ks] = (bf16x8){};
        }
    }
    f32x4 oacc[D / 16];
#pragma unroll
    for (int i = 0; i < D / 16; ++i) oacc[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
    float mrow[4], lrow[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) { mrow[i] = -INFINITY; lrow[i] = 0.f; }
    char* pw = p_lds + wave * 16 * PSTRIDE;

    // K / V tiles are software-pipelined one tile deep: tile t + 1's global loads (block-table entry, then the
    // 16-byte chunks) are issued right after tile t is staged in LDS, so their latency hides behind tile t's
    // MFMAs and softmax instead of opening every tile (short prompt chunks run only a few tiles per workgroup)
    constexpr int CH = KT * D / 8;              // 16-byte chunks per tile
    constexpr int NCH = (CH + NT_C - 1) / NT_C;  // chunks per thread
    constexpr bool KV8 = KVF == KVF_FP8;
    constexpr bool KVQ_ = KVF >= KVF_Q8_0;  // block-quantised rows (kvq.h): raw codes + scales kept in flight
    using KRaw = typename std::conditional<KVQ_, KVQRaw, typename std::conditional<KV8, uint2, uint4>::type>::type;
    KRaw kr[NCH], vr[NCH];
    auto load_tile = [&](int kt0) {
#pragma unroll
        for (int j = 0; j < NCH; ++j) {
            const int id = tid + j * NT_C;
            const int p = id / (D / 8), c = id % (D / 8);
            const int pos = kt0 + p;
            kr[j] = KRaw{};
            vr[j] = KRaw{};
            if (id < CH && pos < kv_end) {
                const int blk = bt[pos / bs], off = pos % bs;
                const size_t eo = (((size_t)blk * Hkv + kvh) * bs + off) * D + c * 8;
                if constexpr (KVQ_) {
                    kr[j] = kvq_load<KVF, D>(kc, eo);
                    vr[j] = kvq_load<KVF, D>(vc, eo);
                } else if constexpr (KV8) {
                    kr[j] = *(const uint2*)((const uint8_t*)kc + eo);
                    vr[j] = *(const uint2*)((const uint8_t*)vc + eo);
                } else {
                    kr[j] = *(const uint4*)((const bf16_t*)kc + eo);
                    vr[j] = *(const uint4*)((const bf16_t*)vc + eo);
                }
            }
        }
    };
    auto store_tile = [&]() {
#pragma unroll
        for (int j = 0; j < NCH; ++j) {
            const int id = tid + j * NT_C;
            if (id >= CH) continue;
            const int p = id / (D / 8), c = id % (D / 8);
            uint4 kv, vv;
            if constexpr (KVQ_) {
                kv = kvq_to_bf16x8<KVF>(kr[j]);
                vv = kvq_to_bf16x8<KVF>(vr[j]);
            } else if constexpr (KV8) {
                kv = fp8x8_to_bf16x8(kr[j]);
                vv = fp8x8_to_bf16x8(vr[j]);
            } else {
                kv = kr[j];
                vv = vr[j];
            }
            *(uint4*)(k_lds + k_lds_off<D>(p, c)) = kv;
            if constexpr (VT == 0) {
                *(uint4*)(v_lds + v_lds_off<D>(p, c >> 1) + 16 * (c & 1)) = vv;
            } else {
                const uint32_t w[4] = {vv.x, vv.y, vv.z, vv.w};
#pragma unroll
                for (int jj = 0; jj < 8; ++jj)
                    *(bf16_t*)(v_lds + (8 * c + jj) * VTSTRIDE + 2 * p) = (bf16_t)(w[jj >> 1] >> (16 * (jj & 1)));
            }
        }
    };
    // key group ksp takes tiles kt_begin + KT (ksp + KSP r); every group runs the same number of rounds (the
    // barriers below are workgroup-wide), a group past the end idles through its last round
    const int n_rounds = kv_end > kt_begin ? (kv_end - kt_begin + KSP * KT - 1) / (KSP * KT) : 0;
    if (kt_begin + ksp * KT < kv_end) load_tile(kt_begin + ksp * KT);
    for (int r = 0; r < n_rounds; ++r) {
        const int kt0 = kt_begin + (KSP * r + ksp) * KT;
        const bool live = kt0 < kv_end;
        // ---- stage this K and V tile (64 keys x D), then request the next one ----
        if (live) store_tile();
        if (kt0 + KSP * KT < kv_end) load_tile(kt0 + KSP * KT);
        __syncthreads();
        if (!live) {
            __syncthreads();
            continue;
        }
        // ---- S = Q K^T : 16 rows x 64 keys ----
        f32x4 sacc[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            sacc[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ks = 0; ks < D / 32; ++ks) {
                const bf16x8 kf = *(const bf16x8*)(k_lds + k_lds_off<D>(16 * t + col, 4 * ks + g));
                sacc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qf[ks], kf, sacc[t], 0, 0, 0);
            }
        }
        // ---- mask + online softmax (rows 4g+i, keys 16t+col) ----
        float rmax[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int qi = row_q0 + 4 * g + i;
            const int qpos = pos_off + qi;
            float mx = -INFINITY;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int kp = kt0 + 16 * t + col;
                float v = sacc[t][i] * qs;
                if (softcap > 0.f) v = sc_l2 * tanhf(v * sc_inv);
                if (kp > qpos || kp >= ctx || qi >= qlen || (window > 0 && kp <= qpos - window)) v = -INFINITY;
                sacc[t][i] = v;
                mx = fmaxf(mx, v);
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
            for (int t = 0; t < 4; ++t) {
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
        // ---- P -> LDS (bf16) ----
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int i = 0; i < 4; ++i)
                *(bf16_t*)(pw + (4 * g + i) * PSTRIDE + (16 * t + col) * 2) = f32_to_bf16(sacc[t][i]);
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): P visible to the wave (same wave reads)
        __builtin_amdgcn_wave_barrier();
        // ---- O += P V ----
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const bf16x8 pa = *(const bf16x8*)(pw + col * PSTRIDE + (32 * ks + 8 * g) * 2);
            const int r0 = 32 * ks + 8 * g;
            const int q4 = col >> 2, p4 = col & 3;
#pragma unroll
            for (int nt = 0; nt < D / 16; ++nt) {
                bf16x8 vb;
                if constexpr (VT == 0) {
                    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                        (MX_LDS s16x4*)(v_lds + v_lds_off<D>(r0 + q4, nt) + 8 * p4));
                    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                        (MX_LDS s16x4*)(v_lds + v_lds_off<D>(r0 + 4 + q4, nt) + 8 * p4));
                    // whole-vector reinterpretation: per-element bf16 bit_casts of the v4i16 result were
                    // miscompiled (hipcc dropped elements 2,3 of each transposed read)
                    const u32x2 l2 = __builtin_bit_cast(u32x2, lo), h2 = __builtin_bit_cast(u32x2, hi);
                    const u32x4 w4 = {l2[0], l2[1], h2[0], h2[1]};
                    vb = __builtin_bit_cast(bf16x8, w4);
                } else {
                    vb = *(const bf16x8*)(v_lds + (16 * nt + col) * VTSTRIDE + r0 * 2);
                }
                oacc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, vb, oacc[nt], 0, 0, 0);
            }
        }
        __syncthreads();
    }
    if constexpr (KSP > 1) {
        // ---- merge the key groups: group 1 parks (m, l, O) in the freed tile buffers, group 0 combines ----
        float* mo = (float*)smem + (wave % GW) * (16 * D + 32);  // [16 rows][D] O, then m[16], l[16]
        if (ksp == 1) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
#pragma unroll
                for (int nt = 0; nt < D / 16; ++nt) mo[(4 * g + i) * D + 16 * nt + col] = oacc[nt][i];
                if (col == 0) {
                    mo[16 * D + 4 * g + i] = mrow[i];
                    mo[16 * D + 16 + 4 * g + i] = lrow[i];
                }
            }
        }
        __syncthreads();
        if (ksp == 1) return;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float m1 = mo[16 * D + 4 * g + i], l1 = mo[16 * D + 16 + 4 * g + i];
            const float mn = fmaxf(mrow[i], m1);
            const float a0 = mn == -INFINITY ? 0.f : exp2f(mrow[i] - mn), a1 = mn == -INFINITY ? 0.f : exp2f(m1 - mn);
            lrow[i] = lrow[i] * a0 + l1 * a1;
#pragma unroll
            for (int nt = 0; nt < D / 16; ++nt)
                oacc[nt][i] = oacc[nt][i] * a0 + mo[(4 * g + i) * D + 16 * nt + col] * a1;
        }
    }
    // ---- write O / l ----
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int qi = row_q0 + 4 * g + i;
        if (qi >= qlen) continue;
        const float inv = lrow[i] > 0.f ? 1.f / lrow[i] : 0.f;
#pragma unroll
        for (int nt = 0; nt < D / 16; ++nt)
            out[((size_t)(qbeg + qi) * Hq + hq) * D + 16 * nt + col] = f32_to_act<F16>(oacc[nt][i] * inv);
    }
}

template <int D, int GW, int VT, int KVF, int KSP = 1>
static void launch_prefill_t(dim3 grid, int threads, size_t lds, const bf16_t* q, const void* kc, const void* vc,
                             const int* bt, int bt_stride, const int* tile_seq, const int* tile_q0, const int* cu_q,
                             const int* ctx_lens, int Hq, int Hkv, int bs, float scale, int window, float softcap,
                             bf16_t* out, hipStream_t st) {
    MX_ACT_DISPATCH({
        if (lds > 65536) {  // D=256 tiles / key-split tiles (73-82 KB): opt in to the large LDS allocation once
            static bool opted = false;
            if (!opted) {
                (void)hipFuncSetAttribute((const void*)attn_prefill_kernel<D, GW, VT, F16, KVF, KSP>,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
                opted = true;
            }
        }
        attn_prefill_kernel<D, GW, VT, F16, KVF, KSP><<<grid, threads, lds, st>>>(
            q, kc, vc, bt, bt_stride, tile_seq, tile_q0, cu_q, ctx_lens, Hq, Hkv, Hq / Hkv, bs, scale, window,
            softcap, out);
    });
}

template <int D, int GW>
static int launch_prefill(const bf16_t* q, const void* kc, const void* vc, const int* bt, int bt_stride,
                          const int* tile_seq, const int* tile_q0, int n_tiles, const int* cu_q,
                          const int* ctx_lens, int Hq, int Hkv, int bs, float scale, int window, float softcap,
                          bf16_t* out, int vmode, int kv8, hipStream_t st) {
    constexpr int NW = GW >= 3 ? GW : 4;
    dim3 grid(n_tiles, Hq / GW);
    const size_t lds0 = 2 * 64 * D * 2 + NW * 16 * (64 + 8) * 2;
    const size_t lds1 = 64 * D * 2 + D * (64 + 8) * 2 + NW * 16 * (64 + 8) * 2;
    // key split when the grid leaves most CUs idle (short prompt chunks): bf16 cache, V image, D = 128, one wave
    // per head and GW = 4 (2 x 4 waves = 512 threads, the kernel's launch bound; the merge buffer, 4 x (16 D + 32)
    // floats, fits the two tile buffers)
    if constexpr (D == 128 && GW == 4) {
        static const bool ks_on = !getenv("MX_PREFILL_KSPLIT") || atoi(getenv("MX_PREFILL_KSPLIT")) != 0;
        if (ks_on && vmode == 0 && !kv8 && (long)n_tiles * (Hq / GW) < 256) {
            launch_prefill_t<D, GW, 0, KVF_BF16, 2>(grid, 2 * NW * 64, 2 * (2 * 64 * D * 2) + 2 * NW * 16 * (64 + 8) * 2,
                                                 q, kc, vc, bt, bt_stride, tile_seq, tile_q0, cu_q, ctx_lens, Hq, Hkv,
                                                 bs, scale, window, softcap, out, st);
            MXK_CHECK_LAUNCH();
        }
    }
#define PFL(VT_, K8_)                                                                                          \
    launch_prefill_t<D, GW, VT_, K8_>(grid, NW * 64, VT_ ? lds1 : lds0, q, kc, vc, bt, bt_stride, tile_seq,    \
                                      tile_q0, cu_q, ctx_lens, Hq, Hkv, bs, scale, window, softcap, out, st)
#define PFK(VT_)                                                                                                \
    {                                                                                                           \
        if (kv8 == KVF_FP8) PFL(VT_, KVF_FP8);                                                                  \
        else if (kv8 == KVF_Q8_0) PFL(VT_, KVF_Q8_0);                                                           \
        else if (kv8 == KVF_Q4_0) PFL(VT_, KVF_Q4_0);                                                           \
        else if (kv8 == KVF_Q4_1) PFL(VT_, KVF_Q4_1);                                                           \
        else if (kv8 == KVF_Q5_0) PFL(VT_, KVF_Q5_0);                                                           \
        else if (kv8 == KVF_Q5_1) PFL(VT_, KVF_Q5_1);                                                           \
        else if (kv8 == KVF_IQ4_NL) PFL(VT_, KVF_IQ4_NL);                                                       \
        else PFL(VT_, KVF_BF16);                                                                                \
    }
    if (vmode == 0) PFK(0) else PFK(1)
#undef PFK
#undef PFL
    MXK_CHECK_LAUNCH();
}

// rows per workgroup for the host-side tile map: 16 * (NW / GW)
extern "C" int mxk_attn_prefill_rows(int Hq, int Hkv) {
    const int G = Hq / Hkv;
    const int GW = G <= 8 ? G : 8;
    const int NW = GW >= 3 ? GW : 4;
    return 16 * (NW / GW);
}

extern "C" int mxk_attn_prefill(const bf16_t* q, const void* kc, const void* vc, const int* bt, int bt_stride,
                                const int* tile_seq, const int* tile_q0, int n_tiles, const int* cu_q,
                                const int* ctx_lens, int Hq, int Hkv, int D, int bs, float scale, int window,
                                float softcap, bf16_t* out, int vmode, int kv8, hipStream_t st) {
    if (n_tiles <= 0) return 0;
    if (Hq % Hkv) return (int)hipErrorInvalidValue;
    const int G = Hq / Hkv;
    const int GW = G <= 8 ? G : 8;
    if (G > 8 && G % 8) return (int)hipErrorInvalidValue;
#define PF(D_, GW_) \
    if (D == D_ && GW == GW_) return launch_prefill<D_, GW_>(q, kc, vc, bt, bt_stride, tile_seq, tile_q0, n_tiles, cu_q, ctx_lens, Hq, Hkv, bs, scale, window, softcap, out, vmode, kv8, st);
    PF(128, 1) PF(128, 2) PF(128, 3) PF(128, 4) PF(128, 5) PF(128, 6) PF(128, 7) PF(128, 8)
    PF(64, 1) PF(64, 2) PF(64, 4) PF(64, 8)
    PF(256, 1) PF(256, 2) PF(256, 4)
#undef PF
    return (int)hipErrorInvalidValue;
}

// debug probe: semantics of ds_read_b64_tr_b16 on this device. LDS holds value r*16+c at row r
// (16 rows), column c (16 cols), 32-byte rows; lane l supplies row (l&15)>>2 (+4*(l>>4)),
// columns 4*(l&3). out[l*4 + e] = element e returned to lane l.
__global__ void probe_tr16_kernel(short* out) {
    __shared__ __attribute__((aligned(16))) short lds[16 * 16];
    for (int i = threadIdx.x; i < 256; i += 64) lds[i] = (short)i;
    __syncthreads();
    const int l = threadIdx.x;
    const int row = ((l & 15) >> 2) + 4 * (l >> 4);
    const int colg = 4 * (l & 3);
    s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((MX_LDS s16x4*)(lds + row * 16 + colg));
    for (int e = 0; e < 4; ++e) out[l * 4 + e] = v[e];
}
extern "C" int mxk_probe_tr16(short* out, hipStream_t st) {
    probe_tr16_kernel<<<1, 64, 0, st>>>(out);
    MXK_CHECK_LAUNCH();
}
