// rope_kv.hip — fused bias + RoPE + paged KV-cache append (K8 + K10 of SURVEY §2.6).
//
// Consumes the fp32 QKV projection of T tokens ([T, (Hq + 2*Hkv) * D], written by the qgemm/qgemv
// F32 epilogue), applies the optional QKV bias (Qwen2), rotates Q and K, writes Q as bf16 for the
// attention kernel and scatters K/V into the paged cache:
//   cache layout  [num_blocks][Hkv][block_size][D] bf16 — a kv-head's block is one contiguous
//   block_size*D*2-byte run, so decode attention streams it with 16-byte loads.
// Rotation: theta_i = pos * inv_freq[i] (the host folds freq_base, linear/llama3/YaRN scaling into
// inv_freq and the YaRN magnitude correction into attn_factor; grpc-server.cpp:2419-2439 is the
// reference's parameter surface). Modes: NORM (adjacent pairs, llama) and NEOX (half split).
// QKN (Qwen3): per-head RMSNorm of every q and k head (weights qn / kn over head_dim) applied
// after the bias and before the rotation — one wave per head computes the head's rms into LDS,
// so the normalisation costs one extra read of the row instead of a separate kernel.
#include "mx_common.h"

// Grid (T, NG): workgroup (t, g) handles heads [g*HPG, (g+1)*HPG) of the Hq+Hkv rotated heads and
// its share of the Hkv V heads, so short decode batches still spread over the CUs. ZERO: after
// reading its rows the kernel writes them back as zeros — the fp32 QKV buffer is the target of the
// next layer's split-K GEMM (atomic accumulate), which then needs no separate zero-fill launch.
template <bool NEOX, bool HAS_BIAS, bool QKN, bool ZERO, bool KV8>
__global__ __launch_bounds__(256) void rope_kv_kernel(float* __restrict__ qkv, const float* __restrict__ bias,
                                                      const int* __restrict__ pos, const int* __restrict__ slots,
                                                      const float* __restrict__ inv_freq, float attn_factor,
                                                      int Hq, int Hkv, int D, int rot_dim, bf16_t* __restrict__ qo,
                                                      void* __restrict__ kc, void* __restrict__ vc,
                                                      int block_size, const float* __restrict__ qn,
                                                      const float* __restrict__ kn, float eps) {
    __shared__ float cs[256], sn[256], rsh[QKN ? 256 : 1];
    const int t = blockIdx.x;
    const int nh = Hq + Hkv;
    const int hpg = (nh + gridDim.y - 1) / gridDim.y, vpg = (Hkv + gridDim.y - 1) / gridDim.y;
    const int h_lo = blockIdx.y * hpg, h_hi = min(nh, h_lo + hpg);
    const int v_lo = blockIdx.y * vpg, v_hi = min(Hkv, v_lo + vpg);
    const int p = pos[t];
    const int half = rot_dim / 2;
    for (int i = threadIdx.x; i < half; i += 256) {
        float s, c;
        sincosf((float)p * inv_freq[i], &s, &c);
        cs[i] = c * attn_factor;
        sn[i] = s * attn_factor;
    }
    const int W = (Hq + 2 * Hkv) * D;
    float* row = qkv + (size_t)t * W;
    if constexpr (QKN) {
        const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
        for (int h = h_lo + wave; h < h_hi; h += 4) {
            float ss = 0.f;
            for (int d = lane; d < D; d += 64) {
                float x = row[h * D + d];
                if (HAS_BIAS) x += bias[h * D + d];
                ss += x * x;
            }
            ss = wave_sum(ss);
            if (lane == 0) rsh[h] = rsqrtf(ss / D + eps);
        }
    }
    __syncthreads();
    const int slot = slots[t];
    const int blk = slot >= 0 ? slot / block_size : 0, off = slot >= 0 ? slot % block_size : 0;
    // rotate q and k heads: one thread per output element; dims >= rot_dim pass through.
    const int total = (h_hi - h_lo) * D;
    for (int idx = threadIdx.x; idx < total; idx += 256) {
        const int h = h_lo + idx / D, d = idx % D;
        float x = row[h * D + d];
        if (HAS_BIAS) x += bias[h * D + d];
        float nscale = 1.f;
        const float* nw = nullptr;
        if constexpr (QKN) {
            nscale = rsh[h];
            nw = h < Hq ? qn : kn;
            x *= nscale * nw[d];
        }
        float y = x;
        if (d < rot_dim) {
            int pd, fi;
            bool first;
            if (NEOX) { first = d < half; pd = first ? d + half : d - half; fi = first ? d : d - half; }
            else { first = (d & 1) == 0; pd = first ? d + 1 : d - 1; fi = d >> 1; }
            float xp = row[h * D + pd];
            if (HAS_BIAS) xp += bias[h * D + pd];
            if constexpr (QKN) xp *= nscale * nw[pd];
            const float c = cs[fi], s = sn[fi];
            y = first ? (x * c - xp * s) : (xp * s + x * c);
        }
        if (h < Hq) {
            qo[((size_t)t * Hq + h) * D + d] = f32_to_bf16(y);
        } else if (slot >= 0) {
            const int kh = h - Hq;
            const size_t e = (((size_t)blk * Hkv + kh) * block_size + off) * D + d;
            if constexpr (KV8) ((uint8_t*)kc)[e] = f32_to_fp8(y);
            else ((bf16_t*)kc)[e] = f32_to_bf16(y);
        }
    }
    float* vr = row + (Hq + Hkv) * D;
    if (slot >= 0) {
        for (int idx = v_lo * D + threadIdx.x; idx < v_hi * D; idx += 256) {
            const int kh = idx / D, d = idx % D;
            float v = vr[idx];
            if (HAS_BIAS) v += bias[(Hq + Hkv) * D + idx];
            const size_t e = (((size_t)blk * Hkv + kh) * block_size + off) * D + d;
            if constexpr (KV8) ((uint8_t*)vc)[e] = f32_to_fp8(v);
            else ((bf16_t*)vc)[e] = f32_to_bf16(v);
        }
    }
    if constexpr (ZERO) {
        __syncthreads();  // every read of this group's q/k elements (incl. rotation partners) is done
        for (int idx = h_lo * D + threadIdx.x; idx < h_hi * D; idx += 256) row[idx] = 0.f;
        for (int idx = v_lo * D + threadIdx.x; idx < v_hi * D; idx += 256) vr[idx] = 0.f;
    }
}

// Vectorised variant for the common case (rot_dim == D in {64, 128}): each thread owns whole rotation pairs — 4
// consecutive dims (NORM: two adjacent pairs) or 4 dims + their partners D/2 away (NEOX) — so every element is loaded
// once as a float4, written as 8-byte bf16 / 4-byte fp8 runs, and the head / dim split is shifts instead of
// divisions. QKN (Qwen3 / Gemma-3 per-head RMSNorm of q and k before the rotation): a head's UPH threads are
// consecutive lanes of one wave, so its sum of squares is a UPH-lane shuffle reduction of the values already in
// registers (no LDS pass, no second read of the row).
template <int D, bool NEOX, bool HAS_BIAS, bool ZERO, bool KV8, bool QKN = false>
__global__ __launch_bounds__(256) void rope_kv4_kernel(float* __restrict__ qkv, const float* __restrict__ bias,
                                                       const int* __restrict__ pos, const int* __restrict__ slots,
                                                       const float* __restrict__ inv_freq, float attn_factor, int Hq,
                                                       int Hkv, bf16_t* __restrict__ qo, void* __restrict__ kc,
                                                       void* __restrict__ vc, int block_size,
                                                       const float* __restrict__ qn = nullptr,
                                                       const float* __restrict__ kn = nullptr, float eps = 0.f) {
    constexpr int HALF = D / 2;
    constexpr int UPH = NEOX ? D / 8 : D / 4;  // work units per head
    constexpr int USH = UPH == 8 ? 3 : UPH == 16 ? 4 : 5;
    static_assert((1 << USH) == UPH, "units per head");
    __shared__ float cs[HALF], sn[HALF];
    const int t = blockIdx.x;
    const int nh = Hq + Hkv;
    const int hpg = (nh + gridDim.y - 1) / gridDim.y, vpg = (Hkv + gridDim.y - 1) / gridDim.y;
    const int h_lo = blockIdx.y * hpg, h_hi = min(nh, h_lo + hpg);
    const int v_lo = blockIdx.y * vpg, v_hi = min(Hkv, v_lo + vpg);
    const int W = (Hq + 2 * Hkv) * D;
    float* row = qkv + (size_t)t * W;
    auto ld4 = [&](int e) {
        float4 x = *(const float4*)(row + e);
        if (HAS_BIAS) {
            const float4 b = *(const float4*)(bias + e);
            x.x += b.x; x.y += b.y; x.z += b.z; x.w += b.w;
        }
        return x;
    };
    const int total = (h_hi - h_lo) << USH;
    // the first unit's row elements are requested before the rotation table is built: their latency overlaps the
    // sincosf work and the table barrier
    float4 a0 = {0.f, 0.f, 0.f, 0.f}, b0 = {0.f, 0.f, 0.f, 0.f};
    if (threadIdx.x < total) {
        const int h = h_lo + (threadIdx.x >> USH), u = threadIdx.x & (UPH - 1);
        a0 = ld4(h * D + 4 * u);
        if constexpr (NEOX) b0 = ld4(h * D + 4 * u + HALF);
    }
    const int p = pos[t];
    for (int i = threadIdx.x; i < HALF; i += 256) {
        float sv, cv;
        sincosf((float)p * inv_freq[i], &sv, &cv);
        cs[i] = cv * attn_factor;
        sn[i] = sv * attn_factor;
    }
    __syncthreads();
    const int slot = slots[t];
    const int blk = slot >= 0 ? slot / block_size : 0, off = slot >= 0 ? slot % block_size : 0;
    auto st4 = [&](int h, int d, float4 y) {
        if (h < Hq) {
            uint2 o = {pack_bf16x2(y.x, y.y), pack_bf16x2(y.z, y.w)};
            *(uint2*)(qo + ((size_t)t * Hq + h) * D + d) = o;
        } else if (slot >= 0) {
            const size_t e = (((size_t)blk * Hkv + (h - Hq)) * block_size + off) * D + d;
            if constexpr (KV8) {
                ((uint8_t*)kc)[e] = f32_to_fp8(y.x); ((uint8_t*)kc)[e + 1] = f32_to_fp8(y.y);
                ((uint8_t*)kc)[e + 2] = f32_to_fp8(y.z); ((uint8_t*)kc)[e + 3] = f32_to_fp8(y.w);
            } else {
                uint2 o = {pack_bf16x2(y.x, y.y), pack_bf16x2(y.z, y.w)};
                *(uint2*)((bf16_t*)kc + e) = o;
            }
        }
    };
    const float4 z4 = {0.f, 0.f, 0.f, 0.f};
    // ZERO: every element is read by exactly one thread, which zeroes it after use (the next layer's split GEMM
    // accumulates into the buffer) — no block barrier, no wait for the other threads' stores
    for (int idx = threadIdx.x; idx < total; idx += 256) {
        const int h = h_lo + (idx >> USH), u = idx & (UPH - 1);
        if constexpr (NEOX) {
            const int d = 4 * u;  // dims d..d+3 and their partners d+HALF..
            float4 a = idx == threadIdx.x ? a0 : ld4(h * D + d), b = idx == threadIdx.x ? b0 : ld4(h * D + d + HALF);
            if constexpr (QKN) {
                const float ss = group_sum<UPH>(a.x * a.x + a.y * a.y + a.z * a.z + a.w * a.w + b.x * b.x + b.y * b.y +
                                                b.z * b.z + b.w * b.w);
                const float rs = rsqrtf(ss / D + eps);
                const float* nw = h < Hq ? qn : kn;
                const float4 na = *(const float4*)(nw + d), nb = *(const float4*)(nw + d + HALF);
                a.x *= rs * na.x; a.y *= rs * na.y; a.z *= rs * na.z; a.w *= rs * na.w;
                b.x *= rs * nb.x; b.y *= rs * nb.y; b.z *= rs * nb.z; b.w *= rs * nb.w;
            }
            float4 ya, yb;
            ya.x = a.x * cs[d] - b.x * sn[d];         yb.x = b.x * cs[d] + a.x * sn[d];
            ya.y = a.y * cs[d + 1] - b.y * sn[d + 1]; yb.y = b.y * cs[d + 1] + a.y * sn[d + 1];
            ya.z = a.z * cs[d + 2] - b.z * sn[d + 2]; yb.z = b.z * cs[d + 2] + a.z * sn[d + 2];
            ya.w = a.w * cs[d + 3] - b.w * sn[d + 3]; yb.w = b.w * cs[d + 3] + a.w * sn[d + 3];
            st4(h, d, ya);
            st4(h, d + HALF, yb);
            if constexpr (ZERO) {
                *(float4*)(row + h * D + d) = z4;
                *(float4*)(row + h * D + d + HALF) = z4;
            }
        } else {
            const int d = 4 * u, f = 2 * u;  // pairs (d, d+1) and (d+2, d+3): frequencies f, f+1
            float4 x = idx == threadIdx.x ? a0 : ld4(h * D + d);
            if constexpr (QKN) {
                const float ss = group_sum<UPH>(x.x * x.x + x.y * x.y + x.z * x.z + x.w * x.w);
                const float rs = rsqrtf(ss / D + eps);
                const float4 nw = *(const float4*)((h < Hq ? qn : kn) + d);
                x.x *= rs * nw.x; x.y *= rs * nw.y; x.z *= rs * nw.z; x.w *= rs * nw.w;
            }
            float4 y;
            y.x = x.x * cs[f] - x.y * sn[f];
            y.y = x.y * cs[f] + x.x * sn[f];
            y.z = x.z * cs[f + 1] - x.w * sn[f + 1];
            y.w = x.w * cs[f + 1] + x.z * sn[f + 1];
            st4(h, d, y);
            if constexpr (ZERO) *(float4*)(row + h * D + d) = z4;
        }
    }
    float* vr = row + (Hq + Hkv) * D;
    for (int idx = v_lo * (D / 4) + threadIdx.x; idx < v_hi * (D / 4); idx += 256) {
        const int kh = idx / (D / 4), d = (idx % (D / 4)) * 4;
        if (slot >= 0) {
            float4 v = *(const float4*)(vr + kh * D + d);
            if (HAS_BIAS) {
                const float4 b = *(const float4*)(bias + (Hq + Hkv) * D + kh * D + d);
                v.x += b.x; v.y += b.y; v.z += b.z; v.w += b.w;
            }
            const size_t e = (((size_t)blk * Hkv + kh) * block_size + off) * D + d;
            if constexpr (KV8) {
                ((uint8_t*)vc)[e] = f32_to_fp8(v.x); ((uint8_t*)vc)[e + 1] = f32_to_fp8(v.y);
                ((uint8_t*)vc)[e + 2] = f32_to_fp8(v.z); ((uint8_t*)vc)[e + 3] = f32_to_fp8(v.w);
            } else {
                uint2 o = {pack_bf16x2(v.x, v.y), pack_bf16x2(v.z, v.w)};
                *(uint2*)((bf16_t*)vc + e) = o;
            }
        }
        if constexpr (ZERO) *(float4*)(vr + kh * D + d) = z4;
    }
}

extern "C" int mxk_rope_kv(float* qkv, const float* bias, const int* pos, const int* slots,
                           const float* inv_freq, float attn_factor, int T, int Hq, int Hkv, int D, int rot_dim,
                           int neox, bf16_t* qo, void* kc, void* vc, int block_size, const float* qn,
                           const float* kn, float eps, int zero_after, int kv_fp8, hipStream_t st) {
    if (T <= 0) return 0;
    if (rot_dim > 512 || (rot_dim & 1) || D & 1) return (int)hipErrorInvalidValue;
    const bool qkn = qn != nullptr && kn != nullptr;
    if (qkn && Hq + Hkv > 256) return (int)hipErrorInvalidValue;
    // enough workgroups for the 256 CUs even at small decode batches, >= 1 head per group
    int ng = (512 + T - 1) / T;
    ng = max(1, min(ng, min(8, Hkv)));
    const dim3 grid(T, ng);
    if (rot_dim == D && (D == 64 || D == 128) && !(((uintptr_t)qkv) & 15) && !(((uintptr_t)bias) & 15) &&
        (!qkn || (!(((uintptr_t)qn) & 15) && !(((uintptr_t)kn) & 15)))) {
#define RK4(D_, N_, B_, Z_, K8_)                                                                                         \
    do {                                                                                                                 \
        if (qkn) rope_kv4_kernel<D_, N_, B_, Z_, K8_, true><<<grid, 256, 0, st>>>(qkv, bias, pos, slots, inv_freq,       \
                                                                                  attn_factor, Hq, Hkv, qo, kc, vc,      \
                                                                                  block_size, qn, kn, eps);              \
        else rope_kv4_kernel<D_, N_, B_, Z_, K8_><<<grid, 256, 0, st>>>(qkv, bias, pos, slots, inv_freq, attn_factor,    \
                                                                        Hq, Hkv, qo, kc, vc, block_size);                \
    } while (0)
#define RK4Z(D_, N_, B_) { if (zero_after) { if (kv_fp8) RK4(D_, N_, B_, true, true); else RK4(D_, N_, B_, true, false); } \
                           else { if (kv_fp8) RK4(D_, N_, B_, false, true); else RK4(D_, N_, B_, false, false); } }
#define RK4B(D_, N_) { if (bias) RK4Z(D_, N_, true) else RK4Z(D_, N_, false) }
        if (D == 128) { if (neox) RK4B(128, true) else RK4B(128, false) }
        else { if (neox) RK4B(64, true) else RK4B(64, false) }
#undef RK4B
#undef RK4Z
#undef RK4
        MXK_CHECK_LAUNCH();
    }
#define RKZ(N_, B_, Q_, K8_) { if (zero_after) rope_kv_kernel<N_, B_, Q_, true, K8_><<<grid, 256, 0, st>>>(qkv, bias, pos, slots, inv_freq, attn_factor, Hq, Hkv, D, rot_dim, qo, kc, vc, block_size, qn, kn, eps); \
    else rope_kv_kernel<N_, B_, Q_, false, K8_><<<grid, 256, 0, st>>>(qkv, bias, pos, slots, inv_freq, attn_factor, Hq, Hkv, D, rot_dim, qo, kc, vc, block_size, qn, kn, eps); }
#define RK(N_, B_, Q_) { if (kv_fp8) RKZ(N_, B_, Q_, true) else RKZ(N_, B_, Q_, false) }
#define RKQ(N_, B_) { if (qkn) RK(N_, B_, true) else RK(N_, B_, false) }
    if (neox) { if (bias) RKQ(true, true) else RKQ(true, false) }
    else { if (bias) RKQ(false, true) else RKQ(false, false) }
#undef RKQ
#undef RK
#undef RKZ
    MXK_CHECK_LAUNCH();
}

// Copy whole KV blocks (prefix-cache copy-on-write / beam fork): dst[i] <- src[i] for all layers
// handled by the caller (one launch per layer cache tensor).
__global__ __launch_bounds__(256) void copy_blocks_kernel(bf16_t* __restrict__ cache, const int* __restrict__ src,
                                                          const int* __restrict__ dst, int block_elems) {
    const int b = blockIdx.y;
    const size_t so = (size_t)src[b] * block_elems, dO = (size_t)dst[b] * block_elems;
    for (int i = (blockIdx.x * 256 + threadIdx.x) * 8; i < block_elems; i += gridDim.x * 256 * 8)
        *(uint4*)(cache + dO + i) = *(const uint4*)(cache + so + i);
}

extern "C" int mxk_copy_blocks(bf16_t* cache, const int* src, const int* dst, int n, int block_elems,
                               hipStream_t st) {
    if (n <= 0) return 0;
    if (block_elems % 8) return (int)hipErrorInvalidValue;
    dim3 grid(min(64, (block_elems / 8 + 255) / 256), n);
    copy_blocks_kernel<<<grid, 256, 0, st>>>(cache, src, dst, block_elems);
    MXK_CHECK_LAUNCH();
}
