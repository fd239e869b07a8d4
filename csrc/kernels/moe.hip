// moe.hip — mixture-of-experts routing for Mixtral / Qwen2-MoE / Qwen3-MoE style FFNs
// (llama.cpp's build_moe_ffn: ggml_soft_max -> ggml_top_k -> ggml_mul_mat_id).
//
// Everything stays on the device so the MoE layer is graph-capturable:
//   1. moe_route   one wave per token: softmax over the E router logits held in registers
//                  (E/64 per lane), k rounds of wave arg-max (ties -> lower expert id), optional
//                  renormalisation of the k selected probabilities (Mixtral, Qwen3-MoE) or not
//                  (Qwen2-MoE). Out: ids/weights [T, k].
//   2. moe_sort    one 1024-thread workgroup: LDS histogram of the T*k pairs per expert, exclusive
//                  scan -> off[E+1] and the per-expert tile prefix tile_start[E+1] (ceil(n_e/BM)),
//                  then a counting-sort scatter -> sorted_tok[P] (token row of each sorted pair)
//                  and inv_pos[P] (pair -> sorted row). Row order inside an expert does not affect
//                  any result: GEMM rows are independent and the combine below sums in fixed order.
//   3. mxk_moe_qgemm16 (qgemm16.hip, grouped mode): gate|up SwiGLU over sorted rows gathered from
//                  the normed hidden state, then down projection into a [P, H] fp32 buffer.
//   4. moe_combine h[t] += sum_j w[t, j] * Y[inv_pos[t*k + j]] in j order (deterministic; no
//                  atomics on the residual stream).
#include "mx_common.h"

// one wave routes one token: softmax over the row's E logits, k rounds of arg-max, optional renormalisation.
// SC1: the row was written by other workgroups in this launch — read it with agent-scope (sc1) loads
template <int VPL, bool SC1 = false>
MX_DEV void route_row(const float* row, int E, int k, int renorm, int* ids, float* wts, int lane) {
    float v[VPL];
    float mx = -INFINITY;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
        const int e = lane + 64 * i;
        if constexpr (SC1)
            v[i] = e < E ? __hip_atomic_load((float*)row + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : -INFINITY;
        else
            v[i] = e < E ? row[e] : -INFINITY;
        mx = fmaxf(mx, v[i]);
    }
    mx = wave_max(mx);
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
        const int e = lane + 64 * i;
        v[i] = e < E ? __expf(v[i] - mx) : -1.f;  // probabilities are >= 0; -1 marks padding
        s += e < E ? v[i] : 0.f;
    }
    s = wave_sum(s);
    const float inv = 1.f / s;
    float picked = 0.f, my_p = 0.f;
    int my_id = 0;
    for (int j = 0; j < k; ++j) {
        float best = -2.f;
        int bi = 0x7fffffff;
#pragma unroll
        for (int i = 0; i < VPL; ++i) {
            const int e = lane + 64 * i;
            if (v[i] > best) { best = v[i]; bi = e; }
        }
        // wave arg-max: larger value wins, equal values -> smaller index
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const float ob = __shfl_xor(best, o);
            const int oi = __shfl_xor(bi, o);
            if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
        }
        if (bi >= E) {  // NaN logits: keep the index valid for the sort / GEMM, contribute nothing
            bi = 0;
            best = 0.f;
        }
#pragma unroll
        for (int i = 0; i < VPL; ++i)
            if (lane + 64 * i == bi) v[i] = -2.f;  // remove from later rounds
        const float p = best * inv;
        picked += p;
        if (lane == j) {
            my_id = bi;
            my_p = p;
        }
    }
    if (lane < k) {
        ids[lane] = my_id;
        wts[lane] = renorm ? my_p / picked : my_p;
    }
}

template <int VPL>
__global__ __launch_bounds__(256) void moe_route_kernel(const float* __restrict__ logits, int ldl, int T, int E,
                                                        int k, int renorm, int* __restrict__ ids,
                                                        float* __restrict__ wts) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int t = blockIdx.x * 4 + wave;
    if (t >= T) return;
    route_row<VPL>(logits + (size_t)t * ldl, E, k, renorm, ids + (size_t)t * k, wts + (size_t)t * k, lane);
}

extern "C" int mxk_moe_route(const float* logits, int ldl, int T, int E, int k, int renorm, int* ids, float* wts,
                             hipStream_t st);

// Router GEMV: logits[t, e] = x[t] . wr[e] (fp32 router rows, 16-bit hidden rows). Workgroup (token block, expert
// block): TT tokens' rows staged in LDS, one expert per wave — the wave's fp32 router row (H floats) is requested in
// full before any FMA, so a decode step's router costs one load latency instead of one per 256 columns (the first
// form, one workgroup walking every expert, took 177 us per layer at batch 1: profiles/r6_moe_qwen3_30b.md).
// The top-k routing then runs as moe_route_kernel over the logits.
// With `tickets` (one zeroed int per token block): the last expert-block workgroup of a token block to finish runs the
// top-k routing of its tokens (route_row, one wave per token) — router + route in one launch; it re-arms the ticket.
// NRM: the FFN RMSNorm fused in front — the workgroup reads its tokens' fp32 residual rows `hs`, normalises them
// (x = hs / rms(hs) * gamma, rounded to the 16-bit activation type exactly as the norm kernel stores it) into its LDS
// rows, and the expert-block-0 workgroups also write them to `x` for the expert GEMMs: no separate norm launch.
template <int TT, bool F16, int VPL, bool NRM>
__global__ __launch_bounds__(256) void moe_router_kernel(bf16_t* __restrict__ x, int ldx,
                                                         const float* __restrict__ wr, int T, int H, int E,
                                                         float* __restrict__ logits, int* __restrict__ tickets, int k,
                                                         int renorm, int* __restrict__ ids, float* __restrict__ wts,
                                                         const float* __restrict__ hs, int ldh,
                                                         const float* __restrict__ gamma, float eps) {
    extern __shared__ __attribute__((aligned(16))) char rsm[];
    bf16_t* xs = (bf16_t*)rsm;  // [TT][H]
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int t0 = blockIdx.x * TT, nt = min(TT, T - t0);
    const int e = blockIdx.y * 4 + wave;
    // the wave's router row (first 2048 columns) is requested before the rows are staged / normalised: its load
    // latency overlaps that work instead of following it
    const float* w = wr + (size_t)min(e, E - 1) * H;
    float4 w4[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int c = 256 * j + lane * 4;
        w4[j] = (c < H && e < E) ? *(const float4*)(w + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if constexpr (NRM) {
        __shared__ float s_ss[TT];
        if (threadIdx.x < TT) s_ss[threadIdx.x] = 0.f;
        __syncthreads();
        for (int i = threadIdx.x * 8; i < TT * H; i += 256 * 8) {
            const int t = i / H, c = i % H;
            if (t < nt) {
                const float* r = hs + (size_t)(t0 + t) * ldh + c;
                const float4 a = *(const float4*)r, b = *(const float4*)(r + 4);
                atomicAdd(&s_ss[t], a.x * a.x + a.y * a.y + a.z * a.z + a.w * a.w + b.x * b.x + b.y * b.y +
                                        b.z * b.z + b.w * b.w);
            }
        }
        __syncthreads();
        for (int i = threadIdx.x * 8; i < TT * H; i += 256 * 8) {
            const int t = i / H, c = i % H;
            if (t < nt) {
                const float rs = rsqrtf(s_ss[t] / (float)H + eps);
                const float* r = hs + (size_t)(t0 + t) * ldh + c;
                const float4 a = *(const float4*)r, b = *(const float4*)(r + 4);
                const float4 ga = *(const float4*)(gamma + c), gb = *(const float4*)(gamma + c + 4);
                uint4 o;
                o.x = pack_act2<F16>(a.x * rs * ga.x, a.y * rs * ga.y);
                o.y = pack_act2<F16>(a.z * rs * ga.z, a.w * rs * ga.w);
                o.z = pack_act2<F16>(b.x * rs * gb.x, b.y * rs * gb.y);
                o.w = pack_act2<F16>(b.z * rs * gb.z, b.w * rs * gb.w);
                *(uint4*)(xs + i) = o;
                if (blockIdx.y == 0) *(uint4*)(x + (size_t)(t0 + t) * ldx + c) = o;
            }
        }
    } else {
        for (int i = threadIdx.x * 8; i < TT * H; i += 256 * 8) {
            const int t = i / H, c = i % H;
            if (t < nt) *(uint4*)(xs + i) = *(const uint4*)(x + (size_t)(t0 + t) * ldx + c);
        }
    }
    __syncthreads();
    float acc[TT];
#pragma unroll
    for (int t = 0; t < TT; ++t) acc[t] = 0.f;
    for (int c0 = 0; c0 < H && e < E; c0 += 256 * 8) {  // 8 float4 per lane in flight per 2048-column pass
        if (c0 > 0) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int c = c0 + 256 * j + lane * 4;
                w4[j] = c < H ? *(const float4*)(w + c) : make_float4(0.f, 0.f, 0.f, 0.f);
            }
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int c = c0 + 256 * j + lane * 4;
            if (c >= H) break;
#pragma unroll
            for (int t = 0; t < TT; ++t) {
                if (t < nt) {
                    const uint2 raw = *(const uint2*)(xs + t * H + c);
                    float a0, a1, a2, a3;
                    unpack_act2<F16>(raw.x, a0, a1);
                    unpack_act2<F16>(raw.y, a2, a3);
                    acc[t] += w4[j].x * a0 + w4[j].y * a1 + w4[j].z * a2 + w4[j].w * a3;
                }
            }
        }
    }
#pragma unroll
    for (int t = 0; t < TT; ++t) {
        if (t < nt) {
            const float s = wave_sum(acc[t]);
            if (lane == 0 && e < E) {
                if (tickets)  // read by another workgroup of this launch: an sc1 store
                    __hip_atomic_store(logits + (size_t)(t0 + t) * E + e, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                else
                    logits[(size_t)(t0 + t) * E + e] = s;
            }
        }
    }
    if (!tickets) return;
    // fence-free hand-off (MI355X_MICROARCH.md inter-workgroup visibility, row 1): every wave's sc1 stores complete,
    // a barrier, ONE agent-scope atomic add per workgroup; the workgroup whose add came last routes with sc1 loads
    __shared__ int s_last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const int old = __hip_atomic_fetch_add(&tickets[blockIdx.x], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = old == (int)gridDim.y - 1;
        if (s_last) __hip_atomic_store(&tickets[blockIdx.x], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!s_last) return;
    for (int t = wave; t < nt; t += 4)
        route_row<VPL, true>(logits + (size_t)(t0 + t) * E, E, k, renorm, ids + (size_t)(t0 + t) * k,
                             wts + (size_t)(t0 + t) * k, lane);
}

// x 16-bit [T, H] (the normed hidden state), wr fp32 [E, H] -> logits fp32 [T, E] (workspace) -> ids / wts [T, k];
// H % 256 == 0. tickets: ceil(T / 8) zeroed ints (left zeroed) to route in the same launch, or null (a second launch).
// hs (fp32 [T, H] residual rows, ldh) + gamma: x is the OUTPUT, hs's RMSNorm (eps) written by the router itself.
extern "C" int mxk_moe_router(void* x, int ldx, const float* wr, int T, int H, int E, int k, int renorm, int* ids,
                              float* wts, float* logits, int* tickets, const float* hs, int ldh, const float* gamma,
                              float eps, hipStream_t st) {
    if (T <= 0) return 0;
    if (k < 1 || k > 64 || k > E || H % 256 || ldx % 8 || ((uintptr_t)x & 15) || ((uintptr_t)wr & 15) || !logits)
        return (int)hipErrorInvalidValue;
    const bool nrm = hs != nullptr;
    if (nrm && (!gamma || ldh % 4 || ((uintptr_t)hs & 15) || ((uintptr_t)gamma & 15))) return (int)hipErrorInvalidValue;
    constexpr int TT = 8;
    const size_t lds = (size_t)TT * H * 2;
    if (lds > 160 * 1024) return (int)hipErrorInvalidValue;
    const dim3 grid((T + TT - 1) / TT, (E + 3) / 4);
    if (E > 512) return (int)hipErrorInvalidValue;
#define MRK2(V, N_)                                                                                                  \
    do {                                                                                                             \
        static bool attr = false;                                                                                    \
        if (!attr && lds > 64 * 1024) {                                                                              \
            (void)hipFuncSetAttribute((const void*)moe_router_kernel<TT, F16, V, N_>,                                \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);                         \
            attr = true;                                                                                             \
        }                                                                                                            \
        moe_router_kernel<TT, F16, V, N_><<<grid, 256, lds, st>>>((bf16_t*)x, ldx, wr, T, H, E, logits, tickets, k,    \
                                                                  renorm, ids, wts, hs, ldh, gamma, eps);            \
    } while (0)
#define MRK(V) MX_ACT_DISPATCH({ if (nrm) MRK2(V, true); else MRK2(V, false); })
    if (E <= 64) MRK(1);
    else if (E <= 128) MRK(2);
    else if (E <= 256) MRK(4);
    else MRK(8);
#undef MRK
#undef MRK2
    {
        const int err = (int)hipGetLastError();
        if (err) return err;
    }
    if (tickets || !ids) return 0;  // routed by the last workgroup of each token block / logits only (route_sort)
    return mxk_moe_route(logits, E, T, E, k, renorm, ids, wts, st);
}

extern "C" int mxk_moe_route(const float* logits, int ldl, int T, int E, int k, int renorm, int* ids, float* wts,
                             hipStream_t st) {
    if (T <= 0) return 0;
    if (k < 1 || k > 64 || k > E) return (int)hipErrorInvalidValue;
    const int blocks = (T + 3) / 4;
#define MR(V) moe_route_kernel<V><<<blocks, 256, 0, st>>>(logits, ldl, T, E, k, renorm, ids, wts)
    if (E <= 64) MR(1);
    else if (E <= 128) MR(2);
    else if (E <= 256) MR(4);
    else if (E <= 512) MR(8);
    else return (int)hipErrorInvalidValue;
#undef MR
    MXK_CHECK_LAUNCH();
}

__global__ __launch_bounds__(1024) void moe_sort_kernel(const int* __restrict__ ids, int P, int k, int E, int BM,
                                                        int* __restrict__ off, int* __restrict__ tile_start,
                                                        int* __restrict__ sorted_tok, int* __restrict__ inv_pos,
                                                        const float* __restrict__ wts, float* __restrict__ sorted_wt) {
    extern __shared__ int sm[];
    int* cnt = sm;         // [E]
    int* cur = sm + E;     // [E]
    for (int e = threadIdx.x; e < E; e += 1024) cnt[e] = 0;
    __syncthreads();
    for (int p = threadIdx.x; p < P; p += 1024) atomicAdd(&cnt[min(max(ids[p], 0), E - 1)], 1);
    __syncthreads();
    if (threadIdx.x == 0) {
        int o = 0, ts = 0;
        for (int e = 0; e < E; ++e) {
            const int c = cnt[e];
            off[e] = o;
            tile_start[e] = ts;
            cur[e] = o;
            o += c;
            ts += (c + BM - 1) / BM;
        }
        off[E] = o;
        tile_start[E] = ts;
    }
    __syncthreads();
    for (int p = threadIdx.x; p < P; p += 1024) {
        const int pos = atomicAdd(&cur[min(max(ids[p], 0), E - 1)], 1);
        sorted_tok[pos] = p / k;
        inv_pos[p] = pos;
        if (sorted_wt) sorted_wt[pos] = wts[p];
    }
}

extern "C" int mxk_moe_sort(const int* ids, int P, int k, int E, int BM, int* off, int* tile_start, int* sorted_tok,
                            int* inv_pos, const float* wts, float* sorted_wt, hipStream_t st) {
    if (E <= 0 || E > 4096 || BM <= 0 || (sorted_wt && !wts)) return (int)hipErrorInvalidValue;
    moe_sort_kernel<<<1, 1024, 2 * E * sizeof(int), st>>>(ids, P, k, E, BM, off, tile_start, sorted_tok, inv_pos, wts,
                                                          sorted_wt);
    MXK_CHECK_LAUNCH();
}

// Decode-sized batches (T <= 64): routing and the counting sort in ONE workgroup — each of the 16 waves routes tokens
// wave, wave + 16, .. (route_row), the pairs' experts stay in LDS, then the same histogram / scan / scatter as
// moe_sort_kernel. One launch instead of two per MoE layer.
template <int VPL>
__global__ __launch_bounds__(1024) void moe_route_sort_kernel(const float* __restrict__ logits, int ldl, int T, int E,
                                                              int k, int renorm, int* __restrict__ ids,
                                                              float* __restrict__ wts, int BM, int* __restrict__ off,
                                                              int* __restrict__ tile_start,
                                                              int* __restrict__ sorted_tok, int* __restrict__ inv_pos,
                                                              float* __restrict__ sorted_wt) {
    extern __shared__ int rs_sm[];
    int* cnt = rs_sm;            // [E]
    int* cur = rs_sm + E;        // [E]
    int* sid = rs_sm + 2 * E;    // [T k] routed experts
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int e = threadIdx.x; e < E; e += 1024) cnt[e] = 0;
    for (int t = wave; t < T; t += 16) {
        route_row<VPL>(logits + (size_t)t * ldl, E, k, renorm, ids + (size_t)t * k, wts + (size_t)t * k, lane);
    }
    __syncthreads();
    // the routed ids as this workgroup wrote them (same workgroup: visible after the barrier; first touch of the lines)
    const int P = T * k;
    for (int p = threadIdx.x; p < P; p += 1024) {
        const int e = min(max(__hip_atomic_load(ids + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP), 0), E - 1);
        sid[p] = e;
        atomicAdd(&cnt[e], 1);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int o = 0, ts = 0;
        for (int e = 0; e < E; ++e) {
            const int c = cnt[e];
            off[e] = o;
            tile_start[e] = ts;
            cur[e] = o;
            o += c;
            ts += (c + BM - 1) / BM;
        }
        off[E] = o;
        tile_start[E] = ts;
    }
    __syncthreads();
    for (int p = threadIdx.x; p < P; p += 1024) {
        const int pos = atomicAdd(&cur[sid[p]], 1);
        sorted_tok[pos] = p / k;
        inv_pos[p] = pos;
        if (sorted_wt) sorted_wt[pos] = __hip_atomic_load(wts + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
}

extern "C" int mxk_moe_route_sort(const float* logits, int ldl, int T, int E, int k, int renorm, int* ids, float* wts,
                                  int BM, int* off, int* tile_start, int* sorted_tok, int* inv_pos, float* sorted_wt,
                                  hipStream_t st) {
    if (T <= 0) return 0;
    if (k < 1 || k > 64 || k > E || E > 512 || BM <= 0 || T * k > 8192) return (int)hipErrorInvalidValue;
    const size_t lds = (size_t)(2 * E + T * k) * sizeof(int);
#define MRS(V) moe_route_sort_kernel<V><<<1, 1024, lds, st>>>(logits, ldl, T, E, k, renorm, ids, wts, BM, off, tile_start, \
                                                             sorted_tok, inv_pos, sorted_wt)
    if (E <= 64) MRS(1);
    else if (E <= 128) MRS(2);
    else if (E <= 256) MRS(4);
    else MRS(8);
#undef MRS
    MXK_CHECK_LAUNCH();
}

// h[t, :] (+)= sum_j w[t, j] * Y[inv_pos[t*k + j], :]   (fp32; `accumulate` adds into h; inv_pos null: Y rows in
// pair order t*k + j, as the grouped decode GEMV writes them)
__global__ __launch_bounds__(256) void moe_combine_kernel(const float* __restrict__ Y, int ldy,
                                                          const int* __restrict__ inv_pos,
                                                          const float* __restrict__ wts, int k, int H,
                                                          float* __restrict__ h, int ldh, int accumulate) {
    const int t = blockIdx.x;
    for (int c = threadIdx.x * 4; c < H; c += 1024) {
        float4 acc = accumulate ? *(const float4*)(h + (size_t)t * ldh + c) : (float4){0.f, 0.f, 0.f, 0.f};
        for (int j = 0; j < k; ++j) {
            const float w = wts[(size_t)t * k + j];
            const size_t row = inv_pos ? (size_t)inv_pos[(size_t)t * k + j] : (size_t)t * k + j;
            const float4 y = *(const float4*)(Y + row * ldy + c);
            acc.x = fmaf(w, y.x, acc.x);
            acc.y = fmaf(w, y.y, acc.y);
            acc.z = fmaf(w, y.z, acc.z);
            acc.w = fmaf(w, y.w, acc.w);
        }
        *(float4*)(h + (size_t)t * ldh + c) = acc;
    }
}

extern "C" int mxk_moe_combine(const float* Y, int ldy, const int* inv_pos, const float* wts, int T, int k, int H,
                               float* h, int ldh, int accumulate, hipStream_t st) {
    if (T <= 0) return 0;
    if (H % 4 || ldy % 4 || ldh % 4) return (int)hipErrorInvalidValue;
    moe_combine_kernel<<<T, 256, 0, st>>>(Y, ldy, inv_pos, wts, k, H, h, ldh, accumulate);
    MXK_CHECK_LAUNCH();
}
