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

template <int VPL>
__global__ __launch_bounds__(256) void moe_route_kernel(const float* __restrict__ logits, int ldl, int T, int E,
                                                        int k, int renorm, int* __restrict__ ids,
                                                        float* __restrict__ wts) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int t = blockIdx.x * 4 + wave;
    if (t >= T) return;
    const float* row = logits + (size_t)t * ldl;
    float v[VPL];
    float mx = -INFINITY;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
        const int e = lane + 64 * i;
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
        ids[(size_t)t * k + lane] = my_id;
        wts[(size_t)t * k + lane] = renorm ? my_p / picked : my_p;
    }
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
                                                        int* __restrict__ sorted_tok, int* __restrict__ inv_pos) {
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
    }
}

extern "C" int mxk_moe_sort(const int* ids, int P, int k, int E, int BM, int* off, int* tile_start, int* sorted_tok,
                            int* inv_pos, hipStream_t st) {
    if (E <= 0 || E > 4096 || BM <= 0) return (int)hipErrorInvalidValue;
    moe_sort_kernel<<<1, 1024, 2 * E * sizeof(int), st>>>(ids, P, k, E, BM, off, tile_start, sorted_tok, inv_pos);
    MXK_CHECK_LAUNCH();
}

// h[t, :] (+)= sum_j w[t, j] * Y[inv_pos[t*k + j], :]   (fp32; `accumulate` adds into h)
__global__ __launch_bounds__(256) void moe_combine_kernel(const float* __restrict__ Y, int ldy,
                                                          const int* __restrict__ inv_pos,
                                                          const float* __restrict__ wts, int k, int H,
                                                          float* __restrict__ h, int ldh, int accumulate) {
    const int t = blockIdx.x;
    for (int c = threadIdx.x * 4; c < H; c += 1024) {
        float4 acc = accumulate ? *(const float4*)(h + (size_t)t * ldh + c) : (float4){0.f, 0.f, 0.f, 0.f};
        for (int j = 0; j < k; ++j) {
            const float w = wts[(size_t)t * k + j];
            const float4 y = *(const float4*)(Y + (size_t)inv_pos[(size_t)t * k + j] * ldy + c);
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
