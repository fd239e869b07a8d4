// sampling.hip — fused on-GPU token sampler (K13 of SURVEY §2.6).
//
// The reference samples on the CPU over the full 128k-vocab logits of every slot every step
// (grpc-server.cpp:2038 common_sampler_sample). Here one 1024-thread workgroup per sequence does the
// whole chain on the device with no sort:
//   sparse penalties/bias (repeat, presence, frequency, logit_bias: host passes unique (tok, count,
//   bias) triples per row)  ->  grammar allow-mask  ->  temperature  ->  top-k / top-p / min-p /
//   typical-p / mirostat-v2 truncation, each as a threshold found by bisection on the value axis
//   ->  Gumbel-max draw over the kept set (exactly a categorical sample of the renormalised
//   distribution), or argmax when greedy.
// Output: token id and its log-probability under the final (truncated, tempered) distribution.
#include "mx_common.h"

struct SampleParams {
    float temperature;  // <= 0 -> greedy
    int top_k;          // <= 0 -> off
    float top_p;        // >= 1 -> off
    float min_p;        // <= 0 -> off
    float typical_p;    // >= 1 -> off
    float mirostat_tau;  // mirostat v2 truncation mu (already 2*tau on first step); <= 0 -> off
    float repeat_penalty;
    float presence_penalty;
    float frequency_penalty;
    int pen_offset;  // into the sparse penalty arrays
    int pen_count;
    unsigned long long seed;
};

MX_DEV uint32_t mix32(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL;
    x ^= x >> 33;
    return (uint32_t)x;
}
MX_DEV float gumbel(uint64_t seed, uint32_t i) {
    const uint32_t r = mix32(seed * 0x9E3779B97F4A7C15ULL + i);
    const float u = ((float)(r >> 8) + 0.5f) * (1.f / 16777216.f);
    return -__logf(-__logf(u));
}

constexpr int SNT = 1024;

MX_DEV float bsum(float v, float* red) {
    v = wave_sum(v);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < SNT / 64; ++i) t += red[i];
    __syncthreads();
    return t;
}
MX_DEV float bmax(float v, float* red) {
    v = wave_max(v);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    float t = -INFINITY;
#pragma unroll
    for (int i = 0; i < SNT / 64; ++i) t = fmaxf(t, red[i]);
    __syncthreads();
    return t;
}

// sparse penalties + logit bias, in place (unique tokens per row -> no write conflicts)
MX_DEV void apply_penalties(float* x, int V, const SampleParams& P, const int* pen_tok, const int* pen_cnt,
                            const float* pen_bias) {
    for (int i = threadIdx.x; i < P.pen_count; i += SNT) {
        const int t = pen_tok[P.pen_offset + i];
        if (t < 0 || t >= V) continue;
        const int c = pen_cnt[P.pen_offset + i];
        float v = x[t];
        if (c > 0) {
            if (P.repeat_penalty != 1.f) v = v > 0.f ? v / P.repeat_penalty : v * P.repeat_penalty;
            v -= P.frequency_penalty * (float)c + P.presence_penalty;
        }
        v += pen_bias[P.pen_offset + i];
        x[t] = v;
    }
    __syncthreads();
}

// General chain by bisection on the value axis (every pass streams the whole row): typical-p, mirostat,
// and the rare rows whose truncation keeps more candidates than the fast path's LDS holds.
MX_DEV void sample_row_bisect(float* __restrict__ x, int V, const SampleParams& P, const uint32_t* am,
                              int row, int* __restrict__ out_tok, float* __restrict__ out_logp, float* red, float* rv,
                              int* ri) {
    const bool greedy = P.temperature <= 0.f;
    const float itemp = greedy ? 1.f : 1.f / P.temperature;
    auto val = [&](int i) -> float {
        float v = x[i];
        if (am && !((am[i >> 5] >> (i & 31)) & 1u)) return -INFINITY;
        return v * itemp;
    };
    // 2. max and log-sum-exp of the tempered distribution
    float mx = -INFINITY;
    for (int i = threadIdx.x; i < V; i += SNT) mx = fmaxf(mx, val(i));
    mx = bmax(mx, red);
    float thr = -INFINITY;  // keep tokens with val >= thr
    if (!greedy) {
        // top-k: largest thr with count(val >= thr) >= k, by bisection on [mx - 64, mx]
        if (P.top_k > 0 && P.top_k < V) {
            float lo = mx - 80.f, hi = mx;
            for (int it = 0; it < 28; ++it) {
                const float mid = 0.5f * (lo + hi);
                float c = 0.f;
                for (int i = threadIdx.x; i < V; i += SNT) c += val(i) >= mid ? 1.f : 0.f;
                c = bsum(c, red);
                if (c >= (float)P.top_k) lo = mid; else hi = mid;
            }
            thr = fmaxf(thr, lo);
        }
        float Z = 0.f;
        for (int i = threadIdx.x; i < V; i += SNT) { const float v = val(i); Z += v >= thr ? __expf(v - mx) : 0.f; }
        Z = bsum(Z, red);
        // min-p: keep p >= min_p * p_max  <=>  val >= mx + log(min_p)
        if (P.min_p > 0.f && P.min_p <= 1.f) thr = fmaxf(thr, mx + __logf(P.min_p));
        // top-p: largest thr with mass(val >= thr) >= top_p * Z
        if (P.top_p < 1.f && P.top_p > 0.f) {
            float lo = fmaxf(thr, mx - 80.f), hi = mx;
            for (int it = 0; it < 28; ++it) {
                const float mid = 0.5f * (lo + hi);
                float s = 0.f;
                for (int i = threadIdx.x; i < V; i += SNT) { const float v = val(i); s += v >= mid ? __expf(v - mx) : 0.f; }
                s = bsum(s, red);
                if (s >= P.top_p * Z) lo = mid; else hi = mid;
            }
            thr = fmaxf(thr, lo);
        }
        // typical-p: keep tokens whose surprise is closest to the entropy, cumulative mass >= typical_p
        if (P.typical_p < 1.f && P.typical_p > 0.f) {
            const float lZ = __logf(Z);
            float H = 0.f;
            for (int i = threadIdx.x; i < V; i += SNT) {
                const float v = val(i);
                if (v >= thr) { const float lp = v - mx - lZ; H -= __expf(lp) * lp; }
            }
            H = bsum(H, red);
            // bisection on eps: keep |(-lp) - H| <= eps
            float lo = 0.f, hi = 80.f;
            for (int it = 0; it < 28; ++it) {
                const float mid = 0.5f * (lo + hi);
                float s = 0.f;
                for (int i = threadIdx.x; i < V; i += SNT) {
                    const float v = val(i);
                    if (v >= thr) { const float lp = v - mx - lZ; s += fabsf(-lp - H) <= mid ? __expf(lp) : 0.f; }
                }
                s = bsum(s, red);
                if (s >= P.typical_p) hi = mid; else lo = mid;
            }
            // encode the typical band into the value test below via a second bound: keep v with
            // |-(v - mx - lZ) - H| <= hi.  (applied in the draw loop)
            thr = fmaxf(thr, -INFINITY);
            // stash in shared for the draw
            if (threadIdx.x == 0) { rv[0] = hi; rv[1] = H; rv[2] = lZ; }
            __syncthreads();
        }
        // mirostat v2: keep tokens with surprise -log2 p <= mu
        if (P.mirostat_tau > 0.f) {
            const float lZ = __logf(Z);
            // -log2(p) <= mu  <=>  v >= mx + lZ - mu*ln2
            thr = fmaxf(thr, mx + lZ - P.mirostat_tau * 0.69314718f);
            thr = fminf(thr, mx);  // always keep the argmax
        }
    }
    const bool typ = !greedy && P.typical_p < 1.f && P.typical_p > 0.f;
    float tb = 0.f, tH = 0.f, tlZ = 0.f;
    if (typ) { tb = rv[0]; tH = rv[1]; tlZ = rv[2]; }
    __syncthreads();
    // 3. draw: argmax of v (+ Gumbel noise) over the kept set
    float best = -INFINITY;
    int bi = 0x7fffffff;
    for (int i = threadIdx.x; i < V; i += SNT) {
        const float v = val(i);
        if (v < thr || v == -INFINITY) continue;
        if (typ && fabsf(-(v - mx - tlZ) - tH) > tb && v < mx) continue;
        const float sc = greedy ? v : v + gumbel(P.seed, (uint32_t)i);
        if (sc > best || (sc == best && i < bi)) { best = sc; bi = i; }
    }
    // block argmax
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float ob = __shfl_xor(best, o, 64);
        const int oi = __shfl_xor(bi, o, 64);
        if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
    }
    if ((threadIdx.x & 63) == 0) { rv[threadIdx.x >> 6] = best; ri[threadIdx.x >> 6] = bi; }
    __syncthreads();
    if (threadIdx.x == 0) {
        float b = rv[0];
        int id = ri[0];
        for (int w = 1; w < SNT / 64; ++w)
            if (rv[w] > b || (rv[w] == b && ri[w] < id)) { b = rv[w]; id = ri[w]; }
        if (id == 0x7fffffff) id = 0;
        out_tok[row] = id;
        rv[0] = (float)id;
    }
    __syncthreads();
    if (out_logp) {
        // log-prob of the chosen token under the tempered, truncated distribution
        const int id = (int)rv[0];
        float Z = 0.f;
        for (int i = threadIdx.x; i < V; i += SNT) {
            const float v = val(i);
            if (v >= thr && v != -INFINITY) Z += __expf(v - mx);
        }
        Z = bsum(Z, red);
        if (threadIdx.x == 0) out_logp[row] = val(id) - mx - __logf(fmaxf(Z, 1e-30f));
    }
}

// ---- fast path: histogram -> candidate set in LDS -> exact truncation on the candidates ----------------
// Streams the row three times (max, histogram of the distance to the max with per-bin exp mass, candidate
// gather) instead of the ~60 passes of the bisection chain: at 128 rows x 128k vocabulary that is ~40 us
// instead of ~2.5 ms per step. The histogram picks the lowest bin that must be kept (top-k by count,
// top-p by mass, min-p by value); every token at or above it is gathered (value, id) into LDS, sorted
// (bitonic, descending), truncated exactly, and drawn by the same Gumbel-max as the bisection path, so
// both paths pick the same token for the same kept set.
constexpr int SHB = 2048;           // histogram bins over d = max - v in [0, SHR)
constexpr float SHR = 48.f;         // exp(-48) ~ 1e-21: mass beyond is negligible
constexpr int SCAP = 4096;          // candidate capacity (power of two for the bitonic sort)

__global__ __launch_bounds__(SNT) void sample_kernel(float* __restrict__ logits, int ld, int V,
                                                     const SampleParams* __restrict__ params,
                                                     const int* __restrict__ pen_tok,
                                                     const int* __restrict__ pen_cnt,
                                                     const float* __restrict__ pen_bias,
                                                     const uint32_t* __restrict__ allow_mask, int mask_ld,
                                                     int* __restrict__ out_tok, float* __restrict__ out_logp) {
    __shared__ float red[SNT / 64];
    __shared__ float rv[SNT / 64];
    __shared__ int ri[SNT / 64];
    __shared__ unsigned hcnt[SHB];
    __shared__ float hmass[SHB];
    __shared__ float cv[SCAP];
    __shared__ int ci[SCAP];
    __shared__ int s_n, s_bin;
    const int row = blockIdx.x;
    const SampleParams P = params[row];
    float* x = logits + (size_t)row * ld;
    const uint32_t* am = allow_mask ? allow_mask + (size_t)row * mask_ld : nullptr;
    apply_penalties(x, V, P, pen_tok, pen_cnt, pen_bias);
    const bool greedy = P.temperature <= 0.f;
    const bool fast_ok = !greedy && !(P.typical_p < 1.f && P.typical_p > 0.f) && !(P.mirostat_tau > 0.f) &&
                         ((P.top_k > 0 && P.top_k <= SCAP) || (P.top_p < 1.f && P.top_p > 0.f) || P.min_p > 0.f);
    if (!fast_ok) {
        sample_row_bisect(x, V, P, am, row, out_tok, out_logp, red, rv, ri);
        return;
    }
    const float itemp = 1.f / P.temperature;
    auto val = [&](int i, float v) -> float {
        if (am && !((am[i >> 5] >> (i & 31)) & 1u)) return -INFINITY;
        return v * itemp;
    };
    const bool vec = ((((uintptr_t)x) & 15) == 0);
    const int V4 = vec ? (V & ~3) : 0;
    // pass 1: max
    float mx = -INFINITY;
    for (int i = threadIdx.x * 4; i < V4; i += SNT * 4) {
        const float4 a = *(const float4*)(x + i);
        mx = fmaxf(fmaxf(fmaxf(mx, val(i, a.x)), val(i + 1, a.y)), fmaxf(val(i + 2, a.z), val(i + 3, a.w)));
    }
    for (int i = V4 + threadIdx.x; i < V; i += SNT) mx = fmaxf(mx, val(i, x[i]));
    mx = bmax(mx, red);
    for (int b = threadIdx.x; b < SHB; b += SNT) { hcnt[b] = 0u; hmass[b] = 0.f; }
    __syncthreads();
    // pass 2: histogram of d = mx - v (count and exp mass per bin); Z over the whole row
    constexpr float BW = SHR / (float)SHB, IBW = (float)SHB / SHR;
    float Zt = 0.f;
    auto hist = [&](float v) {
        if (v == -INFINITY) return;
        const float e = __expf(v - mx);
        Zt += e;
        const int b = (int)fminf((float)(SHB - 1), (mx - v) * IBW);  // float clamp: no int overflow
        atomicAdd(&hcnt[b], 1u);
        atomicAdd(&hmass[b], e);
    };
    for (int i = threadIdx.x * 4; i < V4; i += SNT * 4) {
        const float4 a = *(const float4*)(x + i);
        hist(val(i, a.x)); hist(val(i + 1, a.y)); hist(val(i + 2, a.z)); hist(val(i + 3, a.w));
    }
    for (int i = V4 + threadIdx.x; i < V; i += SNT) hist(val(i, x[i]));
    const float Z = bsum(Zt, red);
    // lowest bin that must be gathered. With top-k on, the candidates must hold the whole top-k set: top-p's
    // target mass is top_p x the top-k set's mass (the bisection chain's semantics), so its mass is needed even
    // where min-p later trims the set. With top-k off the target is top_p x Z (Z: the whole row) and the
    // candidates stop at that mass; min-p caps the search wherever the top-k mass is not needed.
    const bool tk = P.top_k > 0 && P.top_k < V, tp = P.top_p < 1.f && P.top_p > 0.f;
    if (threadIdx.x == 0) {
        int lim = SHB - 1;
        if (P.min_p > 0.f && P.min_p <= 1.f && !(tk && tp)) lim = min(lim, (int)(-__logf(P.min_p) * IBW));
        unsigned c = 0;
        float m = 0.f;
        int b = 0;
        for (; b < lim; ++b) {
            c += hcnt[b];
            m += hmass[b];
            if (tk) {
                if (c >= (unsigned)P.top_k) break;
            } else if (tp && m >= P.top_p * Z) {
                break;
            }
        }
        s_bin = b;
        s_n = 0;
    }
    __syncthreads();
    const float cut = mx - ((float)s_bin + 1.01f) * BW;  // gather every v > cut (a superset of the kept set)
    // pass 3: gather candidates
    auto gather = [&](int i, float v) {
        if (v == -INFINITY || !(v > cut || v == mx)) return;
        const int k = atomicAdd(&s_n, 1);
        if (k < SCAP) { cv[k] = v; ci[k] = i; }
    };
    for (int i = threadIdx.x * 4; i < V4; i += SNT * 4) {
        const float4 a = *(const float4*)(x + i);
        gather(i, val(i, a.x)); gather(i + 1, val(i + 1, a.y)); gather(i + 2, val(i + 2, a.z)); gather(i + 3, val(i + 3, a.w));
    }
    for (int i = V4 + threadIdx.x; i < V; i += SNT) gather(i, val(i, x[i]));
    __syncthreads();
    const int n = s_n;
    if (n > SCAP) {  // a flat distribution: more candidates than LDS holds
        sample_row_bisect(x, V, P, am, row, out_tok, out_logp, red, rv, ri);
        return;
    }
    // bitonic sort of the candidates, descending by value (ties: ascending id), padded to a power of two
    int np = 1;
    while (np < n) np <<= 1;
    for (int k = n + threadIdx.x; k < np; k += SNT) { cv[k] = -INFINITY; ci[k] = 0x7fffffff; }
    __syncthreads();
    for (int size = 2; size <= np; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int t = threadIdx.x; t < np / 2; t += SNT) {
                const int lo = 2 * t - (t & (stride - 1)), hi = lo + stride;
                const bool desc = (lo & size) == 0;
                const float a = cv[lo], bb = cv[hi];
                const int ia = ci[lo], ib = ci[hi];
                const bool a_first = a > bb || (a == bb && ia < ib);
                if (a_first != desc) { cv[lo] = bb; cv[hi] = a; ci[lo] = ib; ci[hi] = ia; }
            }
            __syncthreads();
        }
    }
    // exact truncation on the sorted candidates (thread 0: at most SCAP steps), then Gumbel-max draw
    if (threadIdx.x == 0) {
        // same semantics as the bisection chain: top-k (ties at the k-th value kept), then top-p's target
        // mass is top_p x the top-k set's mass, measured over the set that also passes min-p
        int keep = n;
        if (P.top_k > 0 && P.top_k < keep) {
            const float kv = cv[P.top_k - 1];
            keep = P.top_k;
            while (keep < n && cv[keep] == kv) ++keep;
        }
        float zk = Z;  // top-k off: the whole row's mass
        if (tp && tk) {
            zk = 0.f;
            for (int k = 0; k < keep; ++k) zk += __expf(cv[k] - mx);
        }
        if (P.min_p > 0.f && P.min_p <= 1.f) {
            const float mv = mx + __logf(P.min_p);
            while (keep > 1 && cv[keep - 1] < mv) --keep;
        }
        if (P.top_p < 1.f && P.top_p > 0.f) {
            float cum = 0.f;
            int k = 0;
            while (k < keep) {
                cum += __expf(cv[k] - mx);
                ++k;
                if (cum >= P.top_p * zk) break;
            }
            while (k < keep && cv[k] == cv[k - 1]) ++k;  // equal values stay together
            keep = max(1, k);
        }
        s_n = keep;
    }
    __syncthreads();
    const int keep = s_n;
    float best = -INFINITY, zk = 0.f;
    int bi = 0x7fffffff;
    for (int k = threadIdx.x; k < keep; k += SNT) {
        const float sc = cv[k] + gumbel(P.seed, (uint32_t)ci[k]);
        zk += __expf(cv[k] - mx);
        if (sc > best || (sc == best && ci[k] < bi)) { best = sc; bi = ci[k]; }
    }
    zk = bsum(zk, red);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float ob = __shfl_xor(best, o, 64);
        const int oi = __shfl_xor(bi, o, 64);
        if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
    }
    if ((threadIdx.x & 63) == 0) { rv[threadIdx.x >> 6] = best; ri[threadIdx.x >> 6] = bi; }
    __syncthreads();
    if (threadIdx.x == 0) {
        float b = rv[0];
        int id = ri[0];
        for (int w = 1; w < SNT / 64; ++w)
            if (rv[w] > b || (rv[w] == b && ri[w] < id)) { b = rv[w]; id = ri[w]; }
        if (id == 0x7fffffff) id = 0;
        out_tok[row] = id;
        if (out_logp) out_logp[row] = val(id, x[id]) - mx - __logf(fmaxf(zk, 1e-30f));
    }
}

extern "C" int mxk_sample(float* logits, int ld, int B, int V, const SampleParams* params, const int* pen_tok,
                          const int* pen_cnt, const float* pen_bias, const uint32_t* allow_mask, int mask_ld,
                          int* out_tok, float* out_logp, hipStream_t st) {
    if (B <= 0) return 0;
    sample_kernel<<<B, SNT, 0, st>>>(logits, ld, V, params, pen_tok, pen_cnt, pen_bias, allow_mask, mask_ld, out_tok,
                                     out_logp);
    MXK_CHECK_LAUNCH();
}

extern "C" int mxk_sample_params_size() { return (int)sizeof(SampleParams); }

// ---- small batches with top-k on: the vocabulary split over many workgroups ----------------------------
// One workgroup per row reads the 128k-entry row from one CU (~0.2 ms at batch 1). With top-k <= TK_CAP on,
// every quantity the chain needs lives in the global top-k set (top-p's target is top_p x the top-k mass,
// min-p is relative to the max), and the global top-k is contained in the union of per-slice top-ks:
//   tk_slice_kernel  (B x S workgroups): slice max, slice histogram, gather + sort the slice's top-k
//   tk_merge_kernel  (B workgroups):     merge the S x k candidates, truncate exactly, Gumbel-max draw.
constexpr int TK_CAP = 64, TK_NT = 256, TK_HB = 1024;
constexpr float TK_HR = 48.f;

__global__ __launch_bounds__(TK_NT) void tk_penalty_kernel(float* logits, int ld, int V, const SampleParams* params,
                                                          const int* pen_tok, const int* pen_cnt, const float* pen_bias) {
    const SampleParams P = params[blockIdx.x];
    float* x = logits + (size_t)blockIdx.x * ld;
    for (int i = threadIdx.x; i < P.pen_count; i += TK_NT) {
        const int t = pen_tok[P.pen_offset + i];
        if (t < 0 || t >= V) continue;
        const int c = pen_cnt[P.pen_offset + i];
        float v = x[t];
        if (c > 0) {
            if (P.repeat_penalty != 1.f) v = v > 0.f ? v / P.repeat_penalty : v * P.repeat_penalty;
            v -= P.frequency_penalty * (float)c + P.presence_penalty;
        }
        v += pen_bias[P.pen_offset + i];
        x[t] = v;
    }
}

__global__ __launch_bounds__(TK_NT) void tk_slice_kernel(const float* __restrict__ logits, int ld, int V,
                                                        const SampleParams* __restrict__ params,
                                                        const uint32_t* __restrict__ allow_mask, int mask_ld,
                                                        float* __restrict__ cand_v, int* __restrict__ cand_i,
                                                        int* __restrict__ cand_n, float2* __restrict__ slice_z) {
    __shared__ float red[TK_NT / 64], zred[TK_NT / 64];
    __shared__ unsigned hcnt[TK_HB];
    __shared__ float cv[2 * TK_CAP * 4];
    __shared__ int ci[2 * TK_CAP * 4];
    __shared__ int s_n, s_bin;
    const int row = blockIdx.x, S = gridDim.y, sl = blockIdx.y;
    const SampleParams P = params[row];
    const int K = P.temperature <= 0.f ? 1 : min(P.top_k, TK_CAP);
    const float itemp = P.temperature <= 0.f ? 1.f : 1.f / P.temperature;
    const float* x = logits + (size_t)row * ld;
    const uint32_t* am = allow_mask ? allow_mask + (size_t)row * mask_ld : nullptr;
    const int L = (V + S - 1) / S, i0 = sl * L, i1 = min(V, i0 + L);
    auto val = [&](int i) -> float {
        if (am && !((am[i >> 5] >> (i & 31)) & 1u)) return -INFINITY;
        return x[i] * itemp;
    };
    float mx = -INFINITY;
    for (int i = i0 + threadIdx.x; i < i1; i += TK_NT) mx = fmaxf(mx, val(i));
    mx = wave_max(mx);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
    for (int b = threadIdx.x; b < TK_HB; b += TK_NT) hcnt[b] = 0u;
    __syncthreads();
    mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    constexpr float IBW = (float)TK_HB / TK_HR, BW = TK_HR / (float)TK_HB;
    float zs = 0.f;  // the slice's share of the row's partition function (greedy rows report log-softmax)
    for (int i = i0 + threadIdx.x; i < i1; i += TK_NT) {
        const float v = val(i);
        if (!(v > -INFINITY)) continue;  // masked (and NaN)
        zs += __expf(v - mx);
        atomicAdd(&hcnt[(int)fminf((float)(TK_HB - 1), (mx - v) * IBW)], 1u);
    }
    zs = wave_sum(zs);
    if ((threadIdx.x & 63) == 0) zred[threadIdx.x >> 6] = zs;
    __syncthreads();
    if (threadIdx.x == 0) slice_z[row * S + sl] = make_float2(mx, zred[0] + zred[1] + zred[2] + zred[3]);
    if (threadIdx.x == 0) {
        unsigned c = 0;
        int b = 0;
        for (; b < TK_HB - 1; ++b) {
            c += hcnt[b];
            if (c >= (unsigned)K) break;
        }
        s_bin = b;
        s_n = 0;
    }
    __syncthreads();
    // fewer than K entries within TK_HR of the slice max (a sparse allow mask): take every entry
    const float cut = s_bin == TK_HB - 1 ? -INFINITY : mx - ((float)s_bin + 1.01f) * BW;
    constexpr int CAPL = 2 * TK_CAP * 4;
    for (int i = i0 + threadIdx.x; i < i1; i += TK_NT) {
        const float v = val(i);
        if (v == -INFINITY || !(v > cut || v == mx)) continue;  // (an all-masked slice gathers nothing)
        const int k = atomicAdd(&s_n, 1);
        if (k < CAPL) { cv[k] = v; ci[k] = i; }
    }
    __syncthreads();
    const int n = min(s_n, CAPL);  // a bin holding > CAPL - K entries: the first CAPL are kept (exactly
                                   // representable ties beyond are the only loss; the histogram bins are
                                   // 0.047 logits wide)
    int np = 1;
    while (np < n) np <<= 1;
    for (int k = n + threadIdx.x; k < np; k += TK_NT) { cv[k] = -INFINITY; ci[k] = 0x7fffffff; }
    __syncthreads();
    for (int size = 2; size <= np; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int t = threadIdx.x; t < np / 2; t += TK_NT) {
                const int lo = 2 * t - (t & (stride - 1)), hi = lo + stride;
                const bool desc = (lo & size) == 0;
                const float a = cv[lo], bb = cv[hi];
                const int ia = ci[lo], ib = ci[hi];
                const bool a_first = a > bb || (a == bb && ia < ib);
                if (a_first != desc) { cv[lo] = bb; cv[hi] = a; ci[lo] = ib; ci[hi] = ia; }
            }
            __syncthreads();
        }
    }
    // this slice's top-K plus every entry tied with its K-th value (top-k keeps ties)
    int keep = min(n, K);
    if (keep > 0) while (keep < n && keep < 2 * K && cv[keep] == cv[keep - 1]) ++keep;
    const size_t base = ((size_t)row * S + sl) * (2 * TK_CAP);
    for (int k = threadIdx.x; k < keep; k += TK_NT) { cand_v[base + k] = cv[k]; cand_i[base + k] = ci[k]; }
    if (threadIdx.x == 0) cand_n[row * S + sl] = keep;
}

__global__ __launch_bounds__(1024) void tk_merge_kernel(const float* __restrict__ logits, int ld,
                                                       const SampleParams* __restrict__ params, int S,
                                                       const float* __restrict__ cand_v, const int* __restrict__ cand_i,
                                                       const int* __restrict__ cand_n, const float2* __restrict__ slice_z,
                                                       int* __restrict__ out_tok, float* __restrict__ out_logp) {
    constexpr int CAP = 4096;
    __shared__ float cv[CAP];
    __shared__ int ci[CAP];
    __shared__ int s_off[65], s_keep;
    __shared__ float red[16], rv[16];
    __shared__ int ri[16];
    const int row = blockIdx.x;
    const SampleParams P = params[row];
    const bool greedy = P.temperature <= 0.f;
    const int K = greedy ? 1 : min(P.top_k, TK_CAP);
    if (threadIdx.x == 0) {
        int o = 0;
        for (int s = 0; s < S; ++s) { s_off[s] = o; o += cand_n[row * S + s]; }
        s_off[S] = min(o, CAP);
    }
    __syncthreads();
    const int n = s_off[S];
    for (int s = 0; s < S; ++s) {
        const int c = min(cand_n[row * S + s], CAP - s_off[s]);
        for (int k = threadIdx.x; k < c; k += 1024) {
            cv[s_off[s] + k] = cand_v[((size_t)row * S + s) * (2 * TK_CAP) + k];
            ci[s_off[s] + k] = cand_i[((size_t)row * S + s) * (2 * TK_CAP) + k];
        }
    }
    int np = 1;
    while (np < n) np <<= 1;
    for (int k = n + threadIdx.x; k < np; k += 1024) { cv[k] = -INFINITY; ci[k] = 0x7fffffff; }
    __syncthreads();
    for (int size = 2; size <= np; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int t = threadIdx.x; t < np / 2; t += 1024) {
                const int lo = 2 * t - (t & (stride - 1)), hi = lo + stride;
                const bool desc = (lo & size) == 0;
                const float a = cv[lo], bb = cv[hi];
                const int ia = ci[lo], ib = ci[hi];
                const bool a_first = a > bb || (a == bb && ia < ib);
                if (a_first != desc) { cv[lo] = bb; cv[hi] = a; ci[lo] = ib; ci[hi] = ia; }
            }
            __syncthreads();
        }
    }
    const float mx = cv[0];
    if (threadIdx.x == 0) {  // the bisection chain's semantics (see sample_kernel)
        int keep = n;
        if (K < keep) {
            const float kv = cv[K - 1];
            keep = K;
            while (keep < n && cv[keep] == kv) ++keep;
        }
        float zk = 0.f;
        const bool tp = P.top_p < 1.f && P.top_p > 0.f;
        if (tp)
            for (int k = 0; k < keep; ++k) zk += __expf(cv[k] - mx);
        if (P.min_p > 0.f && P.min_p <= 1.f) {
            const float mv = mx + __logf(P.min_p);
            while (keep > 1 && cv[keep - 1] < mv) --keep;
        }
        if (tp) {
            float cum = 0.f;
            int k = 0;
            while (k < keep) {
                cum += __expf(cv[k] - mx);
                ++k;
                if (cum >= P.top_p * zk) break;
            }
            while (k < keep && cv[k] == cv[k - 1]) ++k;
            keep = max(1, k);
        }
        s_keep = keep;
    }
    __syncthreads();
    const int keep = s_keep;
    float best = -INFINITY, zk = 0.f;
    int bi = 0x7fffffff;
    for (int k = threadIdx.x; k < keep; k += 1024) {
        const float sc = greedy ? cv[k] : cv[k] + gumbel(P.seed, (uint32_t)ci[k]);
        zk += __expf(cv[k] - mx);
        if (sc > best || (sc == best && ci[k] < bi)) { best = sc; bi = ci[k]; }
    }
    zk = wave_sum(zk);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = zk;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float ob = __shfl_xor(best, o, 64);
        const int oi = __shfl_xor(bi, o, 64);
        if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
    }
    if ((threadIdx.x & 63) == 0) { rv[threadIdx.x >> 6] = best; ri[threadIdx.x >> 6] = bi; }
    __syncthreads();
    if (threadIdx.x == 0) {
        float b = rv[0], z = red[0];
        int id = ri[0];
        for (int w = 1; w < 16; ++w) {
            z += red[w];
            if (rv[w] > b || (rv[w] == b && ri[w] < id)) { b = rv[w]; id = ri[w]; }
        }
        if (id == 0x7fffffff) id = 0;
        out_tok[row] = id;
        if (out_logp) {
            if (greedy) {  // log-softmax over the whole (allowed) row, from the slices' (max, sum exp)
                float M = -INFINITY, Z = 0.f;
                for (int s2 = 0; s2 < S; ++s2) M = fmaxf(M, slice_z[row * S + s2].x);
                for (int s2 = 0; s2 < S; ++s2) {
                    const float2 m = slice_z[row * S + s2];
                    if (m.x > -INFINITY) Z += m.y * __expf(m.x - M);
                }
                out_logp[row] = logits[(size_t)row * ld + id] - M - __logf(fmaxf(Z, 1e-30f));
            } else {
                out_logp[row] = logits[(size_t)row * ld + id] / P.temperature - mx - __logf(fmaxf(z, 1e-30f));
            }
        }
    }
}

// B rows, S slices per row (<= 64, S * 2 * max top_k <= 4096 so the merge holds every candidate); every row
// must have top_k in [1, TK_CAP] or be greedy, no typical-p / mirostat (the caller checks).
// cand_v / cand_i: [B][S][2*TK_CAP] scratch, cand_n / slice_z: [B][S].
extern "C" int mxk_sample_topk_split(float* logits, int ld, int B, int V, const SampleParams* params, int has_pen,
                                     const int* pen_tok, const int* pen_cnt, const float* pen_bias,
                                     const uint32_t* allow_mask, int mask_ld, int S, float* cand_v, int* cand_i,
                                     int* cand_n, float2* slice_z, int* out_tok, float* out_logp, hipStream_t st) {
    if (B <= 0) return 0;
    if (S < 1 || S > 64) return (int)hipErrorInvalidValue;
    if (has_pen) tk_penalty_kernel<<<B, TK_NT, 0, st>>>(logits, ld, V, params, pen_tok, pen_cnt, pen_bias);
    tk_slice_kernel<<<dim3(B, S), TK_NT, 0, st>>>(logits, ld, V, params, allow_mask, mask_ld, cand_v, cand_i, cand_n,
                                                  slice_z);
    tk_merge_kernel<<<B, 1024, 0, st>>>(logits, ld, params, S, cand_v, cand_i, cand_n, slice_z, out_tok, out_logp);
    MXK_CHECK_LAUNCH();
}
extern "C" int mxk_sample_topk_cap() { return TK_CAP; }

// greedy argmax over rows (fast path used by the decode graph when every row is greedy)
__global__ __launch_bounds__(1024) void argmax_kernel(const float* __restrict__ x, int ld, int V,
                                                      int* __restrict__ out, unsigned long long* __restrict__ keys,
                                                      int off) {
    __shared__ float rv[16];
    __shared__ int ri[16];
    const float* r = x + (size_t)blockIdx.x * ld;
    float best = -INFINITY;
    int bi = 0x7fffffff;
    auto take = [&](float v, int i) {
        if (v > best) { best = v; bi = i; }  // ascending i per lane: the first maximum wins ties
    };
    int tail = 0;
    if ((((uintptr_t)r) & 15) == 0) {
        // 16-B loads, two in flight per lane (one block streams the row: at batch 1 a scalar loop was
        // load-latency bound, ~39 us for a 128k vocabulary)
        const int V4 = V & ~3;
        int i = threadIdx.x * 4;
        for (; i + 4096 < V4; i += 8192) {
            const float4 a = *(const float4*)(r + i), c = *(const float4*)(r + i + 4096);
            take(a.x, i); take(a.y, i + 1); take(a.z, i + 2); take(a.w, i + 3);
            take(c.x, i + 4096); take(c.y, i + 4097); take(c.z, i + 4098); take(c.w, i + 4099);
        }
        if (i < V4) {
            const float4 a = *(const float4*)(r + i);
            take(a.x, i); take(a.y, i + 1); take(a.z, i + 2); take(a.w, i + 3);
        }
        tail = V4;
    }
    for (int i = tail + threadIdx.x; i < V; i += 1024) take(r[i], i);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float ob = __shfl_xor(best, o, 64);
        const int oi = __shfl_xor(bi, o, 64);
        if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
    }
    if ((threadIdx.x & 63) == 0) { rv[threadIdx.x >> 6] = best; ri[threadIdx.x >> 6] = bi; }
    __syncthreads();
    if (threadIdx.x == 0) {
        float b = rv[0];
        int id = ri[0];
        for (int w = 1; w < 16; ++w)
            if (rv[w] > b || (rv[w] == b && ri[w] < id)) { b = rv[w]; id = ri[w]; }
        if (keys) {
            // vocabulary shard: (value, global index) as one orderable 64-bit key, larger = better
            // (higher value, then lower index)
            const uint32_t u = __float_as_uint(b);
            const uint32_t hi = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
            const uint32_t gi = id == 0x7fffffff ? 0xFFFFFFFFu : (uint32_t)(id + off);
            keys[blockIdx.x] = ((unsigned long long)(id == 0x7fffffff ? 0u : hi) << 32) | (0xFFFFFFFFu - gi);
        } else {
            out[blockIdx.x] = id == 0x7fffffff ? 0 : id;
        }
    }
}

extern "C" int mxk_argmax(const float* x, int ld, int B, int V, int* out, hipStream_t st) {
    if (B <= 0) return 0;
    argmax_kernel<<<B, 1024, 0, st>>>(x, ld, V, out, nullptr, 0);
    MXK_CHECK_LAUNCH();
}

// tensor-parallel greedy head: each rank reduces its [B, V_shard] logits to one key per row
// (mxk_argmax_keys), the keys are all-gathered ([tp, B] x 8 bytes instead of the B x V fp32 logits),
// and mxk_argmax_merge picks the winner per row: the same token as an argmax over the gathered logits.
extern "C" int mxk_argmax_keys(const float* x, int ld, int B, int V, int off, unsigned long long* keys,
                               hipStream_t st) {
    if (B <= 0) return 0;
    argmax_kernel<<<B, 1024, 0, st>>>(x, ld, V, nullptr, keys, off);
    MXK_CHECK_LAUNCH();
}

__global__ void argmax_merge_kernel(const unsigned long long* __restrict__ keys, int tp, int B, int* __restrict__ out) {
    const int row = blockIdx.x * blockDim.x + threadIdx.x;
    if (row >= B) return;
    unsigned long long k = 0;
    for (int r = 0; r < tp; ++r) k = max(k, keys[(size_t)r * B + row]);
    const uint32_t gi = 0xFFFFFFFFu - (uint32_t)(k & 0xFFFFFFFFull);
    out[row] = gi == 0xFFFFFFFFu ? 0 : (int)gi;
}

extern "C" int mxk_argmax_merge(const unsigned long long* keys, int tp, int B, int* out, hipStream_t st) {
    if (B <= 0) return 0;
    argmax_merge_kernel<<<(B + 255) / 256, 256, 0, st>>>(keys, tp, B, out);
    MXK_CHECK_LAUNCH();
}
