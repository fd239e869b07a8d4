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
    int pend;        // overlap pipeline: index of this row's still-in-flight previous token in pend_tok (-1: none);
                     // the host's sparse counts lag that token by one, it is counted here
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

// sparse penalties + logit bias, in place (unique tokens per row -> no write conflicts). `pend_tok`: the
// tokens of the previous, still-in-flight step (overlap pipeline); the row's one pending token counts once
// more (an entry already in the list, or a penalty-only entry of count 1).
template <int NT>
MX_DEV void penalize(float* x, int V, const SampleParams& P, const int* pen_tok, const int* pen_cnt,
                     const float* pen_bias, const int* pend_tok, int* s_found) {
    const int tp = (P.pend >= 0 && pend_tok) ? pend_tok[P.pend] : -1;
    const bool pens = P.repeat_penalty != 1.f || P.presence_penalty != 0.f || P.frequency_penalty != 0.f;
    if (threadIdx.x == 0) *s_found = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < P.pen_count; i += NT) {
        const int t = pen_tok[P.pen_offset + i];
        if (t < 0 || t >= V) continue;
        int c = pen_cnt[P.pen_offset + i];
        if (t == tp) {
            *s_found = 1;
            if (pens) ++c;
        }
        float v = x[t];
        if (c > 0) {
            if (P.repeat_penalty != 1.f) v = v > 0.f ? v / P.repeat_penalty : v * P.repeat_penalty;
            v -= P.frequency_penalty * (float)c + P.presence_penalty;
        }
        v += pen_bias[P.pen_offset + i];
        x[t] = v;
    }
    __syncthreads();
    if (threadIdx.x == 0 && pens && tp >= 0 && tp < V && !*s_found) {
        float v = x[tp];
        if (P.repeat_penalty != 1.f) v = v > 0.f ? v / P.repeat_penalty : v * P.repeat_penalty;
        x[tp] = v - P.frequency_penalty - P.presence_penalty;
    }
    __syncthreads();
}

MX_DEV void apply_penalties(float* x, int V, const SampleParams& P, const int* pen_tok, const int* pen_cnt,
                            const float* pen_bias, const int* pend_tok) {
    __shared__ int s_found;
    penalize<SNT>(x, V, P, pen_tok, pen_cnt, pen_bias, pend_tok, &s_found);
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
                                                     int* __restrict__ out_tok, float* __restrict__ out_logp,
                                                     const int* __restrict__ pend_tok) {
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
    apply_penalties(x, V, P, pen_tok, pen_cnt, pen_bias, pend_tok);
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
                          int* out_tok, float* out_logp, const int* pend_tok, hipStream_t st) {
    if (B <= 0) return 0;
    sample_kernel<<<B, SNT, 0, st>>>(logits, ld, V, params, pen_tok, pen_cnt, pen_bias, allow_mask, mask_ld, out_tok,
                                     out_logp, pend_tok);
    MXK_CHECK_LAUNCH();
}

extern "C" int mxk_sample_params_size() { return (int)sizeof(SampleParams); }

// ---- top-k on (the reference default, top_k 40): the vocabulary split over B x S workgroups -------------
// One workgroup per row (sample_kernel) reads the 128k-entry row from one CU and builds an LDS histogram
// whose hot bins serialise on atomics (227 us at 128 rows). With top-k <= TK_CAP on, every quantity the
// chain needs lives in the global top-k set (top-p's target is top_p x the top-k mass, min-p is relative to
// the max), and the global top-k set is contained in the union of the per-slice top-k sets:
//   tk_slice_kernel (B x S workgroups of 256): the slice (NV values per thread) held in registers, one LDS
//     histogram of the distance below the slice max picks the whole bins that hold the slice's top-K
//     (candidates written unsorted; key bisection only for a bin denser than the capacity);
//   tk_merge_kernel (B workgroups of 1024): the S x <= TK_CAPS candidates in registers, the same histogram
//     against the row max for the global top-K's bins, a one-pass rank sort of the <= 256 kept values in
//     LDS, exact top-K / min-p / top-p truncation, Gumbel-max draw.
//     A row whose slices overflowed falls back to the full-row bisection chain (sample_row_bisect).
constexpr int TK_CAP = 64, TK_NT = 256, TK_NV = 32, TK_CAPS = 2 * TK_CAP, TK_MNT = 1024, TK_MV = 8;
constexpr int TK_SLICE = TK_NT * TK_NV;  // vocabulary entries per slice at the default TK_NV (see tk_nv)
// values per thread of the slice kernel, chosen at run time (MX_TK_NV = 16 | 32): 32 (8192-entry slices) takes 144
// VGPRs (3 waves per SIMD), 16 (4096-entry slices, twice the workgroups and merge candidates) 80 VGPRs
static int tk_nv() {
    static int nv = [] {
        const char* e = getenv("MX_TK_NV");
        return e && atoi(e) == 16 ? 16 : 32;
    }();
    return nv;
}
constexpr float TK_HR = 48.f;            // values more than this below the slice max are never candidates

MX_DEV uint32_t ord_key(float v) {  // order-preserving float -> uint (NaN / -inf / masked -> 0)
    if (!(v > -INFINITY)) return 0u;
    const uint32_t b = __float_as_uint(v);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

__global__ __launch_bounds__(TK_NT) void tk_penalty_kernel(float* logits, int ld, int V, const SampleParams* params,
                                                          const int* pen_tok, const int* pen_cnt, const float* pen_bias,
                                                          const int* pend_tok) {
    __shared__ int s_found;
    const SampleParams P = params[blockIdx.x];
    penalize<TK_NT>(logits + (size_t)blockIdx.x * ld, V, P, pen_tok, pen_cnt, pen_bias, pend_tok, &s_found);
}

MX_DEV uint32_t tk_key(uint32_t u) { return u; }
MX_DEV uint32_t tk_key(float v) { return ord_key(v); }

// block-wide count of keys >= t over NV registers per thread (keys, or floats keyed on the fly);
// `red` double-buffered by the caller's parity
template <int NT, int NV, typename T>
MX_DEV int tk_count(const T (&u)[NV], uint32_t t, int* red, int par) {
    int c = 0;
#pragma unroll
    for (int j = 0; j < NV; ++j) c += tk_key(u[j]) >= t ? 1 : 0;
    c = wave_sum_i(c);
    if ((threadIdx.x & 63) == 0) red[par * (NT / 64) + (threadIdx.x >> 6)] = c;
    __syncthreads();
    int s = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) s += red[par * (NT / 64) + w];
    return s;
}

// largest key T with count(keys >= T) >= K, searched in [lo, hi) (count(>= lo) known = c_lo >= K,
// count(>= hi) < K). exact = false: stop as soon as count(>= T) <= cap (a superset of the top-K set that
// fits); exact = true: stop only at the K-th key itself (or when count(>= T) == K, which is the same set).
template <int NT, int NV, typename T>
MX_DEV uint32_t tk_bisect(const T (&u)[NV], int K, uint32_t lo, uint32_t hi, int& c_lo, int cap, bool exact,
                          int* red, int par) {
    while (hi - lo > 1u) {
        if (exact ? c_lo == K : c_lo <= cap) break;
        const uint32_t mid = lo + ((hi - lo) >> 1);
        const int c = tk_count<NT, NV, T>(u, mid, red, par);
        par ^= 1;
        if (c >= K) { lo = mid; c_lo = c; }
        else hi = mid;
    }
    return lo;
}

// Candidate selection by one LDS histogram of the distance below the max (TK_NB bins of 1/TK_BPU logit unit;
// beyond that no bin): one wave scans the bins from the top for the first cumulative count >= K, and
// everything in bins <= that one is the candidate set — 4 block barriers instead of a ~20-step bisection
// (round 3: 45 + 33 us at 128 rows). A bin too dense for the capacity (flat rows, exact ties) or a row with
// fewer than K values inside the histogram range falls back to the bisection on the key axis.
constexpr int TK_NB = 256;

constexpr float TK_BPU = 8.f;  // bins per logit unit: 256 bins cover 32 units below the max

MX_DEV int tk_bin(float mx, float v) {  // monotone in v (0 = the top), TK_NB = outside the range / masked
    const float d = (mx - v) * TK_BPU;
    return d < (float)TK_NB ? (int)d : TK_NB;  // -inf / NaN: the compare fails
}
// bin(v) <= b  <=>  (mx - v) * TK_BPU < b + 1 (truncation of a non-negative value): one sub, mul and compare
MX_DEV bool tk_in(float mx, float v, int b) { return (mx - v) * TK_BPU < (float)(b + 1); }

// first bin b (scanning from the top) whose cumulative count reaches K: {b, cum(b)}; {TK_NB, total} if none.
// Called by one full wave; hist[TK_NB] in LDS.
MX_DEV int2 tk_scan_bins(const int* hist, int K) {
    const int lane = threadIdx.x & 63;
    int4 h = *(const int4*)(hist + 4 * lane);  // bins 4 lane .. 4 lane + 3
    const int own = h.x + h.y + h.z + h.w;
    int inc = own;  // inclusive prefix over lanes
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(inc, o, 64);
        if (lane >= o) inc += t;
    }
    const int exc = inc - own;
    const unsigned long long hit = __ballot(inc >= K);
    if (!hit) return make_int2(TK_NB, __shfl(inc, 63, 64));
    const int L = __builtin_ctzll(hit);
    int b = 4 * L, c = __shfl(exc, L, 64);
    const int4 hl = make_int4(__shfl(h.x, L, 64), __shfl(h.y, L, 64), __shfl(h.z, L, 64), __shfl(h.w, L, 64));
    c += hl.x;
    if (c < K) { ++b; c += hl.y; }
    if (c < K) { ++b; c += hl.z; }
    if (c < K) { ++b; c += hl.w; }
    return make_int2(b, c);
}

// block barrier for LDS hand-offs only: __syncthreads() also waits for every outstanding global store of the
// wave (vmcnt(0) before the barrier), which after the candidate writes cost several microseconds per slice
MX_DEV void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ int g_tk_trace;                    // phase timestamps of workgroup (0, 0) (tools/time_sampler.py --trace)
__device__ unsigned long long g_tk_ts[16];
#define TK_TS(k)                                                                                         \
    if (g_tk_trace && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {                          \
        volatile unsigned long long* ts_ = g_tk_ts;                                                      \
        ts_[k] = wall_clock64();                                                                         \
    }

// VEC = 4: each thread's values come in float4 loads (1 KB per wave instruction instead of 256 B); value
// j of the thread is vocabulary entry i0 + VEC (floor(j / VEC) TK_NT + thread) + j % VEC
template <int VEC, bool MASK, int NV>
__global__ __launch_bounds__(TK_NT) void tk_slice_kernel(const float* __restrict__ logits, int ld, int V,
                                                        const SampleParams* __restrict__ params,
                                                        const uint32_t* __restrict__ allow_mask, int mask_ld,
                                                        float* __restrict__ cand_v, int* __restrict__ cand_i,
                                                        int* __restrict__ cand_n, float2* __restrict__ slice_z) {
    __shared__ float fred[2 * TK_NT / 64];
    __shared__ int red[2 * TK_NT / 64];
    __shared__ __attribute__((aligned(16))) int hist[TK_NB], hist2[TK_NB];
    __shared__ int s_n, s_b, s_fb;
    const int row = blockIdx.x, S = gridDim.y, sl = blockIdx.y;
    const SampleParams P = params[row];
    const int K = P.temperature <= 0.f ? 1 : min(P.top_k, TK_CAP);
    const float itemp = P.temperature <= 0.f ? 1.f : 1.f / P.temperature;
    const float* x = logits + (size_t)row * ld;
    const uint32_t* am = MASK ? allow_mask + (size_t)row * mask_ld : nullptr;
    TK_TS(0)
    const int i0 = sl * (NV * TK_NT), i1 = min(V, i0 + NV * TK_NT);
    float v[NV];
    float mx = -INFINITY;
    auto gidx = [&](int j) { return i0 + VEC * ((j / VEC) * TK_NT + (int)threadIdx.x) + j % VEC; };
    // branch-free loads (clamped index, masked after): a conditional load per value made the compiler wait
    // for each one before the next (vmcnt(0) per load, ~1 us of HBM latency each)
    if constexpr (VEC == 4) {  // slice lengths are multiples of 4 here (V % 4 == 0)
#pragma unroll
        for (int j = 0; j < NV / 4; ++j) {
            const f32x4 q = __builtin_nontemporal_load(
                (const f32x4*)(x + min(i0 + 4 * (j * TK_NT + (int)threadIdx.x), i1 - 4)));
            v[4 * j] = q[0];
            v[4 * j + 1] = q[1];
            v[4 * j + 2] = q[2];
            v[4 * j + 3] = q[3];
        }
    } else {
#pragma unroll
        for (int j = 0; j < NV; ++j) v[j] = __builtin_nontemporal_load(x + min(gidx(j), i1 - 1));
    }
    if constexpr (MASK) {  // grammar rows (a separate instantiation: the mask words cost registers)
        uint32_t w[NV];
#pragma unroll
        for (int j = 0; j < NV; ++j) w[j] = am[min(gidx(j), i1 - 1) >> 5];
#pragma unroll
        for (int j = 0; j < NV; ++j)
            if (!((w[j] >> (gidx(j) & 31)) & 1u)) v[j] = -INFINITY;
    }
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        v[j] = gidx(j) < i1 ? v[j] * itemp : -INFINITY;
        mx = fmaxf(mx, v[j]);
    }
    TK_TS(1)
    const float tmax = mx;  // this thread's largest value
    mx = wave_max(mx);
    if ((threadIdx.x & 63) == 0) fred[threadIdx.x >> 6] = mx;
    hist[threadIdx.x] = 0;  // TK_NB == TK_NT
    hist2[threadIdx.x] = 0;
    if (threadIdx.x == 0) s_n = 0;
    __syncthreads();
#pragma unroll
    for (int w = 0; w < TK_NT / 64; ++w) mx = fmaxf(mx, fred[w]);
    // pass 1: the threads' maxima only (one atomic per thread). Its K-th largest is a lower bound of the
    // slice's K-th largest value (K threads each hold a value >= it), so only values in bins <= that
    // bin go into pass 2 — a few hundred LDS atomics instead of one per value on flat rows
    {
        const int tb = tk_bin(mx, tmax);
        if (tb < TK_NB) atomicAdd(&hist[tb], 1);
    }
    float zs = 0.f;  // the slice's share of the row's partition function (log-probs of greedy rows only)
    if (P.temperature <= 0.f) {
#pragma unroll
        for (int j = 0; j < NV; ++j)
            if (v[j] > -INFINITY) zs += __expf(v[j] - mx);
    }
    zs = wave_sum(zs);
    if ((threadIdx.x & 63) == 0) fred[TK_NT / 64 + (threadIdx.x >> 6)] = zs;
    __syncthreads();
    if (threadIdx.x < 64) {
        const int2 bc = tk_scan_bins(hist, K);
        if (threadIdx.x == 0) s_b = bc.x;  // TK_NB: fewer than K threads hold a value in range
    }
    __syncthreads();
    const int bA = s_b;
    TK_TS(2)
    const size_t base = ((size_t)row * S + sl) * TK_CAPS;
    // direct compaction at the pass-1 bound: every value in bins <= bA (>= K of them). Each lane counts its
    // own and reserves its range with ONE LDS atomic (a returning atomic per value made every lane wait ~100
    // cycles per value); the usual case ends here. Too many (clustered maxima) -> pass 2 below.
    if (threadIdx.x == 0) {
        float z = 0.f;
#pragma unroll
        for (int w = 0; w < TK_NT / 64; ++w) z += fred[TK_NT / 64 + w];
        slice_z[row * S + sl] = make_float2(mx, z);
    }
    if (bA < TK_NB) {
        int myc = 0;
#pragma unroll
        for (int j = 0; j < NV; ++j) myc += tk_in(mx, v[j], bA) ? 1 : 0;
        int off = myc ? atomicAdd(&s_n, myc) : 0;
        if (myc && off + myc <= TK_CAPS) {
#pragma unroll
            for (int j = 0; j < NV; ++j) {
                if (tk_in(mx, v[j], bA)) {
                    cand_v[base + off] = v[j];
                    cand_i[base + off] = gidx(j);
                    ++off;
                }
            }
        }
        lds_barrier();  // the reservations are done; the candidate stores need no ordering within the block
        const int tot = s_n;
        TK_TS(3)
        if (tot <= TK_CAPS) {
            if (threadIdx.x == 0) cand_n[row * S + sl] = tot;
            TK_TS(4)
            return;
        }
        lds_barrier();  // every lane has read s_n
        if (threadIdx.x == 0) s_n = 0;
        // pass 2: histogram of the values in bins <= bA, the first bin reaching K
#pragma unroll
        for (int j = 0; j < NV; ++j) {  // bins recomputed (not held: 32 more VGPRs would cost occupancy)
            const int bj = tk_bin(mx, v[j]);
            if (bj <= bA) atomicAdd(&hist2[bj], 1);
        }
        __syncthreads();
        if (threadIdx.x < 64) {
            const int2 bc = tk_scan_bins(hist2, K);
            if (threadIdx.x == 0) {
                s_b = bc.x;
                s_fb = bc.x == TK_NB || bc.y > TK_CAPS;
            }
        }
        __syncthreads();
        if (!s_fb) {
            const int b = s_b;
            myc = 0;
#pragma unroll
            for (int j = 0; j < NV; ++j) myc += tk_in(mx, v[j], b) ? 1 : 0;
            off = myc ? atomicAdd(&s_n, myc) : 0;  // <= TK_CAPS in total by the scan
#pragma unroll
            for (int j = 0; j < NV; ++j) {
                if (tk_in(mx, v[j], b)) {
                    cand_v[base + off] = v[j];
                    cand_i[base + off] = gidx(j);
                    ++off;
                }
            }
            __syncthreads();
            if (threadIdx.x == 0) cand_n[row * S + sl] = s_n;
            return;
        }
        __syncthreads();
        if (threadIdx.x == 0) s_n = 0;
        __syncthreads();
    }
    // fallback: bisection on the order-preserving key (computed from the values on the fly)
    uint32_t lo = mx > -INFINITY ? ord_key(mx - TK_HR) : 0u;
    const uint32_t hi = mx > -INFINITY ? ord_key(mx) + 1u : 1u;
    int c_lo = tk_count<TK_NT, NV, float>(v, lo, red, 0);
    if (c_lo >= K) lo = tk_bisect<TK_NT, NV, float>(v, K, lo, hi, c_lo, TK_CAPS, false, red, 1);
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        const uint32_t uj = ord_key(v[j]);
        if (uj >= lo && uj != 0u) {
            const int k = atomicAdd(&s_n, 1);
            if (k < TK_CAPS) {
                cand_v[base + k] = v[j];
                cand_i[base + k] = gidx(j);
            }
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) cand_n[row * S + sl] = s_n > TK_CAPS ? (TK_CAPS | (1 << 30)) : s_n;  // bit 30: ties overflowed
}

__global__ __launch_bounds__(TK_MNT) void tk_merge_kernel(float* __restrict__ logits, int ld, int V,
                                                         const SampleParams* __restrict__ params, int S,
                                                         const uint32_t* __restrict__ allow_mask, int mask_ld,
                                                         const float* __restrict__ cand_v, const int* __restrict__ cand_i,
                                                         const int* __restrict__ cand_n, const float2* __restrict__ slice_z,
                                                         int* __restrict__ out_tok, float* __restrict__ out_logp) {
    constexpr int KC = 256;  // kept-set capacity (top-k <= 64 plus the rest of the K-th value's bin)
    __shared__ __attribute__((aligned(16))) float cv[KC];
    __shared__ __attribute__((aligned(16))) int ci[KC];
    __shared__ float sv[KC];
    __shared__ int si[KC];
    __shared__ __attribute__((aligned(16))) int hist[TK_NB];
    __shared__ int s_cnt[64], s_keep, s_n, s_ovf, s_b, s_fb;
    __shared__ float s_mx, s_Z;
    __shared__ float red[2 * TK_MNT / 64], rv[TK_MNT / 64], rbv[TK_MNT / 64];
    __shared__ int ired[2 * TK_MNT / 64], ri[TK_MNT / 64];
    const int row = blockIdx.x;
    const SampleParams P = params[row];
    const bool greedy = P.temperature <= 0.f;
    const int K = greedy ? 1 : min(P.top_k, TK_CAP);
    // candidate position t = (slice t / TK_CAPS, entry t % TK_CAPS), valid below that slice's count. The loads
    // are unconditional (clamped; validity applied once the counts are known) and issued before the count /
    // max prologue, so the two round trips overlap; positions past S x TK_CAPS are skipped (uniform branch)
    float v[TK_MV];
    int id[TK_MV], bin[TK_MV];
#pragma unroll
    for (int j = 0; j < TK_MV; ++j) {
        if (j * TK_MNT < S * TK_CAPS) {
            const int t = j * TK_MNT + threadIdx.x, s = min(t / TK_CAPS, S - 1), e = t % TK_CAPS;
            const size_t src = ((size_t)row * S + s) * TK_CAPS + e;
            v[j] = cand_v[src];
            id[j] = cand_i[src];
        } else {
            v[j] = -INFINITY;
            id[j] = 0x7fffffff;
        }
    }
    if (threadIdx.x < TK_NB) hist[threadIdx.x] = 0;
    if (threadIdx.x < 64) {  // one wave: per-slice counts, overflow flags and the row max (largest slice max)
        const int s = threadIdx.x;
        const int c = s < S ? cand_n[row * S + s] : 0;
        const float sm = s < S ? slice_z[row * S + s].x : -INFINITY;
        s_cnt[s] = c & 0xFFFF;
        const unsigned long long ov = __ballot((c >> 30) != 0);
        const float m = wave_max(sm);
        if (s == 0) { s_ovf = ov != 0; s_n = 0; s_mx = m; }
    }
    __syncthreads();
    if (s_ovf) {  // exact ties beyond a slice's capacity (flat / degenerate rows): the full-row chain
        float* x = logits + (size_t)row * ld;
        const uint32_t* am = allow_mask ? allow_mask + (size_t)row * mask_ld : nullptr;
        sample_row_bisect(x, V, P, am, row, out_tok, out_logp, red, rv, ri);
        return;
    }
    const float mx = s_mx;
#pragma unroll
    for (int j = 0; j < TK_MV; ++j) {
        const int t = j * TK_MNT + threadIdx.x, s = t / TK_CAPS, e = t % TK_CAPS;
        if (!(s < S && e < s_cnt[min(s, 63)])) { v[j] = -INFINITY; id[j] = 0x7fffffff; }
        bin[j] = tk_bin(mx, v[j]);
        if (bin[j] < TK_NB) atomicAdd(&hist[bin[j]], 1);
    }
    __syncthreads();
    if (threadIdx.x < 64) {
        const int2 bc = tk_scan_bins(hist, K);
        if (threadIdx.x == 0) {
            s_b = bc.x;
            s_fb = bc.x == TK_NB || bc.y > KC;
        }
    }
    __syncthreads();
    int nk;
    if (!s_fb) {  // every candidate in bins <= b: a superset of the top-K (whole bins), at most KC
        const int b = s_b;
        int myc = 0;
#pragma unroll
        for (int j = 0; j < TK_MV; ++j) myc += bin[j] <= b ? 1 : 0;
        int k = myc ? atomicAdd(&s_n, myc) : 0;  // one returning LDS atomic per lane (see tk_slice_kernel)
#pragma unroll
        for (int j = 0; j < TK_MV; ++j) {
            if (bin[j] <= b) {
                cv[k] = v[j];
                ci[k] = id[j];
                ++k;
            }
        }
        __syncthreads();
        nk = s_n;
    } else {  // exact global top-K by key bisection (ties at the K-th value kept)
        uint32_t u[TK_MV];
#pragma unroll
        for (int j = 0; j < TK_MV; ++j) u[j] = ord_key(v[j]);
        int c_lo = tk_count<TK_MNT, TK_MV, uint32_t>(u, 1u, ired, 0);
        uint32_t T = 1u;
        if (c_lo > K) T = tk_bisect<TK_MNT, TK_MV, uint32_t>(u, K, 1u, ord_key(mx) + 1u, c_lo, 0, true, ired, 1);
#pragma unroll
        for (int j = 0; j < TK_MV; ++j) {
            if (u[j] >= T && u[j] != 0u) {
                const int k = atomicAdd(&s_n, 1);
                if (k < KC) { cv[k] = v[j]; ci[k] = id[j]; }
            }
        }
        __syncthreads();
        if (s_n > KC) {  // more exact ties at the K-th value than the kept-set buffer holds
            float* x = logits + (size_t)row * ld;
            const uint32_t* am = allow_mask ? allow_mask + (size_t)row * mask_ld : nullptr;
            sample_row_bisect(x, V, P, am, row, out_tok, out_logp, red, rv, ri);
            return;
        }
        nk = s_n;
    }
    // rank sort of the <= KC kept values (descending value, ascending id): one comparison pass per element
    if (threadIdx.x < KC) {  // pad to a multiple of 4 for the vector reads (pads rank below every real value)
        if (threadIdx.x >= nk) { cv[threadIdx.x] = -INFINITY; ci[threadIdx.x] = 0x7fffffff; }
    }
    __syncthreads();
    if (threadIdx.x < nk) {
        const float a = cv[threadIdx.x];
        const int ia = ci[threadIdx.x];
        int r = 0;
        const int n4 = (nk + 3) & ~3;
        for (int k = 0; k < n4; k += 4) {  // broadcast LDS reads, 4 candidates per step
            const float4 bv = *(const float4*)(cv + k);
            const int4 bi4 = *(const int4*)(ci + k);
            r += (bv.x > a || (bv.x == a && bi4.x < ia)) ? 1 : 0;
            r += (bv.y > a || (bv.y == a && bi4.y < ia)) ? 1 : 0;
            r += (bv.z > a || (bv.z == a && bi4.z < ia)) ? 1 : 0;
            r += (bv.w > a || (bv.w == a && bi4.w < ia)) ? 1 : 0;
        }
        sv[r] = a;
        si[r] = ia;
    }
    __syncthreads();
    if (threadIdx.x < 64) {  // one wave, 4 sorted entries per lane: top-K (ties at the K-th value kept), then
        const int lane = threadIdx.x;  // the bisection chain's semantics (min-p, then top-p over the top-K mass)
        float sv4[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) sv4[i] = sv[4 * lane + i];  // entries >= nk are never used below
        // first index in [k, lim) whose value differs from sv[k - 1] (sorted: the end of its tie run), else lim
        auto tie_end = [&](int k, int lim) {
            if (k <= 0 || k >= lim) return k;
            const float tv = sv[k - 1];
            int f = 0x7fffffff;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int idx = 4 * lane + i;
                if (idx >= k && idx < lim && sv4[i] != tv) f = min(f, idx);
            }
            for (int o = 32; o > 0; o >>= 1) f = min(f, __shfl_xor(f, o, 64));
            return f == 0x7fffffff ? lim : f;
        };
        int keep = tie_end(min(K, nk), nk);
        const bool tp = P.top_p < 1.f && P.top_p > 0.f;
        float zk = 0.f;
        if (tp) {
#pragma unroll
            for (int i = 0; i < 4; ++i) zk += 4 * lane + i < keep ? __expf(sv4[i] - mx) : 0.f;
            zk = wave_sum(zk);
        }
        if (P.min_p > 0.f && P.min_p <= 1.f) {  // the values below mx + log(min_p) are a suffix of the kept run
            const float mv = mx + __logf(P.min_p);
            int c = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i) c += (4 * lane + i < keep && sv4[i] >= mv) ? 1 : 0;
            keep = max(1, wave_sum_i(c));
        }
        if (tp) {  // smallest prefix whose mass reaches top_p x zk: inclusive scan over the lanes' 4-entry sums
            float e[4], own = 0.f;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                e[i] = 4 * lane + i < keep ? __expf(sv4[i] - mx) : 0.f;
                own += e[i];
            }
            float inc = own;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const float t = __shfl_up(inc, o, 64);
                if (lane >= o) inc += t;
            }
            const float target = P.top_p * zk;
            float cum = inc - own;
            int f = 0x7fffffff;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                cum += e[i];
                if (f == 0x7fffffff && 4 * lane + i < keep && cum >= target) f = 4 * lane + i;
            }
            for (int o = 32; o > 0; o >>= 1) f = min(f, __shfl_xor(f, o, 64));
            const int k = f == 0x7fffffff ? keep : f + 1;
            keep = max(1, tie_end(k, keep));
        }
        if (lane == 0) s_keep = keep;
    }
    __syncthreads();
    const int keep = s_keep;
    float best = -INFINITY, bv = -INFINITY, zk = 0.f;  // bv: the winner's (scaled) logit, for its log-prob
    int bi = 0x7fffffff;
    for (int k = threadIdx.x; k < keep; k += TK_MNT) {
        const float sc = greedy ? sv[k] : sv[k] + gumbel(P.seed, (uint32_t)si[k]);
        zk += __expf(sv[k] - mx);
        if (sc > best || (sc == best && si[k] < bi)) { best = sc; bi = si[k]; bv = sv[k]; }
    }
    zk = wave_sum(zk);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = zk;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float ob = __shfl_xor(best, o, 64), obv = __shfl_xor(bv, o, 64);
        const int oi = __shfl_xor(bi, o, 64);
        if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; bv = obv; }
    }
    if ((threadIdx.x & 63) == 0) { rv[threadIdx.x >> 6] = best; ri[threadIdx.x >> 6] = bi; rbv[threadIdx.x >> 6] = bv; }
    __syncthreads();
    if (out_logp && greedy && threadIdx.x < 64) {  // greedy log-softmax over the whole (allowed) row, from the
        const int s2 = threadIdx.x;                // slices' (max, sum exp); mx is the row max
        const float2 m = s2 < S ? slice_z[row * S + s2] : make_float2(-INFINITY, 0.f);
        const float Z = wave_sum(m.x > -INFINITY ? m.y * __expf(m.x - mx) : 0.f);
        if (s2 == 0) s_Z = Z;  // read below by this same lane
    }
    if (threadIdx.x == 0) {
        float b = rv[0], z = red[0], tv = rbv[0];
        int tok = ri[0];
        for (int w = 1; w < TK_MNT / 64; ++w) {
            z += red[w];
            if (rv[w] > b || (rv[w] == b && ri[w] < tok)) { b = rv[w]; tok = ri[w]; tv = rbv[w]; }
        }
        if (tok == 0x7fffffff) {  // nothing kept (every value masked): token 0, its logit read back
            tok = 0;
            tv = logits[(size_t)row * ld] * (greedy ? 1.f : 1.f / P.temperature);
        }
        out_tok[row] = tok;
        // the winner's value is its logit x 1/T as the slices scaled it: no dependent read of the row
        if (out_logp) out_logp[row] = tv - mx - __logf(fmaxf(greedy ? s_Z : z, 1e-30f));
    }
}

// B rows, S = ceil(V / TK_SLICE) slices per row (<= 64 and S * TK_CAPS <= TK_MNT * TK_MV); every row must have
// top_k in [1, TK_CAP] or be greedy, no typical-p / mirostat (the caller checks). cand_v / cand_i:
// [B][S][TK_CAPS] scratch, cand_n / slice_z: [B][S].
extern "C" int mxk_sample_topk_split(float* logits, int ld, int B, int V, const SampleParams* params, int has_pen,
                                     const int* pen_tok, const int* pen_cnt, const float* pen_bias,
                                     const uint32_t* allow_mask, int mask_ld, int S, float* cand_v, int* cand_i,
                                     int* cand_n, float2* slice_z, int* out_tok, float* out_logp, const int* pend_tok,
                                     hipStream_t st) {
    if (B <= 0) return 0;
    const int slice = tk_nv() * TK_NT;
    if (S != (V + slice - 1) / slice || S > 64 || S * TK_CAPS > TK_MNT * TK_MV) return (int)hipErrorInvalidValue;
    if (has_pen) tk_penalty_kernel<<<B, TK_NT, 0, st>>>(logits, ld, V, params, pen_tok, pen_cnt, pen_bias, pend_tok);
    const bool v4 = V % 4 == 0 && ld % 4 == 0 && ((uintptr_t)logits & 15) == 0;
#define TK_SLICE_LAUNCH(VEC_, MASK_, NV_)                                                                             \
    tk_slice_kernel<VEC_, MASK_, NV_><<<dim3(B, S), TK_NT, 0, st>>>(logits, ld, V, params, allow_mask, mask_ld,      \
                                                                    cand_v, cand_i, cand_n, slice_z)
    if (tk_nv() == 16) {
        if (allow_mask) {
            if (v4) TK_SLICE_LAUNCH(4, true, 16);
            else TK_SLICE_LAUNCH(1, true, 16);
        } else {
            if (v4) TK_SLICE_LAUNCH(4, false, 16);
            else TK_SLICE_LAUNCH(1, false, 16);
        }
    } else {
        if (allow_mask) {
            if (v4) TK_SLICE_LAUNCH(4, true, 32);
            else TK_SLICE_LAUNCH(1, true, 32);
        } else {
            if (v4) TK_SLICE_LAUNCH(4, false, 32);
            else TK_SLICE_LAUNCH(1, false, 32);
        }
    }
#undef TK_SLICE_LAUNCH
    tk_merge_kernel<<<B, TK_MNT, 0, st>>>(logits, ld, V, params, S, allow_mask, mask_ld, cand_v, cand_i, cand_n, slice_z,
                                          out_tok, out_logp);
    MXK_CHECK_LAUNCH();
}
extern "C" int mxk_sample_topk_slice() { return tk_nv() * TK_NT; }
// debug: enable / read the per-phase wall-clock stamps of tk_slice_kernel's workgroup (0, 0) (100 MHz ticks)
extern "C" int mxk_sample_trace(int on, unsigned long long* out16) {
    if (out16) return (int)hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_tk_ts), sizeof(unsigned long long) * 16);
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_tk_trace), &on, sizeof(int));
}
extern "C" int mxk_sample_topk_caps() { return TK_CAPS; }
extern "C" int mxk_sample_topk_cap() { return TK_CAP; }

// greedy argmax over rows (fast path used by the decode graph when every row is greedy)
__global__ __launch_bounds__(1024) void argmax_kernel(const float* __restrict__ x, int ld, int V,
                                                      int* __restrict__ out, unsigned long long* __restrict__ keys,
                                                      int off, const int* __restrict__ gate = nullptr) {
    if (gate && *gate == 0) return;  // graph-captured head of a step whose rows are all sampled
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

// the same, skipped on the device when *gate == 0 (a step-graph input: the greedy fast path's argmax runs only on
// steps that use it)
extern "C" int mxk_argmax_gated(const float* x, int ld, int B, int V, int* out, const int* gate, hipStream_t st) {
    if (B <= 0) return 0;
    argmax_kernel<<<B, 1024, 0, st>>>(x, ld, V, out, nullptr, 0, gate);
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
