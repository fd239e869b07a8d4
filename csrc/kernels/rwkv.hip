// rwkv.hip — RWKV-6 ("Finch") token-shift mixing and WKV recurrence for the continuous-batching
// engine. Reference: llama.cpp's rwkv6 graph (llm_build_rwkv6 time/channel mix, GGML_OP_RWKV_WKV6
// in ggml-cuda wkv.cu), which the reference serves through its llama-cpp backend
// (fixture tests/models_fixtures/rwkv.yaml, gallery rwkv-6-world-7b).
//
// Ragged step layout as in ssm.hip: `n_dec` single-row decode segments, then prefill chunks from
// `pf_cu`; a segment's state slot is slots[row0] / slot_div, slot < 0 = hipGraph padding (state left
// alone), positions[row0] == 0 = sequence start (state treated as zero).
//
//  * rwkv_shift_mix: out[m] = x + sx * (maa[m] + dm[m]) with sx = x_prev - x, for n_mix lerp
//    vectors at once (the 5 time-mix inputs, or the 2 channel-mix inputs), straight to the act16
//    GEMM operands. x_prev comes from the row above or, at a segment start, from the carried shift
//    state; the call that computes sx also saves it (sx_out) and stores the segment's last row as
//    the new shift state.
//  * rwkv_wkv6: one wave64 per (segment, head), lane j owns column j of the 64x64 state in VGPRs.
//    Per step r/k/decay land in LDS and are read back as broadcast float4s; y_j = Σ_i r_i (u_i k_i
//    v_j + S_ij), S_ij = w_i S_ij + k_i v_j with w = exp(-exp(w_raw)). The head's GroupNorm (ln_x,
//    eps 64e-5) is a 64-lane shuffle reduction over the same lanes and the SiLU gate multiplies in
//    before the act16 store, so the output projection reads the finished operand.
#include "mx_common.h"

MX_DEV void rwkv_segment(int s, int n_dec, const int* __restrict__ pf_cu, int& row0, int& len) {
    if (s < n_dec) {
        row0 = s;
        len = 1;
    } else {
        const int k = s - n_dec;
        row0 = n_dec + pf_cu[k];
        len = pf_cu[k + 1] - pf_cu[k];
    }
}

template <bool F16>
__global__ __launch_bounds__(256) void rwkv_shift_mix_kernel(const float* __restrict__ x, int ldx,
                                                             float* __restrict__ shift_state,  // [slots, C]
                                                             const float* __restrict__ sx_in,  // [T, C] or null
                                                             float* __restrict__ sx_out,  // [T, C] or null
                                                             const float* __restrict__ maa,  // [n_mix, C]
                                                             const float* __restrict__ dm,  // [n_mix, T, C] or null
                                                             uint16_t* __restrict__ out,  // [n_mix, T, C]
                                                             int n_mix, const int* __restrict__ slots,
                                                             const int* __restrict__ positions, int slot_div,
                                                             int n_dec, const int* __restrict__ pf_cu, int T, int C) {
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= C) return;
    int row0, len;
    rwkv_segment(blockIdx.y, n_dec, pf_cu, row0, len);
    if (len <= 0) return;
    const int slot = slots[row0];
    const bool keep = slot >= 0;
    float* st = keep ? shift_state + (size_t)(slot / slot_div) * C + c : nullptr;
    float prev = 0.f;
    if (!sx_in && keep && positions[row0] != 0) prev = *st;
    const size_t TC = (size_t)T * C;
    for (int t = 0; t < len; ++t) {
        const int r = row0 + t;
        const float xv = x[(size_t)r * ldx + c];
        float sx;
        if (sx_in) {
            sx = sx_in[(size_t)r * C + c];
        } else {
            sx = prev - xv;
            prev = xv;
            if (sx_out) sx_out[(size_t)r * C + c] = sx;
        }
        for (int m = 0; m < n_mix; ++m) {
            float mu = maa[(size_t)m * C + c];
            if (dm) mu += dm[m * TC + (size_t)r * C + c];
            out[m * TC + (size_t)r * C + c] = f32_to_act<F16>(fmaf(sx, mu, xv));
        }
    }
    if (!sx_in && keep) *st = prev;
}

MX_DEV float wave_sum64(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

template <bool F16>
__global__ __launch_bounds__(64) void rwkv_wkv6_kernel(const float* __restrict__ r, const float* __restrict__ k,
                                                       const float* __restrict__ v, const float* __restrict__ w,
                                                       const float* __restrict__ g, int ld,  // [T, C] rows
                                                       const float* __restrict__ u,  // [C] (time_first)
                                                       float* __restrict__ state,  // [slots, H, 64, 64]
                                                       const float* __restrict__ lnw, const float* __restrict__ lnb,
                                                       float ln_eps, uint16_t* __restrict__ out, int ldo,
                                                       const int* __restrict__ slots,
                                                       const int* __restrict__ positions, int slot_div, int n_dec,
                                                       const int* __restrict__ pf_cu, int H) {
    constexpr int N = 64;
    __shared__ __attribute__((aligned(16))) float sr[N], sk[N], sw[N], su[N];
    const int j = threadIdx.x;
    const int h = blockIdx.x;
    int row0, len;
    rwkv_segment(blockIdx.y, n_dec, pf_cu, row0, len);
    if (len <= 0) return;
    const int slot = slots[row0];
    const bool keep = slot >= 0;
    const bool reset = !keep || positions[row0] == 0;
    const int c = h * N + j;
    float* st = keep ? state + ((size_t)(slot / slot_div) * H + h) * N * N + j : nullptr;
    float S[N];
#pragma unroll
    for (int i = 0; i < N; ++i) S[i] = reset ? 0.f : st[(size_t)i * N];
    su[j] = u[c];
    const float gw = lnw[c], gb = lnb[c];
    for (int t = 0; t < len; ++t) {
        const size_t row = (size_t)(row0 + t) * ld + c;
        __syncthreads();  // previous step's LDS reads are done
        sr[j] = r[row];
        sk[j] = k[row];
        sw[j] = __expf(-__expf(w[row]));
        const float vj = v[row];
        const float gj = g[row];
        __syncthreads();
        float y = 0.f;
        const float4* r4 = reinterpret_cast<const float4*>(sr);
        const float4* k4 = reinterpret_cast<const float4*>(sk);
        const float4* w4 = reinterpret_cast<const float4*>(sw);
        const float4* u4 = reinterpret_cast<const float4*>(su);
#pragma unroll
        for (int q = 0; q < N / 4; ++q) {
            const float4 rr = r4[q], kk = k4[q], ww = w4[q], uu = u4[q];
            const float rv[4] = {rr.x, rr.y, rr.z, rr.w}, kv_[4] = {kk.x, kk.y, kk.z, kk.w};
            const float wv[4] = {ww.x, ww.y, ww.z, ww.w}, uv[4] = {uu.x, uu.y, uu.z, uu.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int i = 4 * q + e;
                const float kv = kv_[e] * vj;
                y = fmaf(rv[e], fmaf(uv[e], kv, S[i]), y);
                S[i] = fmaf(wv[e], S[i], kv);
            }
        }
        // per-head GroupNorm (ln_x) over the 64 lanes, affine, then the SiLU gate
        const float mean = wave_sum64(y) * (1.f / N);
        const float d = y - mean;
        const float var = wave_sum64(d * d) * (1.f / N);
        const float yn = fmaf(d * rsqrtf(var + ln_eps), gw, gb);
        out[(size_t)(row0 + t) * ldo + c] = f32_to_act<F16>(yn * gj);
    }
    if (keep) {
#pragma unroll
        for (int i = 0; i < N; ++i) st[(size_t)i * N] = S[i];
    }
}

extern "C" int mxk_rwkv_shift_mix(const float* x, int ldx, float* shift_state, const float* sx_in, float* sx_out,
                                  const float* maa, const float* dm, uint16_t* out, int n_mix, const int* slots,
                                  const int* positions, int slot_div, int n_dec, const int* pf_cu, int n_pf, int T,
                                  int C, hipStream_t st) {
    const int S = n_dec + n_pf;
    if (S == 0) return 0;
    dim3 grid((C + 255) / 256, S);
    MX_ACT_DISPATCH((rwkv_shift_mix_kernel<F16><<<grid, 256, 0, st>>>(x, ldx, shift_state, sx_in, sx_out, maa, dm,
                                                                        out, n_mix, slots, positions, slot_div, n_dec,
                                                                        pf_cu, T, C)));
    return (int)hipGetLastError();
}

extern "C" int mxk_rwkv_wkv6(const float* r, const float* k, const float* v, const float* w, const float* g, int ld,
                             const float* u, float* state, const float* lnw, const float* lnb, float ln_eps,
                             uint16_t* out, int ldo, const int* slots, const int* positions, int slot_div, int n_dec,
                             const int* pf_cu, int n_pf, int H, int head_size, hipStream_t st) {
    const int S = n_dec + n_pf;
    if (S == 0) return 0;
    if (head_size != 64) return (int)hipErrorInvalidValue;
    dim3 grid(H, S);
    MX_ACT_DISPATCH((rwkv_wkv6_kernel<F16><<<grid, 64, 0, st>>>(r, k, v, w, g, ld, u, state, lnw, lnb, ln_eps, out,
                                                                  ldo, slots, positions, slot_div, n_dec, pf_cu, H)));
    return (int)hipGetLastError();
}
