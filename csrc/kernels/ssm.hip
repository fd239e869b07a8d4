// ssm.hip — Mamba (selective state-space) mixer kernels for the continuous-batching LLM engine.
//
// The reference runs Mamba GGUFs through llama.cpp's GGML_OP_SSM_CONV / GGML_OP_SSM_SCAN
// (ggml-cuda ssm-conv.cu / ssm-scan.cu) and HF Mamba checkpoints through the
// transformers backend (backend/python/transformers/backend.py, Type "Mamba"). Here one engine step
// is a ragged batch: `n_dec` single-token decode rows first, then prefill chunks delimited by
// `pf_cu` (offsets relative to the first prefill row). Every segment owns one recurrent-state slot
// = slots[row0] / slot_div (the engine gives a recurrent model one cache "block" per sequence, so
// the paged block id *is* the state slot); slot < 0 marks a hipGraph padding row (state untouched),
// positions[row0] == 0 marks a sequence start (state reset, no separate zeroing launch).
//
//  * ssm_conv: causal depthwise conv (width KC) + bias + SiLU over x = xz[:, :Di], one lane per
//    channel streaming the segment's rows with the KC-1 previous inputs in registers; the window
//    is carried across chunks in conv_state [slots, KC-1, Di] (coalesced per row). Emits fp32 (for
//    the scan) and act16 (the x_proj GEMM operand) in one pass.
//  * ssm_scan: the selective scan with dt_proj + softplus, the D skip and the SiLU(z) gate fused:
//    16 lanes per channel (one per state dim, d_state = 16), 4 channels per wave64. Per step a lane
//    does R/16 FMAs of dt_proj (its W_dt slice lives in VGPRs), one exp, two FMAs for h, and the
//    C·h reduction is 4 xor-shuffles inside the 16-lane group. Loads of step t+1 are independent
//    of h, so the only serial chain is the h update. Output y is act16 for out_proj.
#include "mx_common.h"

MX_DEV void ssm_segment(int s, int n_dec, const int* __restrict__ pf_cu, int& row0, int& len) {
    if (s < n_dec) {
        row0 = s;
        len = 1;
    } else {
        const int k = s - n_dec;
        row0 = n_dec + pf_cu[k];
        len = pf_cu[k + 1] - pf_cu[k];
    }
}


template <bool F16, int KC>
__global__ __launch_bounds__(256) void ssm_conv_kernel(const float* __restrict__ xz, int ldxz,
                                                       const float* __restrict__ w,  // [Di, KC]
                                                       const float* __restrict__ bias,  // [Di]
                                                       float* __restrict__ state,  // [slots, KC-1, Di]
                                                       const int* __restrict__ slots,
                                                       const int* __restrict__ positions, int slot_div, int n_dec,
                                                       const int* __restrict__ pf_cu, float* __restrict__ xc,
                                                       uint16_t* __restrict__ xc16, int ldo16, int Di) {
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= Di) return;
    int row0, len;
    ssm_segment(blockIdx.y, n_dec, pf_cu, row0, len);
    if (len <= 0) return;
    const int slot = slots[row0];
    const bool keep = slot >= 0;
    const bool reset = !keep || positions[row0] == 0;
    float* st = keep ? state + (size_t)(slot / slot_div) * (KC - 1) * Di + c : nullptr;
    float win[KC - 1];
#pragma unroll
    for (int k = 0; k < KC - 1; ++k) win[k] = reset ? 0.f : st[(size_t)k * Di];
    float wk[KC];
#pragma unroll
    for (int k = 0; k < KC; ++k) wk[k] = w[c * KC + k];
    const float b = bias ? bias[c] : 0.f;
    float xn = xz[(size_t)row0 * ldxz + c];
    for (int t = 0; t < len; ++t) {
        const int r = row0 + t;
        const float x = xn;
        if (t + 1 < len) xn = xz[(size_t)(r + 1) * ldxz + c];
        float acc = fmaf(wk[KC - 1], x, b);
#pragma unroll
        for (int k = 0; k < KC - 1; ++k) acc = fmaf(wk[k], win[k], acc);
#pragma unroll
        for (int k = 0; k < KC - 2; ++k) win[k] = win[k + 1];
        win[KC - 2] = x;
        const float y = silu_f(acc);
        xc[(size_t)r * Di + c] = y;
        xc16[(size_t)r * ldo16 + c] = f32_to_act<F16>(y);
    }
    if (keep) {
#pragma unroll
        for (int k = 0; k < KC - 1; ++k) st[(size_t)k * Di] = win[k];
    }
}

// softplus with torch's threshold (F.softplus beta=1, threshold=20)
MX_DEV float softplus_f(float x) { return x > 20.f ? x : log1pf(__expf(x)); }

template <bool F16, int RPL>
__global__ __launch_bounds__(64) void ssm_scan_kernel(const float* __restrict__ xc,  // [T, Di]
                                                      const float* __restrict__ dbc, int lddbc,  // [T, R+2N]
                                                      const float* __restrict__ wdt,  // [Di, R]
                                                      const float* __restrict__ dt_bias,  // [Di]
                                                      const float* __restrict__ A,  // [Di, 16] (= -exp(A_log))
                                                      const float* __restrict__ Dskip,  // [Di]
                                                      const float* __restrict__ xz, int ldxz,  // z = xz[:, Di:]
                                                      float* __restrict__ state,  // [slots, Di, 16]
                                                      const int* __restrict__ slots,
                                                      const int* __restrict__ positions, int slot_div, int n_dec,
                                                      const int* __restrict__ pf_cu, uint16_t* __restrict__ y16,
                                                      int ldy, int Di, int R) {
    constexpr int NS = 16;
    const int n = threadIdx.x & (NS - 1);
    const int c = blockIdx.x * 4 + (threadIdx.x >> 4);
    if (c >= Di) return;  // Di % 4 == 0 (host-checked): whole 16-lane groups leave together
    int row0, len;
    ssm_segment(blockIdx.y, n_dec, pf_cu, row0, len);
    if (len <= 0) return;
    const int slot = slots[row0];
    const bool keep = slot >= 0;
    const bool reset = !keep || positions[row0] == 0;
    float* st = keep ? state + ((size_t)(slot / slot_div) * Di + c) * NS + n : nullptr;
    float h = reset ? 0.f : *st;
    const float a = A[c * NS + n];
    const float dsk = Dskip[c];
    const float db = dt_bias[c];
    float wr[RPL];  // lane n holds W_dt[c, n + 16 j]
#pragma unroll
    for (int j = 0; j < RPL; ++j) {
        const int k = n + NS * j;
        wr[j] = k < R ? wdt[(size_t)c * R + k] : 0.f;
    }
    const int offB = R, offC = R + NS;
    for (int t = 0; t < len; ++t) {
        const int r = row0 + t;
        const float* row = dbc + (size_t)r * lddbc;
        float dp = 0.f;
#pragma unroll
        for (int j = 0; j < RPL; ++j) {
            const int k = n + NS * j;
            if (k < R) dp = fmaf(wr[j], row[k], dp);
        }
        const float x = xc[(size_t)r * Di + c];
        const float Bn = row[offB + n];
        const float Cn = row[offC + n];
        // dt = softplus(W_dt row · dt_low + bias): 16-lane sum, every lane ends with the total
        dp += __shfl_xor(dp, 1, 16);
        dp += __shfl_xor(dp, 2, 16);
        dp += __shfl_xor(dp, 4, 16);
        dp += __shfl_xor(dp, 8, 16);
        const float dt = softplus_f(dp + db);
        h = fmaf(__expf(dt * a), h, dt * Bn * x);
        float p = Cn * h;
        p += __shfl_xor(p, 1, 16);
        p += __shfl_xor(p, 2, 16);
        p += __shfl_xor(p, 4, 16);
        p += __shfl_xor(p, 8, 16);
        if (n == 0) {
            const float z = xz[(size_t)r * ldxz + Di + c];
            y16[(size_t)r * ldy + c] = f32_to_act<F16>(fmaf(dsk, x, p) * silu_f(z));
        }
    }
    if (keep) *st = h;
}

extern "C" int mxk_ssm_conv(const float* xz, int ldxz, const float* w, const float* bias, float* state, int kc,
                            const int* slots, const int* positions, int slot_div, int n_dec, const int* pf_cu,
                            int n_pf, float* xc, uint16_t* xc16, int ldo16, int Di, hipStream_t st) {
    const int S = n_dec + n_pf;
    if (S == 0) return 0;
    dim3 grid((Di + 255) / 256, S);
    if (kc != 4) return (int)hipErrorInvalidValue;
    MX_ACT_DISPATCH((ssm_conv_kernel<F16, 4><<<grid, 256, 0, st>>>(xz, ldxz, w, bias, state, slots, positions,
                                                                     slot_div, n_dec, pf_cu, xc, xc16, ldo16, Di)));
    return (int)hipGetLastError();
}

extern "C" int mxk_ssm_scan(const float* xc, const float* dbc, int lddbc, const float* wdt, const float* dt_bias,
                            const float* A, const float* Dskip, const float* xz, int ldxz, float* state,
                            const int* slots, const int* positions, int slot_div, int n_dec, const int* pf_cu,
                            int n_pf, uint16_t* y16, int ldy, int Di, int R, int d_state, hipStream_t st) {
    const int S = n_dec + n_pf;
    if (S == 0) return 0;
    if (d_state != 16 || Di % 4 != 0 || R <= 0 || R > 256) return (int)hipErrorInvalidValue;
    dim3 grid(Di / 4, S);
#define SSM_SCAN(RPL_)                                                                                        \
    MX_ACT_DISPATCH((ssm_scan_kernel<F16, RPL_><<<grid, 64, 0, st>>>(xc, dbc, lddbc, wdt, dt_bias, A, Dskip, xz, \
                                                                      ldxz, state, slots, positions, slot_div,  \
                                                                      n_dec, pf_cu, y16, ldy, Di, R)))
    if (R <= 16) SSM_SCAN(1);
    else if (R <= 64) SSM_SCAN(4);
    else if (R <= 128) SSM_SCAN(8);
    else SSM_SCAN(16);
#undef SSM_SCAN
    return (int)hipGetLastError();
}
