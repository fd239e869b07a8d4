// diffusion.hip — normalisation / modulation kernels for the diffusion models (SD3 MMDiT, SD UNet,
// VAE) and other adaLN transformers:
//
//  * layernorm_mod:  y = LN(x) * (1 + scale[b]) + shift[b]   (adaLN-Zero / AdaLayerNormContinuous)
//                    fp32 residual stream in, act16 out; per-sample modulation rows from the
//                    conditioning GEMM (fp32 or act16), two-pass variance from registers.
//  * gate_add:       x[b, s, :] += gate[b, :] * y[b, s, :]  (gated residual, act16 y, fp32 x)
//  * GroupNorm NHWC: a wide stats pass (grid over spatial chunks x samples, per-group partials
//                    reduced in LDS, fp64 atomics into [N, G, 2]) + an elementwise apply pass with
//                    optional fused SiLU, act16 in / act16 out. The old one-workgroup-per-group
//                    kernel left most of the 256 CUs idle at VAE resolutions (HW up to 1M).
#include "mx_common.h"

// ---------------------------------------------------------------------------------------------
// LayerNorm + modulation
template <bool F16, int PER>
__global__ __launch_bounds__(256) void layernorm_mod_kernel(const float* __restrict__ x, int ldx,
                                                            const float* __restrict__ scale,
                                                            const float* __restrict__ shift, int ldm,
                                                            int rows_per_b, uint16_t* __restrict__ out, int ldo,
                                                            int H, float eps) {
    __shared__ float red[4];
    const int row = blockIdx.x;
    const int b = row / rows_per_b;
    const float* xr = x + (size_t)row * ldx;
    float v[PER];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const int c = threadIdx.x + 256 * i;
        v[i] = c < H ? xr[c] : 0.f;
        s += v[i];
    }
    s = block_sum<256>(s, red);
    const float mean = s / H;
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const int c = threadIdx.x + 256 * i;
        const float d = c < H ? v[i] - mean : 0.f;
        ss += d * d;
    }
    ss = block_sum<256>(ss, red);
    const float rs = rsqrtf(ss / H + eps);
    const float* sc = scale ? scale + (size_t)b * ldm : nullptr;
    const float* sh = shift ? shift + (size_t)b * ldm : nullptr;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const int c = threadIdx.x + 256 * i;
        if (c < H) {
            float y = (v[i] - mean) * rs;
            if (sc) y *= 1.f + sc[c];
            if (sh) y += sh[c];
            out[(size_t)row * ldo + c] = f32_to_act<F16>(y);
        }
    }
}

extern "C" int mxk_layernorm_mod(const float* x, int ldx, const float* scale, const float* shift, int ldm,
                                 int rows_per_b, uint16_t* out, int ldo, int rows, int H, float eps, hipStream_t st) {
    if (rows <= 0) return 0;
    if (H > 256 * 16 || rows_per_b <= 0) return (int)hipErrorInvalidValue;
#define LNM(P) layernorm_mod_kernel<F16, P><<<rows, 256, 0, st>>>(x, ldx, scale, shift, ldm, rows_per_b, out, ldo, H, eps)
    MX_ACT_DISPATCH({
        if (H <= 1024) LNM(4);
        else if (H <= 2048) LNM(8);
        else LNM(16);
    });
#undef LNM
    MXK_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------------------------
// gated residual: x (fp32) += gate[b] * y (act16), 8 columns per thread
template <bool F16>
__global__ __launch_bounds__(256) void gate_add_kernel(float* __restrict__ x, int ldx, const uint16_t* __restrict__ y,
                                                       int ldy, const float* __restrict__ gate, int ldg,
                                                       int rows_per_b, int rows, int H) {
    const int cpr = H / 8;
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (size_t)rows * cpr) return;
    const int row = (int)(i / cpr), c = (int)(i % cpr) * 8;
    const int b = row / rows_per_b;
    const uint4 yv = *(const uint4*)(y + (size_t)row * ldy + c);
    const uint32_t yw[4] = {yv.x, yv.y, yv.z, yv.w};
    float* xr = x + (size_t)row * ldx + c;
    float4 a = *(float4*)xr, bq = *(float4*)(xr + 4);
    float xs[8] = {a.x, a.y, a.z, a.w, bq.x, bq.y, bq.z, bq.w};
    const float* g = gate ? gate + (size_t)b * ldg + c : nullptr;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        float lo, hi;
        unpack_act2<F16>(yw[k], lo, hi);
        xs[2 * k] += (g ? g[2 * k] : 1.f) * lo;
        xs[2 * k + 1] += (g ? g[2 * k + 1] : 1.f) * hi;
    }
    *(float4*)xr = make_float4(xs[0], xs[1], xs[2], xs[3]);
    *(float4*)(xr + 4) = make_float4(xs[4], xs[5], xs[6], xs[7]);
}

extern "C" int mxk_gate_add(float* x, int ldx, const uint16_t* y, int ldy, const float* gate, int ldg, int rows_per_b,
                            int rows, int H, hipStream_t st) {
    if (rows <= 0) return 0;
    if (H % 8 || ldx % 4 || ldy % 8) return (int)hipErrorInvalidValue;
    const size_t n = (size_t)rows * (H / 8);
    MX_ACT_DISPATCH(gate_add_kernel<F16><<<(unsigned)((n + 255) / 256), 256, 0, st>>>(x, ldx, y, ldy, gate, ldg,
                                                                                      rows_per_b, rows, H));
    MXK_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------------------------
// GroupNorm over NHWC act16
constexpr int GN_MAXG = 32;

template <bool F16>
__global__ __launch_bounds__(256) void gn_stats_kernel(const uint16_t* __restrict__ x, int HW, int C, int G,
                                                       int rows_per_block, double* __restrict__ stats) {
    __shared__ float gs[GN_MAXG], gss[GN_MAXG];
    const int n = blockIdx.y;
    const int cpr = C / 8;                 // 8-channel chunks per pixel row
    const int tpr = cpr < 256 ? cpr : 256; // threads per pixel row (wider rows: each thread loops chunks)
    const int rpi = 256 / tpr;             // pixel rows per iteration
    const int t = threadIdx.x;
    if (t < GN_MAXG) { gs[t] = 0.f; gss[t] = 0.f; }
    __syncthreads();
    const int p0 = blockIdx.x * rows_per_block;
    const int p1 = min(HW, p0 + rows_per_block);
    const int pr = t / tpr;
    for (int cc = t % tpr; pr < rpi && cc < cpr; cc += tpr) {
        float s[8] = {0, 0, 0, 0, 0, 0, 0, 0}, ss[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        const uint16_t* xb = x + (size_t)n * HW * C + cc * 8;
        for (int p = p0 + pr; p < p1; p += rpi) {
            const uint4 v = *(const uint4*)(xb + (size_t)p * C);
            const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                float lo, hi;
                unpack_act2<F16>(w[k], lo, hi);
                s[2 * k] += lo;
                ss[2 * k] += lo * lo;
                s[2 * k + 1] += hi;
                ss[2 * k + 1] += hi * hi;
            }
        }
        const int cg = C / G;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int g = (cc * 8 + k) / cg;
            atomicAdd(&gs[g], s[k]);
            atomicAdd(&gss[g], ss[k]);
        }
    }
    __syncthreads();
    if (t < G) {
        atomicAdd(&stats[((size_t)n * G + t) * 2], (double)gs[t]);
        atomicAdd(&stats[((size_t)n * G + t) * 2 + 1], (double)gss[t]);
    }
}

template <bool F16, bool SILU>
__global__ __launch_bounds__(256) void gn_apply_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y,
                                                       const float* __restrict__ gamma,
                                                       const float* __restrict__ beta,
                                                       const double* __restrict__ stats, int HW, int C, int G,
                                                       float eps, size_t total8) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= total8) return;
    const int cpr = C / 8;
    const int c0 = (int)(i % cpr) * 8;
    const int n = (int)(i / ((size_t)HW * cpr));
    const int cg = C / G;
    const double cnt = (double)HW * cg;
    const uint4 v = *(const uint4*)(x + i * 8);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    uint32_t o[4];
    int gprev = -1;
    float mean = 0.f, rs = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        float e[2];
        unpack_act2<F16>(w[k], e[0], e[1]);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int c = c0 + 2 * k + j;
            const int g = c / cg;
            if (g != gprev) {
                const double m = stats[((size_t)n * G + g) * 2] / cnt;
                const double var = fmax(stats[((size_t)n * G + g) * 2 + 1] / cnt - m * m, 0.0);
                mean = (float)m;
                rs = rsqrtf((float)var + eps);
                gprev = g;
            }
            float r = (e[j] - mean) * rs * gamma[c] + beta[c];
            if (SILU) r = silu_f(r);
            e[j] = r;
        }
        o[k] = pack_act2<F16>(e[0], e[1]);
    }
    *(uint4*)(y + i * 8) = make_uint4(o[0], o[1], o[2], o[3]);
}

// x, y: act16 [N, HW, C] (NHWC / channels_last), y may alias x. workspace: N*G*2 doubles.
extern "C" int mxk_groupnorm16(const uint16_t* x, uint16_t* y, const float* gamma, const float* beta, int N, int HW,
                               int C, int G, float eps, int silu, double* ws, hipStream_t st) {
    if (N <= 0 || HW <= 0) return 0;
    if (C % 8 || C % G || G > GN_MAXG) return (int)hipErrorInvalidValue;
    hipMemsetAsync(ws, 0, sizeof(double) * N * G * 2, st);
    const int rpi = 256 / (C / 8 < 256 ? C / 8 : 256);
    int rows_per_block = max(rpi * 8, (HW + 255) / 256);          // >= 8 iterations, <= 256 blocks per sample
    rows_per_block = (rows_per_block + rpi - 1) / rpi * rpi;
    dim3 g1((HW + rows_per_block - 1) / rows_per_block, N);
    const size_t total8 = (size_t)N * HW * (C / 8);
    const unsigned g2 = (unsigned)((total8 + 255) / 256);
    MX_ACT_DISPATCH({
        gn_stats_kernel<F16><<<g1, 256, 0, st>>>(x, HW, C, G, rows_per_block, ws);
        if (silu) gn_apply_kernel<F16, true><<<g2, 256, 0, st>>>(x, y, gamma, beta, ws, HW, C, G, eps, total8);
        else gn_apply_kernel<F16, false><<<g2, 256, 0, st>>>(x, y, gamma, beta, ws, HW, C, G, eps, total8);
    });
    MXK_CHECK_LAUNCH();
}

// ---- Mix-FFN (Sana GLUMBConv) middle: depthwise 3x3 over 2*Ch channels + GLU -----------------------------
// x 16-bit NHWC [B, H, W, 2*Ch] (optionally SiLU applied on load: the 1x1 expansion's activation), w fp32
// [2*Ch][9], b fp32 [2*Ch]; out 16-bit [B, H, W, Ch] = dw(x)[c] * silu(dw(x)[Ch + c]). Two channels per
// thread (4-byte loads), zero padding at the borders. Memory bound: each input element is read by its 9
// neighbours through L1/L2, the expanded activation never round-trips through HBM twice.
template <bool F16>
__global__ __launch_bounds__(256) void dwconv3_glu_kernel(const uint16_t* __restrict__ x, const float* __restrict__ w,
                                                          const float* __restrict__ b, uint16_t* __restrict__ out,
                                                          int B, int H, int W, int Ch, int silu_in) {
    const int pairs = Ch >> 1;
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    const long long total = (long long)B * H * W * pairs;
    if (i >= total) return;
    const int cp = (int)(i % pairs);
    const long long pix = i / pairs;
    const int px = (int)(pix % W), py = (int)((pix / W) % H), bb = (int)(pix / ((long long)W * H));
    const int c = 2 * cp, C2 = 2 * Ch;
    float v0 = b[c], v1 = b[c + 1], g0 = b[Ch + c], g1 = b[Ch + c + 1];
#pragma unroll
    for (int dy = -1; dy <= 1; ++dy) {
        const int yy = py + dy;
        if (yy < 0 || yy >= H) continue;
#pragma unroll
        for (int dx = -1; dx <= 1; ++dx) {
            const int xx = px + dx;
            if (xx < 0 || xx >= W) continue;
            const int t = (dy + 1) * 3 + (dx + 1);
            const uint16_t* p = x + (((size_t)bb * H + yy) * W + xx) * C2;
            float a0, a1, h0, h1;
            unpack_act2<F16>(*(const uint32_t*)(p + c), a0, a1);
            unpack_act2<F16>(*(const uint32_t*)(p + Ch + c), h0, h1);
            if (silu_in) {
                a0 = a0 / (1.f + __expf(-a0)); a1 = a1 / (1.f + __expf(-a1));
                h0 = h0 / (1.f + __expf(-h0)); h1 = h1 / (1.f + __expf(-h1));
            }
            v0 += a0 * w[c * 9 + t];
            v1 += a1 * w[(c + 1) * 9 + t];
            g0 += h0 * w[(Ch + c) * 9 + t];
            g1 += h1 * w[(Ch + c + 1) * 9 + t];
        }
    }
    const float o0 = v0 * (g0 / (1.f + __expf(-g0))), o1 = v1 * (g1 / (1.f + __expf(-g1)));
    *(uint32_t*)(out + (size_t)pix * Ch + c) = pack_act2<F16>(o0, o1);
}

extern "C" int mxk_dwconv3_glu(const uint16_t* x, const float* w, const float* b, uint16_t* out, int B, int H, int W,
                               int Ch, int silu_in, hipStream_t st) {
    if ((long long)B * H * W == 0) return 0;
    if (Ch & 1) return (int)hipErrorInvalidValue;
    const long long total = (long long)B * H * W * (Ch / 2);
    const int grid = (int)((total + 255) / 256);
    MX_ACT_DISPATCH((dwconv3_glu_kernel<F16><<<grid, 256, 0, st>>>(x, w, b, out, B, H, W, Ch, silu_in)));
    return (int)hipGetLastError();
}
