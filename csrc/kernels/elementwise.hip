// elementwise.hip — small fused element-wise kernels (K11/K12 of SURVEY §2.6) used outside the
// fused GEMM epilogues: SwiGLU/GeGLU on separate gate/up buffers, GELU, residual adds, fp32<->bf16
// casts and embedding-row gathers for dense (f32/f16/bf16) tables. All loads are 16-byte vectors.
#include "mx_common.h"

// library-wide 16-bit activation format (see mx_common.h): 0 bf16, 1 f16
int g_mx_act_f16 = 0;
extern "C" int mxk_set_act_f16(int on) {
    const int prev = g_mx_act_f16;
    g_mx_act_f16 = on ? 1 : 0;
    return prev;
}
extern "C" int mxk_get_act_f16() { return g_mx_act_f16; }

// y[m, f] = act(g[m, f]) * u[m, f]; g/u bf16 with row stride ld_in, out bf16
template <int ACT, bool F16>
__global__ __launch_bounds__(256) void glu_kernel(const bf16_t* __restrict__ g, const bf16_t* __restrict__ u,
                                                  int ld_in, bf16_t* __restrict__ y, int ld_out, int F) {
    const int m = blockIdx.y;
    const int f = (blockIdx.x * 256 + threadIdx.x) * 8;
    if (f >= F) return;
    const uint4 gr = *(const uint4*)(g + (size_t)m * ld_in + f);
    const uint4 ur = *(const uint4*)(u + (size_t)m * ld_in + f);
    const uint32_t gw[4] = {gr.x, gr.y, gr.z, gr.w}, uw[4] = {ur.x, ur.y, ur.z, ur.w};
    uint32_t o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        float g0, g1, u0, u1;
        unpack_act2<F16>(gw[j], g0, g1);
        unpack_act2<F16>(uw[j], u0, u1);
        float a0, a1;
        if (ACT == 0) { a0 = silu_f(g0); a1 = silu_f(g1); }
        else if (ACT == 1) { a0 = gelu_tanh_f(g0); a1 = gelu_tanh_f(g1); }
        else { a0 = gelu_erf_f(g0); a1 = gelu_erf_f(g1); }
        o[j] = pack_act2<F16>(a0 * u0, a1 * u1);
    }
    *(uint4*)(y + (size_t)m * ld_out + f) = make_uint4(o[0], o[1], o[2], o[3]);
}

extern "C" int mxk_glu(int act, const bf16_t* g, const bf16_t* u, int ld_in, bf16_t* y, int ld_out, int M, int F,
                       hipStream_t st) {
    if (M <= 0) return 0;
    if (F % 8) return (int)hipErrorInvalidValue;
    dim3 grid((F / 8 + 255) / 256, M);
    MX_ACT_DISPATCH({
        if (act == 0) glu_kernel<0, F16><<<grid, 256, 0, st>>>(g, u, ld_in, y, ld_out, F);
        else if (act == 1) glu_kernel<1, F16><<<grid, 256, 0, st>>>(g, u, ld_in, y, ld_out, F);
        else glu_kernel<2, F16><<<grid, 256, 0, st>>>(g, u, ld_in, y, ld_out, F);
    });
    MXK_CHECK_LAUNCH();
}

// SwiGLU over a gate|up product whose columns are interleaved in 16-column groups (the layout of
// the fused gate_up weight): y[m, 32*(f/16) + f%16] = gate, y[m, 32*(f/16) + 16 + f%16] = up.
template <bool F16, int EPI>
__global__ __launch_bounds__(256) void swiglu_il16_kernel(const bf16_t* __restrict__ y, int ldy,
                                                          bf16_t* __restrict__ out, int ldo, int F) {
    const int m = blockIdx.y;
    const int f = (blockIdx.x * 256 + threadIdx.x) * 8;  // 8 features: half of a 16-group
    if (f >= F) return;
    const int grp = f >> 4, sub = f & 15;
    const bf16_t* base = y + (size_t)m * ldy + grp * 32 + sub;
    const uint4 gr = *(const uint4*)base;
    const uint4 ur = *(const uint4*)(base + 16);
    const uint32_t gw[4] = {gr.x, gr.y, gr.z, gr.w}, uw[4] = {ur.x, ur.y, ur.z, ur.w};
    uint32_t o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        float g0, g1, u0, u1;
        unpack_act2<F16>(gw[j], g0, g1);
        unpack_act2<F16>(uw[j], u0, u1);
        o[j] = pack_act2<F16>(glu_gate_f<EPI>(g0) * u0, glu_gate_f<EPI>(g1) * u1);
    }
    *(uint4*)(out + (size_t)m * ldo + f) = make_uint4(o[0], o[1], o[2], o[3]);
}

// gelu: 0 SwiGLU, 1 GeGLU (gelu tanh)
extern "C" int mxk_swiglu_il16(const bf16_t* y, int ldy, bf16_t* out, int ldo, int M, int F, int gelu,
                               hipStream_t st) {
    if (M <= 0) return 0;
    if (F % 16) return (int)hipErrorInvalidValue;
    dim3 grid((F / 8 + 255) / 256, M);
    if (gelu) MX_ACT_DISPATCH((swiglu_il16_kernel<F16, 4><<<grid, 256, 0, st>>>(y, ldy, out, ldo, F)));
    else MX_ACT_DISPATCH((swiglu_il16_kernel<F16, 3><<<grid, 256, 0, st>>>(y, ldy, out, ldo, F)));
    MXK_CHECK_LAUNCH();
}

// in-place activation on fp32 (act: 0 silu, 1 gelu-tanh, 2 gelu-erf, 3 relu)
__global__ __launch_bounds__(256) void act_f32_kernel(float* __restrict__ x, size_t n, int act) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        float v = x[i];
        if (act == 0) v = silu_f(v);
        else if (act == 1) v = gelu_tanh_f(v);
        else if (act == 2) v = gelu_erf_f(v);
        else v = fmaxf(v, 0.f);
        x[i] = v;
    }
}

extern "C" int mxk_act_f32(float* x, size_t n, int act, hipStream_t st) {
    if (!n) return 0;
    const int grid = (int)min((size_t)4096, (n + 255) / 256);
    act_f32_kernel<<<grid, 256, 0, st>>>(x, n, act);
    MXK_CHECK_LAUNCH();
}

// fp32 -> act16 (bf16 or f16, library mode) cast of a [rows, cols] view with strides
template <bool F16>
__global__ __launch_bounds__(256) void cast_f32_bf16_kernel(const float* __restrict__ x, int ldx,
                                                            bf16_t* __restrict__ y, int ldy, int cols) {
    const int r = blockIdx.y;
    for (int c = (blockIdx.x * 256 + threadIdx.x) * 4; c < cols; c += gridDim.x * 256 * 4) {
        const float4 v = *(const float4*)(x + (size_t)r * ldx + c);
        uint2 p;
        p.x = pack_act2<F16>(v.x, v.y);
        p.y = pack_act2<F16>(v.z, v.w);
        *(uint2*)(y + (size_t)r * ldy + c) = p;
    }
}

extern "C" int mxk_cast_f32_bf16(const float* x, int ldx, bf16_t* y, int ldy, int rows, int cols, hipStream_t st) {
    if (rows <= 0) return 0;
    if (cols % 4) return (int)hipErrorInvalidValue;
    dim3 grid(min(64, (cols / 4 + 255) / 256), rows);
    MX_ACT_DISPATCH(cast_f32_bf16_kernel<F16><<<grid, 256, 0, st>>>(x, ldx, y, ldy, cols));
    MXK_CHECK_LAUNCH();
}

// gather rows of a dense table: dtype 0 f32, 1 f16, 2 bf16 -> fp32 out (the residual stream)
__global__ __launch_bounds__(256) void gather_rows_kernel(const void* __restrict__ tab, int dtype,
                                                          const int* __restrict__ ids, int H, float scale,
                                                          float* __restrict__ out) {
    const int r = blockIdx.x;
    const size_t base = (size_t)ids[r] * H;
    for (int c = threadIdx.x; c < H; c += 256) {
        float v;
        if (dtype == 0) v = ((const float*)tab)[base + c];
        else if (dtype == 1) v = half_to_f32(((const uint16_t*)tab)[base + c]);
        else v = bf16_to_f32(((const uint16_t*)tab)[base + c]);
        out[(size_t)r * H + c] = v * scale;
    }
}

extern "C" int mxk_gather_rows(const void* tab, int dtype, const int* ids, int n, int H, float scale, float* out,
                               hipStream_t st) {
    if (n <= 0) return 0;
    gather_rows_kernel<<<n, 256, 0, st>>>(tab, dtype, ids, H, scale, out);
    MXK_CHECK_LAUNCH();
}

// scale fp32 rows in place (embedding scale for Gemma-style models) and add bias vectors
__global__ __launch_bounds__(256) void add_bias_f32_kernel(float* __restrict__ x, int ld, const float* __restrict__ b,
                                                           int cols) {
    const int r = blockIdx.y;
    for (int c = blockIdx.x * 256 + threadIdx.x; c < cols; c += gridDim.x * 256) x[(size_t)r * ld + c] += b[c];
}

extern "C" int mxk_add_bias_f32(float* x, int ld, const float* b, int rows, int cols, hipStream_t st) {
    if (rows <= 0) return 0;
    dim3 grid(min(64, (cols + 255) / 256), rows);
    add_bias_f32_kernel<<<grid, 256, 0, st>>>(x, ld, b, cols);
    MXK_CHECK_LAUNCH();
}

// h (fp32 residual) += y (16-bit activations), 4 elements per thread: the residual add of a row-parallel
// projection when no fused all-reduce+add kernel runs (TP rehearsal on one GPU, RCCL fallback) — one pass,
// instead of PyTorch's mixed-dtype templated add
template <bool F16>
__global__ __launch_bounds__(256) void add_act_into_f32_kernel(const uint16_t* __restrict__ y, int ldy,
                                                               float* __restrict__ h, int ldh, int cols) {
    const int r = blockIdx.y;
    for (int c = (blockIdx.x * 256 + threadIdx.x) * 4; c < cols; c += gridDim.x * 256 * 4) {
        const uint2 raw = *(const uint2*)(y + (size_t)r * ldy + c);
        float4 o = *(float4*)(h + (size_t)r * ldh + c);
        float a0, a1, a2, a3;
        unpack_act2<F16>(raw.x, a0, a1);
        unpack_act2<F16>(raw.y, a2, a3);
        o.x += a0; o.y += a1; o.z += a2; o.w += a3;
        *(float4*)(h + (size_t)r * ldh + c) = o;
    }
}

extern "C" int mxk_add_act_into_f32(const uint16_t* y, int ldy, float* h, int ldh, int rows, int cols, hipStream_t st) {
    if (rows <= 0) return 0;
    if ((cols & 3) || (ldy & 3) || (ldh & 3) || ((uintptr_t)y & 7) || ((uintptr_t)h & 15)) return (int)hipErrorInvalidValue;
    dim3 grid(min(16, (cols + 1023) / 1024), rows);
    MX_ACT_DISPATCH(add_act_into_f32_kernel<F16><<<grid, 256, 0, st>>>(y, ldy, h, ldh, cols));
    MXK_CHECK_LAUNCH();
}

// overlap-mode decode inputs: tokens[dst[i]] = prev[src[i]] (the previous, still unread step's samples) — one launch
// for what index_select + index_copy + two index casts took four
__global__ __launch_bounds__(256) void fix_tokens_kernel(int* __restrict__ tokens, const int* __restrict__ dst,
                                                         const int* __restrict__ src, const int* __restrict__ prev,
                                                         int n) {
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) tokens[dst[i]] = prev[src[i]];
}

extern "C" int mxk_fix_tokens(int* tokens, const int* dst, const int* src, const int* prev, int n, hipStream_t st) {
    if (n <= 0) return 0;
    fix_tokens_kernel<<<(n + 255) / 256, 256, 0, st>>>(tokens, dst, src, prev, n);
    MXK_CHECK_LAUNCH();
}

// gather selected rows of an fp32 matrix (last-token-of-each-sequence selection before the LM head)
__global__ __launch_bounds__(256) void select_rows_f32_kernel(const float* __restrict__ x, int ld,
                                                              const int* __restrict__ idx, int cols,
                                                              float* __restrict__ y, int ldy) {
    const int r = blockIdx.x;
    const float* src = x + (size_t)idx[r] * ld;
    for (int c = threadIdx.x * 4; c < cols; c += 1024) *(float4*)(y + (size_t)r * ldy + c) = *(const float4*)(src + c);
}

extern "C" int mxk_select_rows_f32(const float* x, int ld, const int* idx, int n, int cols, float* y, int ldy,
                                   hipStream_t st) {
    if (n <= 0) return 0;
    if (cols % 4) return (int)hipErrorInvalidValue;
    select_rows_f32_kernel<<<n, 256, 0, st>>>(x, ld, idx, cols, y, ldy);
    MXK_CHECK_LAUNCH();
}
