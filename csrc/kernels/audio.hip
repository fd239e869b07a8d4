// audio.hip — recurrent / vocoder kernels for the speech workers (silero VAD, VITS TTS).
//
//  * lstm_scan: a persistent LSTM recurrence. One workgroup per sequence, 4*H threads (one per
//    gate row). Thread j keeps row j of W_hh in VGPRs for the whole scan (H=128 -> 128 fp32
//    registers), the hidden state lives in LDS and is read as broadcast float4s, so a time step is
//    H FMAs per lane + two barriers and no HBM traffic besides the precomputed input gates
//    gx[t] = W_ih x_t + b_ih + b_hh (one hipBLASLt GEMM over all steps, done by the caller).
//    HEAD fuses silero's decoder (ReLU -> 1x1 conv -> sigmoid) into the scan, so the only output
//    is one speech probability per step. Replaces the reference's per-window onnxruntime call
//    (silero-vad-go speech.Detector.infer), which re-enters the runtime 31 times per second of
//    audio.
//    H <= 128: a 4H-thread workgroup keeps its W_hh rows in registers only up to 2 waves / SIMD.
#include "mx_common.h"

MX_DEV float sigmoid_f(float x) { return 1.f / (1.f + __expf(-x)); }
MX_DEV float tanh_f(float x) {
    const float e = __expf(-2.f * fabsf(x));
    const float t = (1.f - e) / (1.f + e);
    return copysignf(t, x);
}

template <int H, bool HEAD>
__global__ __launch_bounds__(4 * H) void lstm_scan_kernel(const float* __restrict__ gx,   // [B, T, 4H]
                                                          const float* __restrict__ whh,  // [4H, H]
                                                          float* __restrict__ h_io,       // [B, H]
                                                          float* __restrict__ c_io,       // [B, H]
                                                          const float* __restrict__ head_w,  // [H]
                                                          float head_b,
                                                          float* __restrict__ out,  // HEAD ? [B, T] : [B, T, H]
                                                          int T) {
    constexpr int G = 4 * H;
    __shared__ __attribute__((aligned(16))) float sh_h[H];
    __shared__ float sh_g[G];
    __shared__ float sh_red[2 * (H / 64 > 0 ? H / 64 : 1)];
    const int j = threadIdx.x;
    const int b = blockIdx.x;
    float w[H];
    {
        const float4* wr = reinterpret_cast<const float4*>(whh + (size_t)j * H);
#pragma unroll
        for (int i = 0; i < H / 4; ++i) {
            const float4 v = wr[i];
            w[4 * i] = v.x;
            w[4 * i + 1] = v.y;
            w[4 * i + 2] = v.z;
            w[4 * i + 3] = v.w;
        }
    }
    float c = 0.f, hw = 0.f;
    if (j < H) {
        sh_h[j] = h_io[(size_t)b * H + j];
        c = c_io[(size_t)b * H + j];
        if (HEAD) hw = head_w[j];
    }
    const float* g_row = gx + (size_t)b * T * G;
    float g_next = T > 0 ? g_row[j] : 0.f;
    __syncthreads();
    constexpr int NW = H / 64;
    for (int t = 0; t < T; ++t) {
        if (HEAD && j == 0 && t > 0) {
            float s = head_b;
#pragma unroll
            for (int i = 0; i < NW; ++i) s += sh_red[i];
            out[(size_t)b * T + t - 1] = sigmoid_f(s);
        }
        float acc = g_next;
        if (t + 1 < T) g_next = g_row[(size_t)(t + 1) * G + j];  // prefetch: latency hidden by the dot
        const float4* hv = reinterpret_cast<const float4*>(sh_h);
#pragma unroll
        for (int i = 0; i < H / 4; ++i) {
            const float4 h4 = hv[i];
            acc = fmaf(w[4 * i], h4.x, acc);
            acc = fmaf(w[4 * i + 1], h4.y, acc);
            acc = fmaf(w[4 * i + 2], h4.z, acc);
            acc = fmaf(w[4 * i + 3], h4.w, acc);
        }
        sh_g[j] = acc;
        __syncthreads();
        if (j < H) {  // PyTorch gate order: i, f, g, o
            const float ig = sigmoid_f(sh_g[j]);
            const float fg = sigmoid_f(sh_g[H + j]);
            const float gg = tanh_f(sh_g[2 * H + j]);
            const float og = sigmoid_f(sh_g[3 * H + j]);
            c = fg * c + ig * gg;
            const float h = og * tanh_f(c);
            sh_h[j] = h;
            if (HEAD) {
                const float p = wave_sum(fmaxf(h, 0.f) * hw);
                if ((j & 63) == 0) sh_red[j >> 6] = p;
            } else {
                out[((size_t)b * T + t) * H + j] = h;
            }
        }
        __syncthreads();
    }
    if (j < H) {
        h_io[(size_t)b * H + j] = sh_h[j];
        c_io[(size_t)b * H + j] = c;
    }
    if (HEAD && j == 0 && T > 0) {
        float s = head_b;
#pragma unroll
        for (int i = 0; i < NW; ++i) s += sh_red[i];
        out[(size_t)b * T + T - 1] = sigmoid_f(s);
    }
}

extern "C" int mxk_lstm_scan(const float* gx, const float* whh, float* h_io, float* c_io, const float* head_w,
                             float head_b, float* out, int B, int T, int H, hipStream_t st) {
    if (B <= 0) return 0;
    const bool head = head_w != nullptr;
#define MX_LSTM(HH)                                                                                         \
    if (H == HH) {                                                                                          \
        if (head)                                                                                           \
            lstm_scan_kernel<HH, true><<<B, 4 * HH, 0, st>>>(gx, whh, h_io, c_io, head_w, head_b, out, T);  \
        else                                                                                                \
            lstm_scan_kernel<HH, false><<<B, 4 * HH, 0, st>>>(gx, whh, h_io, c_io, head_w, head_b, out, T); \
        return (int)hipGetLastError();                                                                      \
    }
    MX_LSTM(64)
    MX_LSTM(128)
#undef MX_LSTM
    return (int)hipErrorInvalidValue;
}

// ---------------------------------------------------------------------------------------------
// WaveNet gate (VITS flows / posterior encoder): out[b, c, t] = tanh(x[b, c, t]) * sigmoid(x[b, H + c, t])
// for x [B, 2H, T] -> out [B, H, T]; one read of each half, float4-vectorised along T when T % 4 == 0.
__global__ __launch_bounds__(256) void wavenet_gate_kernel(const float* __restrict__ x, float* __restrict__ out,
                                                           int H, int T, long total4, int vec) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i >= total4) return;
    if (vec) {
        const long e = i * 4;
        const long bc = e / T;  // b * H + c
        const int t = (int)(e - bc * T);
        const long b = bc / H, c = bc - b * H;
        const float4 a = *reinterpret_cast<const float4*>(x + ((b * 2 * H + c) * T + t));
        const float4 g = *reinterpret_cast<const float4*>(x + ((b * 2 * H + H + c) * T + t));
        float4 o;
        o.x = tanh_f(a.x) * sigmoid_f(g.x);
        o.y = tanh_f(a.y) * sigmoid_f(g.y);
        o.z = tanh_f(a.z) * sigmoid_f(g.z);
        o.w = tanh_f(a.w) * sigmoid_f(g.w);
        *reinterpret_cast<float4*>(out + e) = o;
    } else {
        const long bc = i / T;
        const int t = (int)(i - bc * T);
        const long b = bc / H, c = bc - b * H;
        out[i] = tanh_f(x[(b * 2 * H + c) * T + t]) * sigmoid_f(x[(b * 2 * H + H + c) * T + t]);
    }
}

extern "C" int mxk_wavenet_gate(const float* x, float* out, int B, int H, int T, hipStream_t st) {
    const long n = (long)B * H * T;
    if (n == 0) return 0;
    const int vec = (T % 4) == 0;
    const long work = vec ? n / 4 : n;
    wavenet_gate_kernel<<<(unsigned)((work + 255) / 256), 256, 0, st>>>(x, out, H, T, work, vec);
    return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// lstm_bidir_coop: a bidirectional single-layer LSTM whose hidden size is too large for one workgroup's
// registers (Kokoro / StyleTTS 2: H = 256 -> W_hh is 1 MB fp32). Each direction is spread over NB = H / 16
// workgroups; workgroup b owns hidden units [16 b, 16 b + 16), i.e. the 64 gate rows {i, f, g, o} x 16 of
// W_hh, held in registers (thread = row x quarter of the columns). Per time step every workgroup reads the
// previous h (H floats, L2) from a double-buffered global vector, computes its 64 gate pre-activations
// (+ the precomputed input gates gx = W_ih x_t + b_ih + b_hh), updates its 16 cells and publishes its h
// slice; the direction's workgroups then meet at a grid barrier: agent-scope release + relaxed counter
// ticket, relaxed polling + agent-scope acquire (placement independent, any XCD). The 2 x NB workgroups are
// far below one per CU, so all are co-resident; every spin is bounded (err flag, no hang).
// gx: [ND][T][4H] (direction 1 in original time order), whh: [ND][4H][H], hbuf: [ND][2][H] (parity 0 = h0),
// out: [T][ND H] (forward | backward halves), cnt: [ND] zeroed counters; all fp32 except cnt / err. ND = 1 runs a
// unidirectional layer (EnCodec's decoder LSTM: H = 512 for the 24 kHz codec, 128 W_hh columns per thread in
// registers; H = 1024 for MusicGen's 32 kHz codec, rows split over QS = 8 threads -> 512-thread workgroups, still
// 128 columns per thread).
template <int H>
constexpr int lstm_qs() { return H >= 1024 ? 8 : 4; }
template <int H>
__global__ __launch_bounds__(64 * lstm_qs<H>()) void lstm_bidir_coop_kernel(const float* __restrict__ gx,
                                                                            const float* __restrict__ whh, float* hbuf,
                                                                            float* __restrict__ out, unsigned* cnt,
                                                                            int* err, int T) {
    constexpr int QS = lstm_qs<H>();
    constexpr int NB = H / 16, NC = H / QS;  // workgroups per direction, columns per thread
    const int dir = blockIdx.x / NB, wb = blockIdx.x % NB;
    const int od = (int)(gridDim.x / NB) * H;  // output row stride: ND x H
    const int tid = threadIdx.x, row = tid / QS, q = tid % QS;
    const int grow = (row >> 4) * H + wb * 16 + (row & 15);  // gate (row >> 4), unit (row & 15)
    __shared__ float sg[64];
    float w[NC];
    {
        const float4* wr = reinterpret_cast<const float4*>(whh + ((size_t)dir * 4 * H + grow) * H + q * NC);
#pragma unroll
        for (int i = 0; i < NC / 4; ++i) {
            const float4 v = wr[i];
            w[4 * i] = v.x;
            w[4 * i + 1] = v.y;
            w[4 * i + 2] = v.z;
            w[4 * i + 3] = v.w;
        }
    }
    float c = 0.f;
    const float* g_dir = gx + (size_t)dir * T * 4 * H;
    for (int s = 0; s < T; ++s) {
        const int t = dir == 0 ? s : T - 1 - s;
        const float4* hp = reinterpret_cast<const float4*>(hbuf + (size_t)(dir * 2 + (s & 1)) * H + q * NC);
        float acc = q == 0 ? g_dir[(size_t)t * 4 * H + grow] : 0.f;
#pragma unroll
        for (int i = 0; i < NC / 4; ++i) {
            const float4 h4 = hp[i];
            acc = fmaf(w[4 * i], h4.x, acc);
            acc = fmaf(w[4 * i + 1], h4.y, acc);
            acc = fmaf(w[4 * i + 2], h4.z, acc);
            acc = fmaf(w[4 * i + 3], h4.w, acc);
        }
        acc += __shfl_xor(acc, 1, 64);
        acc += __shfl_xor(acc, 2, 64);
        if constexpr (QS == 8) acc += __shfl_xor(acc, 4, 64);
        if (q == 0) sg[row] = acc;
        __syncthreads();
        if (tid < 16) {  // PyTorch gate order: i, f, g, o
            const float ig = sigmoid_f(sg[tid]), fg = sigmoid_f(sg[16 + tid]);
            const float gg = tanh_f(sg[32 + tid]), og = sigmoid_f(sg[48 + tid]);
            c = fg * c + ig * gg;
            const float h = og * tanh_f(c);
            hbuf[(size_t)(dir * 2 + ((s + 1) & 1)) * H + wb * 16 + tid] = h;
            out[(size_t)t * od + dir * H + wb * 16 + tid] = h;
        }
        if (s + 1 == T) break;
        // grid barrier of this direction's NB workgroups (release -> ticket; poll -> acquire)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_fetch_add(&cnt[dir], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned target = (unsigned)(s + 1) * NB;
            int spins = 0;
            while (__hip_atomic_load(&cnt[dir], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
                __builtin_amdgcn_s_sleep(1);
                if (++spins > (1 << 22)) {  // a workgroup never arrived: flag it and run on (no hang)
                    __hip_atomic_fetch_max(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
    }
}

// LSTM scan of ndir = 1 (unidirectional) or 2 (bidirectional) directions, H in {128, 256, 512, 1024}; the caller zeroes
// cnt / err and fills hbuf parity 0 with h0.
extern "C" int mxk_lstm_coop(const float* gx, const float* whh, float* hbuf, float* out, unsigned* cnt, int* err, int T,
                             int H, int ndir, hipStream_t st) {
    if (T <= 0) return 0;
    if (ndir != 1 && ndir != 2) return (int)hipErrorInvalidValue;
    if (H == 1024) lstm_bidir_coop_kernel<1024><<<ndir * (1024 / 16), 512, 0, st>>>(gx, whh, hbuf, out, cnt, err, T);
    else if (H == 512) lstm_bidir_coop_kernel<512><<<ndir * (512 / 16), 256, 0, st>>>(gx, whh, hbuf, out, cnt, err, T);
    else if (H == 256) lstm_bidir_coop_kernel<256><<<ndir * (256 / 16), 256, 0, st>>>(gx, whh, hbuf, out, cnt, err, T);
    else if (H == 128) lstm_bidir_coop_kernel<128><<<ndir * (128 / 16), 256, 0, st>>>(gx, whh, hbuf, out, cnt, err, T);
    else return (int)hipErrorInvalidValue;
    return (int)hipGetLastError();
}

// Bidirectional LSTM scan (H in {128, 256}); the caller zeroes cnt / err and fills hbuf parity 0 with h0.
extern "C" int mxk_lstm_bidir(const float* gx, const float* whh, float* hbuf, float* out, unsigned* cnt, int* err, int T,
                              int H, hipStream_t st) {
    if (H != 128 && H != 256) return (int)hipErrorInvalidValue;
    return mxk_lstm_coop(gx, whh, hbuf, out, cnt, err, T, H, 2, st);
}
