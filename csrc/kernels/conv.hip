// conv.hip — implicit-GEMM 2-D convolution on MFMA for NHWC (channels_last) 16-bit activations
// (UNet / VAE / ControlNet convs, Whisper's conv1d stem as H = 1).
//
//   y[p, co] = act( sum_k W[co, k] * X_im2col[p, k] + bias[co] + tadd[img(p), co] + res[p, co] )
//
// with p = output pixel (n, ho, wo) and k = (kh, kw, ci). The im2col matrix is never materialised:
// every 16-byte chunk of an operand tile (8 channels of one pixel at one filter tap) is fetched straight
// from the NHWC input by `global_load_lds` (LDS-DMA, no VGPR staging), with out-of-image taps pointed
// at a 16-byte zero page, so padding, stride and a fused nearest-2x upsample of the input (the UNet /
// VAE upsamplers: conv(interpolate(x))) cost nothing but address arithmetic.
//
// GEMM orientation: A = weights ([Cout, Kp], Kp = KH*KW*Cp rounded up to the 64-wide k-tile, zero
// padded at pack time), B = pixels, D[cout][pixel] — the 32x32 C/D layout then puts one pixel on each
// lane and 4 consecutive output channels in registers 4g..4g+3, so the epilogue (bias, per-image time
// embedding add, residual add, SiLU) reads / writes 8-byte channel quads of the NHWC output.
//
// Tiles: 4 waves as 2 (cout) x 2 (pixel); each wave TM x TN tiles of 32x32 (mfma_f32_32x32x16 f16/bf16),
// workgroup tile 64*TM couts x 64*TN pixels, k-tile 64 (4 MFMA k-steps). Two LDS stages: the DMA of
// k-tile t+1 is issued before the fragment reads + MFMAs of tile t (one barrier per k-tile). LDS rows
// are 128 B with the chunk index XOR-swizzled by (row >> 1) & 7 on the SOURCE address (the LDS-DMA
// image is lane-linear), so the ds_read_b128 fragment reads are bank-conflict free.
// Grid: cout tiles inner, pixel tiles outer, XCD-aware bijective remap (the cout tiles sharing one
// pixel panel run on one XCD and re-read the input taps from its L2).
#include "mx_common.h"

static constexpr int CV_KT = 64;

struct MxConvP {
    const uint16_t* x;     // [Nb, H, W, Cp]
    const uint16_t* w;     // [Cout, Kp]
    const float* bias;     // [Cout] or null
    const float* tadd;     // [Nb, ldt] fp32 per-image channel add (time embedding) or null
    const uint16_t* res;   // [P, ldr] residual (16-bit) or null
    uint16_t* y;           // [P, ldy]
    const uint16_t* zero;  // >= 16 zero bytes
    int ldt, ldr, ldy;
    int Nb, H, W, Cp, Ho, Wo, Cout, KH, KW, stride, dil, pad_h, pad_w, up, Ktot, Kp, P, n_ct, act;
};

static MX_DEV int cv_off(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }

template <bool F16>
static MX_DEV f32x16 cv_mfma(u32x4 a, u32x4 b, f32x16 c) {
    if constexpr (F16)
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
    else
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

// FASTK: Cp % 64 == 0, so a k-tile never straddles a filter tap (tap is uniform per k-tile)
template <bool F16, int TM, int TN, bool FASTK>
__global__ __launch_bounds__(256) void conv_igemm_kernel(MxConvP p) {
    constexpr int BM = 64 * TM, BN = 64 * TN;
    constexpr int A_BYTES = BM * 128, STAGE = A_BYTES + BN * 128;
    constexpr int AI = BM / 32, BI = BN / 32;  // LDS-DMA wave-instructions per wave per stage (8 rows each)
    extern __shared__ __attribute__((aligned(16))) char smem[];

    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int col = lane & 31, h = lane >> 5;
    const int wm = wave >> 1, wn = wave & 1;

    const int nwg = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    const int ct = lid % p.n_ct, pt = lid / p.n_ct;
    const int co_base = ct * BM, p_base = pt * BN;

    // ---- per-lane source descriptors (k-tile independent) ----
    const uint16_t* wsrc[AI];
#pragma unroll
    for (int i = 0; i < AI; ++i) {
        const int r = (wave * AI + i) * 8 + (lane >> 3);
        const int c = (lane & 7) ^ ((r >> 1) & 7);
        wsrc[i] = p.w + (size_t)min(co_base + r, p.Cout - 1) * p.Kp + c * 8;
    }
    const int HWo = p.Ho * p.Wo;
    const int Hl = p.up ? 2 * p.H : p.H, Wl = p.up ? 2 * p.W : p.W;  // logical (upsampled) input extent
    int hb[BI], wb[BI], nb[BI], kc[BI];
#pragma unroll
    for (int i = 0; i < BI; ++i) {
        const int r = (wave * BI + i) * 8 + (lane >> 3);
        const int pix = p_base + r;
        const int n = pix / HWo, rem = pix - n * HWo;
        const int ho = rem / p.Wo, wo = rem - ho * p.Wo;
        const bool ok = pix < p.P;
        hb[i] = ok ? ho * p.stride - p.pad_h : -(1 << 28);  // rows past P read the zero page
        wb[i] = wo * p.stride - p.pad_w;
        nb[i] = n * p.H;
        kc[i] = ((lane & 7) ^ ((r >> 1) & 7)) * 8;
    }
    auto pix_src = [&](int i, int kh, int kw, int ci) -> const void* {
        // branch-free (a select, not a branch around each DMA): the offset of an out-of-image tap is
        // computed but never dereferenced
        const int hi = hb[i] + kh * p.dil, wi = wb[i] + kw * p.dil;
        const bool ok = (unsigned)hi < (unsigned)Hl && (unsigned)wi < (unsigned)Wl;
        const int hs = p.up ? hi >> 1 : hi, ws = p.up ? wi >> 1 : wi;
        const uint16_t* src = p.x + ((long)(nb[i] + hs) * p.W + ws) * p.Cp + ci;
        return (const void*)(ok ? src : p.zero);
    };

    const int nkt = p.Kp / CV_KT;
    auto issue = [&](int kt, int slot) {
        char* sb = smem + slot * STAGE;
#pragma unroll
        for (int i = 0; i < AI; ++i)
            __builtin_amdgcn_global_load_lds((const void*)(wsrc[i] + kt * CV_KT),
                                             (MX_LDS void*)(sb + (wave * AI + i) * 1024), 16, 0, 0);
        char* bb = sb + A_BYTES;
        if constexpr (FASTK) {
            const int k0 = kt * CV_KT;
            const int tap = k0 / p.Cp, ci0 = k0 - tap * p.Cp;
            const int kh = tap / p.KW, kw = tap - kh * p.KW;
#pragma unroll
            for (int i = 0; i < BI; ++i) {
                // (a call expression as the builtin's pointer argument makes hipcc drop the host stub
                // of this instantiation: keep the named local)
                const void* src = pix_src(i, kh, kw, ci0 + kc[i]);
                __builtin_amdgcn_global_load_lds(src, (MX_LDS void*)(bb + (wave * BI + i) * 1024), 16, 0, 0);
            }
        } else {
#pragma unroll
            for (int i = 0; i < BI; ++i) {
                const int k = kt * CV_KT + kc[i];
                const void* src = (const void*)p.zero;
                if (k < p.Ktot) {
                    const int tap = k / p.Cp, ci = k - tap * p.Cp;
                    const int kh = tap / p.KW, kw = tap - kh * p.KW;
                    src = pix_src(i, kh, kw, ci);
                }
                __builtin_amdgcn_global_load_lds(src, (MX_LDS void*)(bb + (wave * BI + i) * 1024), 16, 0, 0);
            }
        }
    };

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    issue(0, 0);
    __syncthreads();
    int slot = 0;
    for (int kt = 0; kt < nkt; ++kt) {
        if (kt + 1 < nkt) issue(kt + 1, slot ^ 1);
        const char* sa = smem + slot * STAGE;
        const char* sbp = sa + A_BYTES;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            u32x4 af[TM], bf[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) af[i] = *(const u32x4*)(sa + cv_off(wm * 32 * TM + i * 32 + col, 2 * s + h));
#pragma unroll
            for (int j = 0; j < TN; ++j) bf[j] = *(const u32x4*)(sbp + cv_off(wn * 32 * TN + j * 32 + col, 2 * s + h));
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) acc[i][j] = cv_mfma<F16>(af[i], bf[j], acc[i][j]);
        }
        __syncthreads();  // tile kt+1 landed (vmcnt(0)) and every wave is done reading tile kt
        slot ^= 1;
    }

    // ---- epilogue: lane = one pixel, registers 4g..4g+3 = 4 consecutive output channels ----
    const bool vec = (p.Cout & 3) == 0 && (p.ldy & 3) == 0 && (p.res == nullptr || (p.ldr & 3) == 0) &&
                     (p.tadd == nullptr || (p.ldt & 3) == 0);
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int pix = p_base + wn * 32 * TN + j * 32 + col;
        if (pix >= p.P) continue;
        const int img = pix / HWo;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int co0 = co_base + wm * 32 * TM + i * 32 + 8 * g + 4 * h;
                if (co0 >= p.Cout) continue;
                float v[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = acc[i][j][4 * g + e];
                if (vec) {
                    if (p.bias) {
                        const f32x4 b = *(const f32x4*)(p.bias + co0);
#pragma unroll
                        for (int e = 0; e < 4; ++e) v[e] += b[e];
                    }
                    if (p.tadd) {
                        const f32x4 t = *(const f32x4*)(p.tadd + (size_t)img * p.ldt + co0);
#pragma unroll
                        for (int e = 0; e < 4; ++e) v[e] += t[e];
                    }
                    if (p.res) {
                        const u32x2 rr = *(const u32x2*)(p.res + (size_t)pix * p.ldr + co0);
                        float a0, a1, a2, a3;
                        unpack_act2<F16>(rr[0], a0, a1);
                        unpack_act2<F16>(rr[1], a2, a3);
                        v[0] += a0; v[1] += a1; v[2] += a2; v[3] += a3;
                    }
                    if (p.act == 1) {
#pragma unroll
                        for (int e = 0; e < 4; ++e) v[e] = silu_f(v[e]);
                    } else if (p.act == 2) {
#pragma unroll
                        for (int e = 0; e < 4; ++e) v[e] = gelu_erf_f(v[e]);
                    } else if (p.act == 3) {
#pragma unroll
                        for (int e = 0; e < 4; ++e) v[e] = v[e] > 0.f ? v[e] : expm1f(v[e]);
                    } else if (p.act == 4) {
#pragma unroll
                        for (int e = 0; e < 4; ++e) v[e] = v[e] > 0.f ? v[e] : 0.1f * v[e];
                    } else if (p.act == 5) {
#pragma unroll
                        for (int e = 0; e < 4; ++e) v[e] = tanhf(v[e]);
                    }
                    u32x2 o = {pack_act2<F16>(v[0], v[1]), pack_act2<F16>(v[2], v[3])};
                    *(u32x2*)(p.y + (size_t)pix * p.ldy + co0) = o;
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int co = co0 + e;
                        if (co >= p.Cout) break;
                        float t = v[e];
                        if (p.bias) t += p.bias[co];
                        if (p.tadd) t += p.tadd[(size_t)img * p.ldt + co];
                        if (p.res) t += act_to_f32<F16>(p.res[(size_t)pix * p.ldr + co]);
                        if (p.act == 1) t = silu_f(t);
                        else if (p.act == 2) t = gelu_erf_f(t);
                        else if (p.act == 3) t = t > 0.f ? t : expm1f(t);
                        else if (p.act == 4) t = t > 0.f ? t : 0.1f * t;
                        else if (p.act == 5) t = tanhf(t);
                        p.y[(size_t)pix * p.ldy + co] = f32_to_act<F16>(t);
                    }
                }
            }
        }
    }
}

template <bool F16, int TM, int TN, bool FASTK>
static int launch_conv_k(const MxConvP& p, unsigned nwg, hipStream_t st) {
    constexpr int lds = 2 * (64 * TM * 128 + 64 * TN * 128);
    static bool set = false;
    if (!set) {
        (void)hipFuncSetAttribute((const void*)&conv_igemm_kernel<F16, TM, TN, FASTK>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        set = true;
    }
    hipLaunchKernelGGL((conv_igemm_kernel<F16, TM, TN, FASTK>), dim3(nwg), dim3(256), lds, st, p);
    MXK_CHECK_LAUNCH();
}

template <bool F16, int TM, int TN>
static int launch_conv(const MxConvP& p, hipStream_t st) {
    const int n_pt = (p.P + 64 * TN - 1) / (64 * TN);
    const long nwg = (long)p.n_ct * n_pt;
    if (nwg <= 0 || nwg > 0x7fffffff) return (int)hipErrorInvalidValue;
    if (p.Cp % 64 == 0) return launch_conv_k<F16, TM, TN, true>(p, (unsigned)nwg, st);
    return launch_conv_k<F16, TM, TN, false>(p, (unsigned)nwg, st);
}

// Tile configs (tm, tn): 64*tm output channels x 64*tn pixels per workgroup. cfg < 0: auto.
extern "C" int mxk_conv_tile_auto(int P, int Cout) {
    // Largest tile (fewest operand re-reads) whose output-channel padding wastes <= 10 % and whose grid still
    // holds >= 2 workgroups per CU; fitted to tools/bench_conv.py --sweep on MI355X (profiles/r2_conv_sweep.jsonl):
    // SDXL 320-channel levels -> 64x128, 640 @ 64x64 -> 128x64, VAE 128..512 @ >= 128x128 -> 128x128.
    static const int cand[4][2] = {{2, 2}, {2, 1}, {1, 2}, {1, 1}};
    for (const auto& c : cand) {
        const long bm = 64L * c[0], bn = 64L * c[1];
        const long ct = (Cout + bm - 1) / bm, pt = (P + bn - 1) / bn;
        if (ct * bm * 10 <= (long)Cout * 11 && ct * pt >= 512) return c[0] * 16 + c[1];
    }
    return Cout < 64 ? 0x12 : 0x11;  // tiny channel counts (RGB / latent outputs) or small grids
}

// x: [Nb, H, W, Cp] act16 NHWC (Cp % 8 == 0, 16-B aligned); w: [Cout, Kp] act16, k = (kh*KW + kw)*Cp + ci,
// zero for k >= KH*KW*Cp, Kp % 64 == 0; y: [Nb*Ho*Wo, ldy]; res: [Nb*Ho*Wo, ldr] or null; tadd fp32 [Nb, ldt]
// or null; bias fp32 [Cout] or null; up: fused nearest 2x upsample of x; act: 0 none, 1 SiLU, 2 GELU (erf),
// 3 ELU, 4 leaky ReLU (slope 0.1, HiFi-GAN), 5 tanh; dil: filter dilation (both axes).
// zero: >= 16 zero bytes of device memory. cfg: tm*16 + tn, or < 0 for mxk_conv_tile_auto.
extern "C" int mxk_conv2d(const uint16_t* x, int Nb, int H, int W, int Cp, const uint16_t* w, int Cout, int KH, int KW,
                          int Kp, int stride, int dil, int pad_h, int pad_w, int up, int Ho, int Wo, const float* bias,
                          const float* tadd, int ldt, const uint16_t* res, int ldr, uint16_t* y, int ldy, int act,
                          const uint16_t* zero, int cfg, hipStream_t st) {
    if (Nb <= 0 || Ho <= 0 || Wo <= 0 || Cout <= 0) return 0;
    if (Cp % 8 || Kp % CV_KT || Kp < KH * KW * Cp || ((uintptr_t)x & 15) || ((uintptr_t)w & 15) || !zero ||
        stride < 1 || dil < 1 || KH < 1 || KW < 1)
        return (int)hipErrorInvalidValue;
    const long P = (long)Nb * Ho * Wo;
    if (P > 0x7fffffff || (long)Nb * H * W * Cp > 0x7fffffffL * 8) return (int)hipErrorInvalidValue;
    if (cfg < 0) cfg = mxk_conv_tile_auto((int)P, Cout);
    const int tm = cfg >> 4, tn = cfg & 15;
    MxConvP p{x, w, bias, tadd, res, y, zero, ldt, ldr, ldy, Nb, H, W, Cp, Ho, Wo, Cout, KH, KW, stride, dil, pad_h,
            pad_w, up, KH * KW * Cp, Kp, (int)P, (Cout + 64 * tm - 1) / (64 * tm), act};
#define CV_CASE(TM_, TN_)                                                              \
    if (tm == TM_ && tn == TN_) {                                                      \
        MX_ACT_DISPATCH(return launch_conv<F16, TM_, TN_>(p, st));                     \
    }
    CV_CASE(2, 2) CV_CASE(1, 4) CV_CASE(1, 2) CV_CASE(1, 1) CV_CASE(2, 1)
#undef CV_CASE
    return (int)hipErrorInvalidValue;
}

