// qmm2.hip — quantised-weight GEMM, second generation (M >= 16: mixed continuous-batching steps, prefill).
//
//   C[M, N] (+)= A[M, K] · W[N, K]^T,   A f16, W Q4_K / Q6_K in the t32 tiled layout (ops/quant.py tile32)
//
// Why a second kernel: qmm.hip's profile at M = 256 (profiles/r3_pmc_qmm_gate_up_m256.md) showed the
// MFMA pipe busy only ~31 % of the time with 9-15 VALU + 4-7 SALU + 1.2-1.4 LDS instructions per
// 32-cycle MFMA: the kernel was issue-bound, not memory- or MFMA-bound. Everything here is arranged to
// cut the instructions per MFMA:
//   * wave tile = WM MFMA row blocks x WN 32-column weight groups (the workgroup's 4 groups take 4 / WN
//     waves, WN waves split the BM = 32 WM WN rows): every dequantised B fragment (14 packed-f16 VALU) feeds
//     WM MFMAs and every A fragment read from LDS feeds WN. WN = 1 reads each A fragment from LDS once per
//     MFMA — 1 KB per 32-cycle MFMA, 128 B/clk per CU, the whole LDS read rate (the round-4 isolation runs:
//     with MFMA, dequant and global loads all removed the WN = 1, BM = 256 kernel still took 25 of its 95 us
//     on gate_up M = 256). WN = 2 halves that at twice the dequant VALU per MFMA (still < 4);
//   * the k loop is unrolled over one 256-element super-block (4 k-tiles of 64): the Q4_K / Q6_K scale
//     decode of a k-tile has compile-time sub-block indices (bit-field extracts, exact f16 products), the
//     super-block header is DMA'd and read once per super-block (not once per k-tile), and with a 4-slot
//     ring every LDS address is a per-lane base plus an immediate;
//   * the A tile's LDS image is [8-row block][k-step][row][16-B half], so a k-step's fragment read is the
//     same base + k-step * 256 B for every lane (ds_read_b128, conflict-free by an XOR of the half index
//     with the row block's parity), and each A LDS-DMA wave-instruction still reads 8 whole 128-B rows;
//   * every operand arrives by LDS-DMA (one load kind, so the counted `s_waitcnt vmcnt` is exact) into a
//     4-deep ring; dummy (clamped) stages past the end keep the count uniform, so the loop has no
//     data-dependent branches.
// KS = 2 doubles the waves (two per SIMD): wave pair (kh = 0, 1) shares a column group and splits each
// k-tile's four k-steps; their fp32 partials are summed through LDS before the epilogue.
// Reference parity: llama.cpp's MMQ path for these formats (reached via backend/cpp/llama/grpc-server.cpp:2002
// llama_decode); numerics = f16 dequantised weights x f16 activations, fp32 accumulation.
#include "qmm2_impl.h"
int g_qmm2_rot = 0;

extern "C" int mxk_qmm2_set_rot(int r) {
    g_qmm2_rot = r;
    return 0;
}

// isolation builds of the Q4_K SwiGLU kernel ((wm, ks, wn) = (8, 1, 1), (4, 2, 1), (4, 1, 2), (2, 2, 2); no split),
// see DBG above
extern "C" int mxk_qmm2_dbg(int dbg, int wm, int ks, int wn, const uint16_t* A, int lda, const uint8_t* W, int M, int N,
                            int K, void* C, int ldc, hipStream_t st) {
    return qmm2_dbg_q4k(dbg, wm, ks, wn, A, lda, W, M, N, K, C, ldc, st);
}

// A f16 [M, K] (lda % 8 == 0, 16-B aligned), W t32 Q4_K / Q5_K / Q6_K / Q3_K / Q2_K / Q8_0 / MX4F / MX5F [N, K] (N % 32 == 0, K % 256 == 0).
// epi: 0 fp32 store, 1 f16 store, 2 fp32 accumulate (split-K via atomics when splits > 1), 3/4 SwiGLU /
// GeGLU over 16-row interleaved gate|up -> f16 [M, N/2]. wm: 32-row MFMA blocks per wave; wn: 32-column groups
// per wave (BM = 32 wm wn); ks: 1 (4 waves) or 2 (8 waves, k-steps split per wave pair). splits: K split in
// whole super-blocks.
static int qmm2_go(int qtype, int epi, int wm, int ks, int wn, const uint16_t* A, int lda, const uint8_t* W, int M, int N,
                   int K, int splits, void* C, int ldc, hipStream_t st, const Q2Fuse& fu) {
    if (M <= 0) return 0;
    if (K % 256 || (lda & 7) || ((uintptr_t)A & 15) || ((uintptr_t)W & 15) || (N & 31)) return (int)hipErrorInvalidValue;
    if (epi != E16_ADD_F32 && splits != 1) return (int)hipErrorInvalidValue;
    switch (qtype) {
        case MXQ_Q4_K: return qmm2_run_q4k(epi, wm, ks, wn, A, lda, W, M, N, K, splits, C, ldc, st, fu);
        case MXQ_Q5_K: return qmm2_run_q5k(epi, wm, ks, wn, A, lda, W, M, N, K, splits, C, ldc, st, fu);
        case MXQ_Q6_K: return qmm2_run_q6k(epi, wm, ks, wn, A, lda, W, M, N, K, splits, C, ldc, st, fu);
        case MXQ_Q3_K: return qmm2_run_q3k(epi, wm, ks, wn, A, lda, W, M, N, K, splits, C, ldc, st, fu);
        case MXQ_Q2_K: return qmm2_run_q2k(epi, wm, ks, wn, A, lda, W, M, N, K, splits, C, ldc, st, fu);
        case MXQ_Q8_0: return qmm2_run_q80(epi, wm, ks, wn, A, lda, W, M, N, K, splits, C, ldc, st, fu);
        case MXQ_MX4F: return qmm2_run_mx4(epi, wm, ks, wn, A, lda, W, M, N, K, splits, C, ldc, st, fu);
        case MXQ_MX5F: return qmm2_run_mx5(epi, wm, ks, wn, A, lda, W, M, N, K, splits, C, ldc, st, fu);
    }
    return (int)hipErrorInvalidValue;
}

extern "C" int mxk_qmm2(int qtype, int epi, int wm, int ks, int wn, const uint16_t* A, int lda, const uint8_t* W, int M,
                        int N, int K, int splits, void* C, int ldc, hipStream_t st) {
    return qmm2_go(qtype, epi, wm, ks, wn, A, lda, W, M, N, K, splits, C, ldc, st, Q2Fuse{});
}

// mxk_qmm2 with the RMSNorm split across two GEMMs (Q2Fuse in qmm2_impl.h).
// mode 1 (producer; epi must be 2 = fp32 accumulate into the residual C): ss_out / ss_zero rows of 32 floats
// (ss_zero may be null), gamma [N], xn f16 [M, ldxn] (null: only re-zero ss_zero), tick >= ceil(M / 32) * N / 32
// zeroed counters (left zeroed).
// mode 2 (consumer; any epi): rows scaled by rsqrt(ss_in[32 m] * inv_h + eps) before the epilogue.
extern "C" int mxk_qmm2_fused(int qtype, int epi, int wm, int ks, int wn, const uint16_t* A, int lda, const uint8_t* W,
                              int M, int N, int K, int splits, void* C, int ldc, int mode, float* ss_out, float* ss_zero,
                              const float* gamma, uint16_t* xn, int ldxn, unsigned* tick, const float* ss_in,
                              float inv_h, float eps, hipStream_t st) {
    if (mode == 1 && (epi != E16_ADD_F32 || (xn && (!gamma || !ss_out || !tick || (ldxn < N)))))
        return (int)hipErrorInvalidValue;
    if (mode == 2 && !ss_in) return (int)hipErrorInvalidValue;
    if (mode != 1 && mode != 2) return (int)hipErrorInvalidValue;
    Q2Fuse fu;
    fu.mode = mode;
    fu.ss_out = ss_out;
    fu.ss_zero = ss_zero;
    fu.gamma = gamma;
    fu.xn = xn;
    fu.ldxn = ldxn;
    fu.tick = tick;
    fu.ss_in = ss_in;
    fu.inv_h = inv_h;
    fu.eps = eps;
    return qmm2_go(qtype, epi, wm, ks, wn, A, lda, W, M, N, K, splits, C, ldc, st, fu);
}

// mxk_qmm2_fused plus mode bit 4: RoPE (adjacent pairs over the whole head, D = 1 << dsh in {64, 128}; rot = the
// step's [M][D / 2] (cos, sin) x attn_factor table) and the paged
// bf16 KV append in the q|k|v GEMM's epilogue (Q2Fuse in qmm2_impl.h). epi 0 (splits 1) or 2 (split-K into the
// zeroed fp32 C, left zeroed; tick as mode 1). Columns n_off .. n_off + N of the q|k|v row; qo bf16 [M, hq << dsh];
// kc / vc [blocks][hkv][block_size][D] bf16.
extern "C" int mxk_qmm2_rope(int qtype, int epi, int wm, int ks, int wn, const uint16_t* A, int lda, const uint8_t* W,
                             int M, int N, int K, int splits, void* C, int ldc, int mode, const float* ss_in, float inv_h,
                             float eps, unsigned* tick, const int* slots, const float2* rot, const float* bias,
                             uint16_t* qo, uint16_t* kc, uint16_t* vc, int n_off, int dsh, int hq, int hkv,
                             int block_size, hipStream_t st) {
    if (!(mode & 4) || (mode & 1) || (epi != E16_F32 && epi != E16_ADD_F32) || (dsh != 6 && dsh != 7) || !slots ||
        !rot || !qo || !kc || !vc || block_size <= 0 || (splits > 1 && (epi != E16_ADD_F32 || !tick)) ||
        ((mode & 2) && !ss_in) || (n_off & 31))
        return (int)hipErrorInvalidValue;
    Q2Fuse fu;
    fu.mode = mode;
    fu.ss_in = ss_in;
    fu.inv_h = inv_h;
    fu.eps = eps;
    fu.tick = tick;
    fu.slots = slots;
    fu.rot = rot;
    fu.bias = bias;
    fu.qo = qo;
    fu.kc = kc;
    fu.vc = vc;
    fu.n_off = n_off;
    fu.dsh = dsh;
    fu.hq = hq;
    fu.hkv = hkv;
    fu.block_size = block_size;
    return qmm2_go(qtype, epi, wm, ks, wn, A, lda, W, M, N, K, splits, C, ldc, st, fu);
}

// Grouped MoE GEMM on t32 expert stacks (see Q2Group in qmm2_impl.h): A f16 token rows gathered through stok (or the
// P sorted rows themselves when stok is null), W = E experts' [N, K] t32 matrices back to back, tiles / off from
// mxk_moe_sort with BM = 32 wm; C row r = sorted pair r. epi: 0 fp32 store [P, N], 3 / 4 SwiGLU / GeGLU f16 [P, N/2].
extern "C" int mxk_qmm2_grouped(int qtype, int epi, int wm, const uint16_t* A, int lda, const int* stok, const uint8_t* W,
                                int P, int E, int N, int K, const int* tiles, const int* off, void* C, int ldc,
                                const int* otok, const float* owt, hipStream_t st) {
    if (P <= 0) return 0;
    if (K % 256 || (lda & 7) || ((uintptr_t)A & 15) || ((uintptr_t)W & 15) || (N & 31) || E <= 0)
        return (int)hipErrorInvalidValue;
    switch (qtype) {
        case MXQ_Q4_K: return qmm2_grouped_q4k(epi, wm, A, lda, stok, W, P, E, N, K, tiles, off, C, ldc, otok, owt, st);
        case MXQ_Q5_K: return qmm2_grouped_q5k(epi, wm, A, lda, stok, W, P, E, N, K, tiles, off, C, ldc, otok, owt, st);
        case MXQ_Q6_K: return qmm2_grouped_q6k(epi, wm, A, lda, stok, W, P, E, N, K, tiles, off, C, ldc, otok, owt, st);
        case MXQ_Q8_0: return qmm2_grouped_q80(epi, wm, A, lda, stok, W, P, E, N, K, tiles, off, C, ldc, otok, owt, st);
    }
    return (int)hipErrorInvalidValue;
}
