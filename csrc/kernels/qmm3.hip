// qmm3.hip — warp-specialised quantised-weight GEMM (M >= 64: continuous-batching steps, prefill).
//
//   C[M, N] (+)= A[M, K] · W[N, K]^T,   A f16, W Q4_K / Q5_K / Q6_K / Q3_K / Q2_K in the t32 tiled layout
//
// Why a third kernel: qmm2.hip's isolation builds (profiles/r4_qmm2_isolation.md) showed its one-wave-per-SIMD
// instruction stream almost serial: gate_up M = 256 took 88 us, 50 us of it without any MFMA and ~36 us of
// MFMA on top — the MFMA pipe idled whenever its only wave waited on an LDS-DMA count, a barrier, an LDS read
// or the dequant VALU chain, and the dequant (14 packed-f16 VALU per B fragment) was duplicated in every wave
// that shared a column group. Here each workgroup is 8 waves, two per SIMD, with split roles:
//   * 4 producer waves (0-3, one per SIMD): all LDS-DMA (A rows, raw quant bytes, super-block headers) into a
//     3-slot ring, and the dequantisation of ONE column group each into a double-buffered f16 B tile in LDS
//     (each weight decoded once per workgroup; ds_write_b128, lane-linear, conflict-free);
//   * 4 consumer waves (4-7): 2 x 2 over the BM x 128 output tile, (32 WM) rows x 2 groups each, doing only
//     ds_read_b128 of A / B fragments and 32x32x16 f16 MFMAs (WM A + 2 B reads per 2 WM MFMAs).
// One s_barrier per 64-k tile joins the roles: in period t consumers run tile t while producers dequantise
// tile t + 1 (its bytes landed: issued in period t - 1) and issue the DMA of tile t + 2 (slot of tile t - 1,
// released at the previous barrier). A consumer issues the last k-step of tile t's MFMAs AFTER the barrier, so
// they cover the latency of tile t + 1's first fragment reads.
// Same t32 format decoders as qmm2 (qmm2_fmt.h); numerics = f16 dequantised weights x f16 activations, fp32
// accumulation (reference parity: llama.cpp MMQ via backend/cpp/llama/grpc-server.cpp:2002 llama_decode).
#include "qmm3_impl.h"

// isolation builds of the Q4_K SwiGLU kernel (wm 4 / 2, no split), see DBG above
extern "C" int mxk_qmm3_dbg(int dbg, int wm, const uint16_t* A, int lda, const uint8_t* W, int M, int N, int K, void* C,
                            int ldc, hipStream_t st) {
    return qmm3_dbg_q4k(dbg, wm, A, lda, W, M, N, K, C, ldc, st);
}

// A f16 [M, K] (lda % 8 == 0, 16-B aligned), W t32 Q4_K / Q5_K / Q6_K / Q3_K / Q2_K / Q8_0 / MX4F / MX5F [N, K] (N % 32 == 0, K % 256 == 0).
// epi as mxk_qmm2 (split-K only with epi 2). wm: 32-row MFMA blocks per consumer wave, BM = 64 wm (1, 2, 4).
extern "C" int mxk_qmm3(int qtype, int epi, int wm, const uint16_t* A, int lda, const uint8_t* W, int M, int N, int K,
                        int splits, void* C, int ldc, hipStream_t st) {
    if (M <= 0) return 0;
    if (K % 256 || (lda & 7) || ((uintptr_t)A & 15) || ((uintptr_t)W & 15) || (N & 31)) return (int)hipErrorInvalidValue;
    if (epi != E16_ADD_F32 && splits != 1) return (int)hipErrorInvalidValue;
    switch (qtype) {
        case MXQ_Q4_K: return qmm3_run_q4k(epi, wm, A, lda, W, M, N, K, splits, C, ldc, st);
        case MXQ_Q5_K: return qmm3_run_q5k(epi, wm, A, lda, W, M, N, K, splits, C, ldc, st);
        case MXQ_Q6_K: return qmm3_run_q6k(epi, wm, A, lda, W, M, N, K, splits, C, ldc, st);
        case MXQ_Q3_K: return qmm3_run_q3k(epi, wm, A, lda, W, M, N, K, splits, C, ldc, st);
        case MXQ_Q2_K: return qmm3_run_q2k(epi, wm, A, lda, W, M, N, K, splits, C, ldc, st);
        case MXQ_Q8_0: return qmm3_run_q80(epi, wm, A, lda, W, M, N, K, splits, C, ldc, st);
        case MXQ_MX4F: return qmm3_run_mx4(epi, wm, A, lda, W, M, N, K, splits, C, ldc, st);
        case MXQ_MX5F: return qmm3_run_mx5(epi, wm, A, lda, W, M, N, K, splits, C, ldc, st);
    }
    return (int)hipErrorInvalidValue;
}
