// qmm2_q6k.hip — qmm2.hip kernel instances for Q6_K weights (one translation unit per block format, so
// the instances compile in parallel).
#include "qmm2_impl.h"

int qmm2_run_q6k(int epi, int wm, int ks, int wn, const uint16_t* A, int lda, const uint8_t* W, int M, int N, int K, int splits, void* C, int ldc, hipStream_t st, const Q2Fuse& fu) {
    return qmm2_run<MXQ_Q6_K>(epi, wm, ks, wn, A, lda, W, M, N, K, splits, C, ldc, st, fu);
}

int qmm2_grouped_q6k(int epi, int wm, const uint16_t* A, int lda, const int* stok, const uint8_t* W, int P, int E, int N,
                     int K, const int* tiles, const int* off, void* C, int ldc, const int* otok, const float* owt,
                     hipStream_t st) {
    return qmm2_grouped_run<MXQ_Q6_K>(epi, wm, A, lda, stok, W, P, E, N, K, tiles, off, C, ldc, otok, owt, st);
}
