// qmm2_q2k.hip — qmm2.hip kernel instances for Q2_K weights (one translation unit per block format, so
// the instances compile in parallel).
#include "qmm2_impl.h"

int qmm2_run_q2k(int epi, int wm, int ks, int wn, const uint16_t* A, int lda, const uint8_t* W, int M, int N, int K, int splits, void* C, int ldc, hipStream_t st, const Q2Fuse& fu) {
    return qmm2_run<MXQ_Q2_K>(epi, wm, ks, wn, A, lda, W, M, N, K, splits, C, ldc, st, fu);
}
