// qmm2_mx4.hip — qmm2.hip kernel instances for MX4F weights (one translation unit per block format, so
// the instances compile in parallel).
#include "qmm2_impl.h"

int qmm2_run_mx4(int epi, int wm, int ks, int wn, const uint16_t* A, int lda, const uint8_t* W, int M, int N, int K, int splits, void* C, int ldc, hipStream_t st, const Q2Fuse& fu) {
    return qmm2_run<MXQ_MX4F>(epi, wm, ks, wn, A, lda, W, M, N, K, splits, C, ldc, st, fu);
}
