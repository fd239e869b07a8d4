// qmm3_mx5.hip — qmm3.hip kernel instances for MX5F weights (one translation unit per block format, so
// the instances compile in parallel).
#include "qmm3_impl.h"

int qmm3_run_mx5(int epi, int wm, const uint16_t* A, int lda, const uint8_t* W, int M, int N, int K, int splits, void* C, int ldc, hipStream_t st) {
    return qmm3_run<MXQ_MX5F>(epi, wm, A, lda, W, M, N, K, splits, C, ldc, st);
}
