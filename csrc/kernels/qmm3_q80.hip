// qmm3_q80.hip — qmm3.hip kernel instances for Q8_0 weights (one translation unit per block format, so
// the instances compile in parallel).
#include "qmm3_impl.h"

int qmm3_run_q80(int epi, int wm, const uint16_t* A, int lda, const uint8_t* W, int M, int N, int K, int splits, void* C, int ldc, hipStream_t st) {
    return qmm3_run<MXQ_Q8_0>(epi, wm, A, lda, W, M, N, K, splits, C, ldc, st);
}
