// qmm3_q4k.hip — qmm3.hip kernel instances for Q4_K weights (one translation unit per block format, so
// the instances compile in parallel).
#include "qmm3_impl.h"

int qmm3_run_q4k(int epi, int wm, const uint16_t* A, int lda, const uint8_t* W, int M, int N, int K, int splits, void* C, int ldc, hipStream_t st) {
    return qmm3_run<MXQ_Q4_K>(epi, wm, A, lda, W, M, N, K, splits, C, ldc, st);
}

int qmm3_dbg_q4k(int dbg, int wm, const uint16_t* A, int lda, const uint8_t* W, int M, int N, int K, void* C, int ldc,
                 hipStream_t st) {
    switch (dbg) {
        case 0: return launch_q3dbg<0>(wm, A, lda, W, M, N, K, C, ldc, st);
        case 1: return launch_q3dbg<1>(wm, A, lda, W, M, N, K, C, ldc, st);
        case 2: return launch_q3dbg<2>(wm, A, lda, W, M, N, K, C, ldc, st);
        case 4: return launch_q3dbg<4>(wm, A, lda, W, M, N, K, C, ldc, st);
        case 8: return launch_q3dbg<8>(wm, A, lda, W, M, N, K, C, ldc, st);
        case 14: return launch_q3dbg<14>(wm, A, lda, W, M, N, K, C, ldc, st);
        case 15: return launch_q3dbg<15>(wm, A, lda, W, M, N, K, C, ldc, st);
        case 12: return launch_q3dbg<12>(wm, A, lda, W, M, N, K, C, ldc, st);
        case 3: return launch_q3dbg<3>(wm, A, lda, W, M, N, K, C, ldc, st);
        case 30: return launch_q3dbg<30>(wm, A, lda, W, M, N, K, C, ldc, st);
        case 31: return launch_q3dbg<31>(wm, A, lda, W, M, N, K, C, ldc, st);
    }
    return (int)hipErrorInvalidValue;
}
