// qmm2_q4k.hip — qmm2.hip kernel instances for Q4_K weights (one translation unit per block format, so
// the instances compile in parallel).
#include "qmm2_impl.h"

int qmm2_run_q4k(int epi, int wm, int ks, int wn, const uint16_t* A, int lda, const uint8_t* W, int M, int N, int K, int splits, void* C, int ldc, hipStream_t st, const Q2Fuse& fu) {
    return qmm2_run<MXQ_Q4_K>(epi, wm, ks, wn, A, lda, W, M, N, K, splits, C, ldc, st, fu);
}

int qmm2_dbg_q4k(int dbg, int wm, int ks, int wn, const uint16_t* A, int lda, const uint8_t* W, int M, int N, int K, void* C,
                 int ldc, hipStream_t st) {
    switch (dbg) {
        case 0: return launch_dbg<0>(wm, ks, wn, A, lda, W, M, N, K, C, ldc, st);
        case 1: return launch_dbg<1>(wm, ks, wn, A, lda, W, M, N, K, C, ldc, st);
        case 2: return launch_dbg<2>(wm, ks, wn, A, lda, W, M, N, K, C, ldc, st);
        case 3: return launch_dbg<3>(wm, ks, wn, A, lda, W, M, N, K, C, ldc, st);
        case 4: return launch_dbg<4>(wm, ks, wn, A, lda, W, M, N, K, C, ldc, st);
        case 8: return launch_dbg<8>(wm, ks, wn, A, lda, W, M, N, K, C, ldc, st);
        case 12: return launch_dbg<12>(wm, ks, wn, A, lda, W, M, N, K, C, ldc, st);
        case 15: return launch_dbg<15>(wm, ks, wn, A, lda, W, M, N, K, C, ldc, st);
    }
    return (int)hipErrorInvalidValue;
}

int qmm2_grouped_q4k(int epi, int wm, const uint16_t* A, int lda, const int* stok, const uint8_t* W, int P, int E, int N,
                     int K, const int* tiles, const int* off, void* C, int ldc, const int* otok, const float* owt,
                     hipStream_t st) {
    return qmm2_grouped_run<MXQ_Q4_K>(epi, wm, A, lda, stok, W, P, E, N, K, tiles, off, C, ldc, otok, owt, st);
}
