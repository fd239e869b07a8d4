// lds_stage_bench.hip — global -> LDS staging throughput on one MI355X: LDS-DMA (global_load_lds, 16 B per lane)
// against plain 16-byte global loads into VGPRs followed by ds_write_b128, the two ways the quantised GEMMs can
// stage their A operand. Each workgroup streams `iters` 64-k A tiles of `rows` rows (rows x 128 B each) from a
// buffer that stays L2-resident, as the GEMM's column workgroups re-read the shared activation rows.
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/lds_stage_bench tools/lds_stage_bench.hip && /tmp/lds_stage_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define LDS_AS __attribute__((address_space(3)))

template <int ROWS, int MODE, int NW>
__global__ __launch_bounds__(64 * NW) void stage_kernel(const uint4* __restrict__ src, int tiles_in_buf, int iters,
                                                         unsigned* __restrict__ sink) {
    constexpr int TILE = ROWS * 128;           // bytes per 64-k tile of ROWS rows
    constexpr int PER_WAVE = TILE / 1024 / NW;  // 1 KB wave-instructions per wave per tile
    __shared__ __attribute__((aligned(16))) char lds[2 * TILE];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    unsigned acc = 0;
    for (int it = 0; it < iters; ++it) {
        const int t = (it + blockIdx.x) % tiles_in_buf;
        const char* base = (const char*)src + (size_t)t * TILE;
        char* dst = lds + (it & 1) * TILE;
        if constexpr (MODE == 0) {
#pragma unroll
            for (int i = 0; i < PER_WAVE; ++i) {
                const int off = (wave * PER_WAVE + i) * 1024;
                __builtin_amdgcn_global_load_lds((const void*)(base + off + 16 * lane), (LDS_AS void*)(dst + off), 16, 0,
                                                 0);
            }
            __builtin_amdgcn_s_waitcnt(0);
        } else {
            uint4 v[PER_WAVE];
#pragma unroll
            for (int i = 0; i < PER_WAVE; ++i) v[i] = *(const uint4*)(base + (wave * PER_WAVE + i) * 1024 + 16 * lane);
#pragma unroll
            for (int i = 0; i < PER_WAVE; ++i) *(uint4*)(dst + (wave * PER_WAVE + i) * 1024 + 16 * lane) = v[i];
        }
        __syncthreads();
        acc += *(const unsigned*)(dst + 4 * lane);
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

template <int ROWS, int MODE, int NW>
static double run(const uint4* buf, int tiles_in_buf, int iters, unsigned* sink, int nwg) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    stage_kernel<ROWS, MODE, NW><<<nwg, 64 * NW>>>(buf, tiles_in_buf, iters, sink);
    hipEventRecord(a);
    for (int r = 0; r < 5; ++r) stage_kernel<ROWS, MODE, NW><<<nwg, 64 * NW>>>(buf, tiles_in_buf, iters, sink);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0.f;
    hipEventElapsedTime(&ms, a, b);
    const double bytes = 5.0 * nwg * (double)iters * ROWS * 128;
    return bytes / (ms * 1e-3) / 1e12;  // TB/s aggregate into LDS
}

int main() {
    const int tiles = 64;  // 64 tiles of up to 256 rows x 128 B = 2 MB: L2-resident
    uint4* buf;
    unsigned* sink;
    hipMalloc(&buf, (size_t)tiles * 256 * 128);
    hipMemset(buf, 1, (size_t)tiles * 256 * 128);
    hipMalloc(&sink, 4);
    const int nwg = 256, iters = 2000;
    printf("{\"what\": \"global->LDS staging, 256 WGs, L2-resident source\", \"unit\": \"TB/s aggregate\", \"results\": {");
    printf("\"dma_rows128_w4\": %.2f, ", run<128, 0, 4>(buf, tiles, iters, sink, nwg));
    printf("\"vgpr_rows128_w4\": %.2f, ", run<128, 1, 4>(buf, tiles, iters, sink, nwg));
    printf("\"dma_rows256_w8\": %.2f, ", run<256, 0, 8>(buf, tiles, iters, sink, nwg));
    printf("\"vgpr_rows256_w8\": %.2f, ", run<256, 1, 8>(buf, tiles, iters, sink, nwg));
    printf("\"dma_rows128_w8\": %.2f, ", run<128, 0, 8>(buf, tiles, iters, sink, nwg));
    printf("\"vgpr_rows128_w8\": %.2f", run<128, 1, 8>(buf, tiles, iters, sink, nwg));
    printf("}}\n");
    hipFree(buf);
    hipFree(sink);
    return 0;
}
