// allreduce.hip — one-shot all-reduce for small tensor-parallel messages (<= ~1 MB: the two row-parallel
// partial sums per decode layer) over hipIpc-mapped peer buffers on xGMI, instead of an RCCL ring whose
// per-hop latency dominates at these sizes (SURVEY §5 "distributed communication backend").
//
// Protocol ("data is the flag", 8-byte granules): every rank PUSHES each pair of its 16-bit partials to
// every rank (itself included) as one 8-byte system-scope atomic store {tag = epoch, 2 x 16-bit payload}
// into slot [parity][src rank] of the destination's receive buffer (uncached device memory, so a remote
// xGMI write is seen by the owner's polling loads without any fence); then each rank polls its OWN
// receive slots until every granule carries this call's tag and sums them in fp32. No separate flag, no
// barrier: a granule is complete when its tag matches.
//  * epoch lives in device memory (epoch_ctr[0], read at kernel start) and the last workgroup to finish bumps it
//    (ticket in epoch_ctr[1]: every workgroup has read the epoch before it takes its ticket), so a captured hipGraph
//    replays correctly with ONE launch per all-reduce; epoch >= 1, the buffers are zeroed at allocation;
//  * two parity halves: a rank can only start call e+2 (writing parity e%2 again) after it received
//    every peer's call-e+1 data, which each peer pushes only after finishing its call-e reads;
//  * spins are bounded: a peer that never arrives sets *err and the kernel exits (the host raises).
// Grid: <= 128 workgroups (all resident, so no cross-rank scheduling dependency), grid-stride granules.
#include "mx_common.h"

#define MX_AR_MAX_WORLD 8

struct MxArPeers {
    unsigned long long* recv[MX_AR_MAX_WORLD];  // peer receive buffers (IPC-mapped; [rank] = local)
};

// RES: instead of writing the 16-bit sum, add it into an fp32 residual stream (res[2i], res[2i+1]) — the
// row-parallel projection's all-reduce and the residual add in one pass.
template <bool F16, bool RES>
__global__ __launch_bounds__(256) void allreduce_1shot_kernel(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                              int ng, int rank, int world, MxArPeers peers,
                                                              long slot_granules, uint32_t* epoch_ctr,
                                                              int* err, float2* __restrict__ res) {
    const uint32_t epoch = __hip_atomic_load(epoch_ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
    const long par = epoch & 1u;
    const int stride = gridDim.x * blockDim.x;
    // phase 1: push this rank's granules to every rank's slot [par][rank]
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < ng; i += stride) {
        const unsigned long long g = ((unsigned long long)epoch << 32) | in[i];
        for (int p = 0; p < world; ++p) {
            unsigned long long* dst = peers.recv[p] + (par * world + rank) * slot_granules + i;
            __hip_atomic_store(dst, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    // phase 2: gather every rank's granule i from the local receive buffer, sum in fp32
    unsigned long long* local = peers.recv[rank];
    bool dead = false;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < ng && !dead; i += stride) {
        float a = 0.f, b = 0.f;
        for (int p = 0; p < world; ++p) {
            unsigned long long* src = local + (par * world + p) * slot_granules + i;
            unsigned long long g = __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            unsigned spins = 0;
            while ((uint32_t)(g >> 32) != epoch) {
                if (++spins > (1u << 22)) {  // ~seconds: a dead peer, not a slow one
                    __hip_atomic_fetch_max(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    dead = true;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
                g = __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            if (dead) break;
            float lo, hi;
            unpack_act2<F16>((uint32_t)g, lo, hi);
            a += lo;
            b += hi;
        }
        if (dead) break;
        if constexpr (RES) {
            float2 r = res[i];
            r.x += a;
            r.y += b;
            res[i] = r;
        } else {
            out[i] = pack_act2<F16>(a, b);
        }
    }
    // the last workgroup to get here bumps the epoch for the next call and re-arms the ticket. Relaxed atomics: the
    // ticket only has to order the epoch reads (every workgroup read it before taking a ticket); no plain data is
    // published through it, so no release fence (on gfx950 an agent-scope release writes back the whole L2)
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t t = __hip_atomic_fetch_add(epoch_ctr + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (t == gridDim.x - 1) {
            __hip_atomic_store(epoch_ctr + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(epoch_ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// ---- host side ----------------------------------------------------------------------------------
// Receive buffer: 2 parities x world slots x slot_granules 8-byte granules, uncached device memory.
extern "C" int mxk_ar_alloc(size_t bytes, void** ptr) {
    hipError_t e = hipExtMallocWithFlags(ptr, bytes, hipDeviceMallocUncached);
    if (e != hipSuccess) return (int)e;
    return (int)hipMemset(*ptr, 0, bytes);
}
extern "C" int mxk_ar_free(void* ptr) { return (int)hipFree(ptr); }
extern "C" int mxk_ar_ipc_handle(void* ptr, void* out /* 64 B */) {
    return (int)hipIpcGetMemHandle((hipIpcMemHandle_t*)out, ptr);
}
extern "C" int mxk_ar_ipc_open(const void* handle /* 64 B */, void** ptr) {
    hipIpcMemHandle_t h;
    __builtin_memcpy(&h, handle, sizeof(h));
    return (int)hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess);
}
extern "C" int mxk_ar_ipc_close(void* ptr) { return (int)hipIpcCloseMemHandle(ptr); }
extern "C" int mxk_ar_handle_size() { return (int)sizeof(hipIpcMemHandle_t); }

// in/out: n 16-bit elements (n even, 4-B aligned; out may alias in); peers: world receive-buffer pointers
// (host array; [rank] = this rank's own buffer); slot_granules >= n / 2; epoch_ctr: 2 device words {epoch,
// ticket}, zeroed once; err: device word.
extern "C" int mxk_allreduce_1shot(const uint16_t* in, uint16_t* out, int n, int rank, int world,
                                   unsigned long long* const* peers, long slot_granules, uint32_t* epoch_ctr,
                                   int* err, hipStream_t st) {
    if (n <= 0) return 0;
    if ((n & 1) || world < 1 || world > MX_AR_MAX_WORLD || rank < 0 || rank >= world || (long)(n / 2) > slot_granules ||
        ((uintptr_t)in & 3) || ((uintptr_t)out & 3))
        return (int)hipErrorInvalidValue;
    MxArPeers pp{};
    for (int p = 0; p < world; ++p) pp.recv[p] = peers[p];
    const int ng = n / 2;
    int blocks = (ng + 255) / 256;
    if (blocks > 128) blocks = 128;
    MX_ACT_DISPATCH((allreduce_1shot_kernel<F16, false><<<blocks, 256, 0, st>>>(
        (const uint32_t*)in, (uint32_t*)out, ng, rank, world, pp, slot_granules, epoch_ctr, err, nullptr)));
    MXK_CHECK_LAUNCH();
}

// same, but res (fp32, n elements, 8-B aligned) += the sum; `in` is not overwritten.
extern "C" int mxk_allreduce_1shot_add(const uint16_t* in, float* res, int n, int rank, int world,
                                       unsigned long long* const* peers, long slot_granules, uint32_t* epoch_ctr,
                                       int* err, hipStream_t st) {
    if (n <= 0) return 0;
    if ((n & 1) || world < 1 || world > MX_AR_MAX_WORLD || rank < 0 || rank >= world || (long)(n / 2) > slot_granules ||
        ((uintptr_t)in & 3) || ((uintptr_t)res & 7))
        return (int)hipErrorInvalidValue;
    MxArPeers pp{};
    for (int p = 0; p < world; ++p) pp.recv[p] = peers[p];
    const int ng = n / 2;
    int blocks = (ng + 255) / 256;
    if (blocks > 128) blocks = 128;
    MX_ACT_DISPATCH((allreduce_1shot_kernel<F16, true><<<blocks, 256, 0, st>>>(
        (const uint32_t*)in, nullptr, ng, rank, world, pp, slot_granules, epoch_ctr, err, (float2*)res)));
    MXK_CHECK_LAUNCH();
}
