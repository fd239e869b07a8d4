// qmm2_impl.h — kernel templates of qmm2.hip (see there), shared by the per-format translation units.
#pragma once
#include "qmm2_fmt.h"

extern int g_qmm2_rot;  // k-order rotation multiplier per column tile (0: natural order), mxk_qmm2_set_rot

// RMSNorm fused across two GEMMs (M > 4 dense layers: o_proj -> gate|up, down -> next qkv). rmsnorm(x) W^T =
// diag(1 / rms(x)) ((x * g) W^T), so the norm splits into
//   mode 1, the producer (E16_ADD_F32 into the fp32 residual): once a 32-row x 32-column block of the residual is
//     final (splits == 1, or the last of its K splits by a relaxed per-block ticket), its wave writes
//     xn = f16(x * g) (the next GEMM's A operand) and adds the rows' partial sums of squares into ss_out
//     (one 128-byte line per row); workgroup 0 re-zeroes ss_zero (the buffer the previous consumer read);
//   mode 2, the consumer (any epilogue): scales its fp32 accumulators by rsqrt(ss_in[m] * inv_h + eps) per row
//     before the epilogue (SwiGLU's gate and up alike: the scale is linear in both).
// That removes the standalone rmsnorm launches between them (profiles/r6_norm_fusion.md).
struct Q2Fuse {
    int mode = 0;
    float* ss_out = nullptr;
    float* ss_zero = nullptr;
    const float* gamma = nullptr;
    uint16_t* xn = nullptr;
    int ldxn = 0;
    unsigned* tick = nullptr;
    const float* ss_in = nullptr;
    float inv_h = 0.f;
    float eps = 0.f;
    // mode bit 4, the qkv GEMM (E16_F32, or E16_ADD_F32 split-K into the zeroed qkv buffer): RoPE (adjacent pairs,
    // rot_dim = D) and the paged KV append in the epilogue instead of a rope_kv launch; split-K blocks are summed by
    // the last split (ticket, as mode 1), which re-zeroes them. Column n_off + n of the q|k|v row is head
    // (n_off + n) >> dsh.
    const int* slots = nullptr;
    const float2* rot = nullptr;  // [M][D / 2] (cos, sin) x attn_factor of each row's position (one table per step)
    const float* bias = nullptr;
    uint16_t* qo = nullptr;
    uint16_t* kc = nullptr;
    uint16_t* vc = nullptr;
    int n_off = 0, dsh = 7, hq = 0, hkv = 0, block_size = 16;
};
constexpr int Q2F_SS_STRIDE = 32;  // floats between rows of ss_out / ss_in

namespace {

// 16 agent-coherent (sc1) loads in flight at once and one wait: the relaxed __hip_atomic_load form waits for each
// load before issuing the next (measured: +10-40 us per GEMM for a 32 x 128 block per wave). Rows past M load row
// M - 1 (the caller ignores them).
MX_DEV void q2_ld16_sc1(float (&v)[16], const float* base, size_t ld, int m0, int M) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const float* p = base + (size_t)min(m0 + 8 * (r >> 2) + (r & 3), M - 1) * ld;
        asm volatile("global_load_dword %0, %1, off sc1" : "=v"(v[r]) : "v"(p) : "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)"
                 : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7]),
                   "+v"(v[8]), "+v"(v[9]), "+v"(v[10]), "+v"(v[11]), "+v"(v[12]), "+v"(v[13]), "+v"(v[14]), "+v"(v[15])
                 :
                 : "memory");
}

// NS: ring slots (k-tiles of 64): 4, or 8 for the 64-row tiles ("deep ring", ks | 8 in mxk_qmm2) — a 64-row
// stage is only 12-14 KB, and with 4 slots a workgroup keeps ~2 stages (24 KB) in flight: at the ~1.1 us
// issue -> landed latency of LDS-DMA under load that caps the CU at ~30 GB/s, which is what the narrow
// projections measured (qkv M = 256: 768 KB per workgroup in 25 us). 8 slots keep 6 stages in flight.
// NG: 32-column groups per workgroup — 4 (128 columns, 4 KS waves), or 8 (256 columns, 8 waves, KS = 1: "wide"
// tiles). The A tile is staged once per workgroup and read by every column group, so the A bytes a CU stages per
// MFMA flop are 1 / (32 NG): the wide tile halves the activation staging that caps large-M GEMMs
// (tools/lds_stage_bench.hip: ~13-19 TB/s of L2 -> LDS staging for the whole chip).
// GPW: column groups each wave stages (and, with WN = GPW, computes): 1, or 2 for the 4-wave wide form whose
// waves cover 64 columns each (one wave per SIMD, all of its registers; the A fragments it reads from LDS serve
// twice the MFMAs)
template <int QT, int WM, int KS, int WN, int NS = 4, int NG = 4, int GPW = 1>
struct Q2Geom {
    using F = Q2F<QT>;
    static_assert(NG == 4 || (NG == 8 && KS == 1), "wide tiles: 8 waves, one per column group");
    static_assert(GPW == 1 || (NG == 8 && WN == 2), "2 groups per wave: the 4-wave wide form");
    static constexpr int BM = GPW == 2 ? 32 * WM : 32 * WM * WN;
    static constexpr int NT = NG == 8 ? 8 / GPW : 4 * KS;   // waves
    static constexpr int A_BYTES = BM * 128;          // one 64-k tile of A
    static constexpr int STAGE = A_BYTES + NG * F::QB; // A + the column groups' quant bytes
    static constexpr int HSZ = NG * F::HB;            // one super-block header slot (NG groups)
    static constexpr int NH = NS >= 6 ? 3 : 2;         // header slots: super-blocks live at once (stages kt .. kt+NS-1)
    static constexpr int LDS = NS * STAGE + NH * HSZ;
    // A LDS-DMA instructions per wave per stage (rounded up: with BM / 8 not a multiple of NT the last wave's spare
    // instructions re-load the tile's last 8-row block into its own slot, identical bytes)
    static constexpr int WA = (BM / 8 + NT - 1) / NT;
    // LDS-DMA instructions per stage of a weight-loading wave (kh == 0) / an A-only wave, by the stage's
    // position in its super-block (JQ == 0 stages also carry the header)
    template <int JQ, bool WL>
    static constexpr int cnt() { return WA + (WL ? GPW * (F::QI + (JQ == 0 ? F::HI : 0)) : 0); }
};


// per-k-step issue schedule: each MFMA followed by one LDS read (the first NDS) and up to NV VALU, so the next
// k-step's fragment reads leave early and the dequant VALU fills the MFMA shadows
constexpr int Q2_VPM = 5;
template <int I, int NM, int NDS, int NV>
MX_DEV void q2_interleave() {
    if constexpr (I < NM) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        if constexpr (I < NDS) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, NV, 0);
        q2_interleave<I + 1, NM, NDS, NV>();
    }
}

// Q2_AEARLY 1: the next k-step's A fragments are read at the TOP of a k-step (all WM reads back to back, then the
// k-step's MFMAs with the dequant VALU in their shadows) instead of one read after each MFMA (0, default). Same-box
// A/B with the asm LDS-DMA (counted lgkmcnt waits either way): within 1 % on every projection, and 0 needs 20
// fewer VGPRs (profiles/r6_qmm2_asm_dma.md)
#ifndef Q2_AEARLY
#define Q2_AEARLY 0
#endif
template <int I, int NM, int NV>
MX_DEV void q2_interleave_mfma() {
    if constexpr (I < NM) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, NV, 0);
        q2_interleave_mfma<I + 1, NM, NV>();
    }
}

// outstanding LDS-DMA instructions of NN consecutive stages from super-block position J0 (a stage: WAI A pieces,
// plus QII quant pieces and, at position 0, HII header pieces for a weight-loading wave)
template <int WAI, int QII, int HII, bool WL, int J0, int NN>
constexpr int q2_cnt_run() {
    int c = 0;
    for (int d = 0; d < NN; ++d) c += WAI + (WL ? QII + (((J0 + d) & 3) == 0 ? HII : 0) : 0);
    return c;
}

// Grouped (mixture-of-experts) mode, GR = true: the rows are token-expert pairs sorted by expert (ops/moe.py,
// moe.hip moe_sort: off[e] .. off[e + 1] are expert e's rows, tiles[e] its first row tile of BM rows), W holds the
// experts' [N, K] t32 matrices back to back (expert e = column groups e N / 32 ..), and A row r is A[stok[r]] (the
// token's normed hidden state; stok == nullptr: A[r], the gate|up activations of pair r for the down projection).
// Output row r is pair r's. The grid covers the maximum row-tile count (P / BM + E, independent of the routing, so a
// captured graph replays any routing); workgroups past tiles[E] exit at once.
struct Q2Group {
    const int* tiles;
    const int* off;
    const int* stok;
    int E;
    // E16_ADD_F32 in grouped mode (the down projection with the MoE combine fused): sorted row r adds
    // owt[r] * its output row into C row otok[r] (the token's residual), fp32 atomics (rows of one token come from
    // different experts' tiles)
    const int* otok = nullptr;
    const float* owt = nullptr;
};


// DBG (isolation builds, tools/prof_qmm.py --q2dbg): 1 no MFMA, 2 no dequant VALU, 4 no A loads, 8 no weight loads
template <int QT, int WM, int KS, int WN, int EPI, int DBG = 0, int NS = 4, int NG = 4, int GPW = 1, bool GR = false,
          bool FU = false>
__global__ __launch_bounds__(NG == 8 ? 512 / GPW : 256 * KS) void qmm2_kernel(const uint16_t* __restrict__ A, int lda,
                                                        const uint8_t* __restrict__ W, int M, int N, int K,
                                                        int n_mt, int splits, int sbps, void* __restrict__ Cv,
                                                        int ldc, int rot_mul, Q2Group grp, Q2Fuse fu = Q2Fuse{}) {
    using G = Q2Geom<QT, WM, KS, WN, NS, NG, GPW>;
    using F = Q2F<QT>;
    constexpr int BM = G::BM, WA = G::WA, STAGE = G::STAGE, A_BYTES = G::A_BYTES;
    static_assert(NS >= 4 && NS <= 8, "ring depth");
    static_assert(WN == 1 || WN == 2, "WN");
    static_assert(KS == 1 || 4 * WM * WN * 16 * 64 * 4 <= G::LDS, "KS = 2 partials fit in the ring");
    static_assert(WA >= 1 && WA * 8 * G::NT >= BM && (WA - 1) * 8 * G::NT < BM, "A tile split");
    static_assert(G::LDS <= 160 * 1024, "LDS");
    static_assert((NS - 2) * G::template cnt<0, true>() <= 63, "vmcnt range");
    // LDS-DMA instructions per stage as issued (the isolation builds drop some)
    constexpr int WAI = (DBG & 4) ? 0 : WA, QII = (DBG & 8) ? 0 : GPW * F::QI, HII = (DBG & 8) ? 0 : GPW * F::HI;
    auto cnt = [](auto jq_c, auto wl_c) constexpr {
        return WAI + (decltype(wl_c)::value ? QII + (decltype(jq_c)::value == 0 ? HII : 0) : 0);
    };
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* const hdr_lds = smem + NS * STAGE;
    // ring slot of k-tile ki = ki % NS; header slot of super-block v = v % NH
    auto hslot_of = [](int v) { return G::NH == 3 ? v % 3 : v & 1; };

    // wave index as a scalar: every LDS-DMA destination (M0) and weight pointer below is then SGPR math
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int h = lane >> 5, col = lane & 31;
    // cg: the column group this wave DMAs; (mw, nw): its compute tile = rows mw * 32 WM .., groups nw * WN + j
    const int cg = wave % NG, kh = NG == 8 ? 0 : wave >> 2;  // (GPW 2: cg = wave, staging groups 2 cg, 2 cg + 1)
    constexpr int NW = NG / WN;
    const int nw = cg % NW, mw = cg / NW;

    // XCD-aware bijective remap: consecutive logical ids (the row tiles and splits of one column panel)
    // run on one XCD and share its L2
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    const int mt = lid % n_mt;
    const int rest = lid / n_mt;
    const int split = rest % splits;
    const int ct = rest / splits;

    const int nsb = K >> 8;
    const int sb0 = split * sbps, sb1 = min(sb0 + sbps, nsb);
    if (sb0 >= sb1) return;
    int m_base = mt * BM;
    const int ngrp = N >> 5;
    size_t g_base = 0;  // grouped: the expert's first column group
    if constexpr (GR) {
        const int tot = grp.tiles[grp.E];
        if (mt >= tot) return;
        int lo = 0, hi = grp.E - 1;  // the expert e with tiles[e] <= mt < tiles[e + 1]
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (grp.tiles[mid] <= mt) lo = mid;
            else hi = mid - 1;
        }
        m_base = grp.off[lo] + (mt - grp.tiles[lo]) * BM;
        M = grp.off[lo + 1];  // rows of this tile: m_base .. min(m_base + BM, M)
        g_base = (size_t)lo * ngrp;
    }
    const int g = min(ct * NG + GPW * cg, ngrp - 1);  // groups past N re-read the last (never stored)
    const uint8_t* wg = W + (g_base + g) * ((size_t)nsb * F::UNIT);
    [[maybe_unused]] const uint8_t* wg2 =
        W + (g_base + min(ct * NG + GPW * cg + 1, ngrp - 1)) * ((size_t)nsb * F::UNIT);

    // A LDS-DMA sources: instruction i of this wave fills 8-row block j = wave * WA + i; lane p writes
    // image slot (k-step p >> 4, row (p >> 1) & 7, half (p & 1) ^ (j & 1)) from 16 B of that row
    uint32_t aoff[WA];
#pragma unroll
    for (int i = 0; i < WA; ++i) {
        const int j = min(wave * WA + i, BM / 8 - 1);
        const int s = lane >> 4, r8 = (lane >> 1) & 7, hh = (lane & 1) ^ (j & 1);
        int row = min(m_base + 8 * j + r8, M - 1);
        if constexpr (GR) {
            if (grp.stok) row = grp.stok[row];
        }
        aoff[i] = (uint32_t)(row * lda + 16 * s + 8 * hh);
    }
    // per-lane fragment read bases (byte offsets within a stage)
    const int rb = col >> 3;
    const uint32_t a_rd = (uint32_t)(mw * WM * 4096 + rb * 1024 + (col & 7) * 32 + ((h ^ (rb & 1)) << 4));
    const uint32_t b_rd = (uint32_t)(A_BYTES + nw * WN * F::QB);  // + j * QB for the wave's group j
    const int hg = nw * WN * F::HB;                                 // header offset of group nw * WN

    // stage issue: the A rows of k-tile `kta` and (weight waves) the quant bytes of super-block `sbw`,
    // quarter JQ, into ring slot `slot`; JQ == 0 stages also bring that super-block's header into header slot
    // `hslot`. Dummy stages past the end pass clamped (valid, never consumed) sources.
    auto issue = [&](int kta, int sbw, int slot, int hslot, auto jq_c, auto wl_c) {
        constexpr int JQ = decltype(jq_c)::value;
        char* sb = smem + slot * STAGE;
        const uint16_t* ak = A + (size_t)kta * 64;
#pragma unroll
        for (int i = 0; i < WAI; ++i)
            q2_dma((const void*)(ak + aoff[i]), (MX_LDS void*)(sb + min(wave * WA + i, BM / 8 - 1) * 1024), 16);
        if constexpr (decltype(wl_c)::value && QII > 0) {
            const uint8_t* u = wg + (size_t)sbw * F::UNIT;
            q2_stage_weights<QT, JQ>(u, sb + A_BYTES + GPW * cg * F::QB, hdr_lds + hslot * G::HSZ + GPW * cg * F::HB,
                                     lane);
            if constexpr (GPW == 2)
                q2_stage_weights<QT, JQ>(wg2 + (size_t)sbw * F::UNIT, sb + A_BYTES + (2 * cg + 1) * F::QB,
                                         hdr_lds + hslot * G::HSZ + (2 * cg + 1) * F::HB, lane);
        }
    };

    f32x16 acc[WM][WN];
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
        for (int j = 0; j < WN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    auto mainloop = [&](auto kh_c, auto wl_c) {
        constexpr int KH = decltype(kh_c)::value;
        using WLc = decltype(wl_c);
        constexpr bool WL = WLc::value;
        using I0 = std::integral_constant<int, 0>;
        using I1 = std::integral_constant<int, 1>;
        using I2 = std::integral_constant<int, 2>;
        using I3 = std::integral_constant<int, 3>;
        // the split's super-blocks are visited in a rotated order (v -> sb0 + (v + rot) % nv): workgroups that
        // run side by side on one XCD (consecutive column tiles) then stream different k ranges of the shared
        // A rows instead of all hitting the same 128-B lines (and L2 channels) at the same time
        const int nv = sb1 - sb0;
        const int rot = rot_mul ? (int)(((unsigned)ct * (unsigned)rot_mul) % (unsigned)nv) : 0;
        auto phys = [&](int v) {
            int p = v + rot;
            if (p >= nv) p -= nv;
            return sb0 + p;
        };
        // stage ki of the virtual k-tile sequence (ki & 3 == KI & 3, compile-time): past the split's end a dummy
        // stage re-reads the last real super-block's tile 3 (valid addresses, never consumed)
        auto issue_stage = [&](int ki, auto jq_c) {
            const int vi = ki >> 2;
            const bool real = vi < nv;
            const int ps = phys(real ? vi : nv - 1);
            issue(ps * 4 + (real ? (ki & 3) : 3), ps, ki % NS, hslot_of(vi), jq_c, WLc{});
        };
        // prologue: stages 0 .. NS - 2, then stage 0 landed
        issue_stage(0, I0{});
        issue_stage(1, I1{});
        issue_stage(2, I2{});
        if constexpr (NS >= 5) issue_stage(3, I3{});
        if constexpr (NS >= 6) issue_stage(4, I0{});
        if constexpr (NS >= 7) issue_stage(5, I1{});
        if constexpr (NS >= 8) issue_stage(6, I2{});
        q2_wait_barrier<q2_cnt_run<WAI, QII, HII, WL, 1, NS - 2>()>();

        // fragment producers (S is a compile-time constant after unrolling)
        auto bfrag = [&](const Q2B<QT>& b, auto jq_c, int S) -> f16x8 {
            constexpr int JQ_ = decltype(jq_c)::value;
            if constexpr (DBG & 2) {
                const u32x2 r2 = (S & 1) ? b.v1 : b.v0;
                return __builtin_bit_cast(f16x8, (u32x4){r2[0], r2[1], r2[0] ^ (uint32_t)S, r2[1]});
            } else {
                switch (S) {
                    case 0: return b.template frag<JQ_, 0>();
                    case 1: return b.template frag<JQ_, 1>();
                    case 2: return b.template frag<JQ_, 2>();
                    default: return b.template frag<JQ_, 3>();
                }
            }
        };
        Q2B<QT> bw[WN];
        f16x8 af[2][WM], bfc[WN];
#pragma unroll
        for (int j = 0; j < WN; ++j) {
            bw[j].load_hdr(hdr_lds + hg + j * F::HB, col, h);
            bw[j].load_q(smem + b_rd + j * F::QB, col, h);
            bw[j].template prep<0>();
            bfc[j] = bfrag(bw[j], I0{}, KH);
        }
#pragma unroll
        for (int i = 0; i < WM; ++i) af[0][i] = *(const f16x8*)(smem + a_rd + i * 4096 + KH * 256);

        // one k-tile (ring slot JQ): the wave's k-steps KH, KH + KS, ...; software-pipelined one k-step deep:
        // k-step S's MFMAs consume A / B fragments read and dequantised during k-step S - KS, while this
        // k-step reads and dequantises those of the next one (on the last k-step: the next tile's first, from
        // ring slot JQ + 1, landed at the top). An explicit per-k-step schedule (q2_interleave) keeps the
        // compiler from sinking the LDS reads next to their MFMAs, which stalled every k-step on lgkmcnt(0).
        auto tile = [&](int sb, auto jq_c) {  // sb: virtual super-block index
            constexpr int JQ = decltype(jq_c)::value;
            constexpr int NJ = (JQ + 1) & 3;
            const int kt = sb * 4 + JQ;
            const int cs = kt % NS, ns = (kt + 1) % NS;  // ring slots of this tile and the next
            // stage kt+1 landed (stages kt+2 .. kt+NS-2 may still be in flight); every wave is past tile kt-1
            q2_wait_barrier<q2_cnt_run<WAI, QII, HII, WL, (JQ + 2) & 3, NS - 3>()>();
            issue_stage(kt + NS - 1, std::integral_constant<int, (JQ + NS - 1) & 3>{});
            // the next tile's quant bytes (and, at a super-block edge, header): slot NJ landed at the wait above
            Q2B<QT> bn[WN];
#pragma unroll
            for (int j = 0; j < WN; ++j) {
                bn[j] = bw[j];
                if constexpr (NJ == 0) bn[j].load_hdr(hdr_lds + hslot_of(sb + 1) * G::HSZ + hg + j * F::HB, col, h);
                bn[j].load_q(smem + ns * STAGE + b_rd + j * F::QB, col, h);
            }
            constexpr int NSTEP = 4 / KS;
#pragma unroll
            for (int t = 0; t < NSTEP; ++t) {
                __builtin_amdgcn_sched_barrier(0);
                const int S = KH + KS * t;  // compile-time after unrolling
                const int cur = t & 1;
                f16x8 bfn[WN];
                if (t + 1 < NSTEP) {
#pragma unroll
                    for (int i = 0; i < WM; ++i)
                        af[cur ^ 1][i] = *(const f16x8*)(smem + cs * STAGE + a_rd + i * 4096 + (S + KS) * 256);
#pragma unroll
                    for (int j = 0; j < WN; ++j) bfn[j] = bfrag(bw[j], jq_c, S + KS);
                } else {
#pragma unroll
                    for (int i = 0; i < WM; ++i)
                        af[cur ^ 1][i] = *(const f16x8*)(smem + ns * STAGE + a_rd + i * 4096 + KH * 256);
#pragma unroll
                    for (int j = 0; j < WN; ++j) {
                        bn[j].template prep<NJ>();
                        bfn[j] = bfrag(bn[j], std::integral_constant<int, NJ>{}, KH);
                    }
                }
#pragma unroll
                for (int j = 0; j < WN; ++j)
#pragma unroll
                    for (int i = 0; i < WM; ++i) {
                        if constexpr (DBG & 1) asm volatile("" ::"v"(af[cur][i]), "v"(bfc[j]));
                        else acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[cur][i], bfc[j], acc[i][j], 0, 0, 0);
                    }
                if constexpr (!(DBG & 1)) {
                    if constexpr (Q2_AEARLY) {
                        __builtin_amdgcn_sched_group_barrier(0x100, WM, 0);  // the next k-step's A reads first
                        q2_interleave_mfma<0, WM * WN, Q2_VPM>();
                    } else {
                        q2_interleave<0, WM * WN, WM, Q2_VPM>();
                    }
                }
#pragma unroll
                for (int j = 0; j < WN; ++j) bfc[j] = bfn[j];
            }
            // NSTEP is even: the next tile's first fragments are in af[0]
#pragma unroll
            for (int j = 0; j < WN; ++j) bw[j] = bn[j];
        };
        for (int sb = 0; sb < nv; ++sb) {
            tile(sb, I0{});
            tile(sb, I1{});
            tile(sb, I2{});
            tile(sb, I3{});
        }
        // drain the dummy stages before the LDS is reused / released
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    };
    using T_ = std::integral_constant<bool, true>;
    using F_ = std::integral_constant<bool, false>;
    if constexpr (KS == 1) {
        mainloop(std::integral_constant<int, 0>{}, T_{});
    } else {
        if (kh == 0) mainloop(std::integral_constant<int, 0>{}, T_{});
        else mainloop(std::integral_constant<int, 1>{}, F_{});
        // sum the k-step halves: kh = 1 waves park their partials in the drained ring
        __syncthreads();
        float* red = (float*)smem + (size_t)cg * (WM * WN * 16 * 64) + lane;
        if (kh == 1) {
#pragma unroll
            for (int i = 0; i < WM; ++i)
#pragma unroll
                for (int j = 0; j < WN; ++j)
#pragma unroll
                    for (int r = 0; r < 16; ++r) red[((i * WN + j) * 16 + r) * 64] = acc[i][j][r];
        }
        __syncthreads();
        if (kh == 1) return;
#pragma unroll
        for (int i = 0; i < WM; ++i)
#pragma unroll
            for (int j = 0; j < WN; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[i][j][r] += red[((i * WN + j) * 16 + r) * 64];
    }

    // ---- epilogue: 32x32 C/D layout: col = lane & 31, row = 8*(r>>2) + 4*(lane>>5) + (r&3) ----
    const int mb = m_base + mw * WM * 32;
    if constexpr (FU && !GR) {
        if (fu.mode & 2) {  // fused RMSNorm, consumer side: the rows' 1 / rms
            // one row per lane (row mb + 32 i + lane % 32), handed to the C/D layout's rows by lane shuffles: one
            // load per 32 rows keeps the register footprint at the kernel's own
#pragma unroll
            for (int i = 0; i < WM; ++i) {
                const int mr = mb + i * 32 + col;
                const float s = mr < M ? fu.ss_in[(size_t)mr * Q2F_SS_STRIDE] : 0.f;
                const float rsl = rsqrtf(s * fu.inv_h + fu.eps);
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const float rs = __shfl(rsl, 8 * (r >> 2) + 4 * h + (r & 3));
#pragma unroll
                    for (int j = 0; j < WN; ++j) acc[i][j][r] *= rs;
                }
            }
        }
    }
    if constexpr (FU && !GR && (EPI == E16_F32 || EPI == E16_ADD_F32)) {
        if (fu.mode & 4) {  // RoPE + KV append epilogue (q|k|v GEMM)
            const int n0 = (ct * NG + nw * WN) * 32;
            if (n0 >= N || mb >= M) return;
            if (splits > 1) {  // sum the splits in C, the last one takes the block (as the fused-norm producer)
#pragma unroll
                for (int j = 0; j < WN; ++j) {
                    if (n0 + j * 32 >= N) break;
#pragma unroll
                    for (int i = 0; i < WM; ++i)
#pragma unroll
                        for (int r = 0; r < 16; ++r) {
                            const int m = mb + i * 32 + 8 * (r >> 2) + 4 * h + (r & 3);
                            if (m < M) atomicAdd((float*)Cv + (size_t)m * ldc + n0 + j * 32 + col, acc[i][j][r]);
                        }
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                const int tk = (mb >> 5) * ngrp + (n0 >> 5);
                unsigned last = 0;
                if (lane == 0)
                    last = __hip_atomic_fetch_add(fu.tick + tk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                           (unsigned)(splits - 1);
                last = __shfl(last, 0);
                if (!last) return;
                if (lane == 0) __hip_atomic_store(fu.tick + tk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            const int D = 1 << fu.dsh, HALF = D >> 1;
            for (int i = 0; i < WM; ++i) {
                const int mr = mb + i * 32;
                if (mr >= M) break;
                // one row per lane, handed out by shuffles (as the row scale above)
                const int sl = mr + col < M ? fu.slots[mr + col] : -1;
#pragma unroll
                for (int j = 0; j < WN; ++j) {
                    if (n0 + j * 32 >= N) break;
                    const int n = n0 + j * 32 + col;
                    const int c = fu.n_off + n, hh = c >> fu.dsh, d = c & (D - 1);
                    const float bn = fu.bias ? fu.bias[c] : 0.f;
                    const bool rotate = hh < fu.hq + fu.hkv;
                    float v[16];
                    if (splits > 1) {
                        float* cp = (float*)Cv + n;
                        q2_ld16_sc1(v, cp, ldc, mr + 4 * h, M);
#pragma unroll
                        for (int r = 0; r < 16; ++r) {
                            const int m = mr + 8 * (r >> 2) + 4 * h + (r & 3);
                            if (m < M) cp[(size_t)m * ldc] = 0.f;  // zero again for the next split-K accumulation
                        }
                    } else {
#pragma unroll
                        for (int r = 0; r < 16; ++r) v[r] = acc[i][j][r];
                    }
                    float2 cs[16];
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int m = min(mr + 8 * (r >> 2) + 4 * h + (r & 3), M - 1);
                        cs[r] = rotate ? fu.rot[(size_t)m * HALF + (d >> 1)] : make_float2(1.f, 0.f);
                    }
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int rr = 8 * (r >> 2) + 4 * h + (r & 3), m = mr + rr;
                        const float x = v[r] + bn;
                        const float partner = __shfl_xor(x, 1);  // the other element of the adjacent pair
                        const int slot = __shfl(sl, rr);
                        const float y = rotate ? ((d & 1) ? partner * cs[r].y + x * cs[r].x : x * cs[r].x - partner * cs[r].y)
                                               : x;
                        if (m < M) {
                            const uint16_t yb = (uint16_t)(pack_bf16x2(y, 0.f) & 0xFFFF);
                            if (hh < fu.hq) {
                                fu.qo[((size_t)m * fu.hq + hh) * D + d] = yb;
                            } else if (slot >= 0) {
                                const bool isk = hh < fu.hq + fu.hkv;
                                const int kvh = hh - fu.hq - (isk ? 0 : fu.hkv);
                                const size_t e = (((size_t)(slot / fu.block_size) * fu.hkv + kvh) * fu.block_size +
                                                  slot % fu.block_size) * D + d;
                                (isk ? fu.kc : fu.vc)[e] = yb;
                            }
                        }
                    }
                }
            }
            return;
        }
    }
#pragma unroll
    for (int j = 0; j < WN; ++j) {
        const int nt = (ct * NG + nw * WN + j) * 32;
        const int n = nt + col;
        if (nt >= N) break;
        if constexpr (GR && EPI == E16_ADD_F32) {
#pragma unroll
            for (int i = 0; i < WM; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int m = mb + i * 32 + 8 * (r >> 2) + 4 * h + (r & 3);
                    if (m < M) atomicAdd((float*)Cv + (size_t)grp.otok[m] * ldc + n, grp.owt[m] * acc[i][j][r]);
                }
            continue;
        }
        if constexpr (EPI == E16_SWIGLU || EPI == E16_GEGLU) {
            // W rows interleaved in 16-row groups: tile columns 0..15 gate, 16..31 up of the same features
#pragma unroll
            for (int i = 0; i < WM; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const float v = acc[i][j][r];
                    const float up = __shfl_xor(v, 16);
                    const int m = mb + i * 32 + 8 * (r >> 2) + 4 * h + (r & 3);
                    if (col < 16 && m < M)
                        ((uint16_t*)Cv)[(size_t)m * ldc + (nt >> 1) + col] = f32_to_act<true>(glu_gate_f<EPI>(v) * up);
                }
            continue;
        }
#pragma unroll
        for (int i = 0; i < WM; ++i) {
            const int m0 = mb + i * 32 + 4 * h;
            if (mb + i * 32 >= M) break;
            float* cf = ((float*)Cv) + (size_t)m0 * ldc + n;
            uint16_t* ch = ((uint16_t*)Cv) + (size_t)m0 * ldc + n;
            auto roff = [&](int r) { return (size_t)(8 * (r >> 2) + (r & 3)) * ldc; };
            if (mb + i * 32 + 32 <= M) {
                if constexpr (EPI == E16_ADD_F32) {
                    if (splits == 1) {
                        float old[16];
#pragma unroll
                        for (int r = 0; r < 16; ++r) old[r] = cf[roff(r)];
#pragma unroll
                        for (int r = 0; r < 16; ++r) cf[roff(r)] = old[r] + acc[i][j][r];
                    } else {
#pragma unroll
                        for (int r = 0; r < 16; ++r) atomicAdd(cf + roff(r), acc[i][j][r]);
                    }
                } else {
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        if constexpr (EPI == E16_F32) cf[roff(r)] = acc[i][j][r];
                        else ch[roff(r)] = f32_to_act<true>(acc[i][j][r]);
                    }
                }
                continue;
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                if (m0 + 8 * (r >> 2) + (r & 3) >= M) continue;
                const float v = acc[i][j][r];
                if constexpr (EPI == E16_F32) cf[roff(r)] = v;
                else if constexpr (EPI == E16_ACT) ch[roff(r)] = f32_to_act<true>(v);
                else if (splits == 1) cf[roff(r)] += v;
                else atomicAdd(cf + roff(r), v);
            }
        }
    }
    if constexpr (FU && EPI == E16_ADD_F32 && !GR) {
        if (fu.mode & 1) {  // fused RMSNorm, producer side
            if (fu.ss_zero && bid == 0 && wave == 0)
                for (int m = lane; m < M; m += 64) fu.ss_zero[(size_t)m * Q2F_SS_STRIDE] = 0.f;
            if (!fu.xn) return;
            // this wave's block is final once every K split has added into it: the adds complete (vmcnt) before a
            // relaxed agent-scope ticket; the last split reads the block with agent-scope loads (no fence: see
            // profiles/r6_fence_free_handoffs.md)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const int n0 = (ct * NG + nw * WN) * 32;
            if (n0 >= N || mb >= M) return;
            if (splits > 1) {
                const int tk = (mb >> 5) * ngrp + (n0 >> 5);
                unsigned last = 0;
                if (lane == 0)
                    last = __hip_atomic_fetch_add(fu.tick + tk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                           (unsigned)(splits - 1);
                last = __shfl(last, 0);
                if (!last) return;
                if (lane == 0) __hip_atomic_store(fu.tick + tk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            // lane = one column, one 32-row block at a time: x * g -> xn, the row's sum of squares over this wave's
            // 32 WN columns -> one atomic per row
            for (int i = 0; i < WM; ++i) {
                const int mr = mb + i * 32;
                if (mr >= M) break;
                float ssr = 0.f;  // sum for row mr + (lane % 32) after the transposing shuffles below
#pragma unroll
                for (int j = 0; j < WN; ++j) {
                    const int n = n0 + j * 32 + col;
                    if (n0 + j * 32 >= N) break;
                    const float g = fu.gamma[n];
                    float sq[16];
                    q2_ld16_sc1(sq, (const float*)Cv + n, ldc, mr + 4 * h, M);
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int m = mr + 8 * (r >> 2) + 4 * h + (r & 3);
                        const float x = m < M ? sq[r] : 0.f;
                        if (m < M)
                            fu.xn[(size_t)m * fu.ldxn + n] = f32_to_act<true>(fminf(fmaxf(x * g, -65504.f), 65504.f));
                        sq[r] = x * x;
                    }
                    // reduce each row's 32 columns (the lanes of this half)
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        float v = sq[r];
                        v += __shfl_xor(v, 1);
                        v += __shfl_xor(v, 2);
                        v += __shfl_xor(v, 4);
                        v += __shfl_xor(v, 8);
                        v += __shfl_xor(v, 16);
                        // lane c of the block's row c: row 8 (r >> 2) + 4 h + (r & 3) lives in half h
                        const int rr = 8 * (r >> 2) + (r & 3);
                        const float v0 = __shfl(v, 0), v1 = __shfl(v, 32);  // the two halves' rows rr and rr + 4
                        if (col == rr) ssr += v0;
                        if (col == rr + 4) ssr += v1;
                    }
                }
                if (lane < 32 && mr + col < M) atomicAdd(fu.ss_out + (size_t)(mr + col) * Q2F_SS_STRIDE, ssr);
            }
        }
    }
}

template <int QT, int WM, int KS, int WN, int EPI, int NS = 4, int NG = 4, int GPW = 1, bool FU = false>
static int launch_qmm2(const uint16_t* A, int lda, const uint8_t* W, int M, int N, int K, int splits, void* C, int ldc,
                       hipStream_t st, const Q2Fuse& fu) {
    using G = Q2Geom<QT, WM, KS, WN, NS, NG, GPW>;
    const int nsb = K >> 8;
    splits = max(1, min(splits, nsb));
    const int sbps = (nsb + splits - 1) / splits;
    splits = (nsb + sbps - 1) / sbps;  // no empty splits
    const int n_ct = (N + 32 * NG - 1) / (32 * NG), n_mt = (M + G::BM - 1) / G::BM;
    const long nwg = (long)n_ct * splits * n_mt;
    if (nwg <= 0 || nwg > 0x7fffffff) return (int)hipErrorInvalidValue;
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)qmm2_kernel<QT, WM, KS, WN, EPI, 0, NS, NG, GPW, false, FU>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS);
        attr_set = true;
    }
    qmm2_kernel<QT, WM, KS, WN, EPI, 0, NS, NG, GPW, false, FU><<<dim3((unsigned)nwg), 64 * G::NT, G::LDS, st>>>(
        A, lda, W, M, N, K, n_mt, splits, sbps, C, ldc, g_qmm2_rot, Q2Group{}, fu);
    MXK_CHECK_LAUNCH();
}

// grouped (MoE) launch: P sorted rows, E experts of N columns each, tiles / off from moe_sort with BM = 32 WM
template <int QT, int WM, int KS, int EPI>
static int launch_qmm2_grouped(const uint16_t* A, int lda, const int* stok, const uint8_t* W, int P, int E, int N, int K,
                               const int* tiles, const int* off, void* C, int ldc, const int* otok, const float* owt,
                               hipStream_t st) {
    if (EPI == E16_ADD_F32 && (!otok || !owt)) return (int)hipErrorInvalidValue;
    using G = Q2Geom<QT, WM, KS, 1>;
    const int n_ct = (N + 127) / 128, n_mt = (P + G::BM - 1) / G::BM + E;
    const long nwg = (long)n_ct * n_mt;
    if (nwg <= 0 || nwg > 0x7fffffff) return (int)hipErrorInvalidValue;
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)qmm2_kernel<QT, WM, KS, 1, EPI, 0, 4, 4, 1, true>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS);
        attr_set = true;
    }
    qmm2_kernel<QT, WM, KS, 1, EPI, 0, 4, 4, 1, true><<<dim3((unsigned)nwg), 64 * G::NT, G::LDS, st>>>(
        A, lda, W, P, N, K, n_mt, 1, K >> 8, C, ldc, 0, Q2Group{tiles, off, stok, E, otok, owt}, Q2Fuse{});
    MXK_CHECK_LAUNCH();
}

// wm 1 (32-row tiles) or 2 (64); epi F32 (the down projection into the [P, H] buffer), ADD_F32 (the down projection
// with the combine fused: weighted atomic adds into the tokens' rows, otok / owt) or SwiGLU / GeGLU (gate|up)
template <int QT>
static int qmm2_grouped_run(int epi, int wm, const uint16_t* A, int lda, const int* stok, const uint8_t* W, int P, int E,
                            int N, int K, const int* tiles, const int* off, void* C, int ldc, const int* otok,
                            const float* owt, hipStream_t st) {
#define Q2G(WM_, EPI_)                                                                                          \
    if (wm == WM_ && epi == EPI_)                                                                               \
        return launch_qmm2_grouped<QT, WM_, 2, EPI_>(A, lda, stok, W, P, E, N, K, tiles, off, C, ldc, otok, owt, st);
    Q2G(1, E16_F32) Q2G(2, E16_F32) Q2G(1, E16_ADD_F32) Q2G(2, E16_ADD_F32) Q2G(1, E16_SWIGLU) Q2G(2, E16_SWIGLU)
    Q2G(1, E16_GEGLU) Q2G(2, E16_GEGLU)
#undef Q2G
    return (int)hipErrorInvalidValue;
}

// ks: 1 / 2 waves per column group; ks | 8 selects the 8-slot ring (64-row tiles only); 17 the wide tiles
template <int QT, int EPI, bool FU = false>
static int dispatch_qmm2(int wm, int ks, int wn, const uint16_t* A, int lda, const uint8_t* W, int M, int N, int K,
                         int splits, void* C, int ldc, hipStream_t st, const Q2Fuse& fu) {
// (configurations whose ring does not fit the LDS for this format — 256-row tiles of Q8_0 — are not compiled)
#define Q2_CASE(WM_, KS_, WN_)                                                                \
    if constexpr (Q2Geom<QT, WM_, KS_, WN_, 4>::LDS <= 160 * 1024)                            \
        if (wm == WM_ && ks == KS_ && wn == WN_)                                              \
            return launch_qmm2<QT, WM_, KS_, WN_, EPI, 4, 4, 1, FU>(A, lda, W, M, N, K, splits, C, ldc, st, fu);
#define Q2_DEEP(WM_, KS_, WN_)                                                                   \
    if constexpr (Q2Geom<QT, WM_, KS_, WN_, 8>::LDS <= 160 * 1024)                               \
        if (wm == WM_ && ks == (KS_ | 8) && wn == WN_)                                           \
            return launch_qmm2<QT, WM_, KS_, WN_, EPI, 8, 4, 1, FU>(A, lda, W, M, N, K, splits, C, ldc, st, fu);
    // (8, 2, 1) / (4, 2, 2) (256-row tiles with 8 waves) exceed the 256 registers a wave has at 2 waves / SIMD
    Q2_CASE(2, 1, 1) Q2_CASE(2, 2, 1) Q2_CASE(4, 1, 1) Q2_CASE(4, 2, 1) Q2_CASE(8, 1, 1)
    Q2_CASE(1, 2, 2) Q2_CASE(2, 1, 2) Q2_CASE(2, 2, 2) Q2_CASE(4, 1, 2)
    // 192-row tiles: M = 384 (a c128 decode batch + a 256-token prompt chunk) in two row tiles, no padding rows
    Q2_CASE(6, 1, 1) Q2_CASE(6, 2, 1) Q2_CASE(3, 2, 2)
    // 224-row tiles: M in (384, 448] (a decode batch + a prompt chunk a little over 256 tokens) in two row tiles
    Q2_CASE(7, 1, 1)
    Q2_DEEP(2, 1, 1) Q2_DEEP(2, 2, 1) Q2_DEEP(1, 2, 2)
    // ks | 32: a 6-slot ring for the 128-row decode tiles (5 stages in flight instead of 3: the LDS-DMA issue ->
    // landed latency, not the MFMA rate, bounds a one-workgroup-per-CU M = 128 GEMM at ~30 GB/s per CU with 4 slots)
#define Q2_R6(WM_, KS_, WN_)                                                                     \
    if constexpr (Q2Geom<QT, WM_, KS_, WN_, 6>::LDS <= 160 * 1024)                               \
        if (wm == WM_ && ks == (KS_ | 32) && wn == WN_)                                          \
            return launch_qmm2<QT, WM_, KS_, WN_, EPI, 6, 4, 1, FU>(A, lda, W, M, N, K, splits, C, ldc, st, fu);
    Q2_R6(4, 1, 1) Q2_R6(4, 2, 1) Q2_R6(2, 2, 2) Q2_R6(2, 1, 2)
#undef Q2_R6
    // ks | 16: wide tiles (8 column groups, 256 columns per workgroup, 8 waves)
#define Q2_WIDE(WM_, WN_)                                                                      \
    if constexpr (Q2Geom<QT, WM_, 1, WN_, 4, 8>::LDS <= 160 * 1024)                           \
        if (wm == WM_ && ks == 17 && wn == WN_)                                                \
            return launch_qmm2<QT, WM_, 1, WN_, EPI, 4, 8, 1, FU>(A, lda, W, M, N, K, splits, C, ldc, st, fu);
    Q2_WIDE(2, 1) Q2_WIDE(4, 1) Q2_WIDE(6, 1) Q2_WIDE(3, 2) Q2_WIDE(7, 1)
    // ks 18: the 4-wave wide form (each wave 64 columns x 32 wm rows)
// (Q4_K / MX4F only: formats whose tile and header each take one DMA instruction; the Q6_K form returned NaNs in
// test_qmm2 and is not compiled)
#define Q2_WIDE4(WM_)                                                                          \
    if constexpr ((QT == MXQ_Q4_K || QT == MXQ_MX4F) && Q2Geom<QT, WM_, 1, 2, 4, 8, 2>::LDS <= 160 * 1024) \
        if (wm == WM_ && ks == 18 && wn == 2)                                                  \
            return launch_qmm2<QT, WM_, 1, 2, EPI, 4, 8, 2, FU>(A, lda, W, M, N, K, splits, C, ldc, st, fu);
    Q2_WIDE4(4) Q2_WIDE4(6) Q2_WIDE4(2)
#undef Q2_WIDE4
#undef Q2_WIDE
#undef Q2_DEEP
#undef Q2_CASE
    return (int)hipErrorInvalidValue;
}

template <int DBG>
static int launch_dbg(int wm, int ks, int wn, const uint16_t* A, int lda, const uint8_t* W, int M, int N, int K, void* C, int ldc,
                      hipStream_t st) {
    constexpr int QT = MXQ_Q4_K, EPI = E16_SWIGLU;
    auto go = [&](auto kern, int bm, int ks, int lds, int ng = 4) {
        (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        const int n_ct = (N + 32 * ng - 1) / (32 * ng), n_mt = (M + bm - 1) / bm;
        kern<<<dim3(n_ct * n_mt), ng == 8 ? 512 : 256 * ks, lds, st>>>(A, lda, W, M, N, K, n_mt, 1, K >> 8, C, ldc,
                                                                      g_qmm2_rot, Q2Group{}, Q2Fuse{});
        return (int)hipGetLastError();
    };
    // ks 17: the wide tiles (8 column groups)
    if (wm == 6 && ks == 17 && wn == 1)
        return go(qmm2_kernel<QT, 6, 1, 1, EPI, DBG, 4, 8>, 192, 1, Q2Geom<QT, 6, 1, 1, 4, 8>::LDS, 8);
    if (wm == 4 && ks == 17 && wn == 1)
        return go(qmm2_kernel<QT, 4, 1, 1, EPI, DBG, 4, 8>, 128, 1, Q2Geom<QT, 4, 1, 1, 4, 8>::LDS, 8);
    if (wm == 3 && ks == 17 && wn == 2)
        return go(qmm2_kernel<QT, 3, 1, 2, EPI, DBG, 4, 8>, 192, 1, Q2Geom<QT, 3, 1, 2, 4, 8>::LDS, 8);
    if (wm == 6 && ks == 18 && wn == 2 && QT == MXQ_Q4_K) {
        auto k4 = qmm2_kernel<QT, 6, 1, 2, EPI, DBG, 4, 8, 2>;
        (void)hipFuncSetAttribute((const void*)k4, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  Q2Geom<QT, 6, 1, 2, 4, 8, 2>::LDS);
        const int n_ct = (N + 255) / 256, n_mt = (M + 191) / 192;
        k4<<<dim3(n_ct * n_mt), 256, Q2Geom<QT, 6, 1, 2, 4, 8, 2>::LDS, st>>>(A, lda, W, M, N, K, n_mt, 1, K >> 8, C, ldc,
                                                                            g_qmm2_rot, Q2Group{}, Q2Fuse{});
        return (int)hipGetLastError();
    }
    if (wm == 8 && ks == 1 && wn == 1) return go(qmm2_kernel<QT, 8, 1, 1, EPI, DBG>, 256, 1, Q2Geom<QT, 8, 1, 1>::LDS);
    if (wm == 4 && ks == 2 && wn == 1) return go(qmm2_kernel<QT, 4, 2, 1, EPI, DBG>, 128, 2, Q2Geom<QT, 4, 2, 1>::LDS);
    if (wm == 4 && ks == 1 && wn == 2) return go(qmm2_kernel<QT, 4, 1, 2, EPI, DBG>, 256, 1, Q2Geom<QT, 4, 1, 2>::LDS);
    if (wm == 2 && ks == 2 && wn == 2) return go(qmm2_kernel<QT, 2, 2, 2, EPI, DBG>, 128, 2, Q2Geom<QT, 2, 2, 2>::LDS);
    return (int)hipErrorInvalidValue;
}


// all epilogues of one block format (each format's instances live in their own translation unit, qmm2_q*.hip)
template <int QT>
static int qmm2_run(int epi, int wm, int ks, int wn, const uint16_t* A, int lda, const uint8_t* W, int M, int N, int K, int splits, void* C, int ldc, hipStream_t st, const Q2Fuse& fu) {
    if (fu.mode != 0) {
        // the fused-RMSNorm forms (separate instances: the plain ones keep their register allocation): the
        // residual-add producer, the fp32 (split-K qkv) and SwiGLU consumers, for the K-quant formats of the
        // Q4_K_M / Q5_K_M / Q6_K / Q8_0 files
        if constexpr (QT == MXQ_Q4_K || QT == MXQ_Q5_K || QT == MXQ_Q6_K || QT == MXQ_Q8_0) {
            switch (epi) {
                case E16_F32: return dispatch_qmm2<QT, E16_F32, true>(wm, ks, wn, A, lda, W, M, N, K, splits, C, ldc, st, fu);
                case E16_ADD_F32: return dispatch_qmm2<QT, E16_ADD_F32, true>(wm, ks, wn, A, lda, W, M, N, K, splits, C, ldc, st, fu);
                case E16_SWIGLU: return dispatch_qmm2<QT, E16_SWIGLU, true>(wm, ks, wn, A, lda, W, M, N, K, splits, C, ldc, st, fu);
            }
        }
        return (int)hipErrorNotSupported;
    }
    switch (epi) {
        case E16_F32: return dispatch_qmm2<QT, E16_F32>(wm, ks, wn, A, lda, W, M, N, K, splits, C, ldc, st, fu);
        case E16_ACT: return dispatch_qmm2<QT, E16_ACT>(wm, ks, wn, A, lda, W, M, N, K, splits, C, ldc, st, fu);
        case E16_ADD_F32: return dispatch_qmm2<QT, E16_ADD_F32>(wm, ks, wn, A, lda, W, M, N, K, splits, C, ldc, st, fu);
        case E16_SWIGLU: return dispatch_qmm2<QT, E16_SWIGLU>(wm, ks, wn, A, lda, W, M, N, K, splits, C, ldc, st, fu);
        case E16_GEGLU: return dispatch_qmm2<QT, E16_GEGLU>(wm, ks, wn, A, lda, W, M, N, K, splits, C, ldc, st, fu);
    }
    return (int)hipErrorInvalidValue;
}

}  // namespace

int qmm2_run_q4k(int epi, int wm, int ks, int wn, const uint16_t* A, int lda, const uint8_t* W, int M, int N, int K, int splits, void* C, int ldc, hipStream_t st, const Q2Fuse& fu);
int qmm2_run_q5k(int epi, int wm, int ks, int wn, const uint16_t* A, int lda, const uint8_t* W, int M, int N, int K, int splits, void* C, int ldc, hipStream_t st, const Q2Fuse& fu);
int qmm2_run_q6k(int epi, int wm, int ks, int wn, const uint16_t* A, int lda, const uint8_t* W, int M, int N, int K, int splits, void* C, int ldc, hipStream_t st, const Q2Fuse& fu);
int qmm2_run_q3k(int epi, int wm, int ks, int wn, const uint16_t* A, int lda, const uint8_t* W, int M, int N, int K, int splits, void* C, int ldc, hipStream_t st, const Q2Fuse& fu);
int qmm2_run_q2k(int epi, int wm, int ks, int wn, const uint16_t* A, int lda, const uint8_t* W, int M, int N, int K, int splits, void* C, int ldc, hipStream_t st, const Q2Fuse& fu);
int qmm2_run_q80(int epi, int wm, int ks, int wn, const uint16_t* A, int lda, const uint8_t* W, int M, int N, int K, int splits, void* C, int ldc, hipStream_t st, const Q2Fuse& fu);
int qmm2_run_mx4(int epi, int wm, int ks, int wn, const uint16_t* A, int lda, const uint8_t* W, int M, int N, int K, int splits, void* C, int ldc, hipStream_t st, const Q2Fuse& fu);
int qmm2_run_mx5(int epi, int wm, int ks, int wn, const uint16_t* A, int lda, const uint8_t* W, int M, int N, int K, int splits, void* C, int ldc, hipStream_t st, const Q2Fuse& fu);
int qmm2_grouped_q4k(int epi, int wm, const uint16_t* A, int lda, const int* stok, const uint8_t* W, int P, int E, int N, int K, const int* tiles, const int* off, void* C, int ldc, const int* otok, const float* owt, hipStream_t st);
int qmm2_grouped_q5k(int epi, int wm, const uint16_t* A, int lda, const int* stok, const uint8_t* W, int P, int E, int N, int K, const int* tiles, const int* off, void* C, int ldc, const int* otok, const float* owt, hipStream_t st);
int qmm2_grouped_q6k(int epi, int wm, const uint16_t* A, int lda, const int* stok, const uint8_t* W, int P, int E, int N, int K, const int* tiles, const int* off, void* C, int ldc, const int* otok, const float* owt, hipStream_t st);
int qmm2_grouped_q80(int epi, int wm, const uint16_t* A, int lda, const int* stok, const uint8_t* W, int P, int E, int N, int K, const int* tiles, const int* off, void* C, int ldc, const int* otok, const float* owt, hipStream_t st);
int qmm2_dbg_q4k(int dbg, int wm, int ks, int wn, const uint16_t* A, int lda, const uint8_t* W, int M, int N, int K, void* C, int ldc, hipStream_t st);
