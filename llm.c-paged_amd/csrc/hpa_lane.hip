// hpa_lane.hip -- the lane-layer launch of the overlapped decode step.
//
// The batch is cut into two micro-batch lanes X and Y.  One launch holds
//   * the paged attention of lane X for layer l (HBM-bound: every CU
//     streams K/V pages), one workgroup per (sequence, head), and
//   * the whole GEMM chain of lane Y -- attproj(l'), fc(l'), fcproj(l') and
//     qkv(l'+1) -- run by a set of persistent chain workgroups that take
//     16x16 output tiles from a queue in dependency order.
// The two roles share the CUs: the chain's latency-bound tiles (load ->
// MFMA chain -> epilogue) fill the issue slots the streaming waves leave,
// and one launch replaces the attention launch plus four GEMM launches of a
// layer (MI355X_MICROARCH.md "boundary": each costs a grid fill and drain).
//
// In-launch hand-offs (cdna_hip_programming.md Guideline 16, R1 form):
//   producer tile: epilogue outputs stored write-through (sc1) -> every wave
//     s_waitcnt vmcnt(0) -> barrier -> one lane adds 1 to the arrival counter
//     of (phase, row block) (relaxed, agent scope);
//   consumer tile: one lane polls the counter of (phase-1, its row block)
//     relaxed with s_sleep until every tile of that row block has arrived,
//     then ONE agent-scope acquire, vmcnt(0), barrier, then plain loads.
// Deadlock freedom: tiles are dequeued from one counter in phase order
// (phase-major, row-block-major inside a phase), and a tile only waits for
// tiles of the previous phase, all dequeued earlier by workgroups that are
// running; attention workgroups never wait.  No residency assumption.
// Every spin is bounded: on expiry the workgroup records a code in ctl[1]
// and goes on (wrong numbers, never a hang); the host checks ctl[1].
// The counters are zeroed by the engine's per-step memset.
//
// Numerics: attention = attn_chunk_body with one chunk (the single-pass
// kernel's tiles and fold, bit-identical output); the chain tiles run the
// fused GEMM bodies with 4 waves, so a row's K summation order is that of
// the 4-wave launches.
#include <string.h>

#include "hpa_attn_body.h"
#include "hpa_gemm_body.h"

namespace {
using hpa_attn::AttnChunk;
using hpa_gemm::FG;

constexpr int kNW = 4;           // waves per workgroup, both roles
constexpr int kMaxPh = 4;        // attproj, fc, fcproj, qkv
constexpr int kMaxRb = 4;        // 16-row blocks per lane (<= 64 rows)
constexpr unsigned kSpinLimit = 1u << 16;  // ~0.1 s of s_sleep polling

struct Chain {
    FG g[kMaxPh];
    int nph;
    int gx[kMaxPh];   // column tiles per phase
    int os[kMaxPh];   // 1: one-shot body (K/16 = 48), 0: looped body
    int gy;           // row blocks of the lane
    int total;        // tiles over all phases
    unsigned* ctl;    // [0] queue head, [1] timeout code, [2 + ph*4 + rb] arrivals
    int nblocks;      // chain workgroups (blocks 0 .. nblocks-1)
};

template <int A, int B>
constexpr int cmax() {
    return A > B ? A : B;
}
constexpr int kLds = cmax<cmax<hpa_attn::attn_lds_floats<kNW>(), hpa_gemm::gemm16_os_lds_floats<kNW>()>(),
                          hpa_gemm::gemm16_lds_floats<kNW, 1, 1>()>();

template <int EPI>
__device__ __forceinline__ void run_tile(const FG& g, int os, int bid, float* smem) {
    if (os)
        hpa_gemm::gemm16_os_body<kNW, EPI, 12, true>(g, bid, smem);
    else
        hpa_gemm::gemm16_body<kNW, EPI, 1, 1, 0, true>(g, bid, smem);
}

template <int P>
__global__ __launch_bounds__(kNW * 64, 3) void lane_layer_kernel(AttnChunk a, Chain c) {
    __shared__ __attribute__((aligned(16))) float smem[kLds];
    __shared__ int s_task;
    const int bid = blockIdx.x;
    if (bid >= c.nblocks) {  // attention role
        if (a.B > 0) hpa_attn::attn_chunk_body<P, kNW>(a, bid - c.nblocks, smem);
        return;
    }
    unsigned* ctl = c.ctl;
    // every branch around a barrier below is on wave-uniform (SGPR) values:
    // the task index comes back through LDS + readfirstlane, and the whole of
    // wave 0 polls, so the compiler emits scalar branches, never exec-masked
    // regions that a wave could skip a barrier in
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    // a counted loop (a workgroup can never draw more than `total` tiles): the
    // compiler's structurisation of an unbounded for(;;) around the barriers
    // hung the chain role in bring-up, the counted form does not
    for (int iter = 0; iter <= c.total; ++iter) {
        if (threadIdx.x == 0) s_task = (int)__hip_atomic_fetch_add(ctl, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        int t = __builtin_amdgcn_readfirstlane(s_task);
        if (t >= c.total) break;
        int ph = 0;
        while (ph + 1 < c.nph && t >= c.gx[ph] * c.gy) {
            t -= c.gx[ph] * c.gy;
            ++ph;
        }
        const int rb = t / c.gx[ph];
        const int cx = t - rb * c.gx[ph];
        if (ph > 0) {  // every tile of (ph-1, rb) must have arrived
            if (wave == 0) {
                const unsigned need = (unsigned)c.gx[ph - 1];
                unsigned* cnt = ctl + 2 + (ph - 1) * kMaxRb + rb;
                unsigned spins = 0;
                for (;;) {
                    const unsigned seen = __builtin_amdgcn_readfirstlane(
                        __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                    if (seen >= need) break;
                    if (++spins > kSpinLimit) {  // code: phase, row block, arrivals seen
                        if (threadIdx.x == 0)
                            __hip_atomic_store(ctl + 1, 0x1000000u | (unsigned)ph << 16 | (unsigned)rb << 8 | min(seen, 255u),
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(2);
                }
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            __syncthreads();
        }
        // the tile's index in the bodies' XCD-ordered grid numbering (xcd_tile)
        const int sbid = (((cx >> 3) * c.gy + rb) << 3) + (cx & 7);
        const FG& g = c.g[ph];
        switch (ph) {
            case 0: run_tile<HPA_FEPI_RESID>(g, c.os[0], sbid, smem); break;
            case 1: run_tile<HPA_FEPI_GELU>(g, c.os[1], sbid, smem); break;
            case 2: run_tile<HPA_FEPI_RESID>(g, c.os[2], sbid, smem); break;
            default: run_tile<HPA_FEPI_QKV>(g, c.os[3], sbid, smem); break;
        }
        // publish: every storing wave drains its sc1 stores, then one arrival
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0)
            __hip_atomic_fetch_add(ctl + 2 + ph * kMaxRb + rb, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

template <int P>
int launch_lane(const AttnChunk& a, const Chain& c) {
    const int grid = c.nblocks + (a.B > 0 ? a.nblocks : 0);
    if (grid == 0) return 0;
    lane_layer_kernel<P><<<grid, kNW * 64, 0, hpa_stream()>>>(a, c);
    HPA_LAUNCH_CHECK();
    return 0;
}

}  // namespace

extern "C" {

int hpa_lane_layer(const HpaAttnChunk* at, const HpaFusedGemm* chain, int nph, unsigned* ctl, int chain_blocks) {
    HPA_REQUIRE(nph >= 0 && nph <= kMaxPh, "lane_layer: 0..4 chain phases");
    HPA_REQUIRE(nph == 0 || (chain && ctl && chain_blocks > 0), "lane_layer: chain needs descriptors, ctl, blocks");
    AttnChunk a;
    memset(&a, 0, sizeof(a));
    int P = 16;
    if (at) {
        HPA_REQUIRE(at->q && at->pool && at->pool->base && at->block_table && at->pos && at->out_frag,
                    "lane_layer: null attention argument");
        const HpaKVPool* pool = at->pool;
        HPA_REQUIRE(pool->dtype == HPA_F32 && pool->head_size == hpa_attn::HS, "lane_layer: fp32 pool, head 64");
        HPA_REQUIRE(at->layer >= 0 && at->layer < pool->num_layers, "lane_layer: layer out of range");
        HPA_REQUIRE(at->B > 0, "lane_layer: B");
        HPA_REQUIRE(((uintptr_t)at->q & 15) == 0 && ((uintptr_t)at->out_frag & 15) == 0,
                    "lane_layer: q / out must be 16-byte aligned");
        a.q = at->q;
        a.layer_base = (const float*)pool->base + (size_t)at->layer * pool->layer_elems;
        a.page_elems = pool->page_elems;
        a.NH = pool->num_heads;
        a.bt = at->block_table;
        a.bt_stride = at->bt_stride;
        a.pos = at->pos;
        a.state = nullptr;  // one chunk: no carried state
        a.out = at->out_frag;
        a.B = at->B;
        a.chunk = 0;
        a.nchunks = 1;
        const float log2e = 1.4426950408889634f;
        a.qscale = (float)(1.0 / sqrt((double)hpa_attn::HS)) * log2e;
        a.m_init = -10000.0f * log2e;  // the reference's maxval = -10000 (paged_infer.c:187)
        a.nblocks = at->B * a.NH;
        P = pool->page_size;
    }
    Chain c;
    memset(&c, 0, sizeof(c));
    c.nph = nph;
    c.ctl = ctl;
    c.nblocks = nph > 0 ? chain_blocks : 0;
    static const int want_epi[kMaxPh] = {HPA_FEPI_RESID, HPA_FEPI_GELU, HPA_FEPI_RESID, HPA_FEPI_QKV};
    for (int i = 0; i < nph; i++) {
        const HpaFusedGemm* gd = &chain[i];
        HPA_REQUIRE(gd->epilogue == want_epi[i], "lane_layer: chain must be attproj, fc, fcproj, qkv");
        if (hpa_gemm::fused_prepare(gd, &c.g[i])) return 1;
        FG& g = c.g[i];
        g.gx = g.ntn;
        g.gy = g.Mp / 16;
        HPA_REQUIRE(g.gy <= kMaxRb, "lane_layer: at most 64 rows per lane");
        HPA_REQUIRE(i == 0 || g.gy == c.gy, "lane_layer: phases must share the row count");
        c.gy = g.gy;
        c.gx[i] = g.ntn;
        c.os[i] = g.K16 == kNW * 12 ? 1 : 0;
        c.total += g.gx * g.gy;
    }
    switch (P) {
        case 8: return launch_lane<8>(a, c);
        case 16: return launch_lane<16>(a, c);
        case 32: return launch_lane<32>(a, c);
        default: return hpa_fail(__FILE__, __LINE__, "lane_layer: page size must be 8, 16 or 32");
    }
}

}  // extern "C"
