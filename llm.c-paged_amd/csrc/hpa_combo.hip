// hpa_combo.hip -- the pipelined decode launch: one context chunk of one
// micro-batch lane's paged attention (HBM-bound) and one fused GEMM of the
// OTHER lane's layer chain (latency-bound) in the same launch, on disjoint
// workgroups.  Two HIP streams did not overlap these (measured ~1.1x kernel
// concurrency); one launch with two roles does by construction -- the
// "stream beside chain" shape of MI355X_MICROARCH.md.  No workgroup waits on
// another: the attention chunks carry their softmax state through memory
// from launch to launch, and the GEMM chain's links are launch boundaries.
#include <string.h>

#include "hpa_attn_body.h"
#include "hpa_gemm_body.h"

namespace {
using hpa_attn::AttnChunk;
using hpa_gemm::FG;

constexpr int kNW = 4;  // waves per workgroup, both roles

template <int A, int B>
constexpr int cmax() {
    return A > B ? A : B;
}

// GK: 0 = no GEMM role, 1 = one-shot (K/16 = 4 * 12), 2 = looped, one row block
template <int P, int EPI, int GK>
__global__ __launch_bounds__(kNW * 64, 2) void combo_kernel(AttnChunk a, FG g) {
    constexpr int LDS = cmax<hpa_attn::attn_lds_floats<kNW>(),
                             GK == 1 ? hpa_gemm::gemm16_os_lds_floats<kNW>()
                                     : (GK == 2 ? hpa_gemm::gemm16_lds_floats<kNW, 1, 1>() : 0)>();
    __shared__ __attribute__((aligned(16))) float smem[LDS];
    // GEMM-role blocks first: the latency-bound chain link is dispatched
    // before the attention blocks take the slots (gblocks % 8 == 0 keeps
    // both roles' b % 8 XCD order)
    const int bid = blockIdx.x;
    const int gblocks = gridDim.x - a.nblocks;
    if (bid >= gblocks) {
        hpa_attn::attn_chunk_body<P, kNW>(a, bid - gblocks, smem);
    } else if constexpr (GK == 1) {
        hpa_gemm::gemm16_os_body<kNW, EPI, 12>(g, bid, smem);
    } else if constexpr (GK == 2) {
        hpa_gemm::gemm16_body<kNW, EPI, 1, 1>(g, bid, smem);
    }
}

template <int P, int EPI, int GK>
int launch_combo(const AttnChunk& a, const FG& g, int gemm_blocks) {
    combo_kernel<P, EPI, GK><<<a.nblocks + gemm_blocks, kNW * 64, 0, hpa_stream()>>>(a, g);
    HPA_LAUNCH_CHECK();
    return 0;
}

template <int P>
int dispatch_combo(const AttnChunk& a, const FG& g, int gemm_blocks, int epi, int gk) {
    if (gk == 0) return launch_combo<P, 0, 0>(a, g, 0);
    switch (epi * 4 + gk) {
        case HPA_FEPI_QKV * 4 + 1: return launch_combo<P, HPA_FEPI_QKV, 1>(a, g, gemm_blocks);
        case HPA_FEPI_RESID * 4 + 1: return launch_combo<P, HPA_FEPI_RESID, 1>(a, g, gemm_blocks);
        case HPA_FEPI_GELU * 4 + 1: return launch_combo<P, HPA_FEPI_GELU, 1>(a, g, gemm_blocks);
        case HPA_FEPI_QKV * 4 + 2: return launch_combo<P, HPA_FEPI_QKV, 2>(a, g, gemm_blocks);
        case HPA_FEPI_RESID * 4 + 2: return launch_combo<P, HPA_FEPI_RESID, 2>(a, g, gemm_blocks);
        case HPA_FEPI_GELU * 4 + 2: return launch_combo<P, HPA_FEPI_GELU, 2>(a, g, gemm_blocks);
        case HPA_FEPI_LOGITS * 4 + 2: return launch_combo<P, HPA_FEPI_LOGITS, 2>(a, g, gemm_blocks);
        default: return hpa_fail(__FILE__, __LINE__, "attn_chunk_with_gemm: unsupported GEMM role");
    }
}

}  // namespace

extern "C" {

size_t hpa_attn_state_elems(int B, int num_heads) {
    return (size_t)B * num_heads * hpa_attn::kStateStride;
}

int hpa_attn_chunk_with_gemm(const HpaAttnChunk* c, const HpaFusedGemm* gd) {
    HPA_REQUIRE(c && c->q && c->pool && c->pool->base && c->block_table && c->pos && c->state && c->out_frag,
                "attn_chunk: null argument");
    const HpaKVPool* pool = c->pool;
    HPA_REQUIRE(pool->dtype == HPA_F32 && pool->head_size == hpa_attn::HS, "attn_chunk: fp32 pool, head 64");
    HPA_REQUIRE(c->layer >= 0 && c->layer < pool->num_layers, "attn_chunk: layer out of range");
    HPA_REQUIRE(c->B > 0 && c->nchunks > 0 && c->chunk >= 0 && c->chunk < c->nchunks, "attn_chunk: chunk");
    HPA_REQUIRE(((uintptr_t)c->q & 15) == 0 && ((uintptr_t)c->out_frag & 15) == 0 && ((uintptr_t)c->state & 15) == 0,
                "attn_chunk: q / out / state must be 16-byte aligned");
    AttnChunk a;
    a.q = c->q;
    a.layer_base = (const float*)pool->base + (size_t)c->layer * pool->layer_elems;
    a.page_elems = pool->page_elems;
    a.NH = pool->num_heads;
    a.bt = c->block_table;
    a.bt_stride = c->bt_stride;
    a.pos = c->pos;
    a.state = c->state;
    a.out = c->out_frag;
    a.B = c->B;
    a.chunk = c->chunk;
    a.nchunks = c->nchunks;
    const float log2e = 1.4426950408889634f;
    a.qscale = (float)(1.0 / sqrt((double)hpa_attn::HS)) * log2e;
    a.m_init = -10000.0f * log2e;  // the reference's maxval = -10000 (paged_infer.c:187)
    a.nblocks = (c->B * a.NH + 7) / 8 * 8;
    FG g;
    memset(&g, 0, sizeof(g));
    int gk = 0, gemm_blocks = 0, epi = 0;
    if (gd) {
        if (hpa_gemm::fused_prepare(gd, &g)) return 1;
        HPA_REQUIRE((gd->waves == 0 || gd->waves == kNW) && (gd->row_blocks == 0 || gd->row_blocks == 1) &&
                        gd->col_tiles <= 1,
                    "attn_chunk: the GEMM role runs 4 waves, one row block, one column tile");
        gk = (g.K16 == kNW * 12 && gd->variant != 1) ? 1 : 2;
        HPA_REQUIRE(gd->variant != 2 || gk == 1, "attn_chunk: one-shot GEMM role needs K = 768");
        epi = gd->epilogue;
        g.gx = g.ntn;
        g.gy = g.Mp / 16;
        gemm_blocks = ((g.gx + 7) / 8) * 8 * g.gy;
    }
    switch (pool->page_size) {
        case 8: return dispatch_combo<8>(a, g, gemm_blocks, epi, gk);
        case 16: return dispatch_combo<16>(a, g, gemm_blocks, epi, gk);
        case 32: return dispatch_combo<32>(a, g, gemm_blocks, epi, gk);
        default: return hpa_fail(__FILE__, __LINE__, "attn_chunk: page size must be 8, 16 or 32");
    }
}

}  // extern "C"
