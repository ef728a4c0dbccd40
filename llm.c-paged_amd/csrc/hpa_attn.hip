// hpa_attn.hip -- paged decode attention for gfx950 (CDNA4, wave64).
//
// Replaces attention_paged (reference paged_infer.c:163-240) for the decode
// step: ONE query row per sequence at absolute position pos[b], keys/values
// of positions 0..pos[b] gathered through the sequence's block table.
//
// Layout (HpaKVPool, hip_paged_attn.h): per (layer, page) K tiles
// [head][16 chunks][P tokens][4 floats] and V tiles [head][P tokens][64].
//
// Work decomposition: one workgroup of NW waves per (sequence, head); the
// context is cut into 64-token tiles, tile `it` goes to wave it % NW.
//  * QK^T, lane-per-token: lane l owns token t0+l.  16 float4 loads per lane
//    (one per 4-dim chunk); a wave-instruction reads P*16 contiguous bytes of
//    each of the 64/P pages it touches (256 B at P=16: two full 128-B lines).
//    The dot product needs no cross-lane reduction.
//  * softmax: online (running max m, per-lane partial sum l), one wave max
//    reduction per tile; exp2 with log2(e) folded into the q pre-scale.  The
//    running max starts at -10000 (in natural-log units) exactly like the
//    reference's `maxval = -10000.0f` (:187), so all-very-negative rows give
//    the same zero output as the reference's expsum==0 branch (:213).
//  * PV, lane-per-dimension: lane (g = l>>4, d4 = l&15) accumulates dims
//    4*d4..4*d4+3 of tokens t0+4i+g (i = 0..15); one wave-instruction reads 4
//    consecutive 256-B token rows = 1 KiB contiguous.  p values arrive by
//    ds_bpermute (__shfl); the 4 lane groups are summed once at the end.
//  * waves combine (m, l, acc) through LDS; wave 0 writes out[b][h*64..+64].
// MFMA is not used: with one query row the QK^T / PV contractions are
// matrix-vector (M = 1), i.e. HBM-bound at ~0.5 FLOP/B; the MFMA path belongs
// to multi-query prefill.
#include <math.h>

#include "hpa_attn_body.h"

namespace {
using namespace hpa_attn;

template <int P, int NW, bool FRAG, bool BF16>
__global__ __launch_bounds__(NW * 64, 3) void paged_attn_decode_f32(
    const float* __restrict__ q, const void* __restrict__ layer_base, size_t page_elems, int NH,
    const int* __restrict__ block_table, int bt_stride, const int* __restrict__ pos,
    float* __restrict__ out, float qscale, float m_init) {
    constexpr int TILE = P * HS;
    __shared__ float s_m[NW];
    __shared__ float s_l[NW];
    __shared__ float4 s_acc[NW * 16];

    const int bh = blockIdx.x;
    const int b = bh / NH;
    const int h = bh - b * NH;
    const int lane = threadIdx.x & 63;
    const int ctx = pos[b] + 1;

    // q is identical in every lane and read-only here: it is loaded with
    // scalar loads into SGPRs (v_fmac takes one SGPR operand), so the 64
    // VGPRs a per-lane copy would cost stay free for K/V loads.  The
    // 1/sqrt(hs) * log2(e) scale is applied to the finished dot (as the
    // reference applies `val *= scale` after the dot, :197).
    const float* __restrict__ qh = q + ((size_t)b * NH + h) * HS;
    const int* bt = block_table + (size_t)b * bt_stride;
    const int n_it = (ctx + 63) >> 6;
    float m = m_init;
    float l = 0.f;
    if constexpr (BF16) {
        const unsigned short* base = reinterpret_cast<const unsigned short*>(layer_base);
        float4 acc[2] = {make_float4(0.f, 0.f, 0.f, 0.f), make_float4(0.f, 0.f, 0.f, 0.f)};
        attn_tiles_bf16<P, NW>(qh, base + (size_t)h * TILE, base + (size_t)(NH + h) * TILE, page_elems, bt, bt_stride, ctx,
                               0, n_it, qscale, m, l, acc);
        if (!attn_fold_bf16<NW>(m, l, acc, s_m, s_l, s_acc)) return;
        const float inv = l == 0.f ? 0.f : 1.f / l;
#pragma unroll
        for (int k = 0; k < 2; ++k) {  // dims 8*lane + 4k .. +3
            const int col = h * HS + 8 * lane + 4 * k;
            const size_t oi = FRAG ? hpa::frag_index(b, col, NH * HS) : (size_t)b * NH * HS + col;
            *reinterpret_cast<float4*>(out + oi) =
                make_float4(acc[k].x * inv, acc[k].y * inv, acc[k].z * inv, acc[k].w * inv);
        }
    } else {
        const float* base = reinterpret_cast<const float*>(layer_base);
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
        attn_tiles<P, NW>(qh, base + (size_t)h * TILE, base + (size_t)(NH + h) * TILE, page_elems, bt, bt_stride, ctx,
                          0, n_it, qscale, m, l, acc);
        if (!attn_fold<NW>(m, l, acc, s_m, s_l, s_acc)) return;
        // out[b][h*64 + 4*lane .. +3]: row-major, or the frag layout the next
        // GEMM reads (4 consecutive columns stay one contiguous float4 there)
        const size_t oi =
            FRAG ? hpa::frag_index(b, h * HS + 4 * lane, NH * HS) : ((size_t)b * NH + h) * HS + 4 * lane;
        const float inv = l == 0.f ? 0.f : 1.f / l;
        *reinterpret_cast<float4*>(out + oi) = make_float4(acc.x * inv, acc.y * inv, acc.z * inv, acc.w * inv);
    }
}

template <int P, bool FRAG, bool BF16>
int launch_decode(const float* q, const HpaKVPool* pool, int layer, const int* bt, int bt_stride,
                  const int* pos, float* out, int B, int nw) {
    const void* base = (const char*)pool->base + (size_t)layer * pool->layer_elems * pool->elem_bytes;
    const float log2e = 1.4426950408889634f;
    const float qscale = (float)(1.0 / sqrt((double)HS)) * log2e;
    const float m_init = -10000.0f * log2e;
    dim3 grid(B * pool->num_heads);
    switch (nw) {
        case 1:
            paged_attn_decode_f32<P, 1, FRAG, BF16><<<grid, 64, 0, hpa_stream()>>>(
                q, base, pool->page_elems, pool->num_heads, bt, bt_stride, pos, out, qscale, m_init);
            break;
        case 2:
            paged_attn_decode_f32<P, 2, FRAG, BF16><<<grid, 128, 0, hpa_stream()>>>(
                q, base, pool->page_elems, pool->num_heads, bt, bt_stride, pos, out, qscale, m_init);
            break;
        case 8:
            paged_attn_decode_f32<P, 8, FRAG, BF16><<<grid, 512, 0, hpa_stream()>>>(
                q, base, pool->page_elems, pool->num_heads, bt, bt_stride, pos, out, qscale, m_init);
            break;
        default:
            paged_attn_decode_f32<P, 4, FRAG, BF16><<<grid, 256, 0, hpa_stream()>>>(
                q, base, pool->page_elems, pool->num_heads, bt, bt_stride, pos, out, qscale, m_init);
            break;
    }
    HPA_LAUNCH_CHECK();
    return 0;
}

int g_attn_waves = 4;

}  // namespace

extern "C" {

// waves per (sequence, head) workgroup: 1, 2, 4 (default) or 8
int hpa_set_attention_waves(int nw) {
    HPA_REQUIRE(nw == 1 || nw == 2 || nw == 4 || nw == 8, "attention waves must be 1, 2, 4 or 8");
    g_attn_waves = nw;
    return 0;
}

static int attn_dispatch(const float* q, const HpaKVPool* pool, int layer, const int* block_table,
                         int bt_stride, const int* pos, float* out, int B, bool frag) {
    HPA_REQUIRE(pool && pool->base, "pool not created");
    HPA_REQUIRE(pool->dtype == HPA_F32 || pool->dtype == HPA_BF16, "decode attention: fp32 or bf16 pool");
    HPA_REQUIRE(pool->head_size == HS, "decode attention requires head_size 64");
    HPA_REQUIRE(layer >= 0 && layer < pool->num_layers, "layer out of range");
    HPA_REQUIRE(B > 0 && q && out && block_table && pos, "bad arguments");
    HPA_REQUIRE(((uintptr_t)q & 15) == 0 && ((uintptr_t)out & 15) == 0, "q/out must be 16-byte aligned");
    const bool bf = pool->dtype == HPA_BF16;
#define HPA_ATTN_CASE(PS)                                                                              \
    case PS:                                                                                            \
        if (bf)                                                                                         \
            return frag ? launch_decode<PS, true, true>(q, pool, layer, block_table, bt_stride, pos, out, B, \
                                                        g_attn_waves)                                   \
                        : launch_decode<PS, false, true>(q, pool, layer, block_table, bt_stride, pos, out, \
                                                         B, g_attn_waves);                              \
        return frag ? launch_decode<PS, true, false>(q, pool, layer, block_table, bt_stride, pos, out, B, \
                                                     g_attn_waves)                                      \
                    : launch_decode<PS, false, false>(q, pool, layer, block_table, bt_stride, pos, out, B, \
                                                      g_attn_waves);
    switch (pool->page_size) {
        HPA_ATTN_CASE(8)
        HPA_ATTN_CASE(16)
        HPA_ATTN_CASE(32)
        HPA_ATTN_CASE(64)
        default: return hpa_fail(__FILE__, __LINE__, "page size must be 8, 16, 32 or 64");
    }
#undef HPA_ATTN_CASE
}

int hpa_paged_attention_decode(const float* q, const HpaKVPool* pool, int layer,
                               const int* block_table, int bt_stride, const int* pos, float* out,
                               int B) {
    return attn_dispatch(q, pool, layer, block_table, bt_stride, pos, out, B, false);
}

int hpa_paged_attention_decode_frag(const float* q, const HpaKVPool* pool, int layer,
                                    const int* block_table, int bt_stride, const int* pos,
                                    float* out_frag, int B) {
    return attn_dispatch(q, pool, layer, block_table, bt_stride, pos, out_frag, B, true);
}

}  // extern "C"
