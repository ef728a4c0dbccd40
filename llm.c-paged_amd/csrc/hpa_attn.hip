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
//  * split context (flash-decoding): when B*NH workgroups
//    cannot keep every CU streaming (B*NH < ~3 per CU), each (sequence, head)
//    is cut into S ranges of its 64-token tiles, one workgroup each.  A range
//    publishes its folded (m, l, acc) record with write-through (sc1) stores,
//    drains them and draws an arrival ticket (agent-scope atomic add); the
//    last arriver of the (sequence, head) merges the S records in range order
//    (sc1 loads: MI355X_MICROARCH.md "Valid forms", row 1) and writes the
//    output, then rewinds the counter for the next launch.  The merge order is
//    fixed, so results do not depend on which range finishes last.
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
    float* __restrict__ out, float qscale, float m_init, int S, float* __restrict__ ws) {
    constexpr int TILE = P * HS;
    __shared__ float s_m[NW];
    __shared__ float s_l[NW];
    __shared__ float4 s_acc[NW * 16];

    const int bh = S == 1 ? (int)blockIdx.x : (int)blockIdx.x / S;
    const int sr = (int)blockIdx.x - bh * S;  // context range of this workgroup
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
    const int n_it_all = (ctx + 63) >> 6;
    const int it0 = S == 1 ? 0 : (int)((long long)sr * n_it_all / S);
    const int n_it = S == 1 ? n_it_all : (int)((long long)(sr + 1) * n_it_all / S);
    float* rec_bh = S == 1 ? nullptr : ws + (size_t)bh * S * kRec;
    int* cnt = S == 1 ? nullptr : reinterpret_cast<int*>(ws + (size_t)gridDim.x * kRec) + bh;
    float m = m_init;
    float l = 0.f;
    if constexpr (BF16) {
        const unsigned short* base = reinterpret_cast<const unsigned short*>(layer_base);
        float4 acc[2] = {make_float4(0.f, 0.f, 0.f, 0.f), make_float4(0.f, 0.f, 0.f, 0.f)};
        attn_tiles_bf16<P, NW>(qh, base + (size_t)h * TILE, base + (size_t)(NH + h) * TILE, page_elems, bt, bt_stride, ctx,
                               it0, n_it, qscale, m, l, acc);
        if (!attn_fold_bf16<NW>(m, l, acc, s_m, s_l, s_acc)) return;
        if (S > 1 && !split_merge<2>(rec_bh, cnt, S, sr, m, l, acc, true)) return;
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
                          it0, n_it, qscale, m, l, acc);
        if (!attn_fold<NW>(m, l, acc, s_m, s_l, s_acc)) return;
        if (S > 1 && !split_merge<1>(rec_bh, cnt, S, sr, m, l, &acc, true)) return;
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
                  const int* pos, float* out, int B, int nw, int S, float* ws) {
    const void* base = (const char*)pool->base + (size_t)layer * pool->layer_elems * pool->elem_bytes;
    const float log2e = 1.4426950408889634f;
    const float qscale = (float)(1.0 / sqrt((double)HS)) * log2e;
    const float m_init = -10000.0f * log2e;
    dim3 grid(B * pool->num_heads * S);
    switch (nw) {
        case 1:
            paged_attn_decode_f32<P, 1, FRAG, BF16><<<grid, 64, 0, hpa_stream()>>>(
                q, base, pool->page_elems, pool->num_heads, bt, bt_stride, pos, out, qscale, m_init, S, ws);
            break;
        case 2:
            paged_attn_decode_f32<P, 2, FRAG, BF16><<<grid, 128, 0, hpa_stream()>>>(
                q, base, pool->page_elems, pool->num_heads, bt, bt_stride, pos, out, qscale, m_init, S, ws);
            break;
        case 8:
            paged_attn_decode_f32<P, 8, FRAG, BF16><<<grid, 512, 0, hpa_stream()>>>(
                q, base, pool->page_elems, pool->num_heads, bt, bt_stride, pos, out, qscale, m_init, S, ws);
            break;
        default:
            paged_attn_decode_f32<P, 4, FRAG, BF16><<<grid, 256, 0, hpa_stream()>>>(
                q, base, pool->page_elems, pool->num_heads, bt, bt_stride, pos, out, qscale, m_init, S, ws);
            break;
    }
    HPA_LAUNCH_CHECK();
    return 0;
}

int g_attn_waves = 0;  // hpa_set_attention_waves: a process-wide override (0: the caller's choice)


}  // namespace

extern "C" {

// waves per (sequence, head) workgroup for every launch of the process: 1,
// 2, 4 or 8 (timing tools); 0 restores the callers' choice
int hpa_set_attention_waves(int nw) {
    HPA_REQUIRE(nw == 0 || nw == 1 || nw == 2 || nw == 4 || nw == 8, "attention waves must be 0, 1, 2, 4 or 8");
    g_attn_waves = nw;
    return 0;
}

// 8 waves when the B*NH*S workgroups leave CUs without one (each workgroup
// then has a CU's memory pipe to itself and its tiles take half the trips),
// else 4.  tools/attn_scan_r3.py, profiles/r3/attn_scan_r3.txt (ctx 1020):
// B = 8, S = 2: 13.02 vs 13.66 us; B = 16, S = 1: 19.11 vs 20.26; B = 32,
// S = 2 (768 workgroups): 38.65 vs 35.33
int hpa_attn_pick_waves(int B, int num_heads, int splits, int num_cus) {
    if (num_cus <= 0) num_cus = 256;
    return (long)B * num_heads * splits <= num_cus ? 8 : 4;
}

static int attn_dispatch(const float* q, const HpaKVPool* pool, int layer, const int* block_table,
                         int bt_stride, const int* pos, float* out, int B, bool frag, int S, void* ws,
                         int waves = 0) {
    HPA_REQUIRE(pool && pool->base, "pool not created");
    HPA_REQUIRE(pool->dtype == HPA_F32 || pool->dtype == HPA_BF16, "decode attention: fp32 or bf16 pool");
    HPA_REQUIRE(pool->head_size == HS, "decode attention requires head_size 64");
    HPA_REQUIRE(layer >= 0 && layer < pool->num_layers, "layer out of range");
    HPA_REQUIRE(B > 0 && q && out && block_table && pos, "bad arguments");
    HPA_REQUIRE(((uintptr_t)q & 15) == 0 && ((uintptr_t)out & 15) == 0, "q/out must be 16-byte aligned");
    HPA_REQUIRE(S >= 1 && S <= HPA_ATTN_MAX_SPLITS && (S == 1 || ws), "decode attention: splits 1..16, workspace");
    const bool bf = pool->dtype == HPA_BF16;
    float* w = (float*)ws;
    HPA_REQUIRE(waves == 0 || waves == 1 || waves == 2 || waves == 4 || waves == 8, "attention waves 1, 2, 4, 8");
    const int nw = g_attn_waves ? g_attn_waves : waves ? waves : 4;
#define HPA_ATTN_CASE(PS)                                                                                      \
    case PS:                                                                                                    \
        if (bf)                                                                                                 \
            return frag ? launch_decode<PS, true, true>(q, pool, layer, block_table, bt_stride, pos, out, B, nw, S, w) \
                        : launch_decode<PS, false, true>(q, pool, layer, block_table, bt_stride, pos, out, B, nw, S, w); \
        return frag ? launch_decode<PS, true, false>(q, pool, layer, block_table, bt_stride, pos, out, B, nw, S, w)     \
                    : launch_decode<PS, false, false>(q, pool, layer, block_table, bt_stride, pos, out, B, nw, S, w);
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
    return attn_dispatch(q, pool, layer, block_table, bt_stride, pos, out, B, false, 1, nullptr);
}

int hpa_paged_attention_decode_frag(const float* q, const HpaKVPool* pool, int layer,
                                    const int* block_table, int bt_stride, const int* pos,
                                    float* out_frag, int B) {
    return attn_dispatch(q, pool, layer, block_table, bt_stride, pos, out_frag, B, true, 1, nullptr);
}

size_t hpa_attn_ws_bytes(int B, int num_heads, int splits) {
    if (B <= 0 || num_heads <= 0 || splits <= 1) return 0;
    const size_t recs = (size_t)B * num_heads * splits * kRec * sizeof(float);
    return recs + (size_t)B * num_heads * splits * sizeof(int);  // counters ([B*NH], padded by the grid size)
}

// Splits by shape (never by context, which varies per sequence and step).
// Measured (tools/attn_scan.py, GPT-2 124M, ctx 1024, profiles/r2/
// attn_scan_c1024.txt): a launch costs ~6 us beyond its streaming time, and
// a CU streams at most ~25 GB/s, so what pays is (1) more CUs streaming when
// B*NH workgroups leave some idle, without (2) ranges so short that the
// merge's extra round trip shows: B = 8 (96 workgroups) 16.7 us single pass,
// 14.2 at 2 ranges, 15.0 at 4, 17.2 at 8; B = 16 (192) 20.6 single, 22.8 at 2;
// B = 32 (384: 1.5 per CU, a second partial round) 37.4 single, 35.9 at 2;
// B >= 64: single pass.  So: as many ranges as keep B*NH*S within one
// workgroup per CU, or 2 when B*NH falls between one and two per CU.
int hpa_attn_pick_splits(int B, int num_heads, int max_ctx, int num_cus) {
    if (B <= 0 || num_heads <= 0) return 1;
    if (num_cus <= 0) num_cus = 256;
    const long bh = (long)B * num_heads;
    if (bh > num_cus && bh < 2L * num_cus) return max_ctx >= 256 ? 2 : 1;
    int s = 1;
    while (s < HPA_ATTN_MAX_SPLITS && bh * s * 2 <= num_cus && (long)(s * 2) * 128 <= (long)max_ctx) s *= 2;
    return s;
}

int hpa_paged_attention_decode_split(const float* q, const HpaKVPool* pool, int layer, const int* block_table,
                                     int bt_stride, const int* pos, float* out, int B, int splits, void* ws,
                                     int out_frag) {
    return attn_dispatch(q, pool, layer, block_table, bt_stride, pos, out, B, out_frag != 0, splits, ws);
}

int hpa_paged_attention_decode_split_w(const float* q, const HpaKVPool* pool, int layer, const int* block_table,
                                       int bt_stride, const int* pos, float* out, int B, int splits, void* ws,
                                       int out_frag, int waves) {
    return attn_dispatch(q, pool, layer, block_table, bt_stride, pos, out, B, out_frag != 0, splits, ws, waves);
}


}  // extern "C"
