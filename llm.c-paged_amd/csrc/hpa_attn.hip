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

#include "hpa_internal.h"

namespace {

constexpr int HS = 64;

typedef float f32x4v __attribute__((ext_vector_type(4)));

// K/V rows are streamed once per step by the one workgroup of their
// (sequence, head): non-temporal loads (MI355X_MICROARCH.md "nt-weights")
__device__ __forceinline__ float4 load_stream(const float* ptr) {
    const f32x4v v = __builtin_nontemporal_load(reinterpret_cast<const f32x4v*>(ptr));
    return make_float4(v.x, v.y, v.z, v.w);
}

template <int P, int NW, bool FRAG>
__global__ __launch_bounds__(NW * 64, 3) void paged_attn_decode_f32(
    const float* __restrict__ q, const float* __restrict__ layer_base, size_t page_elems, int NH,
    const int* __restrict__ block_table, int bt_stride, const int* __restrict__ pos,
    float* __restrict__ out, float qscale, float m_init) {
    static_assert(P % 4 == 0 && 64 % P == 0, "page size must divide 64 and be a multiple of 4");
    constexpr int TILE = P * HS;
    __shared__ float s_m[NW];
    __shared__ float s_l[NW];
    __shared__ float4 s_acc[NW][16];

    const int bh = blockIdx.x;
    const int b = bh / NH;
    const int h = bh - b * NH;
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const int g = lane >> 4;
    const int d4 = lane & 15;
    const int ctx = pos[b] + 1;
    const int* __restrict__ bt = block_table + (size_t)b * bt_stride;

    // q is identical in every lane and read-only here: it is loaded with
    // scalar loads into SGPRs (v_fmac takes one SGPR operand), so the 64
    // VGPRs a per-lane copy would cost stay free for K/V loads.  The
    // 1/sqrt(hs) * log2(e) scale is applied to the finished dot (as the
    // reference applies `val *= scale` after the dot, :197).
    const float* __restrict__ qh = q + ((size_t)b * NH + h) * HS;
    const float* __restrict__ kbase = layer_base + (size_t)h * TILE;
    const float* __restrict__ vbase = layer_base + (size_t)(NH + h) * TILE;
    const int v_lane_off = g * HS + d4 * 4;

    float m = m_init;
    float l = 0.f;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    const int n_it = (ctx + 63) >> 6;

    // one memory round trip per 64-token tile: the tile's page ids were
    // fetched during the previous tile; K and V rows are issued together
    // (both depend only on the page ids), then the next tile's page ids.
    int it = w;
    int pid = 0;
    if (it < n_it) {
        const unsigned t0 = (unsigned)it << 6, tok = t0 + lane;
        pid = bt[(tok < (unsigned)ctx ? tok : t0) / P];
    }
    for (; it < n_it; it += NW) {
        const unsigned t0 = (unsigned)it << 6;
        const unsigned tok = t0 + lane;
        const bool valid = tok < (unsigned)ctx;
        const float* kt = kbase + (size_t)(unsigned)pid * page_elems + (tok % P) * 4;
        float4 kv[16], vv[16];
#pragma unroll
        for (int c = 0; c < 16; ++c) kv[c] = load_stream(kt + c * P * 4);
        // PV operands: lane (g, d4) takes tokens t0 + 4i + g, dims 4*d4..+3.
        // The row address splits into a wave-uniform part (page of tokens
        // t0+4i..+3, slot (4i)%P; t0 % P == 0) and a per-lane offset that is
        // the same for every i, so each load is SGPR base + one shared VGPR.
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int vpid = __builtin_amdgcn_readlane(pid, 4 * i);
            const float* vrow = vbase + (size_t)(unsigned)vpid * page_elems + ((4 * i) % P) * HS;
            vv[i] = (t0 + 4 * i + g) < (unsigned)ctx ? load_stream(vrow + v_lane_off)
                                           : make_float4(0.f, 0.f, 0.f, 0.f);
        }
        {   // next tile's page ids
            const int itn = it + NW;
            const unsigned t0n = (unsigned)itn << 6, tokn = t0n + lane;
            if (itn < n_it) pid = bt[(tokn < (unsigned)ctx ? tokn : t0n) / P];
        }
        // ---- QK^T: lane-per-token over 16 chunks of 4 dims
        float s = 0.f;
#pragma unroll
        for (int c = 0; c < 16; ++c) {
            s = fmaf(qh[4 * c + 0], kv[c].x, s);
            s = fmaf(qh[4 * c + 1], kv[c].y, s);
            s = fmaf(qh[4 * c + 2], kv[c].z, s);
            s = fmaf(qh[4 * c + 3], kv[c].w, s);
        }
        s = valid ? s * qscale : -INFINITY;
        // ---- online softmax (log2 domain)
        const float mt = hpa::wave_max(s);
        const float mn = fmaxf(m, mt);
        const float alpha = exp2f(m - mn);
        const float p = exp2f(s - mn);
        l = fmaf(l, alpha, p);
        acc.x *= alpha;
        acc.y *= alpha;
        acc.z *= alpha;
        acc.w *= alpha;
        m = mn;
        // ---- PV
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const float pi = __shfl(p, 4 * i + g, 64);
            acc.x = fmaf(pi, vv[i].x, acc.x);
            acc.y = fmaf(pi, vv[i].y, acc.y);
            acc.z = fmaf(pi, vv[i].z, acc.z);
            acc.w = fmaf(pi, vv[i].w, acc.w);
        }
    }

    // fold the 4 token groups, then the per-lane sums
#pragma unroll
    for (int o = 16; o <= 32; o <<= 1) {
        acc.x += __shfl_xor(acc.x, o, 64);
        acc.y += __shfl_xor(acc.y, o, 64);
        acc.z += __shfl_xor(acc.z, o, 64);
        acc.w += __shfl_xor(acc.w, o, 64);
    }
    l = hpa::wave_sum(l);

    // out[b][h*64 + 4*lane .. +3]: row-major, or the frag layout the next
    // GEMM reads (4 consecutive columns stay one contiguous float4 there)
    const size_t oi = FRAG ? hpa::frag_index(b, h * HS + 4 * (lane & 15), NH * HS)
                           : ((size_t)b * NH + h) * HS + 4 * (lane & 15);
    float4* o = reinterpret_cast<float4*>(out + oi);
    if constexpr (NW == 1) {
        if (lane < 16) {
            const float inv = l == 0.f ? 0.f : 1.f / l;
            *o = make_float4(acc.x * inv, acc.y * inv, acc.z * inv, acc.w * inv);
        }
    } else {
        if (lane == 0) {
            s_m[w] = m;
            s_l[w] = l;
        }
        if (lane < 16) s_acc[w][lane] = acc;
        __syncthreads();
        if (w == 0 && lane < 16) {
            float M = s_m[0];
#pragma unroll
            for (int i = 1; i < NW; ++i) M = fmaxf(M, s_m[i]);
            float L = 0.f;
            float4 O = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int i = 0; i < NW; ++i) {
                const float f = exp2f(s_m[i] - M);
                L = fmaf(s_l[i], f, L);
                const float4 a = s_acc[i][lane];
                O.x = fmaf(a.x, f, O.x);
                O.y = fmaf(a.y, f, O.y);
                O.z = fmaf(a.z, f, O.z);
                O.w = fmaf(a.w, f, O.w);
            }
            const float inv = L == 0.f ? 0.f : 1.f / L;
            *o = make_float4(O.x * inv, O.y * inv, O.z * inv, O.w * inv);
        }
    }
}

template <int P, bool FRAG>
int launch_decode(const float* q, const HpaKVPool* pool, int layer, const int* bt, int bt_stride,
                  const int* pos, float* out, int B, int nw) {
    const float* base = (const float*)pool->base + (size_t)layer * pool->layer_elems;
    const float log2e = 1.4426950408889634f;
    const float qscale = (float)(1.0 / sqrt((double)HS)) * log2e;
    const float m_init = -10000.0f * log2e;
    dim3 grid(B * pool->num_heads);
    switch (nw) {
        case 1:
            paged_attn_decode_f32<P, 1, FRAG><<<grid, 64, 0, hpa_stream()>>>(
                q, base, pool->page_elems, pool->num_heads, bt, bt_stride, pos, out, qscale, m_init);
            break;
        case 2:
            paged_attn_decode_f32<P, 2, FRAG><<<grid, 128, 0, hpa_stream()>>>(
                q, base, pool->page_elems, pool->num_heads, bt, bt_stride, pos, out, qscale, m_init);
            break;
        case 8:
            paged_attn_decode_f32<P, 8, FRAG><<<grid, 512, 0, hpa_stream()>>>(
                q, base, pool->page_elems, pool->num_heads, bt, bt_stride, pos, out, qscale, m_init);
            break;
        default:
            paged_attn_decode_f32<P, 4, FRAG><<<grid, 256, 0, hpa_stream()>>>(
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
    HPA_REQUIRE(pool->dtype == HPA_F32, "decode attention: fp32 pool expected");
    HPA_REQUIRE(pool->head_size == HS, "decode attention requires head_size 64");
    HPA_REQUIRE(layer >= 0 && layer < pool->num_layers, "layer out of range");
    HPA_REQUIRE(B > 0 && q && out && block_table && pos, "bad arguments");
    HPA_REQUIRE(((uintptr_t)q & 15) == 0 && ((uintptr_t)out & 15) == 0, "q/out must be 16-byte aligned");
#define HPA_ATTN_CASE(PS)                                                                        \
    case PS:                                                                                      \
        return frag ? launch_decode<PS, true>(q, pool, layer, block_table, bt_stride, pos, out, B, \
                                              g_attn_waves)                                        \
                    : launch_decode<PS, false>(q, pool, layer, block_table, bt_stride, pos, out, B, \
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
