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

// ---- balanced form (round 4, VERDICT r3 item 4: small batches) ----
// At B*NH below the CU count the per-(sequence, head) grid leaves CUs idle
// (B = 8: 96 pairs, S = 2 -> 192 workgroups on 256 CUs) and a CU streams at
// most ~25 GB/s, so the launch runs at 3.9 TB/s.  Here the G workgroups
// (one per CU) split the FLATTENED list of 64-token tiles -- pair p = b*NH +
// h holds tiles(b) = ceil((pos[b]+1)/64), pairs in order -- into G equal runs
// [g*T/G, (g+1)*T/G).  A run covers pieces of one or more pairs; each piece is
// folded as a workgroup folds a whole pair, then a pair split over several
// workgroups publishes one record per piece (k = g - the pair's first
// workgroup) and the last arriver merges them in piece order (split_merge:
// the result does not depend on timing); a pair inside one run is written
// directly.  Piece boundaries depend on every sequence's context, so a row's
// sums (not its value beyond fp32 rounding) depend on the batch.
template <int P, int NW, bool FRAG, bool BF16>
__global__ __launch_bounds__(NW * 64, 1) void paged_attn_decode_flat(
    const float* __restrict__ q, const void* __restrict__ layer_base, size_t page_elems, int NH,
    const int* __restrict__ block_table, int bt_stride, const int* __restrict__ pos, float* __restrict__ out,
    float qscale, float m_init, int B, int kmax, float* __restrict__ ws) {
    constexpr int TILE = P * HS;
    __shared__ float s_m[NW];
    __shared__ float s_l[NW];
    __shared__ float4 s_acc[NW * 16];
    __shared__ int s_pref[65];  // tiles of sequences 0..b-1 (b <= 64)
    const int lane = threadIdx.x & 63;
    if (threadIdx.x < 64) {  // inclusive scan of tiles(b) over the lanes
        int t = lane < B ? (pos[lane] + 64) >> 6 : 0;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int u = __shfl_up(t, o, 64);
            if (lane >= o) t += u;
        }
        s_pref[lane + 1] = t;
        if (lane == 0) s_pref[0] = 0;
    }
    __syncthreads();
    const long long T = (long long)NH * s_pref[B];
    // runs of at least one tile: at most T workgroups take part (an empty run
    // would be counted by the merge of a pair it never reaches)
    const int G = (int)min((long long)gridDim.x, T), g = blockIdx.x;
    if (g >= G) return;
    long long lo = (long long)g * T / G;
    const long long hi = (long long)(g + 1) * T / G;
    // the workgroup holding flattened tile t: the largest g' with g' * T / G <= t
    auto wg_of = [&](long long t) { return (int)(((t + 1) * G - 1) / T); };
    int b = 0;
    while (b + 1 < B && (long long)NH * s_pref[b + 1] <= lo) ++b;
    const float* fbase = reinterpret_cast<const float*>(layer_base);
    const unsigned short* hbase = reinterpret_cast<const unsigned short*>(layer_base);
    int* cnt_all = reinterpret_cast<int*>(ws + (size_t)B * NH * kmax * kRec);
    while (lo < hi) {
        while ((long long)NH * s_pref[b + 1] <= lo) ++b;  // the pair's sequence
        const int tb = s_pref[b + 1] - s_pref[b];
        const long long pb = (long long)NH * s_pref[b];   // the sequence's first flattened tile
        const int h = (int)((lo - pb) / tb);
        const long long ps = pb + (long long)h * tb, pe = ps + tb;  // the pair's flattened tiles
        const int it0 = (int)(lo - ps);
        const int it1 = (int)(min(hi, pe) - ps);
        const int bh = b * NH + h;
        const int ctx = pos[b] + 1;
        const float* qh = q + (size_t)bh * HS;
        const int* bt = block_table + (size_t)b * bt_stride;
        const int g0 = wg_of(ps), g1 = wg_of(pe - 1);
        float m = m_init, l = 0.f;
        if constexpr (BF16) {
            float4 acc[2] = {make_float4(0.f, 0.f, 0.f, 0.f), make_float4(0.f, 0.f, 0.f, 0.f)};
            attn_tiles_bf16<P, NW>(qh, hbase + (size_t)h * TILE, hbase + (size_t)(NH + h) * TILE, page_elems, bt,
                                   bt_stride, ctx, it0, it1, qscale, m, l, acc);
            if (attn_fold_bf16<NW>(m, l, acc, s_m, s_l, s_acc) &&
                (g0 == g1 || split_merge<2>(ws + (size_t)bh * kmax * kRec, cnt_all + bh, g1 - g0 + 1, g - g0, m, l,
                                            acc, true))) {
                const float inv = l == 0.f ? 0.f : 1.f / l;
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    const int col = h * HS + 8 * lane + 4 * k;
                    const size_t oi = FRAG ? hpa::frag_index(b, col, NH * HS) : (size_t)b * NH * HS + col;
                    *reinterpret_cast<float4*>(out + oi) =
                        make_float4(acc[k].x * inv, acc[k].y * inv, acc[k].z * inv, acc[k].w * inv);
                }
            }
        } else {
            float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
            attn_tiles<P, NW>(qh, fbase + (size_t)h * TILE, fbase + (size_t)(NH + h) * TILE, page_elems, bt, bt_stride,
                              ctx, it0, it1, qscale, m, l, acc);
            if (attn_fold<NW>(m, l, acc, s_m, s_l, s_acc) &&
                (g0 == g1 ||
                 split_merge<1>(ws + (size_t)bh * kmax * kRec, cnt_all + bh, g1 - g0 + 1, g - g0, m, l, &acc, true))) {
                const size_t oi =
                    FRAG ? hpa::frag_index(b, h * HS + 4 * lane, NH * HS) : ((size_t)b * NH + h) * HS + 4 * lane;
                const float inv = l == 0.f ? 0.f : 1.f / l;
                *reinterpret_cast<float4*>(out + oi) = make_float4(acc.x * inv, acc.y * inv, acc.z * inv, acc.w * inv);
            }
        }
        __syncthreads();  // the fold's LDS is reused by the next piece
        lo = min(hi, pe);
    }
}

// The balanced form with every tile of a run in flight at once: 16 waves,
// wave w takes the run's tile lo + w alone (the host picks this kernel when
// no run can exceed 16 tiles: B*NH*ceil(max_ctx/64) <= 16 G), the waves of a
// piece fold in wave (= tile) order through LDS, and each piece's first wave
// publishes or merges it -- the pieces of a run no longer follow each other.
template <int P, bool FRAG, bool BF16>
__global__ __launch_bounds__(1024, 1) void paged_attn_decode_flat16(
    const float* __restrict__ q, const void* __restrict__ layer_base, size_t page_elems, int NH,
    const int* __restrict__ block_table, int bt_stride, const int* __restrict__ pos, float* __restrict__ out,
    float qscale, float m_init, int B, int kmax, float* __restrict__ ws) {
    constexpr int NW = 16, TILE = P * HS;
    constexpr int KC = BF16 ? 2 : 1;   // float4 chunks per result lane
    constexpr int NL = BF16 ? 8 : 16;  // result lanes of a folded wave
    __shared__ float s_m[NW];
    __shared__ float s_l[NW];
    __shared__ float4 s_acc[NW * 16];
    __shared__ int s_pref[65];
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (threadIdx.x < 64) {
        int t = lane < B ? (pos[lane] + 64) >> 6 : 0;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int u = __shfl_up(t, o, 64);
            if (lane >= o) t += u;
        }
        s_pref[lane + 1] = t;
        if (lane == 0) s_pref[0] = 0;
    }
    __syncthreads();
    const long long T = (long long)NH * s_pref[B];
    const int G = (int)min((long long)gridDim.x, T), g = blockIdx.x;
    if (g >= G) return;
    const long long lo = (long long)g * T / G, hi = (long long)(g + 1) * T / G;
    auto wg_of = [&](long long t) { return (int)(((t + 1) * G - 1) / T); };
    const long long j = lo + w;  // this wave's tile
    const bool act = j < hi;
    int b = 0;
    if (act)
        while ((long long)NH * s_pref[b + 1] <= j) ++b;
    const int tb = max(s_pref[b + 1] - s_pref[b], 1);
    const long long pb = (long long)NH * s_pref[b];
    const int h = act ? (int)((j - pb) / tb) : 0;
    const long long ps = pb + (long long)h * tb, pe = ps + tb;
    const int bh = b * NH + h;
    const int ctx = pos[b] + 1;
    const float* qh = q + (size_t)bh * HS;
    const int* bt = block_table + (size_t)b * bt_stride;
    float m = m_init, l = 0.f;
    float4 acc[KC];
#pragma unroll
    for (int k = 0; k < KC; ++k) acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (act) {
        const int it = (int)(j - ps);
        if constexpr (BF16) {
            const unsigned short* base = reinterpret_cast<const unsigned short*>(layer_base);
            attn_tiles_bf16<P, 1>(qh, base + (size_t)h * TILE, base + (size_t)(NH + h) * TILE, page_elems, bt,
                                  bt_stride, ctx, it, it + 1, qscale, m, l, acc, 0);
        } else {
            const float* base = reinterpret_cast<const float*>(layer_base);
            attn_tiles<P, 1>(qh, base + (size_t)h * TILE, base + (size_t)(NH + h) * TILE, page_elems, bt, bt_stride,
                             ctx, it, it + 1, qscale, m, l, acc[0], 0);
        }
    }
    // the wave's token groups (lane bits above the result lanes), then its sum
#pragma unroll
    for (int o = NL; o <= 32; o <<= 1)
#pragma unroll
        for (int k = 0; k < KC; ++k) {
            acc[k].x += __shfl_xor(acc[k].x, o, 64);
            acc[k].y += __shfl_xor(acc[k].y, o, 64);
            acc[k].z += __shfl_xor(acc[k].z, o, 64);
            acc[k].w += __shfl_xor(acc[k].w, o, 64);
        }
    l = hpa::wave_sum(l);
    if (lane == 0) {
        s_m[w] = m;
        s_l[w] = l;
    }
    if (lane < NL)
#pragma unroll
        for (int k = 0; k < KC; ++k) s_acc[w * 16 + lane * KC + k] = acc[k];
    __syncthreads();
    const long long j0 = max(lo, ps), j1 = min(hi, pe);  // this wave's piece of the run
    if (!act || j != j0 || lane >= NL) return;          // one wave per piece goes on
    const int w0 = (int)(j0 - lo), w1 = (int)(j1 - lo);
    float M = s_m[w0];
    for (int i = w0 + 1; i < w1; ++i) M = fmaxf(M, s_m[i]);
    float L = 0.f;
    float4 O[KC];
#pragma unroll
    for (int k = 0; k < KC; ++k) O[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int i = w0; i < w1; ++i) {  // waves = tiles in order
        const float f = exp2f(s_m[i] - M);
        L = fmaf(s_l[i], f, L);
#pragma unroll
        for (int k = 0; k < KC; ++k) {
            const float4 a = s_acc[i * 16 + lane * KC + k];
            O[k].x = fmaf(a.x, f, O[k].x);
            O[k].y = fmaf(a.y, f, O[k].y);
            O[k].z = fmaf(a.z, f, O[k].z);
            O[k].w = fmaf(a.w, f, O[k].w);
        }
    }
    const int g0 = wg_of(ps), g1 = wg_of(pe - 1);
    int* cnt = reinterpret_cast<int*>(ws + (size_t)B * NH * kmax * kRec) + bh;
    if (g0 != g1 && !split_merge<KC>(ws + (size_t)bh * kmax * kRec, cnt, g1 - g0 + 1, g - g0, M, L, O, true)) return;
    const float inv = L == 0.f ? 0.f : 1.f / L;
#pragma unroll
    for (int k = 0; k < KC; ++k) {
        const int col = h * HS + (BF16 ? 8 * lane + 4 * k : 4 * lane);
        const size_t oi = FRAG ? hpa::frag_index(b, col, NH * HS) : (size_t)b * NH * HS + col;
        *reinterpret_cast<float4*>(out + oi) = make_float4(O[k].x * inv, O[k].y * inv, O[k].z * inv, O[k].w * inv);
    }
}

template <int P, bool FRAG, bool BF16>
int launch_flat(const float* q, const HpaKVPool* pool, int layer, const int* bt, int bt_stride, const int* pos,
                float* out, int B, int nw, int G, int kmax, float* ws) {
    const void* base = (const char*)pool->base + (size_t)layer * pool->layer_elems * pool->elem_bytes;
    const float log2e = 1.4426950408889634f;
    const float qscale = (float)(1.0 / sqrt((double)HS)) * log2e;
    const float m_init = -10000.0f * log2e;
    if (nw == 16)
        paged_attn_decode_flat16<P, FRAG, BF16><<<G, 1024, 0, hpa_stream()>>>(
            q, base, pool->page_elems, pool->num_heads, bt, bt_stride, pos, out, qscale, m_init, B, kmax, ws);
    else if (nw == 8)
        paged_attn_decode_flat<P, 8, FRAG, BF16><<<G, 512, 0, hpa_stream()>>>(
            q, base, pool->page_elems, pool->num_heads, bt, bt_stride, pos, out, qscale, m_init, B, kmax, ws);
    else
        paged_attn_decode_flat<P, 4, FRAG, BF16><<<G, 256, 0, hpa_stream()>>>(
            q, base, pool->page_elems, pool->num_heads, bt, bt_stride, pos, out, qscale, m_init, B, kmax, ws);
    HPA_LAUNCH_CHECK();
    return 0;
}

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

// pieces per pair at most: a pair of t tiles meets at most t + 1 runs
static int flat_kmax(int max_ctx) { return (max_ctx + 63) / 64 + 1; }

size_t hpa_attn_flat_ws_bytes(int B, int num_heads, int max_ctx) {
    if (B <= 0 || num_heads <= 0 || max_ctx <= 0) return 0;
    const size_t pairs = (size_t)B * num_heads;
    return pairs * flat_kmax(max_ctx) * kRec * sizeof(float) + pairs * sizeof(int);
}

int hpa_paged_attention_decode_flat(const float* q, const HpaKVPool* pool, int layer, const int* block_table,
                                    int bt_stride, const int* pos, float* out, int B, int max_ctx, void* ws,
                                    int out_frag, int waves, int workgroups) {
    HPA_REQUIRE(pool && pool->base, "pool not created");
    HPA_REQUIRE(pool->dtype == HPA_F32 || pool->dtype == HPA_BF16, "decode attention: fp32 or bf16 pool");
    HPA_REQUIRE(pool->head_size == HS, "decode attention requires head_size 64");
    HPA_REQUIRE(layer >= 0 && layer < pool->num_layers, "layer out of range");
    HPA_REQUIRE(B > 0 && B <= 64 && q && out && block_table && pos && ws, "decode attention flat: B 1..64, workspace");
    HPA_REQUIRE(max_ctx > 0, "decode attention flat: max_ctx (every pos[b] < max_ctx)");
    HPA_REQUIRE(((uintptr_t)q & 15) == 0 && ((uintptr_t)out & 15) == 0, "q/out must be 16-byte aligned");
    HPA_REQUIRE(waves == 0 || waves == 4 || waves == 8 || waves == 16, "decode attention flat: waves 4, 8 or 16");
    int G = workgroups;
    if (G <= 0) {
        int dev = 0;
        HPA_CHECK(hipGetDevice(&dev));
        HPA_CHECK(hipDeviceGetAttribute(&G, hipDeviceAttributeMultiprocessorCount, dev));
    }
    const int kmax = flat_kmax(max_ctx);
    // 0: 16 waves with every tile of a run in flight when no run can exceed 16
    // tiles (B*NH*ceil(max_ctx/64) <= 16 G), else 4; hpa_set_attention_waves
    // 8 -> 8, any other override -> 4
    const bool fits16 = (long long)B * pool->num_heads * (kmax - 1) <= 16LL * G;
    int nw = waves;
    if (!nw) nw = g_attn_waves == 8 ? 8 : g_attn_waves ? 4 : fits16 ? 16 : 4;
    HPA_REQUIRE(nw != 16 || fits16,
                "decode attention flat: 16 waves need B*NH*ceil(max_ctx/64) <= 16 workgroups");
    const bool bf = pool->dtype == HPA_BF16, frag = out_frag != 0;
    float* w = (float*)ws;
#define HPA_FLAT_CASE(PS)                                                                                       \
    case PS:                                                                                                     \
        if (bf)                                                                                                  \
            return frag ? launch_flat<PS, true, true>(q, pool, layer, block_table, bt_stride, pos, out, B, nw, G, kmax, w) \
                        : launch_flat<PS, false, true>(q, pool, layer, block_table, bt_stride, pos, out, B, nw, G, kmax, w); \
        return frag ? launch_flat<PS, true, false>(q, pool, layer, block_table, bt_stride, pos, out, B, nw, G, kmax, w)     \
                    : launch_flat<PS, false, false>(q, pool, layer, block_table, bt_stride, pos, out, B, nw, G, kmax, w);
    switch (pool->page_size) {
        HPA_FLAT_CASE(8)
        HPA_FLAT_CASE(16)
        HPA_FLAT_CASE(32)
        HPA_FLAT_CASE(64)
        default: return hpa_fail(__FILE__, __LINE__, "page size must be 8, 16, 32 or 64");
    }
#undef HPA_FLAT_CASE
}

}  // extern "C"
