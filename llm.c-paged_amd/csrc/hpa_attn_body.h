// hpa_attn_body.h -- device pieces of the paged decode attention (design
// notes in hpa_attn.hip): the per-wave tile loops (fp32 and bf16 pools) and
// the in-workgroup folds of the online-softmax state.
#pragma once
#include <math.h>

#include "hpa_internal.h"

namespace hpa_attn {

constexpr int HS = 64;

typedef float f32x4v __attribute__((ext_vector_type(4)));

// K/V rows are streamed once per step by the one workgroup of their
// (sequence, head): non-temporal loads (MI355X_MICROARCH.md "nt-weights";
// -DHPA_ATTN_NT=0: default-policy loads, an A/B build)
#ifndef HPA_ATTN_NT
#define HPA_ATTN_NT 1
#endif
constexpr int kCpolNt = HPA_ATTN_NT ? 2 : 0;  // buffer-load cache policy: nt (gfx940+ aux bit 1)
__device__ __forceinline__ float4 load_stream(const float* ptr) {
#if HPA_ATTN_NT
    const f32x4v v = __builtin_nontemporal_load(reinterpret_cast<const f32x4v*>(ptr));
#else
    const f32x4v v = *reinterpret_cast<const f32x4v*>(ptr);
#endif
    return make_float4(v.x, v.y, v.z, v.w);
}

// Page ids of a wave's first tile.  The table load is issued without waiting
// for ctx (pos[b] is itself a load at kernel start: one dependent round trip
// fewer before the K/V stream); lanes past ctx then take lane 0's id (token
// t0 < ctx for every tile below it_end), so garbage entries past the
// sequence's pages are never used as addresses.
template <int P>
__device__ __forceinline__ int first_tile_pid(const int* __restrict__ bt, int bt_len, int ctx, int it,
                                              int it_end) {
    const unsigned tok = ((unsigned)it << 6) + (threadIdx.x & 63);
    const int raw = bt[min(tok / P, (unsigned)bt_len - 1u)];  // inside the table row
    const int lane0 = __builtin_amdgcn_readfirstlane(raw);
    return it < it_end && tok < (unsigned)ctx ? raw : lane0;
}

// Single-buffered form (rounds 1-5; -DHPA_ATTN_SWP=0 builds): the tiles
// it = it_begin + w, it_begin + w + NW, ... < it_end of
// one (sequence, head), folded into this wave's online-softmax state
// (m, l: log2 domain; acc: lane (g = lane>>4, d4 = lane&15) holds dims
// 4*d4..+3 summed over tokens t0 + 4i + g).  One memory round trip per tile:
// the tile's page ids were fetched during the previous tile; K and V rows are
// issued together (both depend only on the page ids), then the next ids.
template <int P, int NW>
__device__ __forceinline__ void attn_tiles_single(const float* __restrict__ qh, const float* __restrict__ kbase,
                                           const float* __restrict__ vbase, size_t page_elems,
                                           const int* __restrict__ bt, int bt_len, int ctx, int it_begin,
                                           int it_end, float qscale, float& m, float& l, float4& acc,
                                           int w = (int)(threadIdx.x >> 6)) {
    static_assert(P % 4 == 0 && 64 % P == 0, "page size must divide 64 and be a multiple of 4");
    const int lane = threadIdx.x & 63;
    const int g = lane >> 4;
    const int d4 = lane & 15;
    const int v_lane_off = g * HS + d4 * 4;
    int it = it_begin + w;
    int pid = first_tile_pid<P>(bt, bt_len, ctx, it, it_end);
    for (; it < it_end; it += NW) {
        const unsigned t0 = (unsigned)it << 6;
        const unsigned tok = t0 + lane;
        const bool valid = tok < (unsigned)ctx;
        const float* kt = kbase + (size_t)(unsigned)pid * page_elems + (tok % P) * 4;
        float4 kv[16], vv[16];
#pragma unroll
        for (int c = 0; c < 16; ++c) kv[c] = load_stream(kt + c * P * 4);
        // PV operands: the row address splits into a wave-uniform part (page
        // of tokens t0+4i..+3, slot (4i)%P; t0 % P == 0) and a per-lane offset
        // that is the same for every i: SGPR base + one shared VGPR per load
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int vpid = __builtin_amdgcn_readlane(pid, 4 * i);
            const float* vrow = vbase + (size_t)(unsigned)vpid * page_elems + ((4 * i) % P) * HS;
            vv[i] = (t0 + 4 * i + g) < (unsigned)ctx ? load_stream(vrow + v_lane_off)
                                                     : make_float4(0.f, 0.f, 0.f, 0.f);
        }
        {  // next tile's page ids
            const int itn = it + NW;
            const unsigned t0n = (unsigned)itn << 6, tokn = t0n + lane;
            if (itn < it_end) pid = bt[(tokn < (unsigned)ctx ? tokn : t0n) / P];
        }
        // QK^T: lane-per-token over 16 chunks of 4 dims (q in SGPRs)
        float s = 0.f;
#pragma unroll
        for (int c = 0; c < 16; ++c) {
            s = fmaf(qh[4 * c + 0], kv[c].x, s);
            s = fmaf(qh[4 * c + 1], kv[c].y, s);
            s = fmaf(qh[4 * c + 2], kv[c].z, s);
            s = fmaf(qh[4 * c + 3], kv[c].w, s);
        }
        s = valid ? s * qscale : -INFINITY;
        // online softmax (log2 domain)
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
        // PV
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const float pi = __shfl(p, 4 * i + g, 64);
            acc.x = fmaf(pi, vv[i].x, acc.x);
            acc.y = fmaf(pi, vv[i].y, acc.y);
            acc.z = fmaf(pi, vv[i].z, acc.z);
            acc.w = fmaf(pi, vv[i].w, acc.w);
        }
    }
}

#ifndef HPA_ATTN_SWP
#define HPA_ATTN_SWP 0  // 1 (A/B builds): the software-pipelined loop (measured slower, profiles/r6/experiments/attn_swp.txt)
#endif

// The 64-token tiles it = it_begin + w, it_begin + w + NW, ... < it_end of
// one (sequence, head), folded into this wave's online-softmax state (m, l:
// log2 domain; acc: lane (g = lane>>4, d4 = lane&15) holds dims 4*d4..+3
// summed over tokens t0 + 4i + g).
// The product runs the single-buffered loop (attn_tiles_single: K and V of a
// tile issued together, one memory round trip per tile).  HPA_ATTN_SWP=1 (A/B
// builds, round 6) software-pipelines it: the next tile's K rows are issued
// as soon as this tile's QK^T has consumed its K registers, and its V rows as
// soon as this tile's PV has consumed the V registers (same registers, same
// arithmetic in the same order: bit-identical).  Measured: faster only at 4
// waves per CU (B = 8, S = 1: 15.6 vs 16.9 us), equal at the engine's picks
// and slower at B = 64 (65.6 vs 64.9 us; step 1.120 vs 1.100 ms,
// profiles/r6/experiments/attn_swp.txt): a CU's K/V stream is not bound by
// the math between tiles.
template <int P, int NW>
__device__ __forceinline__ void attn_tiles(const float* __restrict__ qh, const float* __restrict__ kbase,
                                           const float* __restrict__ vbase, size_t page_elems,
                                           const int* __restrict__ bt, int bt_len, int ctx, int it_begin,
                                           int it_end, float qscale, float& m, float& l, float4& acc,
                                           int w = (int)(threadIdx.x >> 6)) {
#if !HPA_ATTN_SWP
    attn_tiles_single<P, NW>(qh, kbase, vbase, page_elems, bt, bt_len, ctx, it_begin, it_end, qscale, m, l, acc, w);
#else
    static_assert(P % 4 == 0 && 64 % P == 0, "page size must divide 64 and be a multiple of 4");
    const int lane = threadIdx.x & 63;
    const int g = lane >> 4;
    const int d4 = lane & 15;
    const int v_lane_off = g * HS + d4 * 4;
    int it = it_begin + w;
    if (it >= it_end) return;
    int pid = first_tile_pid<P>(bt, bt_len, ctx, it, it_end);
    float4 kv[16], vv[16];
    auto load_k = [&](int itx, int pidx) {
        const unsigned tokx = ((unsigned)itx << 6) + lane;
        const float* kt = kbase + (size_t)(unsigned)pidx * page_elems + (tokx % P) * 4;
#pragma unroll
        for (int c = 0; c < 16; ++c) kv[c] = load_stream(kt + c * P * 4);
    };
    // PV operands: the row address splits into a wave-uniform part (page of
    // tokens t0+4i..+3, slot (4i)%P; t0 % P == 0: the SGPR offset of a buffer
    // load) and a per-lane offset that is the same for every i.  Rows past
    // the context take an out-of-range offset: the buffer load returns 0
    // without a fetch, so the loads need no branch (exec-masked loads kept
    // the loop's registers from fitting once they were carried to the next
    // trip)
    const __amdgpu_buffer_rsrc_t vrsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(vbase), 0, 0x7fffffff,
                                                                           0x00020000);
    auto load_v = [&](int itx, int pidx) {
        const unsigned t0x = (unsigned)itx << 6;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int vpid = __builtin_amdgcn_readlane(pidx, 4 * i);
            const int soff = (int)(((size_t)(unsigned)vpid * page_elems + ((4 * i) % P) * HS) * 4);
            const int voff = (t0x + 4 * i + g) < (unsigned)ctx ? v_lane_off * 4 : (int)0x80000000u;
            const hpa::u32x4 d = __builtin_amdgcn_raw_buffer_load_b128(vrsrc, voff, soff, kCpolNt);
            vv[i] = make_float4(__uint_as_float(d.x), __uint_as_float(d.y), __uint_as_float(d.z), __uint_as_float(d.w));
        }
    };
    auto page_ids = [&](int itx) {  // tile itx's page ids (entry 0 past the range: never used)
        const unsigned t0x = (unsigned)itx << 6, tokx = t0x + lane;
        return bt[itx < it_end ? (tokx < (unsigned)ctx ? tokx : t0x) / P : 0];
    };
    // QK^T: lane-per-token over 16 chunks of 4 dims (q in SGPRs)
    auto qk = [&](int itx) {
        float s = 0.f;
#pragma unroll
        for (int c = 0; c < 16; ++c) {
            s = fmaf(qh[4 * c + 0], kv[c].x, s);
            s = fmaf(qh[4 * c + 1], kv[c].y, s);
            s = fmaf(qh[4 * c + 2], kv[c].z, s);
            s = fmaf(qh[4 * c + 3], kv[c].w, s);
        }
        return ((unsigned)itx << 6) + lane < (unsigned)ctx ? s * qscale : -INFINITY;
    };
    // online softmax (log2 domain), then PV
    auto softmax_pv = [&](float s) {
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
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const float pi = __shfl(p, 4 * i + g, 64);
            acc.x = fmaf(pi, vv[i].x, acc.x);
            acc.y = fmaf(pi, vv[i].y, acc.y);
            acc.z = fmaf(pi, vv[i].z, acc.z);
            acc.w = fmaf(pi, vv[i].w, acc.w);
        }
    };
    load_k(it, pid);
    load_v(it, pid);
    int itn = it + NW;
    int pidn = page_ids(itn);
    while (itn < it_end) {
        const float s = qk(it);
        __builtin_amdgcn_sched_barrier(0);  // K registers consumed before the next K lands in them
        load_k(itn, pidn);
        softmax_pv(s);
        __builtin_amdgcn_sched_barrier(0);  // V registers consumed before the next V lands in them
        load_v(itn, pidn);
        it = itn;
        pid = pidn;
        itn += NW;
        pidn = page_ids(itn);
    }
    softmax_pv(qk(it));
    (void)pid;
#endif
}

// ---- bf16 KV pool (BASELINE config 5): storage only, every product and
// sum in fp32.  K tile [8 chunks][P][8 dims] (a lane-per-token chunk is one
// 16-B load), V tile [P][64] (128 B per token: 8 lanes per row, one wave
// instruction reads 8 consecutive rows = 1 KiB).
__device__ __forceinline__ uint4 load_stream16(const unsigned short* ptr) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(ptr));
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ float bf_lo(unsigned int u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bf_hi(unsigned int u) { return __uint_as_float(u & 0xffff0000u); }

// acc[0], acc[1]: lane (g = lane>>3, d8 = lane&7) holds dims 8*d8..+7 summed
// over tokens t0 + 8i + g
template <int P, int NW>
__device__ __forceinline__ void attn_tiles_bf16(const float* __restrict__ qh,
                                                const unsigned short* __restrict__ kbase,
                                                const unsigned short* __restrict__ vbase, size_t page_elems,
                                                const int* __restrict__ bt, int bt_len, int ctx, int it_begin,
                                                int it_end, float qscale, float& m, float& l, float4* acc,
                                                int w = (int)(threadIdx.x >> 6)) {
    static_assert(P % 8 == 0 && 64 % P == 0, "bf16 pages: page size 8, 16, 32 or 64");
    const int lane = threadIdx.x & 63;
    const int g = lane >> 3;
    const int d8 = lane & 7;
    const int v_lane_off = g * HS + d8 * 8;
    int it = it_begin + w;
    int pid = first_tile_pid<P>(bt, bt_len, ctx, it, it_end);
    for (; it < it_end; it += NW) {
        const unsigned t0 = (unsigned)it << 6;
        const unsigned tok = t0 + lane;
        const bool valid = tok < (unsigned)ctx;
        const unsigned short* kt = kbase + (size_t)(unsigned)pid * page_elems + (tok % P) * 8;
        uint4 kv[8], vv[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) kv[c] = load_stream16(kt + c * P * 8);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int vpid = __builtin_amdgcn_readlane(pid, 8 * i);
            const unsigned short* vrow = vbase + (size_t)(unsigned)vpid * page_elems + ((8 * i) % P) * HS;
            vv[i] = (t0 + 8 * i + g) < (unsigned)ctx ? load_stream16(vrow + v_lane_off) : make_uint4(0, 0, 0, 0);
        }
        {
            const int itn = it + NW;
            const unsigned t0n = (unsigned)itn << 6, tokn = t0n + lane;
            if (itn < it_end) pid = bt[(tokn < (unsigned)ctx ? tokn : t0n) / P];
        }
        float s = 0.f;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            s = fmaf(qh[8 * c + 0], bf_lo(kv[c].x), s);
            s = fmaf(qh[8 * c + 1], bf_hi(kv[c].x), s);
            s = fmaf(qh[8 * c + 2], bf_lo(kv[c].y), s);
            s = fmaf(qh[8 * c + 3], bf_hi(kv[c].y), s);
            s = fmaf(qh[8 * c + 4], bf_lo(kv[c].z), s);
            s = fmaf(qh[8 * c + 5], bf_hi(kv[c].z), s);
            s = fmaf(qh[8 * c + 6], bf_lo(kv[c].w), s);
            s = fmaf(qh[8 * c + 7], bf_hi(kv[c].w), s);
        }
        s = valid ? s * qscale : -INFINITY;
        const float mt = hpa::wave_max(s);
        const float mn = fmaxf(m, mt);
        const float alpha = exp2f(m - mn);
        const float p = exp2f(s - mn);
        l = fmaf(l, alpha, p);
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            acc[k].x *= alpha;
            acc[k].y *= alpha;
            acc[k].z *= alpha;
            acc[k].w *= alpha;
        }
        m = mn;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const float pi = __shfl(p, 8 * i + g, 64);
            acc[0].x = fmaf(pi, bf_lo(vv[i].x), acc[0].x);
            acc[0].y = fmaf(pi, bf_hi(vv[i].x), acc[0].y);
            acc[0].z = fmaf(pi, bf_lo(vv[i].y), acc[0].z);
            acc[0].w = fmaf(pi, bf_hi(vv[i].y), acc[0].w);
            acc[1].x = fmaf(pi, bf_lo(vv[i].z), acc[1].x);
            acc[1].y = fmaf(pi, bf_hi(vv[i].z), acc[1].y);
            acc[1].z = fmaf(pi, bf_lo(vv[i].w), acc[1].z);
            acc[1].w = fmaf(pi, bf_hi(vv[i].w), acc[1].w);
        }
    }
}

// fold for the bf16 layout: the 8 token groups (lane bits 3..5), then the
// waves through LDS (s_acc: [NW][8 lanes][2]); result in wave 0, lanes 0..7
template <int NW>
__device__ __forceinline__ bool attn_fold_bf16(float& m, float& l, float4* acc, float* s_m, float* s_l,
                                               float4* s_acc) {
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
#pragma unroll
    for (int o = 8; o <= 32; o <<= 1)
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            acc[k].x += __shfl_xor(acc[k].x, o, 64);
            acc[k].y += __shfl_xor(acc[k].y, o, 64);
            acc[k].z += __shfl_xor(acc[k].z, o, 64);
            acc[k].w += __shfl_xor(acc[k].w, o, 64);
        }
    l = hpa::wave_sum(l);
    if constexpr (NW == 1) {
        return lane < 8;
    } else {
        if (lane == 0) {
            s_m[w] = m;
            s_l[w] = l;
        }
        if (lane < 8) {
            s_acc[(w * 8 + lane) * 2] = acc[0];
            s_acc[(w * 8 + lane) * 2 + 1] = acc[1];
        }
        __syncthreads();
        if (w != 0 || lane >= 8) return false;
        float M = s_m[0];
#pragma unroll
        for (int i = 1; i < NW; ++i) M = fmaxf(M, s_m[i]);
        float L = 0.f;
        float4 O[2] = {make_float4(0.f, 0.f, 0.f, 0.f), make_float4(0.f, 0.f, 0.f, 0.f)};
#pragma unroll
        for (int i = 0; i < NW; ++i) {
            const float f = exp2f(s_m[i] - M);
            L = fmaf(s_l[i], f, L);
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const float4 a = s_acc[(i * 8 + lane) * 2 + k];
                O[k].x = fmaf(a.x, f, O[k].x);
                O[k].y = fmaf(a.y, f, O[k].y);
                O[k].z = fmaf(a.z, f, O[k].z);
                O[k].w = fmaf(a.w, f, O[k].w);
            }
        }
        m = M;
        l = L;
        acc[0] = O[0];
        acc[1] = O[1];
        return true;
    }
}

// Fold the 4 token groups and the per-lane sums of every wave, then the
// waves (fixed order, through LDS: s_m[NW], s_l[NW], s_acc[NW*16]).  The
// combined state lands in wave 0, lanes 0..15 (returns true there): lane
// holds dims 4*lane..+3.
template <int NW>
__device__ __forceinline__ bool attn_fold(float& m, float& l, float4& acc, float* s_m, float* s_l,
                                          float4* s_acc) {
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
#pragma unroll
    for (int o = 16; o <= 32; o <<= 1) {
        acc.x += __shfl_xor(acc.x, o, 64);
        acc.y += __shfl_xor(acc.y, o, 64);
        acc.z += __shfl_xor(acc.z, o, 64);
        acc.w += __shfl_xor(acc.w, o, 64);
    }
    l = hpa::wave_sum(l);
    if constexpr (NW == 1) {
        return lane < 16;
    } else {
        if (lane == 0) {
            s_m[w] = m;
            s_l[w] = l;
        }
        if (lane < 16) s_acc[w * 16 + lane] = acc;
        __syncthreads();
        if (w != 0 || lane >= 16) return false;
        float M = s_m[0];
#pragma unroll
        for (int i = 1; i < NW; ++i) M = fmaxf(M, s_m[i]);
        float L = 0.f;
        float4 O = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int i = 0; i < NW; ++i) {
            const float f = exp2f(s_m[i] - M);
            L = fmaf(s_l[i], f, L);
            const float4 a = s_acc[i * 16 + lane];
            O.x = fmaf(a.x, f, O.x);
            O.y = fmaf(a.y, f, O.y);
            O.z = fmaf(a.z, f, O.z);
            O.w = fmaf(a.w, f, O.w);
        }
        m = M;
        l = L;
        acc = O;
        return true;
    }
}

// split-context records: [B*NH][S][kRec] floats (m, l, -, -, acc[64]), then
// [B*NH] int arrival counters (zero between launches)
constexpr int kRec = 68;

// Range s of S: publish this workgroup's folded state (K float4 chunks per
// lane in wave 0: chunk k of lane j holds dims 4*(K*j + k)..+3 -- K = 1 for
// the fp32 fold, lanes 0..15; K = 2 for the bf16 fold, lanes 0..7); the last
// arriver merges every range in order and returns true with the merged state
// (rewind: it also zeroes the counter for the next launch).
// Memory model: gfx950 only.  The hand-off is MI355X_MICROARCH.md "Valid
// forms" row 1: 16-byte sc1 (write-through) record stores, drained by
// s_waitcnt vmcnt(0), then an agent-scope relaxed ticket, and sc1 loads by
// the last arriver (L1 bypass); no acquire/release fences, so it relies on
// gfx950's sc1 semantics and on the buffer-load builtins not being speculated
// above the ticket (they are data-dependent on it through the branch).  A
// launch that aborts part-way leaves counters non-zero: the engine re-zeroes
// them after a failure and before a graph recapture (paged_infer.c
// dec_rezero).
template <int K>
__device__ __forceinline__ bool split_merge(float* __restrict__ rec_bh, int* __restrict__ cnt, int S, int s,
                                            float& m, float& l, float4* acc, bool rewind) {
    const int lane = threadIdx.x & 63;
    float* rec = rec_bh + (size_t)s * kRec;
    if (lane == 0) hpa::store_wt16(rec, 0, make_float4(m, l, 0.f, 0.f));
#pragma unroll
    for (int k = 0; k < K; ++k) hpa::store_wt16(rec, (4 + 4 * (K * lane + k)) * 4, acc[k]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every record store drained before the ticket
    int ticket = 0;
    if (lane == 0) ticket = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    ticket = __builtin_amdgcn_readfirstlane(ticket);
    if (ticket != S - 1) return false;
    if (rewind && lane == 0) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch
    // every record's (m, l) head, all in flight together (one after another
    // each would be a cross-XCD round trip), then the acc chunks 8 ranges at a time
    float4 head[HPA_ATTN_MAX_SPLITS];
#pragma unroll
    for (int i = 0; i < HPA_ATTN_MAX_SPLITS; ++i) head[i] = hpa::load_wt16(rec_bh + (size_t)min(i, S - 1) * kRec, 0);
    float M = -INFINITY;
#pragma unroll
    for (int i = 0; i < HPA_ATTN_MAX_SPLITS; ++i)
        if (i < S) M = fmaxf(M, head[i].x);
    float L = 0.f;
    float4 O[K];
#pragma unroll
    for (int k = 0; k < K; ++k) O[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int i0 = 0; i0 < S; i0 += 8) {  // ranges in order: independent of arrival order
        float4 a[8][K];
#pragma unroll
        for (int q = 0; q < 8; ++q)
#pragma unroll
            for (int k = 0; k < K; ++k)
                a[q][k] = hpa::load_wt16(rec_bh + (size_t)min(i0 + q, S - 1) * kRec, (4 + 4 * (K * lane + k)) * 4);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            if (i0 + q >= S) break;
            float hm = head[0].x, hl = head[0].y;
#pragma unroll
            for (int i = 1; i < HPA_ATTN_MAX_SPLITS; ++i)
                if (i == i0 + q) {
                    hm = head[i].x;
                    hl = head[i].y;
                }
            const float f = exp2f(hm - M);
            L = fmaf(hl, f, L);
#pragma unroll
            for (int k = 0; k < K; ++k) {
                O[k].x = fmaf(a[q][k].x, f, O[k].x);
                O[k].y = fmaf(a[q][k].y, f, O[k].y);
                O[k].z = fmaf(a[q][k].z, f, O[k].z);
                O[k].w = fmaf(a[q][k].w, f, O[k].w);
            }
        }
    }
    m = M;
    l = L;
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] = O[k];
    return true;
}

}  // namespace hpa_attn
