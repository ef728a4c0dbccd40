// hpa_pipe.hip -- the decode step's layer loop as ONE persistent launch with
// fixed CU roles and the batch in two halves, software-pipelined (gfx950).
//
// Replaces the 2 x L launches of the chain-form layer loop (the decode
// attention + chain form 6 per layer; reference gpt2_forward,
// paged_infer.c:659-722, one decode row per sequence):
//   attention(l)  attention_paged :163-240
//   attproj(l)    matmul_forward :716 + residual_forward :717
//   fc(l)         layernorm_forward :718 (folded) + matmul :719 + gelu :720
//   fcproj(l)     matmul_forward :721 + residual_forward :722
//   qkv(l+1)      layernorm :696 (folded) + matmul_cached :706 + add_to_cache :710
//
// Why ("Pipelined halves"): the attention is bound by HBM
// (6.5 TB/s on all CUs, 62 us per layer at B = 64) and the GEMM chain by its
// hand-offs and the per-CU operand stream (24 us per layer, HBM nearly idle).
// One after the other they cost 86 us per layer.  Here the two run side by
// side on disjoint CUs, on the two halves of the batch:
//   CUs 0 .. NG-1   (G role, NG = 64: 8 per XCD)  the GEMM chain
//   CUs NG .. 255   (A role, 24 per XCD)          the paged attention
//   slot 0:      A: attention(0, H0)
//   slot 2l+1:   A: attention(l, H1)       G: chain(l, H0)
//   slot 2l+2:   A: attention(l+1, H0)     G: chain(l, H1)
//   chain(l, h) = attproj(l) -> fc(l) -> fcproj(l) -> qkv(l+1) on half h's rows.
// Every dependency is per (layer, half): attention(l, h) waits for qkv(l) of
// half h (chain(l-1, h); layer 0's is the step's first launch), chain(l, h)
// for attention(l, h).  No role ever waits for itself across halves, so the
// pipeline cannot deadlock with every workgroup resident (grid = CU count, one
// 12-wave workgroup per CU: 84 KB of LDS).
//
// Bits: an A unit is paged_attn_decode_f32<P, 4>'s workgroup of one
// (sequence, head) -- tiles w, w+4, .. per wave, the same online softmax and
// wave fold -- and a G unit is chain form 6's 12-wave unit (wave w takes k16
// steps 4w..4w+3 of every tile, folded in wave order; fcproj's 4 K parts in
// part order) holding both row blocks of a half.  A row's result depends on
// neither grouping, so the step equals the chain-form step bit for bit.
//
// Hand-offs inside the launch (MI355X_MICROARCH.md "Valid forms", row 1): every
// handed-over byte is stored sc1 (16-B write-through) and loaded sc1; the
// storing waves drain (vmcnt(0)), a workgroup barrier follows, then ONE lane
// adds to the (layer, half, phase) counter, sharded 8 ways; the consumer's
// wave 0 polls every shard with sc1 loads while the other waves wait at a
// barrier.  Two operands change role here:
//   * q is written in this launch, so the A unit loads it with sc1 vector
//     loads (readfirstlane into SGPRs) instead of scalar loads, whose cache is
//     not refreshed by another CU's stores;
//   * the new token's K / V are appended in this launch: the G role stores
//     them sc1, and the A unit re-reads exactly those bytes with sc1 loads in
//     its last tile (the lane of the new token, the lanes of its V row); every
//     other K / V byte was written by an earlier launch and streams with the
//     non-temporal loads of the stand-alone kernel.
// Every spin is bounded (200 ms): a timeout stores a code in *err and the
// launch ends (outputs garbage, reported by the host).
//
// Measured (round 6, profiles/r6/pipe/README.md): SLOWER than chain form 6 at
// every batch (B = 64: 1.205 vs 1.100 ms per step).  The attention's per-CU
// rate needs all 256 CUs for the chip's HBM rate (a half on 192 CUs: 36-44
// us), and beside that saturating stream the chain's hand-offs and phases cost
// about twice what they cost alone (a half: ~46 us).  Kept, bit-identical and
// tested, in A/B builds only (-DHPA_AB; the product library's entry points
// report it unavailable, and form 7 falls back to form 5).
#include <math.h>
#include <string.h>

#include "hpa_attn_body.h"
#include "hpa_gemm_body.h"

namespace {
using hpa_attn::HS;
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int C = 768, NH = 12, K16 = 48, NCT = 48;  // GPT-2 124M
constexpr int NWV = 12;                              // waves per workgroup (every role)
constexpr int SPW = 4;                               // k16 steps per wave of a K = 768 range
constexpr int kPad = 32;                             // ints per counter shard (one 128-B line)
constexpr long long kSpinTicks = 20000000;           // s_memrealtime is 100 MHz: 200 ms
constexpr int kDefaultG = 64;

// counters of layer l, half h: counter c's 8 shards at ((h*kNC + c)*8 + shard)*kPad
//   QKV    qkv(l) units of the half done (written by chain(l-1, h))
//   ATT    attention(l) units of the half done
//   X1     attproj units done;  H + p: fc units feeding fcproj's K part p done
//   X2     fcproj tile groups combined
// then the fcproj tickets [2 halves][32]
enum { PC_QKV = 0, PC_ATT = 1, PC_X1 = 2, PC_H = 3, PC_X2 = 7, kNC = 8 };
constexpr int kTick = 2 * kNC * 8 * kPad;
constexpr int kLayerInts = kTick + 2 * 32;

struct PA {
    int B, L, NG, NA, stats_mp;
    size_t layer_ctr;
    const HpaPipeLayer* lay;
    float* q;
    char* kv;  // pool base
    size_t layer_bytes, page_elems;
    const int* bt;
    int bt_stride;
    const int* pos;
    float qscale, m_init;
    float *att, *res, *res2, *fch, *slab, *stats_out;
    int* ctr;
    int* err;
    int* err_sticky;
};

template <int HR, int T>
struct GSmem {
    float red[NWV * HR * T * 256];  // [wave][row block][tile][256] accumulators
    float wsum[HR * NWV * 32];      // [row block][wave][16 rows][2] LN row partial sums
    float tile[HR * T * 16 * 17];   // last layer: [row block][tile][16 rows][17] for the LNf statistics
    int s_last;
};
struct ASmem {
    float s_m[3][4], s_l[3][4];
    float4 s_acc[3][64];      // [slot][4 waves x 16 lanes]
    float4 s_q[3][4][16];     // [slot][wave]: q of the unit's (sequence, head)
    int s_cnt[3];
};
template <int HR, int T>
struct PSmem {
    union {
        GSmem<HR, T> g;
        ASmem a;
    };
    int s_ok;
};

__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// diagnostic build (-DHPA_PIPE_TRACE, tools/pipe_trace.py): s_memrealtime of
// workgroup-level events per (layer, half, workgroup); never in the product library
#ifdef HPA_PIPE_TRACE
__device__ unsigned long long g_pipe_trace[2 * 64][256][12];
#define PT_MARK(l, h, k)                                                                            \
    do {                                                                                            \
        if (threadIdx.x == 0 && (l) < 64 && blockIdx.x < 256)                                       \
            g_pipe_trace[2 * (l) + (h)][blockIdx.x][k] = (unsigned long long)__builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define PT_MARK(l, h, k) \
    do {                 \
    } while (0)
#endif

// every storing wave drained (the builtin: the compiler then knows vmcnt is 0)
__device__ __forceinline__ void drain_vm() {
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) expcnt(7) lgkmcnt(15)
    asm volatile("" ::: "memory");
}

__device__ __forceinline__ int wave_sum_int(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ int* ctr_of(const PA& a, int l, int h, int c) {
    return a.ctr + (size_t)l * a.layer_ctr + (size_t)(h * kNC + c) * 8 * kPad;
}

// one lane, after every storing wave's drain and the workgroup barrier
__device__ __forceinline__ void arrive(int* c, int n) {
    __hip_atomic_fetch_add(c + (blockIdx.x & 7) * kPad, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// every thread calls; wave 0 polls the 8 shards of `c` until they sum to
// `expected` (bounded), the others wait at the barrier
template <typename SM>
__device__ __forceinline__ bool wait_sum(const PA& a, const int* c, int expected, int code, SM& sm) {
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (wv == 0) {
        const int lane = threadIdx.x & 63;
        int ok = 0;
        const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
        for (unsigned it = 0;; ++it) {
            int v = lane < 8 ? __hip_atomic_load(c + lane * kPad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
            v = __builtin_amdgcn_readfirstlane(wave_sum_int(v));
            if (v >= expected) {
                ok = 1;
                break;
            }
            if ((it & 7) == 7) {
                const int e = __builtin_amdgcn_readfirstlane(
                    __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                if (e) break;  // another workgroup gave up: follow at once
                if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > kSpinTicks) {
                    if (lane == 0) {
                        atomicCAS(a.err, 0, code);
                        if (a.err_sticky) atomicCAS(a.err_sticky, 0, code);
                    }
                    break;
                }
            }
            __builtin_amdgcn_s_sleep(1);
        }
        if (lane == 0) sm.s_ok = ok;
    }
    lds_barrier();
    const bool ok = sm.s_ok != 0;
    lds_barrier();  // s_ok read before the next wait rewrites it
    return ok;
}

__device__ __forceinline__ float rfl(float x) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(x))); }

// ------------------------------------------------------------------ A role
// one 64-token tile `it` of a wave (hpa_attn::attn_tiles' loop body): K and V
// rows issued together (one memory round trip), the next tile's page ids,
// QK^T lane-per-token, the online softmax, PV lane-per-dimension.  SC1: the
// loads are sc1 (L1-bypassing) buffer loads relative to the layer's slab kvl
// (< 2 GiB) instead of the non-temporal stream.
template <int P, bool SC1>
__device__ __forceinline__ void attn_tile(const PA& a, const char* kvl, const float* kbase, const float* vbase,
                                          const int* bt, int ctx, int n_it, int it, int& pid, const float4* s_q,
                                          float& m, float& lsum, float4& acc) {
    const int lane = threadIdx.x & 63;
    const int g = lane >> 4, d4 = lane & 15;
    const int v_lane_off = g * HS + d4 * 4;
    const size_t pe = a.page_elems;
    const unsigned t0 = (unsigned)it << 6;
    const unsigned tok = t0 + lane;
    const bool valid = tok < (unsigned)ctx;
    const float* kt = kbase + (size_t)(unsigned)pid * pe + (tok % P) * 4;
    float4 kv[16], vv[16];
    if constexpr (SC1) {
        const int koff = (int)((const char*)kt - kvl);
#pragma unroll
        for (int c = 0; c < 16; ++c) kv[c] = hpa::load_wt16(kvl, koff + c * P * 16);
    } else {
#pragma unroll
        for (int c = 0; c < 16; ++c) kv[c] = hpa_attn::load_stream(kt + c * P * 4);
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int vpid = __builtin_amdgcn_readlane(pid, 4 * i);
        const float* vrow = vbase + (size_t)(unsigned)vpid * pe + ((4 * i) % P) * HS;
        if constexpr (SC1)
            vv[i] = (t0 + 4 * i + g) < (unsigned)ctx ? hpa::load_wt16(kvl, (int)((const char*)(vrow + v_lane_off) - kvl))
                                                     : make_float4(0.f, 0.f, 0.f, 0.f);
        else
            vv[i] = (t0 + 4 * i + g) < (unsigned)ctx ? hpa_attn::load_stream(vrow + v_lane_off)
                                                     : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    {  // next tile's page ids
        const int itn = it + 4;
        const unsigned t0n = (unsigned)itn << 6, tokn = t0n + lane;
        if (itn < n_it) pid = bt[(tokn < (unsigned)ctx ? tokn : t0n) / P];
    }
    float s = 0.f;
    int z = 0;  // opaque 0: q is re-read from LDS every tile (hoisted, its 64 VGPRs spilled)
    asm volatile("" : "+s"(z));
#pragma unroll
    for (int c = 0; c < 16; ++c) {
        const float4 qc = s_q[c + z];
        s = fmaf(rfl(qc.x), kv[c].x, s);
        s = fmaf(rfl(qc.y), kv[c].y, s);
        s = fmaf(rfl(qc.z), kv[c].z, s);
        s = fmaf(rfl(qc.w), kv[c].w, s);
    }
    s = valid ? s * a.qscale : -INFINITY;
    const float mt = hpa::wave_max(s);
    const float mn = fmaxf(m, mt);
    const float alpha = exp2f(m - mn);
    const float p = exp2f(s - mn);
    lsum = fmaf(lsum, alpha, p);
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
}

// one attention unit: sequence b, head hh of layer l (kvl = the layer's pool
// slab), run by the 4 waves of `slot`; paged_attn_decode_f32<P, 4>'s tiles,
// softmax and fold (hpa_attn.hip), the fold through LDS by the slot's last
// wave to arrive (no workgroup barrier: the other slot runs on)
template <int P>
__device__ __forceinline__ void attn_unit(const PA& a, const char* kvl, int l, int h, int b, int hh, int slot, int wq,
                                          ASmem& sm) {
    constexpr int TILE = P * HS;
    const int lane = threadIdx.x & 63;
    const int ctx = a.pos[b] + 1;
    // q of (b, hh), stored sc1 in this launch by qkv(l) (or by the first
    // launch): sc1 loads into this wave's LDS (the stand-alone kernel's scalar
    // loads would read the scalar cache, which another CU's stores do not
    // refresh; in SGPRs it overflowed them here), read back per 4-dim chunk
    // as a broadcast
    float4* s_q = &sm.s_q[slot][wq][0];
    if (lane < 16) s_q[lane] = hpa::load_wt16(a.q, ((b * C + hh * HS) + 4 * lane) * 4);
    const float* kbase = reinterpret_cast<const float*>(kvl) + (size_t)hh * TILE;
    const float* vbase = reinterpret_cast<const float*>(kvl) + (size_t)(NH + hh) * TILE;
    const int* bt = a.bt + (size_t)b * a.bt_stride;
    const int n_it = (ctx + 63) >> 6;
    const int it_new = n_it - 1;       // the tile of the token appended in this launch
    float m = a.m_init, lsum = 0.f;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    int it = wq;
    int pid = hpa_attn::first_tile_pid<P>(bt, a.bt_stride, ctx, it, n_it);
    // tiles before the new token's: the stand-alone kernel's non-temporal stream
#pragma unroll 1
    for (; it < it_new; it += 4)
        attn_tile<P, false>(a, kvl, kbase, vbase, bt, ctx, n_it, it, pid, s_q, m, lsum, acc);
    // the new token's tile (one wave): every K / V load sc1, since qkv stored
    // that token's bytes sc1 in this launch (the rest of the tile is older)
    if (it == it_new) attn_tile<P, true>(a, kvl, kbase, vbase, bt, ctx, n_it, it, pid, s_q, m, lsum, acc);
    // hpa_attn::attn_fold<4>: the 4 token groups, the lane sums, then the waves in order
#pragma unroll
    for (int o = 16; o <= 32; o <<= 1) {
        acc.x += __shfl_xor(acc.x, o, 64);
        acc.y += __shfl_xor(acc.y, o, 64);
        acc.z += __shfl_xor(acc.z, o, 64);
        acc.w += __shfl_xor(acc.w, o, 64);
    }
    lsum = hpa::wave_sum(lsum);
    if (lane == 0) {
        sm.s_m[slot][wq] = m;
        sm.s_l[slot][wq] = lsum;
    }
    if (lane < 16) sm.s_acc[slot][wq * 16 + lane] = acc;
    int old = 0;
    if (lane == 0) old = __hip_atomic_fetch_add(&sm.s_cnt[slot], 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
    old = __builtin_amdgcn_readfirstlane(old);
    if ((old & 3) != 3 || lane >= 16) return;
    float M = sm.s_m[slot][0];
#pragma unroll
    for (int i = 1; i < 4; ++i) M = fmaxf(M, sm.s_m[slot][i]);
    float L = 0.f;
    float4 O = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const float f = exp2f(sm.s_m[slot][i] - M);
        L = fmaf(sm.s_l[slot][i], f, L);
        const float4 v = sm.s_acc[slot][i * 16 + lane];
        O.x = fmaf(v.x, f, O.x);
        O.y = fmaf(v.y, f, O.y);
        O.z = fmaf(v.z, f, O.z);
        O.w = fmaf(v.w, f, O.w);
    }
    const float inv = L == 0.f ? 0.f : 1.f / L;
    hpa::store_wt16(a.att, (int)(hpa::frag_index(b, hh * HS + 4 * lane, C) * 4),
                    make_float4(O.x * inv, O.y * inv, O.z * inv, O.w * inv));
    drain_vm();  // this (the only storing) wave drained
    if (lane == 0) arrive(ctr_of(a, l, h, PC_ATT), 1);
}

template <int P, int HR, int T>
__device__ __forceinline__ void a_role(const PA& a, PSmem<HR, T>& smu) {
    ASmem& sm = smu.a;
    const int ab = blockIdx.x - a.NG;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int slot = w >> 2, wq = w & 3;
    if (threadIdx.x < 3) sm.s_cnt[threadIdx.x] = 0;
    constexpr int HB = HR * 16;  // rows per half (padded)
#pragma unroll 1
    for (int l = 0; l < a.L; ++l) {
        const char* kvl = a.kv + (size_t)l * a.layer_bytes;
#pragma unroll 1
        for (int h = 0; h < 2; ++h) {
            // q(l) and layer l's new K / V of the half: the first launch's at
            // l = 0 (a launch boundary), qkv(l) of chain(l-1, h) after
            if (l > 0) {
                if (!wait_sum(a, ctr_of(a, l, h, PC_QKV), 3 * NCT / T, 10, smu)) return;
            } else {
                lds_barrier();  // the slot state of the previous unit is read (and s_cnt set)
            }
            PT_MARK(l, h, 0);
            const int r0 = h * HB, nr = min(a.B, r0 + HB) - r0;
            const int u = ab + slot * a.NA;  // host: nr * NH <= 3 * NA, one unit per slot
            if (u < nr * NH) attn_unit<P>(a, kvl, l, h, r0 + u / NH, u % NH, slot, wq, sm);
            PT_MARK(l, h, 1);
        }
    }
}

// ------------------------------------------------------------------ G role
// the wave's weight fragments of tiles j0 .. j0+TT-1, k16 steps kb + 4w ..
// (K16W steps per tile row); default policy (one unit reads a tile: its
// other reads are the next step's)
template <int TT>
__device__ __forceinline__ void load_wt(const float* W, int K16W, int j0, int kb, int w, float4 (&wr)[TT][SPW]) {
    const float4* wf = reinterpret_cast<const float4*>(W) + ((size_t)j0 * K16W + kb + w * SPW) * 64 + (threadIdx.x & 63);
#pragma unroll
    for (int t = 0; t < TT; ++t)
#pragma unroll
        for (int s = 0; s < SPW; ++s) wr[t][s] = wf[((size_t)t * K16W + s) * 64];
}

// the wave's 4 A fragments of row block rb (sc1: written in this launch)
__device__ __forceinline__ void load_a(const float* A, int K16A, int rb, int kb, int w, float4 (&xv)[SPW]) {
    const int off = ((rb * K16A + kb + w * SPW) * 64 + (int)(threadIdx.x & 63)) * 16;
#pragma unroll
    for (int s = 0; s < SPW; ++s) xv[s] = hpa::load_wt16(A, off + s * 1024);
}

// chain form 6's chains (c6::mfma_regs): each tile one accumulator chain in
// the one-shot order (steps in order, components x, y, z, w); (STATS) the LN
// row partial sums of the fragments
template <int TT, bool STATS>
__device__ __forceinline__ void mfma_rb(const float4 (&xv)[SPW], const float4 (&wr)[TT][SPW], f32x4 (&acc)[TT],
                                        float& fs1, float& fs2) {
#pragma unroll
    for (int t = 0; t < TT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < SPW; ++s)
#pragma unroll
        for (int t = 0; t < TT; ++t) {
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[s].x, wr[t][s].x, acc[t], 0, 0, 0);
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[s].y, wr[t][s].y, acc[t], 0, 0, 0);
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[s].z, wr[t][s].z, acc[t], 0, 0, 0);
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[s].w, wr[t][s].w, acc[t], 0, 0, 0);
        }
    if (STATS)
#pragma unroll
        for (int s = 0; s < SPW; ++s) hpa_gemm::row_sums_add(xv[s], fs1, fs2);
}

// a unit's HR row blocks x TT tiles: A loads of every row block in flight
// before the first MFMA, then the chains; accumulators to LDS
// red[((w*HR + r)*TT + t)*256 + g*64 + lane]
template <int HR, int TT, bool STATS>
__device__ __forceinline__ void unit_mfma(const float* A, int K16A, int rb0, int kb, int w, const float4 (&wr)[TT][SPW],
                                          float* red, float* wsum) {
    float4 xv[HR][SPW];
#pragma unroll
    for (int r = 0; r < HR; ++r) load_a(A, K16A, rb0 + r, kb, w, xv[r]);
    __builtin_amdgcn_sched_barrier(0);
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int r = 0; r < HR; ++r) {
        f32x4 acc[TT];
        float fs1 = 0.f, fs2 = 0.f;
        mfma_rb<TT, STATS>(xv[r], wr, acc, fs1, fs2);
#pragma unroll
        for (int t = 0; t < TT; ++t)
#pragma unroll
            for (int gq = 0; gq < 4; ++gq) red[((w * HR + r) * TT + t) * 256 + gq * 64 + lane] = acc[t][gq];
        if (STATS) hpa_gemm::row_sums_publish(fs1, fs2, wsum + (r * NWV + w) * 32);
    }
}

// epilogue element of (row block r, tile t): row er, columns 4q..4q+3, the
// 12 waves in wave order (c6::fold_t)
template <int HR, int TT>
__device__ __forceinline__ float4 fold(const float* red, int r, int t, int er, int q) {
    const float* p = red + (r * TT + t) * 256 + (er & 3) * 64 + 16 * (er >> 2) + 4 * q;
    float4 v = *reinterpret_cast<const float4*>(p);
#pragma unroll
    for (int w = 1; w < NWV; ++w) {
        const float4 x = *reinterpret_cast<const float4*>(p + w * HR * TT * 256);
        v.x += x.x;
        v.y += x.y;
        v.z += x.z;
        v.w += x.w;
    }
    return v;
}

// LayerNorm-folded value rstd*(acc - mean*c1) + c2 of row er (ln_fold_val<12>)
__device__ __forceinline__ float ln_val(const float* ws, int er, float val, float c1, float c2) {
    float S1 = ws[2 * er], S2 = ws[2 * er + 1];
#pragma unroll
    for (int ww = 1; ww < NWV; ++ww) {
        S1 += ws[ww * 32 + 2 * er];
        S2 += ws[ww * 32 + 2 * er + 1];
    }
    const float m = S1 / C;
    const float rstd = 1.0f / sqrtf(fmaxf(S2 / C - m * m, 0.f) + 1e-5f);
    val = rstd * (val - m * c1);
    val += c2;
    return val;
}
__device__ __forceinline__ float4 ln4(const float* ws, int er, float4 v, float4 c1, float4 c2) {
    v.x = ln_val(ws, er, v.x, c1.x, c2.x);
    v.y = ln_val(ws, er, v.y, c1.y, c2.y);
    v.z = ln_val(ws, er, v.z, c1.z, c2.z);
    v.w = ln_val(ws, er, v.w, c1.w, c2.w);
    return v;
}

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ float4 zero4() { return make_float4(0.f, 0.f, 0.f, 0.f); }

// chain(l, h): one call per (layer, half).  Not inlined into the layer loop:
// inlined, the loop's register allocation kept values of every phase live
// across all of it and spilled (~480 VGPRs); a call gets the straight-line
// body's allocation (~120 VGPRs, as chain form 6).  false: a wait failed.
template <int P, int HR, int T>
__device__ __attribute__((noinline)) bool g_chain(const PA& a, PSmem<HR, T>& smu, int l, int h) {
    GSmem<HR, T>& sm = smu.g;
    constexpr int NGC = 4 * NCT / T;  // fc units (T tiles each) = fcproj units (4 parts x NCT/T groups)
    constexpr int NGD = NCT / T;      // fcproj tile groups per K part
    constexpr int NGE = 3 * NCT / T;  // qkv units
    {
        {
            const int tid = threadIdx.x, bid = blockIdx.x;
            const HpaPipeLayer* ly = a.lay + l;
            const bool last = l + 1 == a.L;
            const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
            // epilogue thread: row block er_r of the unit, tile et, row er, column quad eq
            const int eq1 = tid >> 6, er_r = eq1 / T, et = eq1 - er_r * T, er = (tid & 63) >> 2, eq = tid & 3;
            const bool ethr = tid < HR * T * 64;
            const int er1_r = tid >> 6, er1 = er, eq1b = eq;  // attproj (1 tile): row block er1_r
            const bool ethr1 = tid < HR * 64;
            const int rb0 = h * HR;
            const int nrows = min(a.B, (h + 1) * HR * 16) - h * HR * 16;
            // ---- B: attproj(l): res2 = res + att . Wap^T + b, 1 tile x HR row blocks
            {
                const bool has = bid < NCT;
                const int j = bid;
                float4 wr[1][SPW];
                if (has) load_wt<1>(ly->w_ap, K16, j, 0, w, wr);
                const int row = (rb0 + er1_r) * 16 + er1, col = j * 16 + 4 * eq1b;
                const int fi = (int)(hpa::frag_index(row, col, C) * 4);
                float4 bv = zero4(), rv = zero4();
                if (has && ethr1) {
                    bv = ld4(ly->b_ap + col);
                    rv = hpa::load_wt16(a.res, fi);
                }
                if (!wait_sum(a, ctr_of(a, l, h, PC_ATT), nrows * NH, 1, smu)) return false;
                PT_MARK(l, h, 2);
                if (has) unit_mfma<HR, 1, false>(a.att, K16, rb0, 0, w, wr, sm.red, sm.wsum);
                lds_barrier();
                if (has && ethr1) {
                    float4 v = fold<HR, 1>(sm.red, er1_r, 0, er1, eq1b);
                    v.x += bv.x; v.y += bv.y; v.z += bv.z; v.w += bv.w;
                    const bool live = row < a.B;  // residual_forward(out, res, proj); padded rows stay 0
                    v = live ? make_float4(rv.x + v.x, rv.y + v.y, rv.z + v.z, rv.w + v.w) : zero4();
                    hpa::store_wt16(a.res2, fi, v);
                }
                drain_vm();
                lds_barrier();
                if (tid == 0 && has) arrive(ctr_of(a, l, h, PC_X1), 1);
                PT_MARK(l, h, 3);
            }
            // ---- C: fc(l): fch = gelu(LN2(res2) . Wfc^T + b), LN folded, T tiles x HR row blocks
            {
                const bool has = bid < NGC;
                const int g = bid;
                const int row = (rb0 + er_r) * 16 + er, col = (g * T + et) * 16 + 4 * eq;
                float4 c1 = zero4(), c2 = zero4();
                if (has && ethr) {
                    c1 = ld4(ly->fc_c1 + col);
                    c2 = ld4(ly->fc_c2 + col);
                }
                float4 wr[T][SPW];
                if (has) load_wt<T>(ly->w_fc, K16, g * T, 0, w, wr);
                if (!wait_sum(a, ctr_of(a, l, h, PC_X1), NCT, 2, smu)) return false;
                PT_MARK(l, h, 4);
                if (has) unit_mfma<HR, T, true>(a.res2, K16, rb0, 0, w, wr, sm.red, sm.wsum);
                lds_barrier();
                if (has && ethr) {
                    float4 v = ln4(sm.wsum + er_r * NWV * 32, er, fold<HR, T>(sm.red, er_r, et, er, eq), c1, c2);
                    const bool live = row < a.B;
                    v = live ? make_float4(hpa::gelu_ref(v.x), hpa::gelu_ref(v.y), hpa::gelu_ref(v.z),
                                           hpa::gelu_ref(v.w))
                             : zero4();
                    hpa::store_wt16(a.fch, (int)(hpa::frag_index(row, col, 4 * C) * 4), v);
                }
                drain_vm();
                lds_barrier();
                if (tid == 0 && has) arrive(ctr_of(a, l, h, PC_H + (g * T) / NCT), 1);  // fcproj's K part of these columns
                PT_MARK(l, h, 5);
            }
            // ---- D: fcproj(l), K part p of 4: partials -> slab; the last part of a
            // tile group adds the parts in order + bias + res2 -> res
            {
                const bool has = bid < NGC;
                const int g = bid % NGD, p = bid / NGD;
                const int row = (rb0 + er_r) * 16 + er, col = (g * T + et) * 16 + 4 * eq;
                float4 bv = zero4();
                if (has && ethr) bv = ld4(ly->b_fp + col);
                float4 wr[T][SPW];
                if (has) load_wt<T>(ly->w_fp, 4 * K16, g * T, p * K16, w, wr);
                if (!wait_sum(a, ctr_of(a, l, h, PC_H + (has ? p : 0)), has ? NGD : 0, 3, smu)) return false;
                PT_MARK(l, h, 6);
                if (has) unit_mfma<HR, T, false>(a.fch, 4 * K16, rb0, p * K16, w, wr, sm.red, sm.wsum);
                lds_barrier();
                float4 val = zero4();
                // this part's float4 in the slab: [half][part][group][HR*T*64 threads]
                const int sx = (((h * 4 + p) * NGD + g) * HR * T * 64 + tid) * 16;
                if (has && ethr) {
                    val = fold<HR, T>(sm.red, er_r, et, er, eq);
                    hpa::store_wt16(a.slab, sx, val);
                }
                drain_vm();
                lds_barrier();
                int* tick = a.ctr + (size_t)l * a.layer_ctr + kTick + h * 32;
                if (has && tid == 0) {
                    const int tk = __hip_atomic_fetch_add(tick + g, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    sm.s_last = tk == 3;
                }
                lds_barrier();
                const bool lastp = has && sm.s_last != 0;
                if (lastp && ethr) {
                    float4 pv[4];
                    const int fi = (int)(hpa::frag_index(row, col, C) * 4);
#pragma unroll
                    for (int qq = 0; qq < 4; ++qq)
                        pv[qq] = qq == p ? val : hpa::load_wt16(a.slab, (((h * 4 + qq) * NGD + g) * HR * T * 64 + tid) * 16);
                    const float4 rv = hpa::load_wt16(a.res2, fi);
                    float4 tot = pv[0];
#pragma unroll
                    for (int qq = 1; qq < 4; ++qq) {
                        tot.x += pv[qq].x; tot.y += pv[qq].y; tot.z += pv[qq].z; tot.w += pv[qq].w;
                    }
                    tot.x += bv.x; tot.y += bv.y; tot.z += bv.z; tot.w += bv.w;
                    const bool live = row < a.B;
                    tot = live ? make_float4(rv.x + tot.x, rv.y + tot.y, rv.z + tot.z, rv.w + tot.w) : zero4();
                    hpa::store_wt16(a.res, fi, tot);
                    if (last) {
                        float* tr = sm.tile + ((er_r * T + et) * 16 + er) * 17 + 4 * eq;
                        tr[0] = tot.x; tr[1] = tot.y; tr[2] = tot.z; tr[3] = tot.w;
                    }
                }
                drain_vm();
                lds_barrier();
                if (last && lastp && tid < HR * T * 16) {  // 16-column LNf partial sums of the tiles' rows
                    const int rt = tid >> 4, r = tid & 15;  // rt = row block * T + tile
                    const float* tr = sm.tile + (rt * 16 + r) * 17;
                    float s1 = 0.f, s2 = 0.f;
#pragma unroll
                    for (int c = 0; c < 16; ++c) {
                        s1 += tr[c];
                        s2 += tr[c] * tr[c];
                    }
                    const int j = g * T + rt % T, rr = (rb0 + rt / T) * 16 + r;
                    a.stats_out[((size_t)j * a.stats_mp + rr) * 2] = s1;
                    a.stats_out[((size_t)j * a.stats_mp + rr) * 2 + 1] = s2;
                }
                if (tid == 0 && lastp) arrive(ctr_of(a, l, h, PC_X2), 1);
                PT_MARK(l, h, 7);
            }
            // ---- E: qkv(l+1): LN1 folded; q + this token's K / V of layer l+1, sc1
            if (!last) {
                const bool has = bid < NGE;
                const int g = bid;
                const bool ep = has && ethr;
                const int row = (rb0 + er_r) * 16 + er, col = (g * T + et) * 16 + 4 * eq;
                const bool kvcol = ep && row < a.B && col >= C;
                const int ps = kvcol ? a.pos[row] : 0;  // before the weight loads (vmcnt retires in order)
                float4 c1 = zero4(), c2 = zero4();
                if (ep) {
                    c1 = ld4(ly->qkv_c1 + col);
                    c2 = ld4(ly->qkv_c2 + col);
                }
                float4 wr[T][SPW];
                if (has) load_wt<T>(ly->w_qkv, K16, g * T, 0, w, wr);
                const int page = kvcol ? a.bt[(size_t)row * a.bt_stride + ps / P] : -1;
                if (!wait_sum(a, ctr_of(a, l, h, PC_X2), NGD, 4, smu)) return false;
                PT_MARK(l, h, 8);
                if (has) unit_mfma<HR, T, true>(a.res, K16, rb0, 0, w, wr, sm.red, sm.wsum);
                lds_barrier();
                if (ep && row < a.B) {
                    const float4 v = ln4(sm.wsum + er_r * NWV * 32, er, fold<HR, T>(sm.red, er_r, et, er, eq), c1, c2);
                    if (col < C) {
                        hpa::store_wt16(a.q, (row * C + col) * 4, v);
                    } else if (page >= 0) {  // add_to_cache into layer l+1's page (paged_infer.c:505-573)
                        const int kv = col >= 2 * C;
                        const int c = col - (kv ? 2 * C : C);
                        const int hh = c >> 6, d = c & 63;
                        const int pslot = ps % P;
                        const size_t toff = (size_t)page * a.page_elems + ((size_t)kv * NH + hh) * P * 64 +
                                            (kv == 0 ? ((d >> 2) * P + pslot) * 4 : pslot * 64 + d);
                        hpa::store_wt16(a.kv + (size_t)(l + 1) * a.layer_bytes, (int)(toff * 4), v);
                    }
                }
                drain_vm();
                lds_barrier();
                if (tid == 0 && has) arrive(ctr_of(a, l + 1, h, PC_QKV), 1);
                PT_MARK(l, h, 9);
            }
        }
    }
    return true;
}

template <int P, int HR, int T>
__device__ __forceinline__ void g_role(const PA& a, PSmem<HR, T>& smu) {
#pragma unroll 1
    for (int l = 0; l < a.L; ++l)
#pragma unroll 1
        for (int h = 0; h < 2; ++h)
            if (!g_chain<P, HR, T>(a, smu, l, h)) return;
}

template <int P, int HR, int T>
__global__ __launch_bounds__(768) void decode_pipe_kernel(PA args) {
    const PA& a = *(const PA*)(const void*)__builtin_amdgcn_kernarg_segment_ptr();
    (void)args;
    __shared__ PSmem<HR, T> sm;
    PT_MARK(0, 0, 10);
    if ((int)blockIdx.x < a.NG)
        g_role<P, HR, T>(a, sm);
    else
        a_role<P, HR, T>(a, sm);
}

int g_ncu = 0;
int num_cus() {
    if (!g_ncu) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess) return 0;
        hipDeviceProp_t pr;
        if (hipGetDeviceProperties(&pr, dev) != hipSuccess) return 0;
        g_ncu = pr.multiProcessorCount;
    }
    return g_ncu;
}

template <typename K>
int resident_blocks(K kernel) {
    static int resident = -1;
    if (resident < 0) {
        int nb = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kernel, 768, 0) != hipSuccess) nb = 0;
        resident = nb;
    }
    return resident;
}

constexpr int kT = 3;  // tiles per unit of fc / fcproj / qkv: 64 / 64 / 48 units

template <int P, int HR>
int launch_pipe(PA& a) {
    auto k = decode_pipe_kernel<P, HR, kT>;
    HPA_REQUIRE(resident_blocks(k) >= 1, "decode pipe: the workgroup does not fit a CU");
    decode_pipe_kernel<P, HR, kT><<<a.NG + a.NA, 768, 0, hpa_stream()>>>(a);
    HPA_LAUNCH_CHECK();
    return 0;
}

bool pipe_shape(int B, int ncu, int g_cus, int* HR) {
    const int R = (B + 15) / 16;
    if (B < 1 || B > 64 || (R != 2 && R != 4)) return false;
    const int hr = R / 2;
    if (B <= hr * 16) return false;  // both halves hold rows
    const int na = ncu - g_cus;
    if (g_cus < 4 * NCT / kT || g_cus % 8 || na <= 0) return false;  // every G phase has a unit per workgroup
    if (hr * 16 * NH > 3 * na) return false;                          // an attention unit per A slot
    *HR = hr;
    return true;
}

}  // namespace

extern "C" {

int hpa_decode_pipe_eligible(int B, int C_, int num_heads, int kv_dtype) {
#ifndef HPA_AB
    // measured slower than chain form 6 at every batch (profiles/r6/pipe/):
    // A/B builds only, like the other forms that lost
    (void)B;
    (void)C_;
    (void)num_heads;
    (void)kv_dtype;
    return 0;
#endif
    int hr = 0;
    const int ncu = num_cus();
    return C_ == C && num_heads == NH && kv_dtype == HPA_F32 && ncu > 0 && pipe_shape(B, ncu, kDefaultG, &hr) ? 1 : 0;
}

// trace build only: the stamps of the last launch ([2 * layers][256][12] u64,
// s_memrealtime ticks of 10 ns); host NULL clears them.  1 in the product build.
int hpa_decode_pipe_trace(unsigned long long* host, int layers) {
#ifdef HPA_PIPE_TRACE
    HPA_REQUIRE(layers >= 0 && layers <= 64, "pipe trace: layers 0..64");
    if (!host) {
        static unsigned long long zero[2 * 64 * 256 * 12];
        HPA_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_pipe_trace), zero, sizeof(zero)));
        return 0;
    }
    HPA_CHECK(hipMemcpyFromSymbol(host, HIP_SYMBOL(g_pipe_trace), (size_t)2 * layers * 256 * 12 * 8));
    return 0;
#else
    (void)host;
    (void)layers;
    return 1;
#endif
}

int hpa_decode_pipe_sizes(int B, size_t* out2) {
    HPA_REQUIRE(out2 && B > 0, "decode pipe sizes: bad arguments");
    const int R = (B + 15) / 16, HR = (R + 1) / 2;
    out2[0] = (size_t)2 * 4 * (NCT / kT) * HR * kT * 64 * 4;  // [half][part][group][HR*T*64 threads][4]
    out2[1] = (size_t)kLayerInts;
    return 0;
}

int hpa_decode_pipe(const HpaPipeArgs* h) {
#ifndef HPA_AB
    (void)h;
    return hpa_fail(__FILE__, __LINE__, "decode pipe: the pipelined halves are in A/B builds only (-DHPA_AB)");
#else
    HPA_REQUIRE(h && h->pool && h->pool->base && h->layers, "decode pipe: pool, layer table");
    const HpaKVPool* pool = h->pool;
    HPA_REQUIRE(pool->dtype == HPA_F32 && pool->head_size == HS && pool->num_heads == NH,
                "decode pipe: fp32 pool, 12 heads of 64");
    HPA_REQUIRE(h->num_layers >= 1 && h->num_layers <= pool->num_layers, "decode pipe: layers");
    HPA_REQUIRE(h->q && h->att && h->res && h->res2 && h->fch && h->slab && h->stats_out && h->counters && h->err &&
                    h->block_table && h->pos,
                "decode pipe: null operand");
    HPA_REQUIRE(h->layer_ctr_ints >= (size_t)kLayerInts, "decode pipe: counter block per layer too small");
    const size_t layer_bytes = pool->layer_elems * pool->elem_bytes;
    HPA_REQUIRE(layer_bytes < 0x7fffffffull, "decode pipe: a layer's pages must be < 2 GiB (32-bit offsets)");
    const int ncu = num_cus();
    const int g = h->g_cus > 0 ? h->g_cus : kDefaultG;
    int HR = 0;
    HPA_REQUIRE(pipe_shape(h->B, ncu, g, &HR), "decode pipe: shape (17..64 rows in two halves, CU split)");
    PA a;
    memset(&a, 0, sizeof(a));
    a.B = h->B;
    a.L = h->num_layers;
    a.NG = g;
    a.NA = ncu - g;
    a.stats_mp = h->stats_mp > 0 ? h->stats_mp : (h->B + 15) / 16 * 16;
    a.layer_ctr = h->layer_ctr_ints;
    a.lay = h->layers;
    a.q = h->q;
    a.kv = (char*)pool->base;
    a.layer_bytes = layer_bytes;
    a.page_elems = pool->page_elems;
    a.bt = h->block_table;
    a.bt_stride = h->bt_stride;
    a.pos = h->pos;
    const float log2e = 1.4426950408889634f;
    a.qscale = (float)(1.0 / sqrt((double)HS)) * log2e;
    a.m_init = -10000.0f * log2e;
    a.att = h->att;
    a.res = h->res;
    a.res2 = h->res2;
    a.fch = h->fch;
    a.slab = h->slab;
    a.stats_out = h->stats_out;
    a.ctr = h->counters;
    a.err = h->err;
    a.err_sticky = h->err_sticky;
#define HPA_PIPE_CASE(PS)                                              \
    case PS:                                                           \
        return HR == 2 ? launch_pipe<PS, 2>(a) : launch_pipe<PS, 1>(a);
    switch (pool->page_size) {
        HPA_PIPE_CASE(8)
        HPA_PIPE_CASE(16)
        HPA_PIPE_CASE(32)
        HPA_PIPE_CASE(64)
        default: return hpa_fail(__FILE__, __LINE__, "decode pipe: page size must be 8, 16, 32 or 64");
    }
#undef HPA_PIPE_CASE
#endif
}

}  // extern "C"
