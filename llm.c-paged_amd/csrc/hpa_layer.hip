// hpa_layer.hip -- the decode step's layer as ONE persistent launch (gfx950).
//
// Replaces five launches per layer of the reference layer loop
// (gpt2_forward, paged_infer.c:659-722, one decode row per sequence):
//   A  attention(l)   attention_paged :163-240 (split context, hpa_attn_body.h)
//   B  attproj(l)     matmul_forward :716 + residual_forward :717
//   C  fc(l)          layernorm_forward :718 (folded) + matmul :719 + gelu :720
//   D  fcproj(l)      matmul_forward :721 + residual_forward :722
//   E  qkv(l+1)       layernorm :696 (folded) + matmul_cached :706 + add_to_cache :710
// so a step is embed, qkv(0), L of these, logits, token choice.
//
// Why ("Persistent layer"): every launch of the
// five-kernel layer pays a dispatch + first-round-trip + drain cost, and each
// GEMM starts fetching its weights only after the previous kernel ended.
// Here every phase's weight fragments are loaded into registers before the
// phase's wait, so the weight stream overlaps the hand-off, and the seams
// between phases are in-launch hand-offs.
//
// Geometry: one workgroup of 12 waves per CU (grid = CU count, residency
// checked with the occupancy API), three 4-wave slots.  A phase's units are
// numbered v and dealt v -> (workgroup v % G, slot v / G):
//   A  attention unit (sequence, head, context range; hpa_attn_body.h tiles,
//      folded through LDS by the slot's last wave, split_merge across ranges)
//   B..E  a 16x16 output tile (row block rb, column tile j) over K = C (fc,
//      qkv, attproj) or one of 4 K parts of 4C (fcproj), 4 waves x K/4 each
//      -- the one-shot GEMM kernel's summation order.
// ATTN = false (chain form, the engine's default): no phase A; the attention
// ran as its own launch just before, writing att in frag layout.
// fcproj's K-part partial tiles go to a slab with write-through stores; the
// last part of a tile to draw its ticket sums the parts in part order
// (results independent of arrival order), adds bias and residual.
//
// Hand-offs (MI355X_MICROARCH.md "Valid forms", row 1; cdna_hip_programming.md
// Guideline 16): every byte handed over inside the launch is stored sc1
// (write-through) and loaded sc1 (L1 bypass); each storing wave drains
// (s_waitcnt vmcnt(0)), the workgroup barrier follows, then ONE lane adds to
// the phase counter, sharded over 8 lines by workgroup % 8; the consumer's
// wave 0 polls every shard with sc1 loads, the other waves wait at a barrier.
// Counters are zeroed before every step (a memset node), one block per layer.
// Every spin is bounded: on timeout *err gets the phase code and the launch
// ends (outputs garbage, reported by the host).
#include <math.h>

#include "hpa_attn_body.h"
#include "hpa_gemm_body.h"

namespace {
using hpa_attn::HS;
using hpa_attn::kRec;
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kPad = 32;                // ints per counter shard (one 128-B line)
constexpr int kCtrInts = 4 * 8 * kPad;  // counters ATT, X1, H, X2 x 8 shards
enum { CT_ATT = 0, CT_X1 = 1, CT_H = 2, CT_X2 = 3 };
constexpr long long kSpinTicks = 20000000;  // s_memrealtime is 100 MHz: 200 ms

template <int NH>
struct LD {
    static constexpr int C = 64 * NH;
    static constexpr int K16 = C / 16;  // k16 steps of K = C; also the column tiles of N = C
    static constexpr int NCT = C / 16;
    static constexpr int FP = 4;   // fcproj K parts (C each)
    static constexpr int SW = NH;  // k16 steps per wave: K = C over a slot's 4 waves
};

template <int NH>
struct Smem {
    float red[12 * 256];     // [wave][4 regs][64 lanes] accumulators
    float wsum[12 * 32];     // [wave][16 rows][2] LN row partial sums
    float tile[3 * 16 * 17]; // last layer: [slot][16 rows][17] for the LNf statistics
    float s_m[3][4], s_l[3][4];
    float4 s_acc[3][64];     // [slot][4 waves x 16 lanes] (fp32) / [4 waves x 8 lanes][2] (bf16)
    int s_cnt[3];
    int s_ok;
    int s_last[3];
};

struct KA {
    int B, Mp, R, S, G, last, layer;
    const float* q;
    const void* kv;       // layer l of the pool
    void* kv_next;        // layer l+1
    size_t page_elems;
    const int* bt;
    int bt_stride;
    const int* pos;
    float qscale, m_init;
    float *att, *res, *res2, *fch;
    const float *w_ap, *b_ap, *w_fc, *fc_c1, *fc_c2, *w_fp, *b_fp, *w_qkv, *qkv_c1, *qkv_c2;
    float* q_out;
    float* stats_out;
    float* rec;
    float* slab_fp;
    int* ctr;
    int* err;
    int* err_sticky;
    // chain form 8 (wide layers, GPT-2 XL): tiles per unit and tile groups
    // (padded to a multiple of 8) of attproj, fc, fcproj, qkv
    int xt[4], xng[4];
    // the step's first launch (decode_first6_kernel): the tokens, the
    // embedding tables, and the step's counter block to zero (16-B granules)
    const int* tokens;
    const float *wte, *wpe;
    int4* zero;
    int zero_n4;
};

// diagnostic build (-DHPA_LAYER_TRACE, tools/pl_trace.py): s_memrealtime of
// workgroup-level events per (layer, workgroup); never in the product library
#ifdef HPA_LAYER_TRACE
// (the stamp intrinsic counts as a memory clobber: the trace build loads q
// through vector loads + readfirstlane, HPA_PL_QREG, ~1 us later than the
// product's scalar loads)
#ifndef HPA_PL_QREG
#define HPA_PL_QREG 1
#endif
__device__ unsigned long long g_pl_trace[64][256][16];
// form 8's fc phase of one layer, per wave (s_memtime, shader clock): [0] A
// loads issued, [1 + q] half-tile q's MFMAs issued, [15] loop done
__device__ unsigned long long g_cx_wave[256][12][16];
#define CX_WSTAMP(on, slot)                                                                              \
    do {                                                                                                 \
        if ((on) && (threadIdx.x & 63) == 0 && blockIdx.x < 256)                                         \
            g_cx_wave[blockIdx.x][threadIdx.x >> 6][slot] = (unsigned long long)__builtin_amdgcn_s_memtime(); \
    } while (0)
#define PL_MARK(k)                                                                                     \
    do {                                                                                               \
        if (threadIdx.x == 0 && a.layer < 64 && blockIdx.x < 256)                                      \
            g_pl_trace[a.layer][blockIdx.x][k] = (unsigned long long)__builtin_amdgcn_s_memrealtime(); \
    } while (0)
// stamps taken before the attention are stored after it: a global store in
// front of the q loads would cost them their scalar (s_load) form
#define PL_STAMP(var) const unsigned long long var = (unsigned long long)__builtin_amdgcn_s_memrealtime()
#define PL_STORE(k, var)                                                           \
    do {                                                                           \
        if (threadIdx.x == 0 && a.layer < 64 && blockIdx.x < 256) g_pl_trace[a.layer][blockIdx.x][k] = var; \
    } while (0)
#else
#define PL_MARK(k) \
    do {           \
    } while (0)
#define PL_STAMP(var) \
    do {              \
    } while (0)
#define PL_STORE(k, var) \
    do {                 \
    } while (0)
#define CX_WSTAMP(on, slot) \
    do {                    \
    } while (0)
#endif

__device__ __forceinline__ int wave_sum_int(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// every thread of the workgroup calls; wave 0 polls the 8 shards of counter
// `which` until they sum to `expected` (bounded), the rest wait at the barrier
template <int NH>
__device__ __forceinline__ bool wait_ctr(const KA& a, int which, int expected, int code, Smem<NH>& sm) {
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (wv == 0) {
        const int lane = threadIdx.x & 63;
        const int* c = a.ctr + which * 8 * kPad;
        int ok = 0;
        const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
        for (unsigned it = 0;; ++it) {
#ifndef HPA_PL_POLL
#define HPA_PL_POLL 0
#endif
#if HPA_PL_POLL == 2  /* experiment: returning atomic add of 0 (served at the memory side) */
            int v = lane < 8 ? __hip_atomic_fetch_add(const_cast<int*>(c) + lane * kPad, 0, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT)
                             : 0;
#elif HPA_PL_POLL == 3  /* experiment: system-scope (sc0 sc1) loads */
            int v = lane < 8 ? __hip_atomic_load(c + lane * kPad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0;
#else
            int v = lane < 8 ? __hip_atomic_load(c + lane * kPad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
#endif
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
#ifndef HPA_PL_NOSLEEP
            __builtin_amdgcn_s_sleep(1);
#endif
        }
        if (lane == 0) sm.s_ok = ok;
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // no VMEM drain (see lds_barrier)
    const bool ok = sm.s_ok != 0;
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // s_ok read before the next wait rewrites it
    return ok;
}

// one lane, after every storing wave's drain and the workgroup barrier
__device__ __forceinline__ void arrive(const KA& a, int which, int n) {
    __hip_atomic_fetch_add(a.ctr + which * 8 * kPad + (blockIdx.x & 7) * kPad, n, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ float4 ld_nt(const float4* p) {
    const f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
    return make_float4(v.x, v.y, v.z, v.w);
}

// ------------------------------------------------------------------ phase A
// attention unit u = (sequence, head) x context range, run by the 4 waves of
// `slot`; the slot folds through LDS with a last-arriving-wave counter (no
// workgroup barrier: the other slots and the staging waves run on)
// q of unit u's (sequence, head) as wave-uniform values (SGPRs): loaded
// before the weight DMA is issued (behind an LDS-DMA the compiler no longer
// proves q unclobbered and would keep it in 64 VGPRs)
template <int NH>
__device__ __forceinline__ void load_q(const KA& a, int u, float (&qv)[HS]) {
    const float4* q4 = reinterpret_cast<const float4*>(a.q + (size_t)(u / a.S) * HS);
#pragma unroll
    for (int i = 0; i < HS / 4; ++i) {
        const float4 t = q4[i];
        qv[4 * i + 0] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(t.x)));
        qv[4 * i + 1] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(t.y)));
        qv[4 * i + 2] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(t.z)));
        qv[4 * i + 3] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(t.w)));
    }
}

template <int NH, int P, bool BF>
__device__ __forceinline__ void attn_unit(const KA& a, int u, int slot, int wq, Smem<NH>& sm, const float (&qv)[HS]) {
    constexpr int C = LD<NH>::C;
    constexpr int TILE = P * HS;
    constexpr int K = BF ? 2 : 1;    // float4 chunks of the folded state per lane
    constexpr int NL = 16 / K;       // lanes holding it
    const int lane = threadIdx.x & 63;
    const int S = a.S;
    const int bh = u / S;
    const int sr = u - bh * S;
    const int b = bh / NH;
    const int h = bh - b * NH;
    const int ctx = a.pos[b] + 1;
#ifdef HPA_PL_QREG
    const float* qh = qv;
#else
    (void)qv;
    const float* __restrict__ qh = a.q + (size_t)bh * HS;  // scalar loads beside the first page ids
#endif
    const int* bt = a.bt + (size_t)b * a.bt_stride;
    const int n_all = (ctx + 63) >> 6;
    const int it0 = (int)((long long)sr * n_all / S);
    const int it1 = (int)((long long)(sr + 1) * n_all / S);
    float m = a.m_init, l = 0.f;
    float4 acc[K];
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    if constexpr (BF) {
        const unsigned short* base = reinterpret_cast<const unsigned short*>(a.kv);
        hpa_attn::attn_tiles_bf16<P, 4>(qh, base + (size_t)h * TILE, base + (size_t)(NH + h) * TILE, a.page_elems, bt,
                                        a.bt_stride, ctx, it0, it1, a.qscale, m, l, acc, wq);
#pragma unroll
        for (int o = 8; o <= 32; o <<= 1)
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                acc[k].x += __shfl_xor(acc[k].x, o, 64);
                acc[k].y += __shfl_xor(acc[k].y, o, 64);
                acc[k].z += __shfl_xor(acc[k].z, o, 64);
                acc[k].w += __shfl_xor(acc[k].w, o, 64);
            }
    } else {
        const float* base = reinterpret_cast<const float*>(a.kv);
        hpa_attn::attn_tiles<P, 4>(qh, base + (size_t)h * TILE, base + (size_t)(NH + h) * TILE, a.page_elems, bt,
                                   a.bt_stride, ctx, it0, it1, a.qscale, m, l, acc[0], wq);
#pragma unroll
        for (int o = 16; o <= 32; o <<= 1) {
            acc[0].x += __shfl_xor(acc[0].x, o, 64);
            acc[0].y += __shfl_xor(acc[0].y, o, 64);
            acc[0].z += __shfl_xor(acc[0].z, o, 64);
            acc[0].w += __shfl_xor(acc[0].w, o, 64);
        }
    }
    l = hpa::wave_sum(l);
    if (lane == 0) {
        sm.s_m[slot][wq] = m;
        sm.s_l[slot][wq] = l;
    }
    if (lane < NL)
#pragma unroll
        for (int k = 0; k < K; ++k) sm.s_acc[slot][(wq * NL + lane) * K + k] = acc[k];
    int old = 0;
    if (lane == 0) old = __hip_atomic_fetch_add(&sm.s_cnt[slot], 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
    old = __builtin_amdgcn_readfirstlane(old);
    if (old != 3 || lane >= NL) return;
    // the last wave of the slot: the 4 waves' states in wave order (hpa_attn::attn_fold)
    float M = sm.s_m[slot][0];
#pragma unroll
    for (int i = 1; i < 4; ++i) M = fmaxf(M, sm.s_m[slot][i]);
    float L = 0.f;
    float4 O[K];
#pragma unroll
    for (int k = 0; k < K; ++k) O[k] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const float f = exp2f(sm.s_m[slot][i] - M);
        L = fmaf(sm.s_l[slot][i], f, L);
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const float4 v = sm.s_acc[slot][(i * NL + lane) * K + k];
            O[k].x = fmaf(v.x, f, O[k].x);
            O[k].y = fmaf(v.y, f, O[k].y);
            O[k].z = fmaf(v.z, f, O[k].z);
            O[k].w = fmaf(v.w, f, O[k].w);
        }
    }
    m = M;
    l = L;
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] = O[k];
    if (S > 1) {
        int* tick = a.ctr + kCtrInts + 2 * a.R * LD<NH>::NCT + bh;  // zeroed per step: no rewind
        if (!hpa_attn::split_merge<K>(a.rec + (size_t)bh * S * kRec, tick, S, sr, m, l, acc, false)) return;
    }
    const float inv = l == 0.f ? 0.f : 1.f / l;
#pragma unroll
    for (int k = 0; k < K; ++k) {  // dims (16/NL)*lane + 4k .. +3 of head h, frag layout
        const int col = h * HS + (64 / NL) * lane + 4 * k;
        hpa::store_wt16(a.att, (int)(hpa::frag_index(b, col, C) * 4),
                        make_float4(acc[k].x * inv, acc[k].y * inv, acc[k].z * inv, acc[k].w * inv));
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this (the only storing) wave drained
    if (lane == 0) arrive(a, CT_ATT, 1);
}

// ------------------------------------------------------------------ GEMM units
// A unit is one 16x16 output tile (column tile j, row block rb) over a K range
// of C (the whole K of qkv / attproj / fc, one of 4 parts of fcproj's 4C),
// computed by one 4-wave slot exactly like gemm16_os_kernel<4, *, K16/4>:
// wave wq takes k16 steps [wq*SW, wq*SW+SW), one accumulator chain in k
// order, the 4 waves folded in wave order.  Phase X's units are numbered
// v = (part*R + rb)*NJ + j and dealt v -> workgroup v % G, slot v / G: with
// NJ and G multiples of 8 the row blocks and parts of one weight tile land on
// one XCD (blocks b, b+8 share an XCD) and re-read it from that L2.
// The slot's weight fragments are loaded into registers BEFORE the phase's
// wait (prefetch across the seam); the barriers between phases wait for LDS
// only (lds_barrier), so those loads stay in flight.

// workgroup barrier that does not drain the vector-memory counter (the
// prefetched weights stay in flight); LDS accesses before it are complete
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

struct Unit {
    int j, rb, p;
    bool has;
};
__device__ __forceinline__ Unit unit_of(int v, int n, int NJ, int R) {
    Unit u;
    u.has = v < n;
    const int vv = u.has ? v : 0;
    u.j = vv % NJ;
    const int q = vv / NJ;
    u.rb = q % R;
    u.p = q / R;
    return u;
}

// the wave's weight fragments of column tile j, k16 steps kb + wq*SW ..
// (K16W steps per tile row); non-temporal where one row block reads the tile
template <int SW>
__device__ __forceinline__ void load_w(const float* W, int K16W, int j, int kb, int wq, bool nt, float4 (&wr)[SW]) {
    const float4* wf = reinterpret_cast<const float4*>(W) + ((size_t)j * K16W + kb + wq * SW) * 64 + (threadIdx.x & 63);
    if (nt) {
#pragma unroll
        for (int s = 0; s < SW; ++s) wr[s] = ld_nt(wf + s * 64);
    } else {
#pragma unroll
        for (int s = 0; s < SW; ++s) wr[s] = wf[s * 64];
    }
}

// the wave's A fragments (activation written in this launch: sc1 loads),
// then the one-shot kernel's chain and (STATS) its LN row partial sums
template <int SW, bool STATS>
__device__ __forceinline__ f32x4 unit_mfma(const float* A, int K16A, int rb, int kb, int wq, const float4 (&wr)[SW],
                                           float& fs1, float& fs2) {
    float4 xv[SW];
    const int off = ((rb * K16A + kb + wq * SW) * 64 + (int)(threadIdx.x & 63)) * 16;
#pragma unroll
    for (int s = 0; s < SW; ++s) xv[s] = hpa::load_wt16(A, off + s * 1024);
    __builtin_amdgcn_sched_barrier(0);  // every A load in flight before the first MFMA (see c6::mfma_t)
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < SW; ++s) {
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[s].x, wr[s].x, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[s].y, wr[s].y, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[s].z, wr[s].z, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[s].w, wr[s].w, acc, 0, 0, 0);
    }
    if (STATS)
#pragma unroll
        for (int s = 0; s < SW; ++s) hpa_gemm::row_sums_add(xv[s], fs1, fs2);
    return acc;
}

__device__ __forceinline__ void put_red(float* red, int wv, f32x4 acc) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int g = 0; g < 4; ++g) red[wv * 256 + g * 64 + lane] = acc[g];
}

// element e = wq*64 + lane of the slot's tile, its 4 waves in wave order
// (Epi<4,...>::finish): row 4*(lane>>4) + wq, column lane & 15
__device__ __forceinline__ float fold4(const float* red, int slot, int e) {
    const float* r = red + slot * 4 * 256 + e;
    float v = r[0];
    v += r[256];
    v += r[512];
    v += r[768];
    return v;
}

// units of NWU waves (unit slot us of the workgroup): the waves in wave order
template <int NWU>
__device__ __forceinline__ float foldn(const float* red, int us, int e) {
    const float* r = red + us * NWU * 256 + e;
    float v = r[0];
#pragma unroll
    for (int w = 1; w < NWU; ++w) v += r[w * 256];
    return v;
}

// LayerNorm-folded value: rstd*(acc - mean*c1) + c2 (Epi::apply's order);
// the row partial sums of the NWU waves of unit slot us
template <int NWU = 4>
__device__ __forceinline__ float ln_fold_val(const float* wsum, int us, int lrow, int K, float val, float c1,
                                             float c2) {
    const float* ws = wsum + us * NWU * 32;
    float S1 = ws[2 * lrow], S2 = ws[2 * lrow + 1];
#pragma unroll
    for (int ww = 1; ww < NWU; ++ww) {
        S1 += ws[ww * 32 + 2 * lrow];
        S2 += ws[ww * 32 + 2 * lrow + 1];
    }
    const float m = S1 / K;
    const float rstd = 1.0f / sqrtf(fmaxf(S2 / K - m * m, 0.f) + 1e-5f);
    val = rstd * (val - m * c1);
    val += c2;
    return val;
}

// unit slots of workgroup bid (UPW per workgroup) that hold one of n units
template <int UPW>
__device__ __forceinline__ int units_with(int bid, int G, int n) {
    int k = 0;
#pragma unroll
    for (int s2 = 0; s2 < UPW; ++s2) k += bid + s2 * G < n;
    return k;
}

// every storing wave drained, then one lane counts the slots that stored
__device__ __forceinline__ void publish(const KA& a, int which, int nslots) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();
    if (threadIdx.x == 0 && nslots) arrive(a, which, nslots);
}

// ------------------------------------------------------------------ the kernel
// ATTN = false: the chain only (attproj -> fc -> fcproj -> next qkv); the
// attention ran as its own launch just before (hpa_paged_attention_decode_split
// writing `att` in frag layout), so phase B needs no in-launch wait.
// Waves per GEMM unit, per phase (NB attproj, NCD fc and fcproj, NE qkv): 4
// (three 4-wave slots per workgroup), or wide units in the chain form
// (C = 768): 12 (one unit per workgroup, a phase of <= 256 units) or 6 (two
// per workgroup, <= 512 units).  A unit's K range is split over its waves
// (4 * SW / NWU k16 steps each, folded in wave order): with fewer units than
// 4-wave slots the 4-wave form leaves slots idle and runs longer MFMA chains
// per wave
template <int NWU>
struct UW {  // a wave's place in its phase's unit
    int us, wu, v, e, lrow;
    bool fin;
    __device__ __forceinline__ UW(int wv, int bid, int G, int lane) {
        us = wv / NWU;       // unit slot of the workgroup
        wu = wv - us * NWU;  // wave within the unit
        v = bid + us * G;    // the unit slot's unit
        fin = wu < 4;        // the waves that finish the unit's elements
        e = (wu & 3) * 64 + lane;
        lrow = 4 * (lane >> 4) + (wu & 3);
    }
};

template <int NH, int P, bool BF, bool ATTN, int NB, int NCD, int NE>
__global__ __launch_bounds__(768) void decode_layer_kernel(KA args) {
    using D = LD<NH>;
    constexpr int C = D::C, SW = D::SW, NCT = D::NCT;
    static_assert((NB == 4 && NCD == 4 && NE == 4) ||
                      (!ATTN && (SW * 4) % NB == 0 && (SW * 4) % NCD == 0 && (SW * 4) % NE == 0),
                  "wide units: chain form, K split evenly");
    // fields read where used from the kernarg segment (not all hoisted into
    // SGPRs at entry: the attention keeps q in 64 SGPRs)
    const KA& a = *(const KA*)(const void*)__builtin_amdgcn_kernarg_segment_ptr();
    (void)args;
    __shared__ Smem<NH> sm;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int slot = wv >> 2, wq = wv & 3;
    const int lane = threadIdx.x & 63;
    const int bid = blockIdx.x;
    const int R = a.R, G = a.G;
    const int v = bid + slot * G;           // this slot's attention unit (phase A)
    const int lcol = lane & 15;
    const bool nt = R == 1;                 // one row block: every weight tile read once
    PL_STAMP(t_start);
    if (threadIdx.x < 3) sm.s_cnt[threadIdx.x] = 0;
    __syncthreads();

    // A: attention, one unit (sequence, head, context range) per slot
    if constexpr (ATTN) {
        const bool has = v < a.B * NH * a.S;
        float qv[HS];
#ifdef HPA_PL_QREG
        if (has) load_q<NH>(a, v, qv);
#endif
        PL_STAMP(t_issued);
        if (has) attn_unit<NH, P, BF>(a, v, slot, wq, sm, qv);
        PL_MARK(2);
        PL_STORE(1, t_issued);
    }
    PL_STORE(0, t_start);
    float fs1, fs2;
    // B: attproj(l): res2 = res + att . Wap^T + b
    {
        constexpr int SWU = SW * 4 / NB;
        const UW<NB> uw(wv, bid, G, lane);
        const int us = uw.us, wu = uw.wu, e = uw.e, lrow = uw.lrow;
        const bool fin = uw.fin;
        float4 wr[SWU];
        const Unit u = unit_of(uw.v, NCT * R, NCT, R);
        if (u.has) load_w<SWU>(a.w_ap, D::K16, u.j, 0, wu, nt, wr);
        lds_barrier();
        PL_MARK(3);
        if (ATTN && !wait_ctr<NH>(a, CT_ATT, a.B * NH, 1, sm)) return;
        PL_MARK(4);
        const int row = u.rb * 16 + lrow, col = u.j * 16 + lcol;
        const int fi = (int)(hpa::frag_index(row, col, C) * 4);
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        float bv = 0.f, rv = 0.f;
        if (u.has) {
            if (fin) {
                bv = a.b_ap[col];
                rv = hpa::load_wt4(a.res, fi);
            }
            acc = unit_mfma<SWU, false>(a.att, D::K16, u.rb, 0, wu, wr, fs1, fs2);
        }
        put_red(sm.red, wv, acc);
        lds_barrier();
        if (u.has && fin) {
            float val = foldn<NB>(sm.red, us, e);
            val += bv;
            val = row < a.B ? rv + val : 0.f;  // residual_forward(out, res, proj)
            hpa::store_wt4(a.res2, fi, val);
        }
        publish(a, CT_X1, units_with<12 / NB>(bid, G, NCT * R));
    }
    PL_MARK(5);
    // C: fc(l): fch = gelu(LN2(res2) . Wfc^T + b), LN folded
    {
        constexpr int SWU = SW * 4 / NCD;
        const UW<NCD> uw(wv, bid, G, lane);
        const int us = uw.us, wu = uw.wu, e = uw.e, lrow = uw.lrow;
        const bool fin = uw.fin;
        float4 wr[SWU];
        const Unit u = unit_of(uw.v, 4 * NCT * R, 4 * NCT, R);
        if (u.has) load_w<SWU>(a.w_fc, D::K16, u.j, 0, wu, nt, wr);
        if (!wait_ctr<NH>(a, CT_X1, NCT * R, 2, sm)) return;
        PL_MARK(6);
        const int row = u.rb * 16 + lrow, col = u.j * 16 + lcol;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        float c1 = 0.f, c2 = 0.f;
        fs1 = fs2 = 0.f;
        if (u.has) {
            if (fin) {
                c1 = a.fc_c1[col];
                c2 = a.fc_c2[col];
            }
            acc = unit_mfma<SWU, true>(a.res2, D::K16, u.rb, 0, wu, wr, fs1, fs2);
        }
        hpa_gemm::row_sums_publish(fs1, fs2, sm.wsum + wv * 32);
        put_red(sm.red, wv, acc);
        lds_barrier();
        if (u.has && fin) {
            float val = foldn<NCD>(sm.red, us, e);
            val = ln_fold_val<NCD>(sm.wsum, us, lrow, C, val, c1, c2);
            hpa::store_wt4(a.fch, (int)(hpa::frag_index(row, col, 4 * C) * 4), row < a.B ? hpa::gelu_ref(val) : 0.f);
        }
        publish(a, CT_H, units_with<12 / NCD>(bid, G, 4 * NCT * R));
        PL_MARK(7);
    }
    // D: fcproj(l), K part p of 4: partial tiles -> slab; the last part of
    // (rb, j) adds the parts in order + bias + res2 -> res
    {
        constexpr int SWU = SW * 4 / NCD;
        const UW<NCD> uw(wv, bid, G, lane);
        const int us = uw.us, wu = uw.wu, e = uw.e, lrow = uw.lrow;
        const bool fin = uw.fin;
        float4 wr[SWU];
        const Unit u = unit_of(uw.v, NCT * R * D::FP, NCT, R);
        if (u.has) load_w<SWU>(a.w_fp, 4 * D::K16, u.j, u.p * D::K16, wu, nt, wr);
        if (!wait_ctr<NH>(a, CT_H, 4 * NCT * R, 3, sm)) return;
        PL_MARK(8);
        const int row = u.rb * 16 + lrow, col = u.j * 16 + lcol;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        if (u.has) acc = unit_mfma<SWU, false>(a.fch, 4 * D::K16, u.rb, u.p * D::K16, wu, wr, fs1, fs2);
        put_red(sm.red, wv, acc);
        lds_barrier();
        float val = 0.f;
        const int sofs = ((u.p * R + u.rb) * NCT + u.j) * 256 + e;
        if (u.has && fin) {
            val = foldn<NCD>(sm.red, us, e);
            hpa::store_wt4(a.slab_fp, sofs * 4, val);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        lds_barrier();
        if (u.has && fin && wu == 0 && lane == 0) {
            const int t = __hip_atomic_fetch_add(a.ctr + kCtrInts + R * NCT + u.rb * NCT + u.j, 1, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
            sm.s_last[us] = t == D::FP - 1;
        }
        lds_barrier();
        const bool last = u.has && fin && sm.s_last[us] != 0;
        if (last) {
            float pv[D::FP];
#pragma unroll
            for (int q = 0; q < D::FP; ++q)
                pv[q] = q == u.p ? val : hpa::load_wt4(a.slab_fp, (((q * R + u.rb) * NCT + u.j) * 256 + e) * 4);
            const int fi = (int)(hpa::frag_index(row, col, C) * 4);
            const float rv = hpa::load_wt4(a.res2, fi);
            float tot = pv[0];
#pragma unroll
            for (int q = 1; q < D::FP; ++q) tot += pv[q];
            tot += a.b_fp[col];
            tot = row < a.B ? rv + tot : 0.f;
            hpa::store_wt4(a.res, fi, tot);
            if (a.stats_out) sm.tile[(us * 16 + lrow) * 17 + lcol] = tot;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        lds_barrier();
        if (a.stats_out && wu == 0 && lane < 16 && last) {  // 16-column LNf partial sums of the tile's rows
            const float* tr = sm.tile + (us * 16 + lane) * 17;
            float s1 = 0.f, s2 = 0.f;
#pragma unroll
            for (int c = 0; c < 16; ++c) {
                s1 += tr[c];
                s2 += tr[c] * tr[c];
            }
            const int r = u.rb * 16 + lane;
            a.stats_out[((size_t)u.j * a.Mp + r) * 2] = s1;
            a.stats_out[((size_t)u.j * a.Mp + r) * 2 + 1] = s2;
        }
        if (threadIdx.x == 0) {
            int nd = 0;
            for (int s2 = 0; s2 < 12 / NCD; ++s2) nd += sm.s_last[s2] != 0 && bid + s2 * G < NCT * R * D::FP;
            if (nd) arrive(a, CT_X2, nd);
        }
        PL_MARK(9);
    }
    // E: qkv(l+1): LN1 folded, q + K/V appended into layer l+1's pages
    if (!a.last) {
        constexpr int SWU = SW * 4 / NE;
        const UW<NE> uw(wv, bid, G, lane);
        const int us = uw.us, wu = uw.wu, e = uw.e, lrow = uw.lrow;
        const bool fin = uw.fin;
        float4 wr[SWU];
        const Unit u = unit_of(uw.v, 3 * NCT * R, 3 * NCT, R);
        if (u.has) load_w<SWU>(a.w_qkv, D::K16, u.j, 0, wu, nt, wr);
        if (!wait_ctr<NH>(a, CT_X2, NCT * R, 4, sm)) return;
        PL_MARK(10);
        const int row = u.rb * 16 + lrow, col = u.j * 16 + lcol;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        float c1 = 0.f, c2 = 0.f;
        fs1 = fs2 = 0.f;
        if (u.has) {
            if (fin) {
                c1 = a.qkv_c1[col];
                c2 = a.qkv_c2[col];
            }
            acc = unit_mfma<SWU, true>(a.res, D::K16, u.rb, 0, wu, wr, fs1, fs2);
        }
        hpa_gemm::row_sums_publish(fs1, fs2, sm.wsum + wv * 32);
        put_red(sm.red, wv, acc);
        lds_barrier();
        if (u.has && fin && row < a.B) {
            float val = foldn<NE>(sm.red, us, e);
            val = ln_fold_val<NE>(sm.wsum, us, lrow, C, val, c1, c2);
            if (col < C) {
                a.q_out[(size_t)row * C + col] = val;
            } else {  // K/V of this token into the sequence's page of layer l+1 (add_to_cache)
                const int kv = col >= 2 * C;
                const int c = col - (kv ? 2 * C : C);
                const int hh = c >> 6, d = c & 63;
                const int ps = a.pos[row];
                const int page = a.bt[(size_t)row * a.bt_stride + ps / P];
                if (page >= 0) {
                    const int pslot = ps % P;
                    const size_t toff = (size_t)page * a.page_elems + ((size_t)kv * NH + hh) * P * 64;
                    if constexpr (BF) {
                        unsigned short* kvt = reinterpret_cast<unsigned short*>(a.kv_next) + toff;
                        kvt[kv == 0 ? ((d >> 3) * P + pslot) * 8 + (d & 7) : pslot * 64 + d] = hpa::f32_to_bf16(val);
                    } else {
                        float* kvt = reinterpret_cast<float*>(a.kv_next) + toff;
                        if (kv == 0)
                            kvt[((d >> 2) * P + pslot) * 4 + (d & 3)] = val;
                        else
                            kvt[pslot * 64 + d] = val;
                    }
                }
            }
        }
    }
    PL_MARK(11);
}

// ------------------------------------------------------------------ the chain, multi-tile units (form 6)
// The default chain form for C = 768.  Every phase runs
// units of all 12 waves of a workgroup (one unit per workgroup): a unit is T
// 16-column tiles of one 16-row block (and, for fcproj, one of its 4 K parts)
// over its K range, wave w taking k16 steps 4w .. 4w+3 of every tile -- the
// summation order of the 12-wave units of chain forms 2..5 (a row's result
// depends on neither T nor the batch, so every batch size and every shard
// computes the same rows).  Against the 4-wave units at B = 64:
//   * a workgroup reads its row block's activation ONCE (48 KB) for its T
//     tiles, where three 4-wave slots read three row blocks (144 KB) through
//     the CU's L2 -> CU path;
//   * the epilogue is 16-byte: a thread owns 4 consecutive columns of one
//     row (one float4 of the next GEMM's frag layout, of q, of a K/V page
//     row), so every hand-off store and residual / bias / LN-fold operand load
//     is dwordx4 (was 4 B per lane);
//   * waits are per row block (fcproj: per row block and K part): a unit
//     waits only for the producers of the rows it reads.
// T per phase (host, chain6_tiles): the fewest tiles with units <= workgroups.
#ifndef HPA_C6_DE
#define HPA_C6_DE 0  // A/B builds: bit 0 fcproj, bit 1 qkv k-group waits at 3-4 row blocks as well
#endif
#ifndef HPA_C6_EARLY
#define HPA_C6_EARLY 0  // A/B builds: 1 = non-storing waves prefetch the next phase's weights right after their MFMAs (measured slower, profiles/r6/experiments/c6_early.txt)
#endif
#ifndef HPA_C6_GW
#define HPA_C6_GW 1  // 1: fc / fcproj / qkv wait per 64-column k-group of their A (wave w on its group); 0: per row block (A/B)
#endif
namespace c6 {
constexpr int NW = 12;  // waves per workgroup = waves per unit
constexpr int SPW = 4;  // k16 steps per wave of a K = 768 range (48 / 12)
// wait counters: X1 per row block, H per (row block, K part), X2 per row block
enum { X1 = 0, H = 4, X2 = 20, NCTR = 24 };
constexpr int kCtr = NCTR * 8 * kPad;  // ints of the sharded counters
// HPA_C6_GW: 16-column tiles landed per (row block, 64-column k-group) of each
// phase's A, after the tickets: res2 for fc (12 groups per row block), fch for
// fcproj (48), res for qkv (12); one 128-B line each
constexpr int kGC = 0, kGD = 4 * NW * kPad, kGE = kGD + 4 * 4 * NW * kPad;
constexpr int kGrp = kGE + 4 * NW * kPad;
__device__ __forceinline__ void arrive_tiles(const KA& a, int base, int rb, int groups_per_rb, int j0, int n) {
    for (int t = j0; t < j0 + n; ++t)  // tile t of the row block lands in group t / 4
        __hip_atomic_fetch_add(a.ctr + base + (rb * groups_per_rb + t / 4) * kPad, 1, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
}

struct Smem6 {
    float red[NW * 3 * 256];  // [wave][tile][256] accumulators
    float wsum[NW * 32];      // [wave][16 rows][2] LN row partial sums
    float tile[3 * 16 * 17];  // last layer: [tile][16 rows][17] for the LNf statistics
    int s_ok;
    int s_last;
    int s_ready;  // HPA_C6_GW: k-groups seen ready by wave 0 (bit 12: the wait failed)
};

__device__ __forceinline__ void arrive6(const KA& a, int ctr, int n) {
    __hip_atomic_fetch_add(a.ctr + ctr * 8 * kPad + (blockIdx.x & 7) * kPad, n, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}

// wave 0 polls the 8 shards of counter ctr until they sum to `expected`
// (bounded; the other waves wait at the barrier), as wait_ctr
template <typename SM>
__device__ __forceinline__ bool wait6(const KA& a, int ctr, int expected, int code, SM& sm) {
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (wv == 0) {
        const int lane = threadIdx.x & 63;
        const int* c = a.ctr + ctr * 8 * kPad;
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
                if (e) break;
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
    lds_barrier();
    return ok;
}

// HPA_C6_GW: wave 0 polls the 12 k-group counters of a row block (lane k:
// group k) and publishes the ready set in LDS; wave w goes on as soon as its
// group is in it, so a wave whose producers finished early starts its A loads
// and MFMAs early (the late waves then share the matrix pipe with fewer).
// Bounded like wait6; a failure releases every wave with bit 12 set.
__device__ __forceinline__ bool wait_grp(const KA& a, int base, int expected, int code, Smem6& sm) {
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    volatile int* rdy = &sm.s_ready;
    if (wv == 0) {
        const int lane = threadIdx.x & 63;
        const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
        int fail = 0;
        for (unsigned it = 0;; ++it) {
            const int v = lane < NW ? __hip_atomic_load(a.ctr + base + lane * kPad, __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_AGENT)
                                    : expected;
            const int m = (int)(__ballot(v >= expected) & 0xFFFull);
            if (lane == 0) *rdy = m;
            if (m == 0xFFF) break;
            if ((it & 7) == 7) {
                const int e = __builtin_amdgcn_readfirstlane(
                    __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                if (e) {
                    fail = 1;
                    break;
                }
                if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > kSpinTicks) {
                    if (lane == 0) {
                        atomicCAS(a.err, 0, code);
                        if (a.err_sticky) atomicCAS(a.err_sticky, 0, code);
                    }
                    fail = 1;
                    break;
                }
            }
            __builtin_amdgcn_s_sleep(1);
        }
        if (fail && lane == 0) *rdy = 0x1FFF;
        return !fail;
    }
    int r;
    while (!(((r = *rdy) >> wv) & 1)) __builtin_amdgcn_s_sleep(1);
    return !(r >> 12);
}

// the wave's weight fragments of tiles j0 .. j0+T-1, k16 steps kb + 4w ..
// (NT: non-temporal, one row block reads every tile once; a compile-time
// choice, so the loads carry no branch between them)
template <int T, bool NT>
__device__ __forceinline__ void load_wt(const float* W, int K16W, int j0, int kb, int w, float4 (&wr)[T][SPW]) {
    const float4* wf = reinterpret_cast<const float4*>(W) + ((size_t)j0 * K16W + kb + w * SPW) * 64 + (threadIdx.x & 63);
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
        for (int s = 0; s < SPW; ++s) wr[t][s] = NT ? ld_nt(wf + ((size_t)t * K16W + s) * 64) : wf[((size_t)t * K16W + s) * 64];
}

// the wave's 4 A fragments (sc1: written in this launch or the previous
// one), the T tiles' accumulator chains (each in the one-shot order: steps in
// order, components x, y, z, w), and (STATS) the LN row partial sums
template <int T, bool STATS>
__device__ __forceinline__ void mfma_regs(const float4 (&xv)[SPW], const float4 (&wr)[T][SPW], f32x4 (&acc)[T],
                                          float& fs1, float& fs2);

// the wave's 4 A fragments (sc1: written in this launch or the previous one)
__device__ __forceinline__ void load_a4(const float* A, int K16A, int rb, int kb, int w, float4 (&xv)[SPW]) {
    const int off = ((rb * K16A + kb + w * SPW) * 64 + (int)(threadIdx.x & 63)) * 16;
#pragma unroll
    for (int s = 0; s < SPW; ++s) xv[s] = hpa::load_wt16(A, off + s * 1024);
}

template <int T, bool STATS>
__device__ __forceinline__ void mfma_t(const float* A, int K16A, int rb, int kb, int w, const float4 (&wr)[T][SPW],
                                       f32x4 (&acc)[T], float& fs1, float& fs2) {
    float4 xv[SPW];
    const int off = ((rb * K16A + kb + w * SPW) * 64 + (int)(threadIdx.x & 63)) * 16;
#pragma unroll
    for (int s = 0; s < SPW; ++s) xv[s] = hpa::load_wt16(A, off + s * 1024);
    // all four A loads in flight before the first MFMA: left alone the
    // scheduler interleaves them two at a time with the MFMAs (two dependent
    // round trips instead of one, seen in the gfx950 ISA of round 4)
    __builtin_amdgcn_sched_barrier(0);
    mfma_regs<T, STATS>(xv, wr, acc, fs1, fs2);
}

// the T tiles' accumulator chains over the wave's 4 A fragments (each in the
// one-shot order: steps in order, components x, y, z, w) and (STATS) the LN
// row partial sums
template <int T, bool STATS>
__device__ __forceinline__ void mfma_regs(const float4 (&xv)[SPW], const float4 (&wr)[T][SPW], f32x4 (&acc)[T],
                                          float& fs1, float& fs2) {
#pragma unroll
    for (int t = 0; t < T; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < SPW; ++s)
#pragma unroll
        for (int t = 0; t < T; ++t) {
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[s].x, wr[t][s].x, acc[t], 0, 0, 0);
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[s].y, wr[t][s].y, acc[t], 0, 0, 0);
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[s].z, wr[t][s].z, acc[t], 0, 0, 0);
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[s].w, wr[t][s].w, acc[t], 0, 0, 0);
        }
    if (STATS)
#pragma unroll
        for (int s = 0; s < SPW; ++s) hpa_gemm::row_sums_add(xv[s], fs1, fs2);
}

template <int T>
__device__ __forceinline__ void put_red_t(float* red, int w, const f32x4 (&acc)[T]) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
        for (int g = 0; g < 4; ++g) red[(w * T + t) * 256 + g * 64 + lane] = acc[t][g];
}

// epilogue thread tid < T*64: tile t = tid / 64, row r = (tid % 64) / 4,
// columns 4q .. 4q+3 (q = tid % 4) of that tile; its 4 values summed over the
// 12 waves in wave order (foldn<12>)
template <int T>
__device__ __forceinline__ float4 fold_t(const float* red, int t, int r, int q) {
    const float* p = red + t * 256 + (r & 3) * 64 + 16 * (r >> 2) + 4 * q;
    float4 v = *reinterpret_cast<const float4*>(p);
#pragma unroll
    for (int w = 1; w < NW; ++w) {
        const float4 x = *reinterpret_cast<const float4*>(p + w * T * 256);
        v.x += x.x;
        v.y += x.y;
        v.z += x.z;
        v.w += x.w;
    }
    return v;
}

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

// LN fold of 4 values of row r (ln_fold_val<12>, elementwise)
__device__ __forceinline__ float4 ln_fold4(const float* wsum, int r, float4 v, float4 c1, float4 c2) {
    v.x = ln_fold_val<NW>(wsum, 0, r, 64 * 12, v.x, c1.x, c2.x);
    v.y = ln_fold_val<NW>(wsum, 0, r, 64 * 12, v.y, c1.y, c2.y);
    v.z = ln_fold_val<NW>(wsum, 0, r, 64 * 12, v.z, c1.z, c2.z);
    v.w = ln_fold_val<NW>(wsum, 0, r, 64 * 12, v.w, c1.w, c2.w);
    return v;
}

// every storing wave drained.  The builtin form, not inline asm: the
// compiler must know vmcnt is 0 here, or it waits again before the first
// register it reuses after the stores -- and vmcnt is in order, so that wait
// also drained the next phase's weight prefetch issued in between (seen in
// the gfx950 ISA of round 4: the prefetch had to land before the wait began)
__device__ __forceinline__ void drain_vm() {
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) expcnt(7) lgkmcnt(15)
    asm volatile("" ::: "memory");
}

__device__ __forceinline__ void publish6(const KA& a, int ctr, bool did) {
    drain_vm();
    lds_barrier();
    if (threadIdx.x == 0 && did) arrive6(a, ctr, 1);
}

// the K / V destination of a qkv epilogue lane, resolved while the unit's
// weights stream and before its wait: the token's position, then its page
// (two dependent loads; issued behind the MFMAs they were the epilogue's
// tail).  qkv_pos6 goes before the weight loads (vmcnt retires in order),
// qkv_page6 after them.
__device__ __forceinline__ int qkv_pos6(const KA& a, bool ep, int row, int col) {
    return ep && row < a.B && col >= 768 ? a.pos[row] : 0;
}
template <int P>
__device__ __forceinline__ int qkv_page6(const KA& a, bool ep, int row, int col, int ps) {
    return ep && row < a.B && col >= 768 ? a.bt[(size_t)row * a.bt_stride + ps / P] : -1;
}

// qkv epilogue store of 4 columns col..col+3 of `row` (NH = 12): q row-major,
// or K / V of this token (position ps, page `page` from qkv_pos6 / qkv_page6)
// into the sequence's page of the layer at kv_next (add_to_cache,
// paged_infer.c:505-573)
template <int P, bool BF>
__device__ __forceinline__ void qkv_store6(const KA& a, int row, int col, int ps, int page, float4 v) {
    constexpr int NH = 12, C = 768;
    if (col < C) {
        *reinterpret_cast<float4*>(a.q_out + (size_t)row * C + col) = v;
        return;
    }
    const int kv = col >= 2 * C;
    const int c = col - (kv ? 2 * C : C);
    const int hh = c >> 6, d = c & 63;
    if (page < 0) return;
    const int pslot = ps % P;
    const size_t toff = (size_t)page * a.page_elems + ((size_t)kv * NH + hh) * P * 64;
    if constexpr (BF) {
        unsigned short* kvt = reinterpret_cast<unsigned short*>(a.kv_next) + toff +
                              (kv == 0 ? ((d >> 3) * P + pslot) * 8 + (d & 7) : pslot * 64 + d);
        const unsigned lo = hpa::f32_to_bf16(v.x) | ((unsigned)hpa::f32_to_bf16(v.y) << 16);
        const unsigned hi = hpa::f32_to_bf16(v.z) | ((unsigned)hpa::f32_to_bf16(v.w) << 16);
        *reinterpret_cast<uint2*>(kvt) = make_uint2(lo, hi);
    } else {
        float* kvt = reinterpret_cast<float*>(a.kv_next) + toff + (kv == 0 ? ((d >> 2) * P + pslot) * 4 : pslot * 64 + d);
        *reinterpret_cast<float4*>(kvt) = v;
    }
}

}  // namespace c6

// TC, TD, TE: tiles per unit of fc, fcproj, qkv (NH = 12; attproj 1)
template <int P, bool BF, int TC, int TD, int TE>
__global__ __launch_bounds__(768) void decode_chain6_kernel(KA args) {
    using namespace c6;
    constexpr int C = 768, K16 = 48, NCT = 48;
    const KA& a = *(const KA*)(const void*)__builtin_amdgcn_kernarg_segment_ptr();
    (void)args;
    __shared__ Smem6 sm;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int tid = threadIdx.x;
    const int bid = blockIdx.x;
    const int R = a.R;
    constexpr bool NT = TC == 1 && TD == 1 && TE == 1;  // the one-row-block instantiation: every tile read once
    // k-group waits (HPA_C6_GW): fc always; fcproj and qkv at <= 2 row blocks
    // (B <= 32: -1.5 % / -3.3 % per step at B = 32 / 8; at B = 64 they cost
    // what fc's gains, profiles/r4/kgroup_waits.txt)
    constexpr bool GDE = HPA_C6_GW && TC < 3;
    constexpr bool GD = GDE || (HPA_C6_GW != 0 && (HPA_C6_DE & 1) != 0);  // A/B builds: fcproj / qkv k-group waits
    constexpr bool GE = GDE || (HPA_C6_GW != 0 && (HPA_C6_DE & 2) != 0);  // at 3-4 row blocks too
    // epilogue thread's place: tile et, row er, column quad eq
    const int et = tid >> 6, er = (tid & 63) >> 2, eq = tid & 3;
    int* tick = a.ctr + kCtr;  // fcproj K-part tickets [R][NCT / TD]
    if (HPA_C6_GW && tid == 0) sm.s_ready = 0;  // read first in phase C, after phase B's barriers
    PL_STAMP(t_start);
    PL_STORE(0, t_start);
    float fs1 = 0.f, fs2 = 0.f;
    // every phase's unit of this workgroup (the geometry is fixed per launch)
    constexpr int NGB = NCT, NGC = 4 * NCT / TC, NGD = NCT / TD, NGE = 3 * NCT / TE;
    const bool hasB = bid < R * NGB, hasC = bid < R * NGC, hasD = bid < 4 * R * NGD, hasE = bid < R * NGE;
    const int gB = bid % NGB, rbB = bid / NGB;
    const int gC = bid % NGC, rbC = bid / NGC;
    const int gD = bid % NGD, rbD = (bid / NGD) % R, pD = (bid / NGD) / R;
    const int gE = bid % NGE, rbE = bid / NGE;
    // Early weight prefetch (HPA_C6_EARLY, round 6): a wave that stores
    // nothing in phase X (waves >= T_X: only waves 0..T_X-1 run X's epilogue)
    // issues phase X+1's weight fragments (and epilogue operands) right after
    // its MFMAs of phase X (behind their operand waits), so they stream during
    // X's MFMAs, epilogue and seam instead of being issued at the seam, where
    // the A gather after the
    // wait queued behind them in the CU's memory pipe (MI355X_MICROARCH.md
    // "gather-pass": 1.0-1.7 us queued vs 0.3-0.65 quiet).  Such a wave skips
    // the publish drain (it stored nothing; the drain would wait for its
    // prefetch).  The storing waves keep the round-5 order (drain, then the
    // next phase's operands).  Same loads, same arithmetic: same bits.
    constexpr bool EARLY = HPA_C6_EARLY != 0;
    // B: attproj(l), 1 tile per unit: res2 = res + att . Wap^T + b
    float4 c1C = make_float4(0.f, 0.f, 0.f, 0.f), c2C = c1C;
    float4 wrC[TC][SPW];
    {
        constexpr int T = 1;
        const bool has = hasB;
        const int g = gB, rb = rbB;
        float4 wr[T][SPW];
        if (has) load_wt<T, NT>(a.w_ap, K16, g * T, 0, w, wr);
        const bool ep = has && tid < T * 64;
        const int row = rb * 16 + er, col = (g * T + et) * 16 + 4 * eq;
        const int fx = (int)hpa::frag_index(row, col, C), fi = fx * 4;
        float4 bv = make_float4(0.f, 0.f, 0.f, 0.f), rv = bv;
        if (ep) {
            bv = ld4(a.b_ap + col);
            rv = hpa::load_wt16(a.res, fi);
        }
        PL_MARK(4);
        const bool early = EARLY && w >= T;  // a wave with no store in this phase
        const bool epC = hasC && tid < TC * 64;
        const int colC = (gC * TC + et) * 16 + 4 * eq;
        float4 xv[SPW];
        if (has) load_a4(a.att, K16, rb, 0, w, xv);
        __builtin_amdgcn_sched_barrier(0);
        if (has) {
            f32x4 acc[T];
            mfma_regs<T, false>(xv, wr, acc, fs1, fs2);
            put_red_t<T>(sm.red, w, acc);
        }
        if (early) {  // behind the MFMAs' operand waits (issued here they cannot delay them)
            if (epC) {
                c1C = ld4(a.fc_c1 + colC);
                c2C = ld4(a.fc_c2 + colC);
            }
            if (hasC) load_wt<TC, NT>(a.w_fc, K16, gC * TC, 0, w, wrC);
        }
        lds_barrier();
        if (ep) {
            float4 v = fold_t<T>(sm.red, et, er, eq);
            v.x += bv.x; v.y += bv.y; v.z += bv.z; v.w += bv.w;
            const bool live = row < a.B;  // residual_forward(out, res, proj); padded rows stay 0
            v = live ? make_float4(rv.x + v.x, rv.y + v.y, rv.z + v.z, rv.w + v.w) : make_float4(0.f, 0.f, 0.f, 0.f);
            hpa::store_wt16(a.res2, fi, v);
        }
        PL_MARK(12);
        if (!early) drain_vm();  // the storing waves
        lds_barrier();
        if (HPA_C6_GW) {  // the tile's k-group of fc's A
            if (tid == 0 && has) arrive_tiles(a, kCtr + 4 * NCT + kGC, rb, NW, g, 1);
        } else {
            if (tid == 0 && has) arrive6(a, X1 + rb, 1);
        }
        if (!early) {  // the round-5 order: epilogue operands, then the weights
            if (epC) {
                c1C = ld4(a.fc_c1 + colC);
                c2C = ld4(a.fc_c2 + colC);
            }
            if (hasC) load_wt<TC, NT>(a.w_fc, K16, gC * TC, 0, w, wrC);
        }
    }
    PL_MARK(5);
    // C: fc(l): fch = gelu(LN2(res2) . Wfc^T + b), LN folded; T = TC tiles
    float4 bvD = make_float4(0.f, 0.f, 0.f, 0.f);
    float4 wrD[TD][SPW];
    {
        constexpr int T = TC;
        const bool has = hasC;
        const int g = gC, rb = rbC;
        const bool ep = has && tid < T * 64;
        const int row = rb * 16 + er, col = (g * T + et) * 16 + 4 * eq;
        if (HPA_C6_GW) {
            if (has && !wait_grp(a, kCtr + 4 * NCT + kGC + rb * NW * kPad, 4, 2, sm)) return;
        } else if (!wait6(a, X1 + (has ? rb : 0), has ? NCT : 0, 2, sm)) {
            return;
        }
        PL_MARK(6);
        const bool early = EARLY && w >= T;
        const bool epD = hasD && tid < TD * 64;
        const int colD = (gD * TD + et) * 16 + 4 * eq;
        fs1 = fs2 = 0.f;
        float4 xv[SPW];
        if (has) load_a4(a.res2, K16, rb, 0, w, xv);
        __builtin_amdgcn_sched_barrier(0);
        if (has) {
            f32x4 acc[T];
            mfma_regs<T, true>(xv, wrC, acc, fs1, fs2);
            put_red_t<T>(sm.red, w, acc);
        }
        hpa_gemm::row_sums_publish(fs1, fs2, sm.wsum + w * 32);
        if (early) {
            if (epD) bvD = ld4(a.b_fp + colD);
            if (hasD) load_wt<TD, NT>(a.w_fp, 4 * K16, gD * TD, pD * K16, w, wrD);
        }
        lds_barrier();
        if (GD && tid == 0) sm.s_ready = 0;  // every wave is past fc's wait; read again in fcproj's
        if (ep) {
            float4 v = ln_fold4(sm.wsum, er, fold_t<T>(sm.red, et, er, eq), c1C, c2C);
            const bool live = row < a.B;
            v = live ? make_float4(hpa::gelu_ref(v.x), hpa::gelu_ref(v.y), hpa::gelu_ref(v.z), hpa::gelu_ref(v.w))
                     : make_float4(0.f, 0.f, 0.f, 0.f);
            hpa::store_wt16(a.fch, (int)(hpa::frag_index(row, col, 4 * C) * 4), v);
        }
        PL_MARK(13);
        if (!early) drain_vm();
        lds_barrier();
        if (GD) {  // the tiles' k-groups of fcproj's A (48 per row block)
            if (tid == 0 && has) arrive_tiles(a, kCtr + 4 * NCT + kGD, rb, 4 * NW, g * T, T);
        } else {
            if (tid == 0 && has) arrive6(a, H + rb * 4 + (g * T) / NCT, 1);  // the K part of fcproj these columns feed
        }
        if (!early) {
            if (epD) bvD = ld4(a.b_fp + colD);
            if (hasD) load_wt<TD, NT>(a.w_fp, 4 * K16, gD * TD, pD * K16, w, wrD);
        }
        PL_MARK(7);
    }
    // D: fcproj(l), K part p of 4, T = TD tiles: partial tiles -> slab; the
    // last part of (row block, tile group) adds the parts in order + bias + res2
    float4 wrE[TE][SPW];
    const bool epE = hasE && tid < TE * 64;
    const int rowE = rbE * 16 + er, colE = (gE * TE + et) * 16 + 4 * eq;
    int kps = 0;  // qkv(l+1)'s K/V destination: the row's position (c6::qkv_pos6)
    {
        constexpr int T = TD, NG = NGD;
        const bool has = hasD;
        const int g = gD, rb = rbD, p = pD;
        const bool ep = has && tid < T * 64;
        const int row = rb * 16 + er, col = (g * T + et) * 16 + 4 * eq;
        if (GD) {
            if (has && !wait_grp(a, kCtr + 4 * NCT + kGD + (rb * 4 * NW + p * NW) * kPad, 4, 3, sm)) return;
        } else if (!wait6(a, H + (has ? rb * 4 + p : 0), has ? 4 * NCT / TC / 4 : 0, 3, sm)) {
            return;
        }
        PL_MARK(8);
        const bool early = EARLY && w >= T && !a.last;  // qkv(l+1)'s weights (the storing waves: after the combine)
        float4 xv[SPW];
        if (has) load_a4(a.fch, 4 * K16, rb, p * K16, w, xv);
        __builtin_amdgcn_sched_barrier(0);
        if (has) {
            f32x4 acc[T];
            mfma_regs<T, false>(xv, wrD, acc, fs1, fs2);
            put_red_t<T>(sm.red, w, acc);
        }
        if (early && hasE) load_wt<TE, NT>(a.w_qkv, K16, gE * TE, 0, w, wrE);
        lds_barrier();
        if ((GD || GE) && tid == 0) sm.s_ready = 0;  // every wave is past fcproj's wait; read again in qkv's
        float4 val = make_float4(0.f, 0.f, 0.f, 0.f);
        const int sx = (((p * R + rb) * NG + g) * T * 64 + tid) * 4;  // this part's float4 in the slab (float index)
        if (ep) {
            val = fold_t<T>(sm.red, et, er, eq);
            hpa::store_wt16(a.slab_fp, sx * 4, val);
        }
        PL_MARK(14);
        if (!early) c6::drain_vm();
        lds_barrier();
        if (has && tid == 0) {
            const int tk = __hip_atomic_fetch_add(tick + rb * NG + g, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            sm.s_last = tk == 3;
        }
        lds_barrier();
        const bool last = has && sm.s_last != 0;
        if (last && ep) {
            float4 pv[4];
            const int fx = (int)hpa::frag_index(row, col, C), fi = fx * 4;
#pragma unroll
            for (int qq = 0; qq < 4; ++qq)
                pv[qq] = qq == p ? val : hpa::load_wt16(a.slab_fp, ((((qq * R + rb) * NG + g) * T * 64 + tid) * 4) * 4);
            const float4 rv = hpa::load_wt16(a.res2, fi);
            float4 tot = pv[0];
#pragma unroll
            for (int qq = 1; qq < 4; ++qq) {
                tot.x += pv[qq].x; tot.y += pv[qq].y; tot.z += pv[qq].z; tot.w += pv[qq].w;
            }
            tot.x += bvD.x; tot.y += bvD.y; tot.z += bvD.z; tot.w += bvD.w;
            const bool live = row < a.B;
            tot = live ? make_float4(rv.x + tot.x, rv.y + tot.y, rv.z + tot.z, rv.w + tot.w)
                       : make_float4(0.f, 0.f, 0.f, 0.f);
            hpa::store_wt16(a.res, fi, tot);
            if (a.stats_out) {
                float* tr = sm.tile + (et * 16 + er) * 17 + 4 * eq;
                tr[0] = tot.x; tr[1] = tot.y; tr[2] = tot.z; tr[3] = tot.w;
            }
        }
        if (!early) c6::drain_vm();
        lds_barrier();
        if (a.stats_out && last && tid < T * 16) {  // 16-column LNf partial sums of the tiles' rows
            const int t = tid >> 4, r = tid & 15;
            const float* tr = sm.tile + (t * 16 + r) * 17;
            float s1 = 0.f, s2 = 0.f;
#pragma unroll
            for (int c = 0; c < 16; ++c) {
                s1 += tr[c];
                s2 += tr[c] * tr[c];
            }
            const int j = g * T + t, rr = rb * 16 + r;
            a.stats_out[((size_t)j * a.Mp + rr) * 2] = s1;
            a.stats_out[((size_t)j * a.Mp + rr) * 2 + 1] = s2;
        }
        if (tid == 0 && last) {
            if (GE)
                arrive_tiles(a, kCtr + 4 * NCT + kGE, rb, NW, g * T, T);  // the tiles' k-groups of qkv's A
            else
                arrive6(a, X2 + rb, 1);
        }
        PL_MARK(9);
        if (!a.last) {  // the position before the weights (vmcnt retires in order; the page load needs it)
            kps = qkv_pos6(a, epE, rowE, colE);
            if (!early && hasE) load_wt<TE, NT>(a.w_qkv, K16, gE * TE, 0, w, wrE);
        }
    }
    // E: qkv(l+1), T = TE tiles: LN1 folded, q + K/V appended into layer l+1's pages
    if (!a.last) {
        constexpr int T = TE;
        const bool has = hasE;
        const int rb = rbE;
        const bool ep = epE;
        const int row = rowE, col = colE;
        // the epilogue waves' operands (waves 0..TE-1 store in D too: issued
        // after D's drain, as in round 5): the position (above, ahead of the
        // weights), the LN-fold operands, then the page
        float4 c1 = make_float4(0.f, 0.f, 0.f, 0.f), c2 = c1;
        if (ep) {
            c1 = ld4(a.qkv_c1 + col);
            c2 = ld4(a.qkv_c2 + col);
        }
        const int kpage = qkv_page6<P>(a, ep, row, col, kps);
        if (GE) {
            if (has && !wait_grp(a, kCtr + 4 * NCT + kGE + rb * NW * kPad, 4, 4, sm)) return;
        } else if (!wait6(a, X2 + (has ? rb : 0), has ? NCT / TD : 0, 4, sm)) {
            return;
        }
        PL_MARK(10);
        fs1 = fs2 = 0.f;
        if (has) {
            f32x4 acc[T];
            mfma_t<T, true>(a.res, K16, rb, 0, w, wrE, acc, fs1, fs2);
            put_red_t<T>(sm.red, w, acc);
        }
        hpa_gemm::row_sums_publish(fs1, fs2, sm.wsum + w * 32);
        lds_barrier();
        PL_MARK(15);
        if (ep && row < a.B)
            qkv_store6<P, BF>(a, row, col, kps, kpage, ln_fold4(sm.wsum, er, fold_t<T>(sm.red, et, er, eq), c1, c2));
    }
    PL_MARK(11);
}


// ------------------------------------------------------------------ the step's first launch (form 6)
// embed (encoder_forward, paged_infer.c:41-47: wte[token] + wpe[pos] at the
// absolute position) and layer 0's qkv in ONE launch, which also zeroes the
// step's counter block and error word: was the embed kernel + the one-shot
// qkv GEMM (two launches and a boundary, 4.3 + 9.4 us at B = 64).  The qkv is
// chain form 6's phase E -- (row block, TE tiles) units, LN1 folded, q + K/V
// of the token into layer 0's pages -- with each wave's A fragments built in
// registers from the embedding instead of loaded; the tile group 0 unit of a
// row block also stores the residual stream it built (frag layout, read by
// layer 0's chain launch).  Rows >= B embed as 0 (padded rows stay 0).
template <int P, bool BF, int TE>
__global__ __launch_bounds__(768) void decode_first6_kernel(KA args) {
    using namespace c6;
    constexpr int C = 768, K16 = 48, NCT = 48;
    const KA& a = *(const KA*)(const void*)__builtin_amdgcn_kernarg_segment_ptr();
    (void)args;
    __shared__ Smem6 sm;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int tid = threadIdx.x, lane = tid & 63;
    const int bid = blockIdx.x;
    constexpr int T = TE, NG = 3 * NCT / TE;
    constexpr bool NT = TE == 1;
    const int g = bid % NG, rb = bid / NG;
    // the row's token and position first: the embedding loads depend on them,
    // and vmcnt retires in order, so behind the weight loads they would wait
    // for those too
    const int arow = rb * 16 + (lane & 15);
    const bool live = rb < a.R && arow < a.B;
    const int tok = live ? a.tokens[arow] : 0, ps = live ? a.pos[arow] : 0;
    for (int i = bid * 768 + tid; i < a.zero_n4; i += (int)gridDim.x * 768) a.zero[i] = make_int4(0, 0, 0, 0);
    if (rb >= a.R) return;  // no unit (the grid holds R * NG <= G of them; nothing here waits)
    const int et = tid >> 6, er = (tid & 63) >> 2, eq = tid & 3;
    const bool ep = tid < T * 64;
    const int row = rb * 16 + er, col = (g * T + et) * 16 + 4 * eq;
    const int kps = qkv_pos6(a, ep, row, col);
    float4 c1 = make_float4(0.f, 0.f, 0.f, 0.f), c2 = c1;
    if (ep) {
        c1 = ld4(a.qkv_c1 + col);
        c2 = ld4(a.qkv_c2 + col);
    }
    float4 wr[T][SPW];
    load_wt<T, NT>(a.w_qkv, K16, g * T, 0, w, wr);
    const int kpage = qkv_page6<P>(a, ep, row, col, kps);
    // A fragment of k16 step 4w + s: lane holds row 16 rb + (lane & 15),
    // columns 16 (4w + s) + 4 (lane >> 4) .. + 3 (hpa::frag_index)
    const float4* te = reinterpret_cast<const float4*>(a.wte + (size_t)tok * C) + (lane >> 4);
    const float4* pe = reinterpret_cast<const float4*>(a.wpe + (size_t)ps * C) + (lane >> 4);
    float4 xv[SPW];
#pragma unroll
    for (int s = 0; s < SPW; ++s) {
        const float4 x = te[(w * SPW + s) * 4], y = pe[(w * SPW + s) * 4];
        xv[s] = live ? make_float4(x.x + y.x, x.y + y.y, x.z + y.z, x.w + y.w) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if (g == 0)
#pragma unroll
        for (int s = 0; s < SPW; ++s)
            *reinterpret_cast<float4*>(a.res + ((size_t)(rb * K16 + w * SPW + s) * 64 + lane) * 4) = xv[s];
    float fs1 = 0.f, fs2 = 0.f;
    f32x4 acc[T];
    mfma_regs<T, true>(xv, wr, acc, fs1, fs2);
    put_red_t<T>(sm.red, w, acc);
    hpa_gemm::row_sums_publish(fs1, fs2, sm.wsum + w * 32);
    lds_barrier();
    if (ep && row < a.B)
        qkv_store6<P, BF>(a, row, col, kps, kpage, ln_fold4(sm.wsum, er, fold_t<T>(sm.red, et, er, eq), c1, c2));
}

// ------------------------------------------------------------------ the chain for wide layers (form 8)
// GPT-2 XL (C = 1600, NH = 25): the same persistent
// chain attproj -> fc -> fcproj -> qkv(l+1) as form 6, sized for GEMMs that
// are MFMA-bound (3.9 GFLOP per layer at B = 64, 25 us at the fp32 rate):
//   * one unit of all 12 waves per workgroup = (row block, up to XT_MAX
//     16-column tiles[, fcproj K part]), T per phase chosen on the host so
//     the units fill the CUs (B = 64: attproj 2, fc 7, fcproj 7, qkv 5 tiles);
//     tile groups are padded to a multiple of 8 so the row blocks of a weight
//     tile land on one XCD and re-read it from that L2;
//   * a wave holds its K range of the A rows (K16 / 12 steps, 8 or 9 at XL)
//     once per phase and streams its weight fragments tile by tile, double
//     buffered: the phase's first tile is loaded before its wait;
//   * every tile's accumulators stay in registers until one LDS fold of all
//     T tiles; epilogues are 16-byte as in form 6;
//   * waits per row block; fcproj's 4 K parts (of C each) are combined by the
//     last part to draw its ticket, in part order.
// A wave's K range depends only on K, so a row's sums never depend on B.
#ifndef HPA_CX_SB
#define HPA_CX_SB 1  // A/B builds: 0 = no scheduling barrier after form 8's A loads
#endif
namespace cx {
constexpr int NW = 12;
constexpr int XT_MAX = 7;

template <int MAXS>
__device__ __forceinline__ void ld_tile(const float* W, int K16W, int j, int kb, int s0, int ns, bool nt,
                                        float4 (&wr)[MAXS]) {
    const float4* wf = reinterpret_cast<const float4*>(W) + ((size_t)j * K16W + kb + s0) * 64 + (threadIdx.x & 63);
#pragma unroll
    for (int s = 0; s < MAXS; ++s)
        if (s < ns) wr[s] = nt ? ld_nt(wf + (size_t)s * 64) : wf[(size_t)s * 64];
}

template <int MAXS>
__device__ __forceinline__ f32x4 chain_tile(const float4 (&xv)[MAXS], const float4 (&wr)[MAXS], int ns) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < MAXS; ++s)
        if (s < ns) {
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[s].x, wr[s].x, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[s].y, wr[s].y, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[s].z, wr[s].z, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[s].w, wr[s].w, acc, 0, 0, 0);
        }
    return acc;
}

struct SmemX {
    float red[NW * XT_MAX * 256];
    float wsum[NW * 32];
    float tile[XT_MAX * 16 * 17];
    int s_ok;
    int s_last;
};

// the unit body up to the LDS fold: A (its K range of row block rb, sc1),
// row sums (STATS), then the nt tiles j0.. streamed in half-tiles (HS k16
// steps of the wave's range) through four register sets rotating by name,
// three half-tiles ahead (wr01 holds tile 0, loaded before the caller's
// wait); accumulators -> red[w][t].  One whole tile ahead left the XL fc
// phase at 19 us for 11.7 us of MFMA issue (profiles/r4/traces): a tile's
// 100 KB per CU did not land within one tile's MFMAs; two whole tiles ahead
// need 168 VGPRs + spills.
template <int MAXS>
struct HalfT {
    static constexpr int HS = (MAXS + 1) / 2;
};

template <int MAXS>
__device__ __forceinline__ void ld_half(const float* W, int K16W, int j, int kb, int s0, int ns, int h, bool nt,
                                        float4 (&wr)[HalfT<MAXS>::HS]) {
    constexpr int HS = HalfT<MAXS>::HS;
    const float4* wf = reinterpret_cast<const float4*>(W) + ((size_t)j * K16W + kb + s0 + h * HS) * 64 + (threadIdx.x & 63);
#pragma unroll
    for (int s = 0; s < HS; ++s)
        if (h * HS + s < ns) wr[s] = nt ? ld_nt(wf + (size_t)s * 64) : wf[(size_t)s * 64];
}

template <int MAXS>
__device__ __forceinline__ void chain_half(const float4 (&xv)[MAXS], const float4 (&wr)[HalfT<MAXS>::HS], int ns, int h,
                                           f32x4& acc) {
    constexpr int HS = HalfT<MAXS>::HS;
#pragma unroll
    for (int s = 0; s < HS; ++s)
        if (h * HS + s < ns) {
            const float4 x = xv[h * HS + s];
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x.x, wr[s].x, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x.y, wr[s].y, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x.z, wr[s].z, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x.w, wr[s].w, acc, 0, 0, 0);
        }
}

template <int MAXS>
struct Tile0 {  // tile 0's two halves, loaded before the caller's wait
    float4 h0[HalfT<MAXS>::HS], h1[HalfT<MAXS>::HS];
};

template <int MAXS>
__device__ __forceinline__ void ld_tile0(const float* W, int K16W, int j, int kb, int s0, int ns, bool nt, Tile0<MAXS>& t0) {
    ld_half<MAXS>(W, K16W, j, kb, s0, ns, 0, nt, t0.h0);
    ld_half<MAXS>(W, K16W, j, kb, s0, ns, 1, nt, t0.h1);
}

template <int MAXS, bool STATS>
__device__ __forceinline__ void unit_body(const float* A, int K16A, const float* W, int K16W, int rb, int kb, int j0,
                                          int ntl, int s0, int ns, bool nt, Tile0<MAXS>& t0, float* red,
                                          float& fs1, float& fs2, bool wtrace = false) {
    (void)wtrace;
    constexpr int HS = HalfT<MAXS>::HS;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    float4 xv[MAXS];
    const int off = ((rb * K16A + kb + s0) * 64 + lane) * 16;
#pragma unroll
    for (int s = 0; s < MAXS; ++s)
        if (s < ns) xv[s] = hpa::load_wt16(A, off + s * 1024);
#if HPA_CX_SB
    __builtin_amdgcn_sched_barrier(0);  // every A load in flight before the first MFMA (see mfma_t)
#endif
    CX_WSTAMP(wtrace, 0);
    if (STATS)
#pragma unroll
        for (int s = 0; s < MAXS; ++s)
            if (s < ns) hpa_gemm::row_sums_add(xv[s], fs1, fs2);
    // half-tile q = 2t + h in set q % 4: sets 0, 1 = tile 0 (t0), 2, 3 here
    float4 w2[HS], w3[HS];
    if (ntl > 1) {
        ld_half<MAXS>(W, K16W, j0 + 1, kb, s0, ns, 0, nt, w2);
        ld_half<MAXS>(W, K16W, j0 + 1, kb, s0, ns, 1, nt, w3);
    }
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < 2 * XT_MAX; ++q) {
        const int t = q >> 1, h = q & 1;
        if (t >= ntl) break;
        // half-tile q + 3 into the set half-tile q - 1 used (q % 4 == 0: set 3 is tile 1's half 1, still live)
        const int qn = q + 3;
        if (q >= 1 && (qn >> 1) < ntl) {
            if (qn % 4 == 0)
                ld_half<MAXS>(W, K16W, j0 + (qn >> 1), kb, s0, ns, qn & 1, nt, t0.h0);
            else if (qn % 4 == 1)
                ld_half<MAXS>(W, K16W, j0 + (qn >> 1), kb, s0, ns, qn & 1, nt, t0.h1);
            else if (qn % 4 == 2)
                ld_half<MAXS>(W, K16W, j0 + (qn >> 1), kb, s0, ns, qn & 1, nt, w2);
            else
                ld_half<MAXS>(W, K16W, j0 + (qn >> 1), kb, s0, ns, qn & 1, nt, w3);
        }
        if (q % 4 == 0)
            chain_half<MAXS>(xv, t0.h0, ns, h, acc);
        else if (q % 4 == 1)
            chain_half<MAXS>(xv, t0.h1, ns, h, acc);
        else if (q % 4 == 2)
            chain_half<MAXS>(xv, w2, ns, h, acc);
        else
            chain_half<MAXS>(xv, w3, ns, h, acc);
        CX_WSTAMP(wtrace, 1 + q);
        if (h == 1) {
#pragma unroll
            for (int g = 0; g < 4; ++g) red[(w * XT_MAX + t) * 256 + g * 64 + lane] = acc[g];
            acc = f32x4{0.f, 0.f, 0.f, 0.f};
        }
    }
    CX_WSTAMP(wtrace, 15);
}

// epilogue element of thread tid: tile et = tid / 64 of the unit, row er,
// columns 4 eq .. +3; summed over the 12 waves in wave order
__device__ __forceinline__ float4 fold_x(const float* red, int t, int r, int q) {
    const float* p = red + t * 256 + (r & 3) * 64 + 16 * (r >> 2) + 4 * q;
    float4 v = *reinterpret_cast<const float4*>(p);
#pragma unroll
    for (int w = 1; w < NW; ++w) {
        const float4 x = *reinterpret_cast<const float4*>(p + w * XT_MAX * 256);
        v.x += x.x; v.y += x.y; v.z += x.z; v.w += x.w;
    }
    return v;
}

__device__ __forceinline__ float4 ln_fold4x(const float* wsum, int r, int K, float4 v, float4 c1, float4 c2) {
    v.x = ln_fold_val<NW>(wsum, 0, r, K, v.x, c1.x, c2.x);
    v.y = ln_fold_val<NW>(wsum, 0, r, K, v.y, c1.y, c2.y);
    v.z = ln_fold_val<NW>(wsum, 0, r, K, v.z, c1.z, c2.z);
    v.w = ln_fold_val<NW>(wsum, 0, r, K, v.w, c1.w, c2.w);
    return v;
}

__device__ __forceinline__ bool waitx(const KA& a, int ctr, int expected, int code, SmemX& sm) {
    return c6::wait6<SmemX>(a, ctr, expected, code, sm);
}
}  // namespace cx

template <int NH, int P, bool BF>
__global__ __launch_bounds__(768) void decode_chainx_kernel(KA args) {
    using namespace cx;
    constexpr int C = 64 * NH, K16 = C / 16, NCT = C / 16;
    constexpr int MAXS = (K16 + NW - 1) / NW;
    const KA& a = *(const KA*)(const void*)__builtin_amdgcn_kernarg_segment_ptr();
    (void)args;
    __shared__ SmemX sm;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int tid = threadIdx.x;
    const int bid = blockIdx.x;
    const int R = a.R;
    const bool nt = R == 1;
    const int s0 = w * K16 / NW, ns = (w + 1) * K16 / NW - s0;  // this wave's k16 steps of a K = C range
    const int et = tid >> 6, er = (tid & 63) >> 2, eq = tid & 3;
    int* tick = a.ctr + c6::kCtr;
    PL_STAMP(t_start);
    PL_STORE(0, t_start);
    float fs1 = 0.f, fs2 = 0.f;
    cx::Tile0<MAXS> t0w;
    // B: attproj(l): res2 = res + att . Wap^T + b
    {
        const int T = a.xt[0], NG = a.xng[0];
        const int g = bid % NG, rb = bid / NG, j0 = g * T;
        const bool has = rb < R && j0 < NCT;
        const int ntl = has ? min(T, NCT - j0) : 0;
        if (has) cx::ld_tile0<MAXS>(a.w_ap, K16, j0, 0, s0, ns, nt, t0w);
        const bool ep = tid < ntl * 64;
        const int row = rb * 16 + er, col = (j0 + et) * 16 + 4 * eq;
        const int fi = ep ? (int)(hpa::frag_index(row, col, C) * 4) : 0;
        float4 bv = make_float4(0.f, 0.f, 0.f, 0.f), rv = bv;
        if (ep) {
            bv = c6::ld4(a.b_ap + col);
            rv = hpa::load_wt16(a.res, fi);
        }
        if (has) unit_body<MAXS, false>(a.att, K16, a.w_ap, K16, rb, 0, j0, ntl, s0, ns, nt, t0w, sm.red, fs1, fs2);
        lds_barrier();
        if (ep) {
            float4 v = fold_x(sm.red, et, er, eq);
            v.x += bv.x; v.y += bv.y; v.z += bv.z; v.w += bv.w;
            v = row < a.B ? make_float4(rv.x + v.x, rv.y + v.y, rv.z + v.z, rv.w + v.w) : make_float4(0.f, 0.f, 0.f, 0.f);
            hpa::store_wt16(a.res2, fi, v);
        }
        c6::publish6(a, c6::X1 + rb, has);
    }
    PL_MARK(5);
    // C: fc(l): fch = gelu(LN2(res2) . Wfc^T + b), LN folded
    {
        constexpr int NJ = 4 * NCT;
        const int T = a.xt[1], NG = a.xng[1];
        const int g = bid % NG, rb = bid / NG, j0 = g * T;
        const bool has = rb < R && j0 < NJ;
        const int ntl = has ? min(T, NJ - j0) : 0;
        if (has) cx::ld_tile0<MAXS>(a.w_fc, K16, j0, 0, s0, ns, nt, t0w);
        const bool ep = tid < ntl * 64;
        const int row = rb * 16 + er, col = (j0 + et) * 16 + 4 * eq;
        float4 c1 = make_float4(0.f, 0.f, 0.f, 0.f), c2 = c1;
        if (ep) {
            c1 = c6::ld4(a.fc_c1 + col);
            c2 = c6::ld4(a.fc_c2 + col);
        }
        const int n_b = (NCT + a.xt[0] - 1) / a.xt[0];  // attproj units of a row block
        if (!waitx(a, c6::X1 + (has ? rb : 0), has ? n_b : 0, 2, sm)) return;
        PL_MARK(6);
        fs1 = fs2 = 0.f;
        if (has) unit_body<MAXS, true>(a.res2, K16, a.w_fc, K16, rb, 0, j0, ntl, s0, ns, nt, t0w, sm.red, fs1, fs2,
                                       a.layer == 5);
        hpa_gemm::row_sums_publish(fs1, fs2, sm.wsum + w * 32);
        lds_barrier();
        if (ep) {
            float4 v = ln_fold4x(sm.wsum, er, C, fold_x(sm.red, et, er, eq), c1, c2);
            v = row < a.B ? make_float4(hpa::gelu_ref(v.x), hpa::gelu_ref(v.y), hpa::gelu_ref(v.z), hpa::gelu_ref(v.w))
                          : make_float4(0.f, 0.f, 0.f, 0.f);
            hpa::store_wt16(a.fch, (int)(hpa::frag_index(row, col, 4 * C) * 4), v);
        }
        c6::publish6(a, c6::H + rb * 4, has);
        PL_MARK(7);
    }
    // D: fcproj(l), K part p of 4 (C each): partials -> slab; the last part of
    // (row block, tile group) adds the parts in order + bias + res2 -> res
    {
        const int T = a.xt[2], NG = a.xng[2];
        const int g = bid % NG, q1 = bid / NG, rb = q1 % R, p = q1 / R, j0 = g * T;
        const bool has = p < 4 && j0 < NCT;
        const int ntl = has ? min(T, NCT - j0) : 0;
        if (has) cx::ld_tile0<MAXS>(a.w_fp, 4 * K16, j0, p * K16, s0, ns, nt, t0w);
        const bool ep = tid < ntl * 64;
        const int row = rb * 16 + er, col = (j0 + et) * 16 + 4 * eq;
        float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
        if (ep) bv = c6::ld4(a.b_fp + col);
        const int n_c = (4 * NCT + a.xt[1] - 1) / a.xt[1];  // fc units of a row block
        if (!waitx(a, c6::H + (has ? rb * 4 : 0), has ? n_c : 0, 3, sm)) return;
        PL_MARK(8);
        if (has) unit_body<MAXS, false>(a.fch, 4 * K16, a.w_fp, 4 * K16, rb, p * K16, j0, ntl, s0, ns, nt, t0w, sm.red, fs1, fs2);
        lds_barrier();
        float4 val = make_float4(0.f, 0.f, 0.f, 0.f);
        auto slab_at = [&](int pp) { return (((pp * R + rb) * NCT + j0 + et) * 256 + (tid & 63) * 4) * 4; };
        if (ep) {
            val = fold_x(sm.red, et, er, eq);
            hpa::store_wt16(a.slab_fp, slab_at(p), val);
        }
        c6::drain_vm();
        lds_barrier();
        if (has && tid == 0) {
            const int tk = __hip_atomic_fetch_add(tick + rb * NG + g, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            sm.s_last = tk == 3;
        }
        lds_barrier();
        const bool last = has && sm.s_last != 0;
        if (last && ep) {
            float4 pv[4];
#pragma unroll
            for (int qq = 0; qq < 4; ++qq) pv[qq] = qq == p ? val : hpa::load_wt16(a.slab_fp, slab_at(qq));
            const int fi = (int)(hpa::frag_index(row, col, C) * 4);
            const float4 rv = hpa::load_wt16(a.res2, fi);
            float4 tot = pv[0];
#pragma unroll
            for (int qq = 1; qq < 4; ++qq) {
                tot.x += pv[qq].x; tot.y += pv[qq].y; tot.z += pv[qq].z; tot.w += pv[qq].w;
            }
            tot.x += bv.x; tot.y += bv.y; tot.z += bv.z; tot.w += bv.w;
            tot = row < a.B ? make_float4(rv.x + tot.x, rv.y + tot.y, rv.z + tot.z, rv.w + tot.w)
                            : make_float4(0.f, 0.f, 0.f, 0.f);
            hpa::store_wt16(a.res, fi, tot);
            if (a.stats_out) {
                float* tr = sm.tile + (et * 16 + er) * 17 + 4 * eq;
                tr[0] = tot.x; tr[1] = tot.y; tr[2] = tot.z; tr[3] = tot.w;
            }
        }
        c6::drain_vm();
        lds_barrier();
        if (a.stats_out && last && tid < ntl * 16) {  // 16-column LNf partial sums of the tiles' rows
            const int t = tid >> 4, r = tid & 15;
            const float* tr = sm.tile + (t * 16 + r) * 17;
            float s1 = 0.f, s2 = 0.f;
#pragma unroll
            for (int c = 0; c < 16; ++c) {
                s1 += tr[c];
                s2 += tr[c] * tr[c];
            }
            const int j = j0 + t, rr = rb * 16 + r;
            a.stats_out[((size_t)j * a.Mp + rr) * 2] = s1;
            a.stats_out[((size_t)j * a.Mp + rr) * 2 + 1] = s2;
        }
        if (tid == 0 && last) c6::arrive6(a, c6::X2 + rb, 1);
        PL_MARK(9);
    }
    // E: qkv(l+1): LN1 folded, q + K/V appended into layer l+1's pages
    if (!a.last) {
        constexpr int NJ = 3 * NCT;
        const int T = a.xt[3], NG = a.xng[3];
        const int g = bid % NG, rb = bid / NG, j0 = g * T;
        const bool has = rb < R && j0 < NJ;
        const int ntl = has ? min(T, NJ - j0) : 0;
        const bool ep = tid < ntl * 64;
        const int row = rb * 16 + er, col = (j0 + et) * 16 + 4 * eq;
        // the K/V destination while the weights stream (as c6::qkv_pos6 / qkv_page6)
        const int kps = ep && row < a.B && col >= C ? a.pos[row] : 0;
        if (has) cx::ld_tile0<MAXS>(a.w_qkv, K16, j0, 0, s0, ns, nt, t0w);
        float4 c1 = make_float4(0.f, 0.f, 0.f, 0.f), c2 = c1;
        if (ep) {
            c1 = c6::ld4(a.qkv_c1 + col);
            c2 = c6::ld4(a.qkv_c2 + col);
        }
        const int kpage = ep && row < a.B && col >= C ? a.bt[(size_t)row * a.bt_stride + kps / P] : -1;
        const int n_d = (NCT + a.xt[2] - 1) / a.xt[2];  // fcproj tile groups of a row block
        if (!waitx(a, c6::X2 + (has ? rb : 0), has ? n_d : 0, 4, sm)) return;
        PL_MARK(10);
        fs1 = fs2 = 0.f;
        if (has) unit_body<MAXS, true>(a.res, K16, a.w_qkv, K16, rb, 0, j0, ntl, s0, ns, nt, t0w, sm.red, fs1, fs2);
        hpa_gemm::row_sums_publish(fs1, fs2, sm.wsum + w * 32);
        lds_barrier();
        if (ep && row < a.B) {
            const float4 v = ln_fold4x(sm.wsum, er, C, fold_x(sm.red, et, er, eq), c1, c2);
            if (col < C) {
                *reinterpret_cast<float4*>(a.q_out + (size_t)row * C + col) = v;
            } else {  // K/V of this token into the sequence's page of layer l+1 (add_to_cache)
                const int kv = col >= 2 * C;
                const int c = col - (kv ? 2 * C : C);
                const int hh = c >> 6, d = c & 63;
                if (kpage >= 0) {
                    const int pslot = kps % P;
                    const size_t toff = (size_t)kpage * a.page_elems + ((size_t)kv * NH + hh) * P * 64;
                    if constexpr (BF) {
                        unsigned short* kvt = reinterpret_cast<unsigned short*>(a.kv_next) + toff +
                                              (kv == 0 ? ((d >> 3) * P + pslot) * 8 + (d & 7) : pslot * 64 + d);
                        const unsigned lo = hpa::f32_to_bf16(v.x) | ((unsigned)hpa::f32_to_bf16(v.y) << 16);
                        const unsigned hi = hpa::f32_to_bf16(v.z) | ((unsigned)hpa::f32_to_bf16(v.w) << 16);
                        *reinterpret_cast<uint2*>(kvt) = make_uint2(lo, hi);
                    } else {
                        float* kvt = reinterpret_cast<float*>(a.kv_next) + toff +
                                     (kv == 0 ? ((d >> 2) * P + pslot) * 4 : pslot * 64 + d);
                        *reinterpret_cast<float4*>(kvt) = v;
                    }
                }
            }
        }
    }
    PL_MARK(11);
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

template <int NH>
bool shape_ok(int B, int S, int G) {
    // one unit per slot in every phase: attention B*NH*S, fc and fcproj
    // 4*(C/16)*R units; grid and unit numbering assume G % 8 == 0
    const int R = (B + 15) / 16;
    return B >= 1 && B <= 64 && S >= 1 && S <= HPA_ATTN_MAX_SPLITS && G % 8 == 0 && (long)B * NH * S <= 3L * G &&
           4L * LD<NH>::NCT * R <= 3L * G;
}

// kernel arguments of one layer launch (every form)
void fill_ka(const HpaLayerArgs* h, int G, KA& a) {
    const HpaKVPool* pool = h->pool;
    a.B = h->B;
    a.R = (h->B + 15) / 16;
    a.Mp = h->stats_mp > 0 ? h->stats_mp : a.R * 16;  // the stride of stats_out only
    a.S = h->splits;
    a.G = G;
    a.last = h->last;
    a.layer = h->layer;
    a.q = h->q;
    a.kv = (const char*)pool->base + (size_t)h->layer * pool->layer_elems * pool->elem_bytes;
    a.kv_next = h->last ? nullptr : (char*)pool->base + (size_t)(h->layer + 1) * pool->layer_elems * pool->elem_bytes;
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
    a.w_ap = h->w_ap;
    a.b_ap = h->b_ap;
    a.w_fc = h->w_fc;
    a.fc_c1 = h->fc_c1;
    a.fc_c2 = h->fc_c2;
    a.w_fp = h->w_fp;
    a.b_fp = h->b_fp;
    a.w_qkv = h->w_qkv;
    a.qkv_c1 = h->qkv_c1;
    a.qkv_c2 = h->qkv_c2;
    a.q_out = h->q_out;
    a.stats_out = h->stats_out;
    a.rec = h->rec;
    a.slab_fp = h->slab;
    a.ctr = h->counters;
    a.err = h->err;
    a.err_sticky = h->err_sticky;
}

// blocks per CU of a 768-thread instantiation (occupancy API), cached per kernel
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

template <int NH, int P, bool BF, bool ATTN, int NB = 4, int NCD = 4, int NE = 4>
int launch(const HpaLayerArgs* h, int G) {
    HPA_REQUIRE(resident_blocks(decode_layer_kernel<NH, P, BF, ATTN, NB, NCD, NE>) >= 1,
                "decode layer: the persistent workgroup does not fit a CU");
    KA a;
    fill_ka(h, G, a);
    decode_layer_kernel<NH, P, BF, ATTN, NB, NCD, NE><<<G, 768, 0, hpa_stream()>>>(a);
    HPA_LAUNCH_CHECK();
    return 0;
}

template <int P, bool BF, int TE>
int launch_first6(const HpaLayerArgs* h, int G, const int* tokens, const float* wte, const float* wpe, void* zero,
                  size_t zero_bytes) {
    HPA_REQUIRE(resident_blocks(decode_first6_kernel<P, BF, TE>) >= 1, "decode first: the workgroup does not fit a CU");
    const int R = (h->B + 15) / 16;
    HPA_REQUIRE(R * 144 / TE <= G, "decode first: a unit per workgroup");
    KA a;
    fill_ka(h, G, a);
    a.last = 0;
    a.kv_next = h->pool->base;  // layer 0's pages
    a.tokens = tokens;
    a.wte = wte;
    a.wpe = wpe;
    a.zero = reinterpret_cast<int4*>(zero);
    a.zero_n4 = (int)(zero_bytes / 16);
    decode_first6_kernel<P, BF, TE><<<G, 768, 0, hpa_stream()>>>(a);
    HPA_LAUNCH_CHECK();
    return 0;
}

template <int P, bool BF>
int dispatch_first6_t(const HpaLayerArgs* h, int G, const int* tokens, const float* wte, const float* wpe, void* zero,
                      size_t zero_bytes) {
    switch ((h->B + 15) / 16) {  // qkv tiles per unit as chain form 6's phase E
        case 1: return launch_first6<P, BF, 1>(h, G, tokens, wte, wpe, zero, zero_bytes);
        case 2: return launch_first6<P, BF, 2>(h, G, tokens, wte, wpe, zero, zero_bytes);
        case 3: return launch_first6<P, BF, 2>(h, G, tokens, wte, wpe, zero, zero_bytes);
        case 4: return launch_first6<P, BF, 3>(h, G, tokens, wte, wpe, zero, zero_bytes);
        default: return hpa_fail(__FILE__, __LINE__, "decode first: B <= 64");
    }
}

template <int P, bool BF, int TC, int TD, int TE>
int launch6(const HpaLayerArgs* h, int G) {
    HPA_REQUIRE(resident_blocks(decode_chain6_kernel<P, BF, TC, TD, TE>) >= 1,
                "decode layer: the chain-6 workgroup does not fit a CU");
    const int R = (h->B + 15) / 16;
    HPA_REQUIRE(R * 48 <= G && R * 192 / TC <= G && 4 * R * 48 / TD <= G && R * 144 / TE <= G,
                "decode layer: chain form 6 needs a unit per workgroup in every phase");
    KA a;
    fill_ka(h, G, a);
    decode_chain6_kernel<P, BF, TC, TD, TE><<<G, 768, 0, hpa_stream()>>>(a);
    HPA_LAUNCH_CHECK();
    return 0;
}

// chain form 8: tiles per unit T (<= cx::XT_MAX) and tile groups NG (padded
// to a multiple of 8 where that still fits) of a phase with NJ column tiles
// and `parts` K parts: the fewest tiles with every unit on a workgroup
int pick_xt(int R, int parts, int NJ, int G, int* T, int* NG) {
    for (int pad = 8; pad >= 1; pad /= 8)
        for (int t = (R * parts * NJ + G - 1) / G; t <= cx::XT_MAX; ++t) {
            if (t < 1) continue;
            const int ng = ((NJ + t - 1) / t + pad - 1) / pad * pad;
            if (R * parts * ng <= G) {
                *T = t;
                *NG = ng;
                return 0;
            }
        }
    return 1;
}

int chainx_shape(int B, int NH, int G, int xt[4], int xng[4]) {
    const int R = (B + 15) / 16, nct = 4 * NH;  // C / 16
    return B < 1 || B > 64 || pick_xt(R, 1, nct, G, &xt[0], &xng[0]) || pick_xt(R, 1, 4 * nct, G, &xt[1], &xng[1]) ||
           pick_xt(R, 4, nct, G, &xt[2], &xng[2]) || pick_xt(R, 1, 3 * nct, G, &xt[3], &xng[3]);
}

template <int NH, int P, bool BF>
int launchx(const HpaLayerArgs* h, int G) {
    HPA_REQUIRE(resident_blocks(decode_chainx_kernel<NH, P, BF>) >= 1,
                "decode layer: the chain-8 workgroup does not fit a CU");
    KA a;
    fill_ka(h, G, a);
    HPA_REQUIRE(chainx_shape(h->B, NH, G, a.xt, a.xng) == 0, "decode layer: chain form 8 shape (B <= 64)");
    decode_chainx_kernel<NH, P, BF><<<G, 768, 0, hpa_stream()>>>(a);
    HPA_LAUNCH_CHECK();
    return 0;
}

template <int NH>
int dispatchx(const HpaLayerArgs* h, int G) {
    const bool bf = h->pool->dtype == HPA_BF16;
    switch (h->pool->page_size) {
        case 8: return bf ? launchx<NH, 8, true>(h, G) : launchx<NH, 8, false>(h, G);
        case 16: return bf ? launchx<NH, 16, true>(h, G) : launchx<NH, 16, false>(h, G);
        case 32: return bf ? launchx<NH, 32, true>(h, G) : launchx<NH, 32, false>(h, G);
        case 64: return bf ? launchx<NH, 64, true>(h, G) : launchx<NH, 64, false>(h, G);
        default: return hpa_fail(__FILE__, __LINE__, "decode layer: page size must be 8, 16, 32 or 64");
    }
}

// tiles per unit of fc, fcproj, qkv by row blocks R: the fewest with every
// phase's units <= 256 workgroups (attproj: 1)
template <int P, bool BF>
int dispatch6_t(const HpaLayerArgs* h, int G) {
    switch ((h->B + 15) / 16) {
        case 1: return launch6<P, BF, 1, 1, 1>(h, G);
        case 2: return launch6<P, BF, 2, 2, 2>(h, G);
        case 3: return launch6<P, BF, 3, 3, 2>(h, G);
        case 4: return launch6<P, BF, 3, 3, 3>(h, G);
        default: return hpa_fail(__FILE__, __LINE__, "decode layer: chain form 6 needs B <= 64");
    }
}

int dispatch6(const HpaLayerArgs* h, int G) {
    const bool bf = h->pool->dtype == HPA_BF16;
    switch (h->pool->page_size) {
        case 8: return bf ? dispatch6_t<8, true>(h, G) : dispatch6_t<8, false>(h, G);
        case 16: return bf ? dispatch6_t<16, true>(h, G) : dispatch6_t<16, false>(h, G);
        case 32: return bf ? dispatch6_t<32, true>(h, G) : dispatch6_t<32, false>(h, G);
        case 64: return bf ? dispatch6_t<64, true>(h, G) : dispatch6_t<64, false>(h, G);
        default: return hpa_fail(__FILE__, __LINE__, "decode layer: page size must be 8, 16, 32 or 64");
    }
}

template <int NH, bool ATTN, int NB = 4, int NCD = 4, int NE = 4>
int dispatch_p(const HpaLayerArgs* h, int G) {
    const bool bf = h->pool->dtype == HPA_BF16;
    switch (h->pool->page_size) {
        case 8: return bf ? launch<NH, 8, true, ATTN, NB, NCD, NE>(h, G) : launch<NH, 8, false, ATTN, NB, NCD, NE>(h, G);
        case 16: return bf ? launch<NH, 16, true, ATTN, NB, NCD, NE>(h, G) : launch<NH, 16, false, ATTN, NB, NCD, NE>(h, G);
        case 32: return bf ? launch<NH, 32, true, ATTN, NB, NCD, NE>(h, G) : launch<NH, 32, false, ATTN, NB, NCD, NE>(h, G);
        case 64: return bf ? launch<NH, 64, true, ATTN, NB, NCD, NE>(h, G) : launch<NH, 64, false, ATTN, NB, NCD, NE>(h, G);
        default: return hpa_fail(__FILE__, __LINE__, "decode layer: page size must be 8, 16, 32 or 64");
    }
}

template <int NH>
int dispatch(const HpaLayerArgs* h, int G) {
    if (h->chain_only == 6) {
        if constexpr (NH == 12) return dispatch6(h, G);
        return hpa_fail(__FILE__, __LINE__, "decode layer: chain form 6 needs C = 768");
    }
#ifndef HPA_AB
    // measured slower than the forms the engine picks: in A/B builds only
    if (h->chain_only >= 2)
        return hpa_fail(__FILE__, __LINE__, "decode layer: wide-unit chain forms 2..5 are in A/B builds only (-DHPA_AB)");
    if (!h->chain_only)
        return hpa_fail(__FILE__, __LINE__, "decode layer: the full persistent layer is in A/B builds only (-DHPA_AB)");
    return dispatch_p<NH, false>(h, G);
#else
    if (h->chain_only >= 2) {  // wide units (C = 768), widths (attproj, fc / fcproj, qkv) by chain_only
        if constexpr (LD<NH>::SW % 3 == 0) {
            const int R = (h->B + 15) / 16, nct = LD<NH>::NCT;
            // every phase's units fit its unit slots: attproj R*nct, fc / fcproj 4*R*nct, qkv 3*R*nct
            auto fits = [&](int nb, int ncd, int ne) {
                return R * nct <= 12 / nb * G && 4 * R * nct <= 12 / ncd * G && 3 * R * nct <= 12 / ne * G;
            };
            switch (h->chain_only) {
                case 2:
                    HPA_REQUIRE(fits(12, 12, 12), "decode layer: chain form 2 (12/12/12-wave units) needs B <= 16");
                    return dispatch_p<NH, false, 12, 12, 12>(h, G);
                case 3:
                    HPA_REQUIRE(fits(12, 6, 6), "decode layer: chain form 3 (12/6/6-wave units) needs B <= 32");
                    return dispatch_p<NH, false, 12, 6, 6>(h, G);
                case 4:
                    HPA_REQUIRE(fits(12, 4, 6), "decode layer: chain form 4 (12/4/6-wave units) needs B <= 48");
                    return dispatch_p<NH, false, 12, 4, 6>(h, G);
                case 5:
                    HPA_REQUIRE(fits(12, 4, 4), "decode layer: chain form 5 (12/4/4-wave units) needs B <= 64");
                    return dispatch_p<NH, false, 12, 4, 4>(h, G);
                default:
                    return hpa_fail(__FILE__, __LINE__, "decode layer: chain_only must be 0..6 or 8");
            }
        } else {
            return hpa_fail(__FILE__, __LINE__, "decode layer: wide units need C = 768");
        }
    }
    return h->chain_only ? dispatch_p<NH, false>(h, G) : dispatch_p<NH, true>(h, G);
#endif
}

}  // namespace

extern "C" {

int hpa_decode_layer_eligible(int B, int C, int num_heads, int splits) {
    const int G = num_cus();
    if (G <= 0 || C != 64 * num_heads) return 0;
    if (num_heads == 12) return shape_ok<12>(B, splits, G) ? 1 : 0;
    if (num_heads == 2) return shape_ok<2>(B, splits, G) ? 1 : 0;
    return 0;
}

// the split count measured best for the stand-alone attention
// (hpa_attn_pick_splits: a range of >= 4 tiles per 4-wave unit; short ranges
// pay the merge), halved until every unit has a slot (B*NH*S <= 3 x CUs)
int hpa_decode_layer_pick_splits(int B, int num_heads, int max_ctx) {
    const int G = num_cus();
    if (G <= 0 || B <= 0 || num_heads <= 0) return 1;
    int s = hpa_attn_pick_splits(B, num_heads, max_ctx, G);
    while (s > 1 && (long)B * num_heads * s > 3L * G) s /= 2;
    return s;
}

int hpa_decode_layer_sizes(int B, int C, int num_heads, int splits, size_t* out3) {
    HPA_REQUIRE(out3 && B > 0 && C == 64 * num_heads && splits >= 1, "decode layer sizes: bad arguments");
    const int R = (B + 15) / 16, nct = C / 16;
    out3[0] = (size_t)B * num_heads * splits * kRec;
    out3[1] = (size_t)4 * R * nct * 256;  // fcproj K-part partial tiles
    const size_t ints5 = (size_t)kCtrInts + 2 * (size_t)R * nct + (size_t)B * num_heads;
    const size_t ints6 = (size_t)c6::kCtr + (size_t)4 * nct + c6::kGrp;  // form 6: counters, tickets [4][nct], k-groups
    const size_t ints = ints5 > ints6 ? ints5 : ints6;
    out3[2] = (ints + 31) / 32 * 32;  // whole 128-B lines (memset in multiples of 16 B)
    return 0;
}

// trace build only: form 8's per-wave fc stamps of layer 5 ([256][12][16] u64,
// s_memtime); host NULL clears them.  Returns 1 in the product build.
int hpa_decode_cx_wave_trace(unsigned long long* host) {
#ifdef HPA_LAYER_TRACE
    if (!host) {
        static unsigned long long zero[256 * 12 * 16];
        HPA_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_cx_wave), zero, sizeof(zero)));
        return 0;
    }
    HPA_CHECK(hipMemcpyFromSymbol(host, HIP_SYMBOL(g_cx_wave), sizeof(unsigned long long) * 256 * 12 * 16));
    return 0;
#else
    (void)host;
    return 1;
#endif
}

// trace build only: copy the per-(layer, workgroup) event stamps of the last
// launches ([layers][256][16] u64, s_memrealtime ticks of 10 ns); host NULL
// clears them.  Returns 1 in the product build.
int hpa_decode_layer_trace(unsigned long long* host, int layers) {
#ifdef HPA_LAYER_TRACE
    HPA_REQUIRE(layers >= 0 && layers <= 64, "trace: layers 0..64");
    if (!host) {
        static unsigned long long zero[64 * 256 * 16];
        HPA_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_pl_trace), zero, sizeof(zero)));
        return 0;
    }
    HPA_CHECK(hipMemcpyFromSymbol(host, HIP_SYMBOL(g_pl_trace), (size_t)layers * 256 * 16 * 8));
    return 0;
#else
    (void)host;
    (void)layers;
    return 1;
#endif
}

// the chain forms 6 (C = 768) and 8 (C = 768, 1024, 1280 or 1600): B <= 64, fp32 or
// bf16 pool, a unit per workgroup in every phase
int hpa_decode_chain_eligible(int B, int C, int num_heads, int form) {
    const int G = num_cus();
    if (G <= 0 || C != 64 * num_heads || B < 1 || B > 64) return 0;
    if (form == 6) {
        if (num_heads != 12) return 0;
        const int R = (B + 15) / 16;
        return R * 48 <= G && 4 * R * 48 / (R == 1 ? 1 : R == 2 ? 2 : 3) <= G ? 1 : 0;
    }
    if (form == 8) {  // GPT-2 124M / medium / large / XL widths (C = 768, 1024, 1280, 1600)
        if (num_heads != 12 && num_heads != 16 && num_heads != 20 && num_heads != 25) return 0;
        int xt[4], xng[4];
        return chainx_shape(B, num_heads, G, xt, xng) == 0 ? 1 : 0;
    }
    return 0;
}

int hpa_decode_first(const HpaLayerArgs* h, const int* tokens, const float* wte, const float* wpe, void* zero,
                     size_t zero_bytes) {
    HPA_REQUIRE(h && h->pool && h->pool->base && tokens && wte && wpe, "decode first: null operand");
    const HpaKVPool* pool = h->pool;
    HPA_REQUIRE(pool->dtype == HPA_F32 || pool->dtype == HPA_BF16, "decode first: fp32 or bf16 pool");
    HPA_REQUIRE(h->num_heads == 12 && h->C == 768 && pool->head_size == HS && pool->num_heads == 12,
                "decode first: C = 768, 12 heads of 64");
    HPA_REQUIRE(h->B >= 1 && h->B <= 64, "decode first: 1..64 rows");
    HPA_REQUIRE(h->res && h->w_qkv && h->qkv_c1 && h->qkv_c2 && h->q_out && h->block_table && h->pos,
                "decode first: null operand");
    HPA_REQUIRE(zero_bytes % 16 == 0 && ((size_t)zero & 15) == 0 && zero_bytes / 16 <= 0x7fffffff,
                "decode first: the zeroed block must be whole 16-byte granules");
    const int G = num_cus();
    const bool bf = pool->dtype == HPA_BF16;
    switch (pool->page_size) {
        case 8: return bf ? dispatch_first6_t<8, true>(h, G, tokens, wte, wpe, zero, zero_bytes)
                          : dispatch_first6_t<8, false>(h, G, tokens, wte, wpe, zero, zero_bytes);
        case 16: return bf ? dispatch_first6_t<16, true>(h, G, tokens, wte, wpe, zero, zero_bytes)
                           : dispatch_first6_t<16, false>(h, G, tokens, wte, wpe, zero, zero_bytes);
        case 32: return bf ? dispatch_first6_t<32, true>(h, G, tokens, wte, wpe, zero, zero_bytes)
                           : dispatch_first6_t<32, false>(h, G, tokens, wte, wpe, zero, zero_bytes);
        case 64: return bf ? dispatch_first6_t<64, true>(h, G, tokens, wte, wpe, zero, zero_bytes)
                           : dispatch_first6_t<64, false>(h, G, tokens, wte, wpe, zero, zero_bytes);
        default: return hpa_fail(__FILE__, __LINE__, "decode first: page size must be 8, 16, 32 or 64");
    }
}

int hpa_decode_layer(const HpaLayerArgs* h) {
    HPA_REQUIRE(h && h->pool && h->pool->base, "decode layer: pool");
    const HpaKVPool* pool = h->pool;
    HPA_REQUIRE(pool->dtype == HPA_F32 || pool->dtype == HPA_BF16, "decode layer: fp32 or bf16 pool");
    HPA_REQUIRE(pool->head_size == HS && h->C == h->num_heads * HS, "decode layer: head size 64");
    HPA_REQUIRE(h->layer >= 0 && h->layer < pool->num_layers && (h->last || h->layer + 1 < pool->num_layers),
                "decode layer: layer out of range");
    HPA_REQUIRE(h->q && h->att && h->res && h->res2 && h->fch && h->w_ap && h->b_ap && h->w_fc && h->fc_c1 &&
                    h->fc_c2 && h->w_fp && h->b_fp && h->block_table && h->pos && h->rec && h->slab &&
                    h->counters && h->err,
                "decode layer: null operand");
    HPA_REQUIRE(h->last || (h->w_qkv && h->qkv_c1 && h->qkv_c2 && h->q_out), "decode layer: qkv(l+1) operands");
    HPA_REQUIRE(h->splits >= 1 && h->splits <= HPA_ATTN_MAX_SPLITS, "decode layer: splits 1..16");
    const int G = num_cus();
    if (h->chain_only == 6 || h->chain_only == 8) {
        HPA_REQUIRE(hpa_decode_chain_eligible(h->B, h->C, h->num_heads, h->chain_only),
                    "decode layer: chain form not supported for this shape");
        if (h->chain_only == 8) switch (h->num_heads) {
                case 16: return dispatchx<16>(h, G);
                case 20: return dispatchx<20>(h, G);
                case 25: return dispatchx<25>(h, G);
                default: return dispatchx<12>(h, G);
            }
        return dispatch<12>(h, G);
    }
    HPA_REQUIRE(hpa_decode_layer_eligible(h->B, h->C, h->num_heads, h->splits), "decode layer: shape not supported");
    if (h->num_heads == 12) return dispatch<12>(h, G);
    return dispatch<2>(h, G);
}

}  // extern "C"
