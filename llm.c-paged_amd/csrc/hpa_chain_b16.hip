// hpa_chain_b16.hip -- the decode layer's GEMM chain on bf16 weights (BASELINE
// config 5, "GPT-2 124M bf16 decode", B up to 256) as ONE persistent launch
// per layer:
//     attproj(l) -> fc(l) -> fcproj(l) -> qkv(l+1)
// after the layer's decode-attention launch (reference gpt2_forward,
// paged_infer.c:659-722; the same phases as chain form 6, hpa_layer.hip, which
// is fp32-only with the LayerNorms folded into the weights and B <= 64).
// Replaces four bf16 GEMM launches per layer (qkv / attproj / fc / fcproj,
// 16.5 + 8.8 + 14.0 + 8.8 us at B = 256 in round 4's step).
//
// Design (MI355X first):
//  * one 8-wave workgroup per CU (grid = CU count, residency checked); every
//    phase deals units of (RG 16-row blocks) x (T 16-column tiles) over a K
//    range of 768, one unit per workgroup, its 8 waves splitting K in 3
//    32-deep steps each (v_mfma_f32_16x16x32_bf16) and folding in wave order
//    through LDS -- a row's summation order depends on nothing but the phase,
//    so every batch size and shard gives the same bits for a row;
//  * the weight fragments of a phase (bf16 frag layout, hpa_gemm_bf16.hip)
//    are loaded into registers BEFORE the phase's wait, so the weight stream
//    overlaps the hand-off;
//  * LayerNorm on the operand path with the row statistics computed by the
//    consumer unit from its own A fragments: the unit's 8 waves together hold
//    every column of its rows (no statistics hand-off, no folded weights);
//  * hand-offs: write-through (sc1) stores, drained, a workgroup barrier, one
//    agent-scope arrival per unit on a per-row-block counter line, polled with
//    agent-scope loads (MI355X_MICROARCH.md "Valid forms", row 1);
//  * fcproj (K = 3072) in 4 K parts; the last part of a (row group, tile
//    group) to draw its ticket adds the parts in part order + bias + res2.
// Unit-to-workgroup numbering puts the units sharing a weight tile group on
// one XCD (block b and b+8 share an XCD): the first reads HBM, the rest L2.
// Every spin is bounded (200 ms): a timeout stores a nonzero code in *err
// (and *err_sticky) and ends the launch (outputs then garbage).
#include <math.h>

#include "hpa_gemm_body.h"

namespace {
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));

namespace cb {
constexpr int NW = 8, NT = NW * 64;
constexpr int C = 768, K16 = 48, K32 = 24, NCT = 48;
constexpr int SPW = K32 / NW;  // 32-deep k-steps per wave of a 768 range
constexpr int kPad = 32;       // ints per counter line (128 B)
// counter lines: X1[16] attproj tiles done per row block, H[16][4] fc tile
// groups done per (row block, fcproj K part), X2[16] fcproj combines per row
// block, tickets[4][16] per (fcproj row quad, tile group)
constexpr int kX1 = 0, kH = 16, kX2 = 80, kTick = 96, kLines = 160;
constexpr long long kSpinTicks = 20000000;  // s_memrealtime is 100 MHz: 200 ms
// phase shapes (RG row blocks, T tiles, NG tile groups) by the per-CU operand
// bytes of a unit (fp32 A: 48 KiB per row block, read sc1 -- measured about
// twice the cost per byte of the L2-served weights; bf16 A and weights 24 KiB
// per row block / tile): attproj (1, 3, 16) 48 + 72 KiB, fc (2, 6, 32)
// 96 + 144, fcproj (4, 3, 16) x 4 K parts on bf16 fch 96 + 72, qkv (1, 9, 16)
// 48 + 216 (qkv as (2, 5): 5.2 us against 4.0, fcproj as (2, 6) on fp32 fch
// 4.3 against 2.8, profiles/r5/b16_chain.txt); at 16 row blocks (B = 256)
// every phase has 256 units
constexpr int NG_B = 16, NG_C = 32, NG_D = 16, NG_E = 16;
constexpr int RED_T = 12;  // most tiles per unit (RG x T)

struct Args {
    int B, R, Mp, last, layer;
    const float* att;
    float *res, *res2, *fch;
    const uint4 *w_ap, *w_fc, *w_fp, *w_qkv;
    const float *b_ap, *ln2_w, *ln2_b, *b_fc, *b_fp, *ln1_w, *ln1_b, *b_qkv;
    float* q_out;
    void* kv_next;
    size_t page_elems;
    const int* bt;
    int bt_stride;
    const int* pos;
    float* stats_out;
    int stats_mp;
    float* slab;
    int* ctr;
    int* err;
    int* err_sticky;
    // the step's first launch (FIRST): the tokens, the embedding tables, and
    // the step's counter block to zero (16-byte granules)
    const int* tokens;
    const float *wte, *wpe;
    int4* zero;
    int zero_n4;
};

struct Smem {
    float red[NW * RED_T * 256];  // [wave][unit tile][256] accumulators
    float wsum[NW * 2 * 32];      // [wave][row block][16 rows][2] LN row partial sums
    int s_ok;
    int s_last;
};

// diagnostic build (-DHPA_LAYER_TRACE, tools/pl_trace.py b16): s_memrealtime
// of workgroup-level events per (layer, workgroup), slots as hpa_layer.hip's
// (0 start, 4/6/8/10 phase B/C/D/E wait done, 12/13/14 B/C/D stored,
// 5/7/9 B/C/D arrived, 15 E folded, 11 end); never in the product library
#ifdef HPA_LAYER_TRACE
__device__ unsigned long long g_cb_trace[64][256][16];
#define CB_MARK(k)                                                                                     \
    do {                                                                                               \
        if (threadIdx.x == 0 && a.layer >= 0 && a.layer < 64 && blockIdx.x < 256)                      \
            g_cb_trace[a.layer][blockIdx.x][k] = (unsigned long long)__builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define CB_MARK(k) \
    do {           \
    } while (0)
#endif

__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// every storing wave drained (the builtin form: the compiler then knows
// vmcnt is 0 and does not wait again, past the next phase's weight loads)
__device__ __forceinline__ void drain_vm() {
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) expcnt(7) lgkmcnt(15)
    asm volatile("" ::: "memory");
}

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ float4 add4(float4 a, float4 b) { return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }

__device__ __forceinline__ bf16x8 pack_bf16(float4 a, float4 b) {
    u16x8 u;
    u[0] = hpa::f32_to_bf16(a.x);
    u[1] = hpa::f32_to_bf16(a.y);
    u[2] = hpa::f32_to_bf16(a.z);
    u[3] = hpa::f32_to_bf16(a.w);
    u[4] = hpa::f32_to_bf16(b.x);
    u[5] = hpa::f32_to_bf16(b.y);
    u[6] = hpa::f32_to_bf16(b.z);
    u[7] = hpa::f32_to_bf16(b.w);
    return __builtin_bit_cast(bf16x8, u);
}

// 16-byte sc1 load as raw bits (bf16 operand fragments) / 8-byte sc1 store
__device__ __forceinline__ uint4 load_wt16u(const void* base, int byte_off) {
    const hpa::u32x4 d = __builtin_amdgcn_raw_buffer_load_b128(hpa::wt_rsrc(base), byte_off, 0, hpa::kCpolSc1);
    return make_uint4(d.x, d.y, d.z, d.w);
}
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void store_wt8(void* base, int byte_off, unsigned lo, unsigned hi) {
    const u32x2 d = {lo, hi};
    __builtin_amdgcn_raw_buffer_store_b64(d, hpa::wt_rsrc(base), byte_off, 0, hpa::kCpolSc1);
}

__device__ __forceinline__ void arrive(const Args& a, int line) {
    __hip_atomic_fetch_add(a.ctr + line * kPad, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// wave 0 polls the n (0..4) counter lines base, base + stride, .. until all
// reach `expected` (bounded; the other waves wait at the barrier)
__device__ __forceinline__ bool wait_lines(const Args& a, int base, int stride, int n, int expected, int code,
                                           Smem& sm) {
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (wv == 0) {
        const int lane = threadIdx.x & 63;
        const int line = lane < n ? base + lane * stride : -1;
        int ok = 0;
        const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
        for (unsigned it = 0;; ++it) {
            const int v = line >= 0 ? __hip_atomic_load(a.ctr + line * kPad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                    : expected;
            if (__ballot(v < expected) == 0ull) {
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

// the wave's weight fragments of tiles j0 .. j0+T-1 at 32-deep steps
// kb + SPW*w .. (bf16 frag layout [tile][K32W][64 lanes] of 16 B)
// (tiles past jlast re-read tile jlast: computed, never stored)
template <int T>
__device__ __forceinline__ void load_w(const uint4* W, int K32W, int j0, int kb, int w, uint4 (&wr)[T][SPW],
                                       int jlast = 1 << 20) {
    const uint4* wf = W + ((size_t)kb + w * SPW) * 64 + (threadIdx.x & 63);
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
        for (int s = 0; s < SPW; ++s) wr[t][s] = wf[((size_t)min(j0 + t, jlast) * K32W + s) * 64];
}

// the unit's accumulators: the wave's A fragments of row blocks rb0 .. rb0+RG-1
// (fp32 frag layout, K16A 16-deep steps per row; sc1 loads -- written in this
// launch or the one before; row blocks >= R clamp to R-1, never stored),
// LayerNorm'ed with the rows' statistics over all 768 columns (LN: the 8
// waves' partial sums through LDS, in wave order; one-pass form as
// layernorm_forward's statistics elsewhere in the engine), rounded to bf16,
// then the RG x T chains of 3 MFMAs
// EMB (the step's first launch): A is the embedding wte[token] + wpe[pos]
// (encoder_forward, paged_infer.c:41-47; rows >= B are 0) built in registers
// from ea's tables, and stored to ea->res (frag layout) when store_res
template <int RG, int T, bool LN, bool EMB = false>
__device__ __forceinline__ void unit_mma(const float* A, int K16A, int rb0, int R, int kb, const uint4 (&wr)[T][SPW],
                                         const float* lnw, const float* lnb, Smem& sm, f32x4 (&acc)[RG][T],
                                         const Args* ea = nullptr, bool store_res = false) {
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    float4 xa[RG][SPW][2];
#pragma unroll
    for (int r = 0; r < RG; ++r) {
        const int rb = min(rb0 + r, R - 1);
        if constexpr (EMB) {
            const int row = rb * 16 + (lane & 15);
            const bool live = row < ea->B;
            const float* te = ea->wte + (size_t)(live ? ea->tokens[row] : 0) * C;
            const float* pe = ea->wpe + (size_t)(live ? ea->pos[row] : 0) * C;
#pragma unroll
            for (int s = 0; s < SPW; ++s)
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int col = 32 * (kb + w * SPW + s) + 16 * h + 4 * (lane >> 4);
                    xa[r][s][h] = live ? add4(ld4(te + col), ld4(pe + col)) : make_float4(0.f, 0.f, 0.f, 0.f);
                }
            if (store_res && rb0 + r < R)
#pragma unroll
                for (int s = 0; s < SPW; ++s)
#pragma unroll
                    for (int h = 0; h < 2; ++h)
                        reinterpret_cast<float4*>(ea->res)[(rb * K16A + 2 * (kb + w * SPW + s) + h) * 64 + lane] =
                            xa[r][s][h];
        } else {
#pragma unroll
            for (int s = 0; s < SPW; ++s)
#pragma unroll
                for (int h = 0; h < 2; ++h)
                    xa[r][s][h] = hpa::load_wt16(A, ((rb * K16A + 2 * (kb + w * SPW + s) + h) * 64 + lane) * 16);
        }
    }
    float4 lg[SPW][2], lb[SPW][2];
    if (LN) {
#pragma unroll
        for (int s = 0; s < SPW; ++s)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int k = 32 * (kb + w * SPW + s) + 16 * h + 4 * (lane >> 4);
                lg[s][h] = ld4(lnw + k);
                lb[s][h] = ld4(lnb + k);
            }
    }
    __builtin_amdgcn_sched_barrier(0);  // every operand load in flight before the first use
    float mu[RG], rs[RG];
    if (LN) {
#pragma unroll
        for (int r = 0; r < RG; ++r) {
            float s1 = 0.f, s2 = 0.f;
#pragma unroll
            for (int s = 0; s < SPW; ++s)
#pragma unroll
                for (int h = 0; h < 2; ++h) hpa_gemm::row_sums_add(xa[r][s][h], s1, s2);
            hpa_gemm::row_sums_publish(s1, s2, sm.wsum + (w * RG + r) * 32);
        }
        lds_barrier();
#pragma unroll
        for (int r = 0; r < RG; ++r) {
            float S1 = 0.f, S2 = 0.f;
#pragma unroll
            for (int ww = 0; ww < NW; ++ww) {
                S1 += sm.wsum[(ww * RG + r) * 32 + 2 * (lane & 15)];
                S2 += sm.wsum[(ww * RG + r) * 32 + 2 * (lane & 15) + 1];
            }
            const float m = S1 / C;
            mu[r] = m;
            rs[r] = 1.0f / sqrtf(fmaxf(S2 / C - m * m, 0.f) + 1e-5f);
        }
    }
#pragma unroll
    for (int r = 0; r < RG; ++r)
#pragma unroll
        for (int t = 0; t < T; ++t) acc[r][t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < SPW; ++s) {
        bf16x8 av[RG];
#pragma unroll
        for (int r = 0; r < RG; ++r) {
            float4 x0 = xa[r][s][0], x1 = xa[r][s][1];
            if (LN) {
                x0 = hpa_gemm::ln4(x0, mu[r], rs[r], lg[s][0], lb[s][0]);
                x1 = hpa_gemm::ln4(x1, mu[r], rs[r], lg[s][1], lb[s][1]);
            }
            av[r] = pack_bf16(x0, x1);
        }
#pragma unroll
        for (int t = 0; t < T; ++t) {
            const bf16x8 wb = __builtin_bit_cast(bf16x8, wr[t][s]);
#pragma unroll
            for (int r = 0; r < RG; ++r)
                acc[r][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[r], wb, acc[r][t], 0, 0, 0);
        }
    }
}

// the same on an A already in the bf16 frag layout (K32A 32-deep steps per
// row; fcproj's fch): no LayerNorm, no rounding
template <int RG, int T>
__device__ __forceinline__ void unit_mma_b(const void* A, int K32A, int rb0, int R, int kb, const uint4 (&wr)[T][SPW],
                                           f32x4 (&acc)[RG][T]) {
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint4 xa[RG][SPW];
#pragma unroll
    for (int r = 0; r < RG; ++r) {
        const int rb = min(rb0 + r, R - 1);
#pragma unroll
        for (int s = 0; s < SPW; ++s) xa[r][s] = load_wt16u(A, ((rb * K32A + kb + w * SPW + s) * 64 + lane) * 16);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int r = 0; r < RG; ++r)
#pragma unroll
        for (int t = 0; t < T; ++t) acc[r][t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < SPW; ++s)
#pragma unroll
        for (int t = 0; t < T; ++t) {
            const bf16x8 wb = __builtin_bit_cast(bf16x8, wr[t][s]);
#pragma unroll
            for (int r = 0; r < RG; ++r)
                acc[r][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, xa[r][s]), wb,
                                                                    acc[r][t], 0, 0, 0);
        }
}

template <int RG, int T>
__device__ __forceinline__ void put_red(float* red, const f32x4 (&acc)[RG][T]) {
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
#pragma unroll
    for (int r = 0; r < RG; ++r)
#pragma unroll
        for (int t = 0; t < T; ++t)
#pragma unroll
            for (int g = 0; g < 4; ++g) red[((w * RG + r) * T + t) * 256 + g * 64 + lane] = acc[r][t][g];
}

// epilogue element e of a unit (< RG*T*64): unit tile q = e / 64 (row block
// q / T, tile q % T), row er = (e % 64) / 4 of it, columns 4*eq .. 4*eq+3;
// the 4 values summed over the 8 waves in wave order
template <int RG, int T>
__device__ __forceinline__ float4 fold(const float* red, int e) {
    const int q = e >> 6, er = (e & 63) >> 2, eq = e & 3;
    const float* p = red + q * 256 + (er & 3) * 64 + 16 * (er >> 2) + 4 * eq;
    float4 v = ld4(p);
#pragma unroll
    for (int w = 1; w < NW; ++w) {
        const float4 x = ld4(p + w * RG * T * 256);
        v.x += x.x;
        v.y += x.y;
        v.z += x.z;
        v.w += x.w;
    }
    return v;
}

template <int T>
__device__ __forceinline__ void where(int e, int rb0, int j0, int& row, int& col) {
    const int q = e >> 6;
    row = (rb0 + q / T) * 16 + ((e & 63) >> 2);
    col = (j0 + q % T) * 16 + 4 * (e & 3);
}

// qkv epilogue store of columns col..col+3 of `row`: q row-major, or K / V of
// this token (position ps, page `page`, loaded by phase E before its wait)
// into the sequence's page of layer l+1 (add_to_cache, paged_infer.c:505-573;
// fp32 pool K [chunk of 4][slot][4], bf16 pool K [chunk of 8][slot][8] RNE,
// V [slot][64])
template <int P, bool BF>
__device__ __forceinline__ void qkv_store(const Args& a, int row, int col, int ps, int page, float4 v) {
    constexpr int NH = 12;
    if (col < C) {
        *reinterpret_cast<float4*>(a.q_out + (size_t)row * C + col) = v;
        return;
    }
    const int kv = col >= 2 * C;
    const int c = col - (kv ? 2 * C : C);
    const int hh = c >> 6, d = c & 63;
    if (page < 0) return;  // no page (host bug): never write below the pool
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

}  // namespace cb

// FIRST: the step's first launch -- the counter block zeroed, then only
// phase E on the embedding (layer 0's q and K/V; the tile group 0 unit of a
// row block also stores the residual stream it built): the embed kernel and
// the qkv(0) GEMM in one launch
template <int P, bool BF, bool FIRST>
__global__ __launch_bounds__(512) void decode_chain_b16_kernel(cb::Args args) {
    using namespace cb;
    const Args& a = *(const Args*)(const void*)__builtin_amdgcn_kernarg_segment_ptr();
    (void)args;
    __shared__ Smem sm;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int tid = threadIdx.x;
    const int bid = blockIdx.x;
    const int R = a.R, RH = (a.R + 1) / 2;  // row blocks, row groups of two
    const int Mp = R * 16;
    CB_MARK(0);
    if constexpr (FIRST)
        for (int i = bid * NT + tid; i < a.zero_n4; i += gridDim.x * NT) a.zero[i] = make_int4(0, 0, 0, 0);

    // B: attproj(l): res2 = res + att . Wap^T + b; unit (row block, 3 tiles)
    if constexpr (!FIRST) {
        constexpr int RG = 1, T = 3, NE = RG * T * 64;
        const bool has = bid < R * NG_B;
        const int g = bid % NG_B, rb = bid / NG_B;
        uint4 wr[T][SPW];
        if (has) load_w<T>(a.w_ap, K32, g * T, 0, w, wr);
        const bool ep = has && tid < NE;
        int row, col;
        where<T>(tid, rb, g * T, row, col);
        const int fi = (int)hpa::frag_index(row, col, C) * 4;
        float4 bv = make_float4(0.f, 0.f, 0.f, 0.f), rv = bv;
        if (ep) {
            bv = ld4(a.b_ap + col);
            rv = hpa::load_wt16(a.res, fi);
        }
        CB_MARK(4);
        if (has) {
            f32x4 acc[RG][T];
            unit_mma<RG, T, false>(a.att, K16, rb, R, 0, wr, nullptr, nullptr, sm, acc);
            put_red<RG, T>(sm.red, acc);
        }
        lds_barrier();
        if (ep) {
            const float4 v = add4(fold<RG, T>(sm.red, tid), bv);
            // residual_forward(out, res, proj); padded rows stay 0
            hpa::store_wt16(a.res2, fi, row < a.B ? add4(rv, v) : make_float4(0.f, 0.f, 0.f, 0.f));
        }
        CB_MARK(12);
        drain_vm();
        lds_barrier();
        if (tid == 0 && has) arrive(a, kX1 + rb);
        CB_MARK(5);
    }
    // C: fc(l): fch = gelu(LN2(res2) . Wfc^T + b); unit (2 row blocks, 6 tiles)
    if constexpr (!FIRST) {
        constexpr int RG = 2, T = 6, NE = RG * T * 64;
        const bool has = bid < RH * NG_C;
        const int g = bid % NG_C, rg = bid / NG_C, rb0 = 2 * rg;
        uint4 wr[T][SPW];
        float4 bv[2];
        auto pre = [&]() {
            if (has) load_w<T>(a.w_fc, K32, g * T, 0, w, wr);
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int e = tid + i * NT;
                int row, col;
                where<T>(e, rb0, g * T, row, col);
                bv[i] = has && e < NE ? ld4(a.b_fc + col) : make_float4(0.f, 0.f, 0.f, 0.f);
            }
        };
        pre();
        if (!wait_lines(a, kX1 + rb0, 1, has ? min(2, R - rb0) : 0, NG_B, 2, sm)) return;
        CB_MARK(6);
        if (has) {
            f32x4 acc[RG][T];
            unit_mma<RG, T, true>(a.res2, K16, rb0, R, 0, wr, a.ln2_w, a.ln2_b, sm, acc);
            put_red<RG, T>(sm.red, acc);
        }
        lds_barrier();
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int e = tid + i * NT;
            int row, col;
            where<T>(e, rb0, g * T, row, col);
            if (has && e < NE && row < Mp) {
                float4 v = add4(fold<RG, T>(sm.red, e), bv[i]);
                v = row < a.B ? make_float4(hpa::gelu_ref(v.x), hpa::gelu_ref(v.y), hpa::gelu_ref(v.z), hpa::gelu_ref(v.w))
                              : make_float4(0.f, 0.f, 0.f, 0.f);
                // bf16 frag layout of fch [Mp][4C] (fcproj rounds its A to bf16 anyway: the same
                // bits, half the bytes): columns col..col+3 are half (col >> 4) & 1 of lane
                // (row & 15) + 16 * ((col & 15) >> 2) of the (row block, 32-deep step) fragment
                const int lt = (row & 15) + 16 * ((col & 15) >> 2);
                const int off = (((row >> 4) * (4 * K32) + (col >> 5)) * 64 + lt) * 16 + ((col >> 4) & 1) * 8;
                store_wt8(a.fch, off, hpa::f32_to_bf16(v.x) | ((unsigned)hpa::f32_to_bf16(v.y) << 16),
                          hpa::f32_to_bf16(v.z) | ((unsigned)hpa::f32_to_bf16(v.w) << 16));
            }
        }
        CB_MARK(13);
        drain_vm();
        lds_barrier();
        if (tid == 0 && has) {  // the fcproj K part these 96 columns feed
            const int p = (g * T) / NCT;
            arrive(a, kH + rb0 * 4 + p);
            if (rb0 + 1 < R) arrive(a, kH + (rb0 + 1) * 4 + p);
        }
        CB_MARK(7);
    }
    // D: fcproj(l), K part p of 4: partial tiles -> slab; the last part of a
    // (row quad, tile group) adds the parts in order + bias + res2 -> res
    if constexpr (!FIRST) {
        constexpr int RG = 4, T = 3, NE = RG * T * 64;
        const int RQ = (R + 3) / 4;
        const bool has = bid < RQ * 4 * NG_D;
        const int g = bid % NG_D, p = (bid / NG_D) & 3, rg = bid / (4 * NG_D), rb0 = 4 * rg;
        uint4 wr[T][SPW];
        float4 bv[2];
        auto pre = [&]() {
            if (has) load_w<T>(a.w_fp, 4 * K32, g * T, p * K32, w, wr);
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int e = tid + i * NT;
                int row, col;
                where<T>(e, rb0, g * T, row, col);
                bv[i] = has && e < NE ? ld4(a.b_fp + col) : make_float4(0.f, 0.f, 0.f, 0.f);
            }
        };
        pre();
        if (!wait_lines(a, kH + rb0 * 4 + p, 4, has ? min(4, R - rb0) : 0, NG_C / 4, 3, sm)) return;
        CB_MARK(8);
        if (has) {
            f32x4 acc[RG][T];
            unit_mma_b<RG, T>(a.fch, 4 * K32, rb0, R, p * K32, wr, acc);
            put_red<RG, T>(sm.red, acc);
        }
        lds_barrier();
        float4 val[2];
        const int sbase = ((p * RQ + rg) * NG_D + g) * NE;  // this part's float4s in the slab
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int e = tid + i * NT;
            val[i] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (has && e < NE) {
                val[i] = fold<RG, T>(sm.red, e);
                hpa::store_wt16(a.slab, (sbase + e) * 16, val[i]);
            }
        }
        CB_MARK(14);
        drain_vm();
        lds_barrier();
        if (has && tid == 0) {
            const int tk = __hip_atomic_fetch_add(a.ctr + (kTick + rg * NG_D + g) * kPad, 1, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
            sm.s_last = tk == 3;
        }
        lds_barrier();
        const bool last = has && sm.s_last != 0;
        if (last) {
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int e = tid + i * NT;
                if (e >= NE) continue;  // wave-uniform (NE % 64 == 0)
                int row, col;
                where<T>(e, rb0, g * T, row, col);
                const bool in = row < Mp;
                float4 pv[4];
#pragma unroll
                for (int qq = 0; qq < 4; ++qq)
                    pv[qq] = qq == p ? val[i] : hpa::load_wt16(a.slab, ((((qq * RQ + rg) * NG_D + g) * NE) + e) * 16);
                const int fi = (int)hpa::frag_index(min(row, Mp - 1), col, C) * 4;
                const float4 rv = hpa::load_wt16(a.res2, fi);
                float4 tot = add4(add4(add4(add4(pv[0], pv[1]), pv[2]), pv[3]), bv[i]);
                tot = row < a.B ? add4(rv, tot) : make_float4(0.f, 0.f, 0.f, 0.f);
                if (in) hpa::store_wt16(a.res, fi, tot);
                if (a.stats_out) {  // last layer: 16-column LNf partial sums of the row (4 lanes of a row)
                    float s1 = ((tot.x + tot.y) + tot.z) + tot.w;
                    float s2 = __fmaf_rn(tot.w, tot.w, __fmaf_rn(tot.z, tot.z, __fmaf_rn(tot.y, tot.y, tot.x * tot.x)));
                    s1 += __shfl_xor(s1, 1, 64);
                    s2 += __shfl_xor(s2, 1, 64);
                    s1 += __shfl_xor(s1, 2, 64);
                    s2 += __shfl_xor(s2, 2, 64);
                    if (in && (e & 3) == 0) {
                        const int j = col >> 4;
                        a.stats_out[((size_t)j * a.stats_mp + row) * 2] = s1;
                        a.stats_out[((size_t)j * a.stats_mp + row) * 2 + 1] = s2;
                    }
                }
            }
        }
        drain_vm();
        lds_barrier();
        if (tid == 0 && last)
            for (int r = 0; r < RG && rb0 + r < R; ++r) arrive(a, kX2 + rb0 + r);
        CB_MARK(9);
    }
    // E: qkv(l+1): LN1 on the operand path, q + K/V of the token into layer
    // l+1's pages; unit (row block, 9 tiles)
    if (!a.last) {
        constexpr int RG = 1, T = 9, NE = RG * T * 64, NJ = 3 * NCT;
        const bool has = bid < R * NG_E;
        const int g = bid % NG_E, rb = bid / NG_E;
        uint4 wr[T][SPW];
        float4 bv[2];
        int kps[2], kpage[2];  // K/V destination (position, page), resolved while the weights stream
        auto kv_lane = [&](int i, int& row) __attribute__((always_inline)) {
            const int e = tid + i * NT;
            int col;
            where<T>(e, rb, g * T, row, col);
            return has && e < NE && row < a.B && col >= C && col < 3 * C;
        };
        auto pre = [&]() {
#pragma unroll
            for (int i = 0; i < 2; ++i) {  // positions ahead of the weights (vmcnt retires in order)
                int row;
                kps[i] = kv_lane(i, row) ? a.pos[row] : 0;
            }
            if (has) load_w<T>(a.w_qkv, K32, g * T, 0, w, wr, NJ - 1);
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int e = tid + i * NT;
                int row, col;
                where<T>(e, rb, g * T, row, col);
                bv[i] = has && e < NE && col < 3 * C ? ld4(a.b_qkv + col) : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                int row;
                kpage[i] = kv_lane(i, row) ? a.bt[(size_t)row * a.bt_stride + kps[i] / P] : -1;
            }
        };
        pre();
        if (!FIRST && !wait_lines(a, kX2 + rb, 1, has ? 1 : 0, NG_D, 4, sm)) return;
        CB_MARK(10);
        if (has) {
            f32x4 acc[RG][T];
            unit_mma<RG, T, true, FIRST>(a.res, K16, rb, R, 0, wr, a.ln1_w, a.ln1_b, sm, acc, &a, g == 0);
            put_red<RG, T>(sm.red, acc);
        }
        lds_barrier();
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int e = tid + i * NT;
            int row, col;
            where<T>(e, rb, g * T, row, col);
            if (has && e < NE && row < a.B && col < 3 * C)
                qkv_store<P, BF>(a, row, col, kps[i], kpage[i], add4(fold<RG, T>(sm.red, e), bv[i]));
        }
        CB_MARK(15);
    }
    CB_MARK(11);
}

int g_ncu_b16 = 0;
int num_cus_b16() {
    if (!g_ncu_b16) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess) return 0;
        hipDeviceProp_t pr;
        if (hipGetDeviceProperties(&pr, dev) != hipSuccess) return 0;
        g_ncu_b16 = pr.multiProcessorCount;
    }
    return g_ncu_b16;
}

template <int P, bool BF, bool FIRST = false>
int launch_b16(const HpaChainB16Args* h, int G, const int* tokens = nullptr, const float* wte = nullptr,
               const float* wpe = nullptr, void* zero = nullptr, size_t zero_bytes = 0) {
    static int resident = -1;
    if (resident < 0) {
        int nb = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, decode_chain_b16_kernel<P, BF, FIRST>, 512, 0) !=
            hipSuccess)
            nb = 0;
        resident = nb;
    }
    HPA_REQUIRE(resident >= 1, "decode chain bf16: the workgroup does not fit a CU");
    const HpaKVPool* pool = h->pool;
    cb::Args a;
    a.B = h->B;
    a.R = (h->B + 15) / 16;
    a.Mp = a.R * 16;
    a.last = h->last;
    a.layer = h->layer;
    a.att = h->att;
    a.res = h->res;
    a.res2 = h->res2;
    a.fch = h->fch;
    a.w_ap = reinterpret_cast<const uint4*>(h->w_ap);
    a.w_fc = reinterpret_cast<const uint4*>(h->w_fc);
    a.w_fp = reinterpret_cast<const uint4*>(h->w_fp);
    a.w_qkv = reinterpret_cast<const uint4*>(h->w_qkv);
    a.b_ap = h->b_ap;
    a.ln2_w = h->ln2_w;
    a.ln2_b = h->ln2_b;
    a.b_fc = h->b_fc;
    a.b_fp = h->b_fp;
    a.ln1_w = h->ln1_w;
    a.ln1_b = h->ln1_b;
    a.b_qkv = h->b_qkv;
    a.q_out = h->q_out;
    a.kv_next = h->last ? nullptr : (char*)pool->base + (size_t)(h->layer + 1) * pool->layer_elems * pool->elem_bytes;
    a.page_elems = pool->page_elems;
    a.bt = h->block_table;
    a.bt_stride = h->bt_stride;
    a.pos = h->pos;
    a.stats_out = h->stats_out;
    a.stats_mp = h->stats_mp > 0 ? h->stats_mp : a.Mp;
    a.slab = h->slab;
    a.ctr = h->counters;
    a.err = h->err;
    a.err_sticky = h->err_sticky;
    a.tokens = tokens;
    a.wte = wte;
    a.wpe = wpe;
    a.zero = reinterpret_cast<int4*>(zero);
    a.zero_n4 = (int)(zero_bytes / 16);
    decode_chain_b16_kernel<P, BF, FIRST><<<G, 512, 0, hpa_stream()>>>(a);
    HPA_LAUNCH_CHECK();
    return 0;
}

}  // namespace

extern "C" {

int hpa_decode_chain_b16_eligible(int B, int C, int num_heads) {
    const int G = num_cus_b16();
    const int R = (B + 15) / 16;
    const int RH = (R + 1) / 2, RQ = (R + 3) / 4;
    // every phase's units on a workgroup each
    return G > 0 && C == 768 && num_heads == 12 && B >= 1 && B <= 256 && R * cb::NG_B <= G && RH * cb::NG_C <= G &&
                   RQ * 4 * cb::NG_D <= G
               ? 1
               : 0;
}

int hpa_decode_chain_b16_sizes(int B, size_t* out2) {
    HPA_REQUIRE(out2 && B >= 1 && B <= 256, "decode chain bf16 sizes: 1..256 rows");
    const int R = (B + 15) / 16, RQ = (R + 3) / 4;
    out2[0] = (size_t)4 * RQ * cb::NG_D * 4 * 3 * 256;  // fcproj K-part partial tiles (floats)
    out2[1] = (size_t)cb::kLines * cb::kPad;            // counter ints per layer
    return 0;
}

// trace build only (as hpa_decode_layer_trace): the bf16 chain's stamps
int hpa_decode_chain_b16_trace(unsigned long long* host, int layers) {
#ifdef HPA_LAYER_TRACE
    HPA_REQUIRE(layers >= 0 && layers <= 64, "trace: layers 0..64");
    if (!host) {
        static unsigned long long zero[64 * 256 * 16];
        HPA_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(cb::g_cb_trace), zero, sizeof(zero)));
        return 0;
    }
    HPA_CHECK(hipMemcpyFromSymbol(host, HIP_SYMBOL(cb::g_cb_trace), (size_t)layers * 256 * 16 * 8));
    return 0;
#else
    (void)host;
    (void)layers;
    return 1;
#endif
}

int hpa_decode_chain_b16_first(const HpaChainB16Args* h, const int* tokens, const float* wte, const float* wpe,
                               void* zero, size_t zero_bytes) {
    HPA_REQUIRE(h && h->pool && h->pool->base && tokens && wte && wpe, "decode chain bf16 first: null operand");
    const HpaKVPool* pool = h->pool;
    HPA_REQUIRE(pool->dtype == HPA_F32 || pool->dtype == HPA_BF16, "decode chain bf16 first: fp32 or bf16 pool");
    HPA_REQUIRE(pool->head_size == 64 && pool->num_heads == 12, "decode chain bf16 first: 12 heads of 64");
    HPA_REQUIRE(hpa_decode_chain_b16_eligible(h->B, 768, 12), "decode chain bf16 first: 1..256 rows");
    HPA_REQUIRE(h->res && h->w_qkv && h->b_qkv && h->ln1_w && h->ln1_b && h->q_out && h->block_table && h->pos,
                "decode chain bf16 first: null operand");
    HPA_REQUIRE(zero_bytes % 16 == 0 && ((size_t)zero & 15) == 0 && zero_bytes / 16 <= 0x7fffffff,
                "decode chain bf16 first: the zeroed block must be whole 16-byte granules");
    HpaChainB16Args f = *h;
    f.layer = -1;  // K/V into layer 0's pages (layer + 1)
    f.last = 0;
    const int G = num_cus_b16();
    const bool bf = pool->dtype == HPA_BF16;
    switch (pool->page_size) {
        case 8: return bf ? launch_b16<8, true, true>(&f, G, tokens, wte, wpe, zero, zero_bytes)
                          : launch_b16<8, false, true>(&f, G, tokens, wte, wpe, zero, zero_bytes);
        case 16: return bf ? launch_b16<16, true, true>(&f, G, tokens, wte, wpe, zero, zero_bytes)
                           : launch_b16<16, false, true>(&f, G, tokens, wte, wpe, zero, zero_bytes);
        case 32: return bf ? launch_b16<32, true, true>(&f, G, tokens, wte, wpe, zero, zero_bytes)
                           : launch_b16<32, false, true>(&f, G, tokens, wte, wpe, zero, zero_bytes);
        case 64: return bf ? launch_b16<64, true, true>(&f, G, tokens, wte, wpe, zero, zero_bytes)
                           : launch_b16<64, false, true>(&f, G, tokens, wte, wpe, zero, zero_bytes);
        default: return hpa_fail(__FILE__, __LINE__, "decode chain bf16 first: page size must be 8, 16, 32 or 64");
    }
}

int hpa_decode_chain_b16(const HpaChainB16Args* h) {
    HPA_REQUIRE(h && h->pool && h->pool->base, "decode chain bf16: pool");
    const HpaKVPool* pool = h->pool;
    HPA_REQUIRE(pool->dtype == HPA_F32 || pool->dtype == HPA_BF16, "decode chain bf16: fp32 or bf16 pool");
    HPA_REQUIRE(pool->head_size == 64 && pool->num_heads == 12, "decode chain bf16: 12 heads of 64");
    HPA_REQUIRE(hpa_decode_chain_b16_eligible(h->B, 768, 12), "decode chain bf16: 1..256 rows, a unit per workgroup");
    HPA_REQUIRE(h->layer >= 0 && h->layer < pool->num_layers && (h->last || h->layer + 1 < pool->num_layers),
                "decode chain bf16: layer out of range");
    HPA_REQUIRE(h->att && h->res && h->res2 && h->fch && h->w_ap && h->b_ap && h->ln2_w && h->ln2_b && h->w_fc &&
                    h->b_fc && h->w_fp && h->b_fp && h->block_table && h->pos && h->slab && h->counters && h->err,
                "decode chain bf16: null operand");
    HPA_REQUIRE(h->last || (h->w_qkv && h->b_qkv && h->ln1_w && h->ln1_b && h->q_out),
                "decode chain bf16: qkv(l+1) operands");
    const int G = num_cus_b16();
    const bool bf = pool->dtype == HPA_BF16;
    switch (pool->page_size) {
        case 8: return bf ? launch_b16<8, true>(h, G) : launch_b16<8, false>(h, G);
        case 16: return bf ? launch_b16<16, true>(h, G) : launch_b16<16, false>(h, G);
        case 32: return bf ? launch_b16<32, true>(h, G) : launch_b16<32, false>(h, G);
        case 64: return bf ? launch_b16<64, true>(h, G) : launch_b16<64, false>(h, G);
        default: return hpa_fail(__FILE__, __LINE__, "decode chain bf16: page size must be 8, 16, 32 or 64");
    }
}

}  // extern "C"
