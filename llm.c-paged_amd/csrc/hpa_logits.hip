// hpa_logits.hip -- the logits GEMM (paged_infer.c:727 matmul_forward of
// LNf(residual) by wte, argmax partials for the greedy pick :937-951) as a
// weight-streaming, activation-resident kernel for GPT-2 124M shapes
// (K = C = 768, rows <= 64, N = V = 50257).
//
// Why a kernel of its own: the logits are fp32-MFMA bound (4.94 GFLOP, 31 us
// at 157 TF/s) over 154 MB of wte.  The looped fused GEMM re-reads the
// activation tile for every column tile (308 MB through L2 for 154 MB of
// weights) and keeps one trip in flight per wave, so its waves wait on memory
// half of their lifetime (PMC: SQ_WAIT_INST_ANY 50 % of SQ_WAVE_CYCLES, MFMA
// busy 42 %).  Here:
//   * one persistent workgroup of 8 waves per CU; wave w owns k-steps
//     [6w, 6w+6) of K16 = 48 and holds LNf(x) of all rows for them in 96
//     VGPRs, loaded and normalised once;
//   * the workgroup walks column tiles bid, bid + grid, ...; per tile a wave
//     streams 6 KiB of wte (non-temporal: every byte read once) for the next
//     tile while its 96 MFMAs of the current one run;
//   * the 8 waves' partial tiles fold through double-buffered LDS in wave
//     order (one barrier per tile); each row's 16 columns sit in 16 adjacent
//     lanes, so the per-tile (max, argmax) is four xor-shuffles, and a
//     running (max, argmax) over the workgroup's tiles (visited in increasing
//     column order, strict > keeps the first max) leaves ONE partial per row
//     per workgroup: argmax_final then reads G x rows partials (G = grid)
//     instead of 3142 x rows strided ones (it fetched 12.9 MB for 1.6 MB).
// A row's K order is fixed (8 slices of 96, folded in wave order), so the
// results do not depend on the grid or the batch.  Measured (config 2): 16
// waves of 3 k-steps 62.7 us per launch, of which the LDS fold was ~30 us
// that the MFMAs could not hide (tools/logits_exp.sh: 33.9 us without the
// fold, 36.6 us without the MFMAs); 8 waves halve the fold.
#include <type_traits>

#include "hpa_gemm_body.h"
#ifndef HPA_RES_EXP
#define HPA_RES_EXP 0  // timing experiments (tools/logits_exp.sh); 0 in the product
#endif
// A/B build knobs of the ring form (tools/r4_pick.sh, profiles/r4/logits_walk.txt):
#ifndef HPA_RG_STRIDED
#define HPA_RG_STRIDED 0  // 0: a contiguous run of tiles per workgroup; 1: tiles b, b + G, ... (round 3)
#endif
#ifndef HPA_RG_PRO
#define HPA_RG_PRO 1  // prologue DMAs: 0 tiles 0, 1 at the start; 1 tile 1 after the first barrier; 2 both after it
#endif
#ifndef HPA_RES_NW
#define HPA_RES_NW 16  // waves per workgroup (16: 3 k-steps each, 8: 6)
#endif

namespace hpa_gemm {
namespace {

constexpr int kResNW = HPA_RES_NW;  // waves per workgroup
constexpr int kResS = 48 / kResNW;  // k-steps (of 16) per wave: K16 = 48

__device__ __forceinline__ float4 load_nt4(const float4* ptr) {
    typedef float v4 __attribute__((ext_vector_type(4)));
    const v4 v = __builtin_nontemporal_load(reinterpret_cast<const v4*>(ptr));
    return make_float4(v.x, v.y, v.z, v.w);
}

template <int CTRL>
__device__ __forceinline__ void dpp_argmax(float& bv, int& bi) {
    const float v2 = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(bv), CTRL, 0xF, 0xF, false));
    const int i2 = __builtin_amdgcn_mov_dpp(bi, CTRL, 0xF, 0xF, false);
    const bool take = v2 > bv || (v2 == bv && i2 < bi);
    bv = take ? v2 : bv;
    bi = take ? i2 : bi;
}

// the launch's final pick (HpaFusedGemm.pick_*): every workgroup has stored
// its per-row (max, column) partial write-through; after the drain each draws
// an arrival ticket, and the last reduces the G partials of every row as
// argmax_final_kernel (hpa_fused.hip) does -- the largest value, the lowest
// column among equals, 0 for a row with no finite maximum -- with sc1 loads
// (MI355X_MICROARCH.md "Valid forms" row 1, as the attention's split merge).
// Lane = row, so a wave's load of partial t is one contiguous 8*Mp-byte run;
// wave w takes t = w, w + NWAVES, ..., and the waves' bests fold through
// `scratch` (NWAVES * 64 * 2 words of the kernel's idle LDS) in wave order.
template <int NWAVES>
__device__ __forceinline__ void final_pick(const FG& p, float* scratch) {
    __shared__ int s_last;
    const int G = gridDim.x;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this thread's partial store has landed
    __syncthreads();
    if (threadIdx.x == 0)
        s_last = __hip_atomic_fetch_add(p.pick_count, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == G - 1;
    __syncthreads();
    if (!s_last) return;
    if (threadIdx.x == 0) __hip_atomic_store(p.pick_count, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int m = min(lane, p.Mp - 1);
    const __amdgpu_buffer_rsrc_t rs = hpa::wt_rsrc(p.part_out);
    float bv = -INFINITY;
    int bi = 0x7fffffff;
    for (int t0 = w; t0 < G; t0 += 8 * NWAVES) {  // 8 partials per lane in flight
        u32x2 v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int t = min(t0 + j * NWAVES, G - 1);
            v[j] = __builtin_amdgcn_raw_buffer_load_b64(rs, (t * p.Mp + m) * 8, 0, hpa::kCpolSc1);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float fv = __uint_as_float(v[j].x);
            const int fi = (int)v[j].y;
            const bool take = t0 + j * NWAVES < G && (fv > bv || (fv == bv && fi < bi));
            bv = take ? fv : bv;
            bi = take ? fi : bi;
        }
    }
    scratch[(w * 64 + lane) * 2] = bv;
    scratch[(w * 64 + lane) * 2 + 1] = __int_as_float(bi);
    __syncthreads();
    if (w == 0 && lane < p.M) {
#pragma unroll
        for (int k = 1; k < NWAVES; ++k) {
            const float v2 = scratch[(k * 64 + lane) * 2];
            const int i2 = __float_as_int(scratch[(k * 64 + lane) * 2 + 1]);
            const bool take = v2 > bv || (v2 == bv && i2 < bi);
            bv = take ? v2 : bv;
            bi = take ? i2 : bi;
        }
        const int id = bi == 0x7fffffff ? 0 : bi;
        p.pick_next[lane] = id;
        if (p.pick_tokens) p.pick_tokens[lane] = id;
        if (p.pick_pos) p.pick_pos[lane] += 1;
    }
}

template <int MT>
constexpr int resident_lds_floats() {
    return 2 * kResNW * MT * 256 + 10 * MT * 16;
}

template <int MT>
__global__ __launch_bounds__(kResNW * 64) void logits_resident_kernel(FG p) {
    constexpr int R = MT * 16;
    constexpr int S = kResS;
    __shared__ __attribute__((aligned(16))) float smem[resident_lds_floats<MT>()];
    float* red = smem;                        // [2][16 waves][MT x 4 reg][64 lanes]
    float* lnst = red + 2 * kResNW * MT * 256; // [R][2] mean, rstd
    float* lnscr = lnst + 2 * R;              // [4R][2]
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const int q4 = lane >> 4;
    const int kb0 = w * S;

    // first tile's weights in flight during the LN prologue
    int t = blockIdx.x;
    // three register sets rotate by name (unrolled by 3, never copied): the
    // current tile's weights and the next two tiles' loads in flight
    float4 w0[S], w1[S], w2[S];
    const float4* __restrict__ wbase = reinterpret_cast<const float4*>(p.w) + (size_t)kb0 * 64 + lane;
    const size_t tstride = (size_t)p.K16 * 64;
    if (t < p.ntn) {
#pragma unroll
        for (int s = 0; s < S; ++s) w0[s] = load_nt4(wbase + (size_t)t * tstride + s * 64);
        const int t1 = min(t + (int)gridDim.x, p.ntn - 1);
#pragma unroll
        for (int s = 0; s < S; ++s) w1[s] = load_nt4(wbase + (size_t)t1 * tstride + s * 64);
    }
    // activations of this wave's k range, all row blocks
    float4 a[MT][S];
    const float4* __restrict__ xf = reinterpret_cast<const float4*>(p.x) + (size_t)kb0 * 64 + lane;
    const size_t rbs = (size_t)p.K16 * 64;
#pragma unroll
    for (int r = 0; r < MT; ++r)
#pragma unroll
        for (int s = 0; s < S; ++s) a[r][s] = xf[r * rbs + s * 64];

    // LNf statistics of the R rows: the same partial-sum order as gemm16_body
    if (threadIdx.x < 4 * R) {
        const int r = threadIdx.x >> 2, q = threadIdx.x & 3;
        float s1 = 0.f, s2 = 0.f;
        if (r < p.M) {
            for (int t0 = q; t0 < p.ln_ntiles; t0 += 32) {
                float x1[8], x2[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int tt = min(t0 + 4 * j, p.ln_ntiles - 1);
                    x1[j] = p.ln_stats[((size_t)tt * p.Mp + r) * 2];
                    x2[j] = p.ln_stats[((size_t)tt * p.Mp + r) * 2 + 1];
                }
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    if (t0 + 4 * j < p.ln_ntiles) {
                        s1 += x1[j];
                        s2 += x2[j];
                    }
            }
        }
        lnscr[2 * threadIdx.x] = s1;
        lnscr[2 * threadIdx.x + 1] = s2;
    }
    __syncthreads();
    if (threadIdx.x < R) {
        const float* tt = lnscr + 8 * threadIdx.x;
        const float s1 = (tt[0] + tt[2]) + (tt[4] + tt[6]);
        const float s2 = (tt[1] + tt[3]) + (tt[5] + tt[7]);
        const float m = s1 / p.K;
        const float v = fmaxf(s2 / p.K - m * m, 0.f);
        lnst[2 * threadIdx.x] = m;
        lnst[2 * threadIdx.x + 1] = 1.0f / sqrtf(v + 1e-5f);
    }
    __syncthreads();
    {
        const float4* gw = reinterpret_cast<const float4*>(p.ln_w);
        const float4* gb = reinterpret_cast<const float4*>(p.ln_b);
#pragma unroll
        for (int s = 0; s < S; ++s) {
            const float4 g = gw[4 * (kb0 + s) + q4], b = gb[4 * (kb0 + s) + q4];
#pragma unroll
            for (int r = 0; r < MT; ++r)
                a[r][s] = ln4(a[r][s], lnst[2 * (16 * r + (lane & 15))], lnst[2 * (16 * r + (lane & 15)) + 1], g, b);
        }
    }

    // fold element e = threadIdx.x (< MT*256): row block e>>8, C register
    // (e>>6)&3, lane e&63 -> row 16*(e>>8) + 4*((e&63)>>4) + ((e>>6)&3),
    // column e&15 of the tile; a row's 16 columns are 16 adjacent lanes
    // stores through buffer descriptors: lanes out of range get an offset past
    // num_records and the hardware drops them, so every memory instruction of
    // the loop is unconditional and the compiler's vmcnt before the weight
    // hand-over (wv = wn) leaves this tile's stores in flight (with branches
    // around them it waits for vmcnt(0): a store round trip per tile)
    const __amdgpu_buffer_rsrc_t out_rs =
        __builtin_amdgcn_make_buffer_rsrc(p.out, 0, (int)((size_t)p.M * p.N * 4), 0x00020000);
    const __amdgpu_buffer_rsrc_t part_rs =
        __builtin_amdgcn_make_buffer_rsrc(p.part_out, 0, (int)((size_t)p.ntn * p.Mp * 8), 0x00020000);
    constexpr int kDrop = 0x7ffffff0;
    int it = 0;
    float run_v = -INFINITY;  // this workgroup's running (max, argmax) of row frow (fcol == 0 lanes)
    int run_i = 0x7fffffff;
    auto step = [&](float4 (&wv)[S], float4 (&wn2)[S]) __attribute__((always_inline)) {
#if HPA_RES_EXP == 3
        const int tn2 = t;  // timing experiment: re-read the same tile (L2 hits)
#else
        const int tn2 = min(t + 2 * (int)gridDim.x, p.ntn - 1);  // past the end: a harmless repeat load
#endif
#pragma unroll
        for (int s = 0; s < S; ++s) wn2[s] = load_nt4(wbase + (size_t)tn2 * tstride + s * 64);
        f32x4 acc[MT];
#pragma unroll
        for (int r = 0; r < MT; ++r) acc[r] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < S; ++s)
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int r = 0; r < MT; ++r) {
                    const float xs = q == 0 ? a[r][s].x : q == 1 ? a[r][s].y : q == 2 ? a[r][s].z : a[r][s].w;
                    const float ws = q == 0 ? wv[s].x : q == 1 ? wv[s].y : q == 2 ? wv[s].z : wv[s].w;
#if HPA_RES_EXP == 1
                    acc[r][0] += xs * ws;  // timing experiment: no MFMA
#else
                    acc[r] = __builtin_amdgcn_mfma_f32_16x16x4f32(xs, ws, acc[r], 0, 0, 0);
#endif
                }
#if HPA_RES_EXP == 2
        if (acc[0][0] == 1.2345f) p.out[threadIdx.x] = acc[MT - 1][3];  // timing experiment: no fold
        t += gridDim.x;
        ++it;
        return;
#endif
        // fold the waves' partial tiles in wave order (double-buffered:
        // one barrier per tile)
        float* rb = red + (it & 1) * (kResNW * MT * 256);
#pragma unroll
        for (int r = 0; r < MT; ++r)
#pragma unroll
            for (int g = 0; g < 4; ++g) rb[w * MT * 256 + (r * 4 + g) * 64 + lane] = acc[r][g];
        __syncthreads();
        for (int e = threadIdx.x; e < MT * 256; e += kResNW * 64) {  // whole waves (multiples of 64)
            const int frow = 16 * (e >> 8) + 4 * ((e & 63) >> 4) + ((e >> 6) & 3);
            const int fcol = e & 15;
            float part[kResNW];  // all partials in flight at once, then the fixed-order sum
#pragma unroll
            for (int ww = 0; ww < kResNW; ++ww) part[ww] = rb[ww * MT * 256 + e];
            float val = part[0];
#pragma unroll
            for (int ww = 1; ww < kResNW; ++ww) val += part[ww];
            const int col = t * 16 + fcol;
            const bool live = frow < p.M && col < p.N;
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(val), out_rs,
                                                  live ? (frow * p.N + col) * 4 : kDrop, 0, 0);
            // per-tile (max, argmax) of the row: first max wins (paged_infer.c:937-951)
            float bv = live ? val : -INFINITY;
            int bi = fcol;
            // butterfly over the 16 lanes of the row with DPP (no LDS): mirror
            // within 16, mirror within 8, then quad xor 2 and xor 1 cover all
            // 16 lanes; (max, lowest index) is order-independent
            dpp_argmax<0x140>(bv, bi);  // row_mirror
            dpp_argmax<0x141>(bv, bi);  // row_half_mirror
            dpp_argmax<0x4E>(bv, bi);   // quad_perm [2,3,0,1]
            dpp_argmax<0xB1>(bv, bi);   // quad_perm [1,0,3,2]
            if (bv > run_v) {  // tiles in increasing column order: the first max stays
                run_v = bv;
                run_i = t * 16 + bi;
            }
        }
        t += gridDim.x;
        ++it;
    };
    while (t < p.ntn) {
        step(w0, w2);
        if (t >= p.ntn) break;
        step(w1, w0);
        if (t >= p.ntn) break;
        step(w2, w1);
    }
    // one partial per row: slot blockIdx.x of part_out ([G][Mp][2])
    const int e = threadIdx.x;
    if (e < MT * 256) {
        const int frow = 16 * (e >> 8) + 4 * ((e & 63) >> 4) + ((e >> 6) & 3);
        if ((e & 15) == 0 && frow < p.Mp) {
            typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
            const u32x2 pv = {__float_as_uint(run_v), (unsigned int)run_i};
            __builtin_amdgcn_raw_buffer_store_b64(pv, part_rs, ((int)blockIdx.x * p.Mp + frow) * 8, 0, hpa::kCpolSc1);
        }
    }
    if (p.pick_next) final_pick<kResNW>(p, red);  // the fold buffers are idle now
}

// ---- ring form (round 3, the default): rows split over waves, wte through
// an LDS ring filled by dedicated loader waves ----
// The 16-wave form above splits K over 16 waves, so every 16x16 output tile
// is folded from 16 partial tiles through LDS behind a barrier that all
// waves reach together, and every wave also streams its own wte fragments:
// the matrix pipes idle through each fold (MFMA busy 50 %,
// profiles/r3/mfma_c2.txt).  Here:
//   * 8 computing waves (2 per SIMD) split the ROWS: at 64 rows wave w owns
//     row block w & 3 and K parts {2h, 2h+1} (h = w >> 2) of the 4 parts of
//     192, i.e. 96 VGPRs of LNf(x), one accumulator per part (two MFMA chains);
//   * 4 loader waves stream each 48 KiB column tile of wte ONCE per workgroup
//     into a 3-stage LDS ring by LDS-DMA (global_load_lds_dwordx4, non-
//     temporal), two tiles ahead, and do nothing else: a wave issuing into
//     the saturated per-CU memory queue stalls at issue (~0.25 us per 1 KiB
//     instruction, tools/rg_trace.py), so no computing wave issues a load;
//   * the computing waves read their B fragments from the ring (ds_read_b128);
//   * a tile's result is (p0 + p1) + (p2 + p3) over the 4 K parts: the wave
//     of h = 1 publishes (p2 + p3) (1 KiB) into a double-buffered fold slot;
//     the owner (h = 0) adds it in the NEXT iteration, after that
//     iteration's one barrier, so the epilogue (store, running argmax)
//     overlaps the partner's MFMAs; the per-row argmax keeps a running
//     (max, column) per lane and reduces the 16 lanes once at the end.
// Fewer rows (16 / 32) keep the same per-row arithmetic: one part per wave
// and three published partials, summed in the same order, so a row's logits
// are bit-identical at every batch size (sharded decode = unsharded).
// Measured (tools/rg_trace.py, s_memtime): per tile the computing waves take
// 3.35 us (6144 MFMA cycles per SIMD = 2.98 us at the 2.06 GHz the chip holds
// under this load), the loaders' 48 KiB DMA 3.15 us (15 GB/s per CU beside
// the MFMAs, 25 alone): 3.64 us per iteration, 57.5 us per launch.
// Round 4 (profiles/r4/logits_walk.txt): a workgroup walks a contiguous run of
// tiles (the round-3 walk b, b + G, ... wrote 18.6 MB for 12.9 MB of logits:
// V is odd, so every row segment of a tile shares its end sectors with the
// neighbouring tiles, written from another XCD; now 13.5 MB), loads nothing
// past its run (the walk used to re-load its last tile twice), and issues tile
// 1's DMA after the prologue's activation loads (prologue 5.9 vs 6.8 us); the
// iteration (3.7 us) is MFMA-bound as before.
// diagnostic build (-DHPA_RG_TRACE, tools/rg_trace.py): stamps per workgroup
// -- [0] start, [1] prologue done, [2..15] iteration starts (after the
// barrier), [16] loop end, [17] end -- as s_memrealtime (10 ns) and
// s_memtime (shader clock); sums over the iterations (10 ns ticks): [18]
// wave 4 (a loader) in its vmcnt wait, [19] wave 0 in the barrier, [20]
// wave 0 and [21] wave 4 from the barrier to their fold write; never in the
// product library
#ifdef HPA_RG_TRACE
__device__ unsigned long long g_rg_trace[2][256][24];
#define RG_MARK(k)                                                                                     \
    do {                                                                                               \
        if (threadIdx.x == 0 && blockIdx.x < 256) {                                                    \
            g_rg_trace[0][blockIdx.x][k] = (unsigned long long)__builtin_amdgcn_s_memrealtime();       \
            g_rg_trace[1][blockIdx.x][k] = (unsigned long long)__builtin_amdgcn_s_memtime();           \
        }                                                                                              \
    } while (0)
#else
#define RG_MARK(k) \
    do {           \
    } while (0)
#endif
constexpr int kRgNC = 8;                 // computing waves (2 per SIMD)
constexpr int kRgNW = 12;                // + 4 loader waves
constexpr int kRgK16 = 48;               // K = 768
constexpr int kRgPart = 12;              // k16-steps per K part (4 parts)
constexpr int kRgTileF = kRgK16 * 256;   // floats per 16-column wte tile (48 KiB)
constexpr int kRgLoaders = kRgNW - kRgNC;    // waves kRgNC .. kRgNW-1 load the ring
constexpr int kRgDma = kRgK16 / kRgLoaders;  // LDS-DMA wave-instructions per loader per tile
constexpr int kRgFoldF = 1536;           // floats per fold buffer (max over MT)
constexpr int kRgStages = 3;
constexpr int kRgLdsF = kRgStages * kRgTileF + 2 * kRgFoldF + 10 * 64;
static_assert(kRgLdsF * 4 <= 160 * 1024, "LDS");
static_assert(kRgPart % kRgDma == 0, "DMAs spread evenly over the k-steps");

template <int MT>
struct RgShape {
    static constexpr int MTS = MT == 3 ? 4 : MT;  // row-block slots
    static constexpr int NPW = MTS == 4 ? 2 : 1;  // K parts per wave
    static constexpr int NWC = MTS * 4 / NPW;     // computing waves: 4 (MT 1) or 8
    static_assert(NWC <= kRgNC, "compute waves");
    static constexpr int NSLOT = 4 / NPW - 1;     // published partials per row block
    static_assert(MTS * NSLOT * 256 <= kRgFoldF, "fold buffer");

};

// LDS-DMA of 1 KiB (16 B per lane to lds_addr + 16 * lane), non-temporal.
// Inline asm, so hipcc does not see it: with the builtin it waits vmcnt(0)
// before every ds_read of the ring (it cannot tell the stages apart), which
// drains the prefetch; the kernel counts these loads itself.
__device__ __forceinline__ void rg_dma(const float* src, unsigned lds_addr) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src), "s"(lds_addr)
                 : "memory");
}

// (max, lowest index) step of the per-row butterfly, branch-free
template <int CTRL>
__device__ __forceinline__ void rg_argmax(float& bv, int& bi) {
    const float v2 = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(bv), CTRL, 0xF, 0xF, false));
    const int i2 = __builtin_amdgcn_mov_dpp(bi, CTRL, 0xF, 0xF, false);
    const bool take = (v2 > bv) | ((v2 == bv) & (i2 < bi));
    bv = take ? v2 : bv;
    bi = take ? i2 : bi;
}

template <int MT>
__global__ __launch_bounds__(kRgNW * 64) void logits_ring_kernel(FG p) {
    using S = RgShape<MT>;
    constexpr int NPW = S::NPW;
    constexpr int R = MT * 16;
    __shared__ __attribute__((aligned(16))) float smem[kRgLdsF];
    float* ring = smem;                          // [3][48 k16][64 lanes][4]
    float* fold = smem + kRgStages * kRgTileF;   // [2][row block][slot][64 lanes][4]
    float* lnst = fold + 2 * kRgFoldF;           // [R][2] mean, rstd
    float* lnscr = lnst + 2 * 64;                // [4R][2]
    float* lngb = ring + 2 * kRgTileF;           // prologue only: LNf gamma, beta (stage 2 is idle)
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int r = w % S::MTS;                  // row block
    const int h = (w / S::MTS) % (4 / NPW);    // part group
    const bool rvalid = w < S::NWC && r < MT;
    const bool owner = rvalid && h == 0;
    const bool loader = w >= kRgNW - kRgLoaders;
    const int G = gridDim.x;
    const int ntn = p.ntn;
#if HPA_RG_STRIDED
    int t = blockIdx.x;  // tiles b, b + G, ...
    constexpr int tstep = 0;
    const int tend = ntn;
#else
    // a contiguous run of column tiles per workgroup (the first ntn % G take
    // one more): a row's 64-byte segments of neighbouring tiles share 32-byte
    // sectors (V is odd, so rows are not sector aligned), and written from
    // one L2 in consecutive iterations they merge there instead of leaving
    // as partial-sector writes from different XCDs
    const int tq = ntn / G, trm = ntn % G;
    int t = (int)blockIdx.x * tq + min((int)blockIdx.x, trm);
    constexpr int tstep = 1;
    const int tend = t + tq + ((int)blockIdx.x < trm ? 1 : 0);
#endif
    const int TS = tstep ? 1 : G;  // tile stride of the walk

    const float* wl = p.w + lane * 4 + (w - (kRgNW - kRgLoaders)) * 256;  // loaders: their 1 KiB chunks
    const unsigned ring_lds = __builtin_amdgcn_readfirstlane(
        (unsigned)(size_t)(__attribute__((address_space(3))) float*)ring);
    // loader chunk j of a tile = k16-step (w - 4) + 4 j
    auto dma_src = [&](int tile) __attribute__((always_inline)) {
        return wl + (size_t)tile * kRgTileF;  // tile < tend: nothing is loaded past the workgroup's tiles
    };
    auto dma_dst = [&](int stage) __attribute__((always_inline)) {
        return ring_lds + (unsigned)(stage * kRgTileF + (w - (kRgNW - kRgLoaders)) * 256) * 4;
    };
    RG_MARK(0);
    // the loaders' DMA of tile t + d * TS (d = 0, 1) into stage d, if the walk has it
    auto dma_pro = [&](int d) __attribute__((always_inline)) {
        if (t + d * TS < tend) {
            const float* src = dma_src(t + d * TS);
            const unsigned dst = dma_dst(d);
#pragma unroll
            for (int j = 0; j < kRgDma; ++j) rg_dma(src + kRgLoaders * j * 256, dst + kRgLoaders * j * 1024);
        }
    };
    if (loader && HPA_RG_PRO < 2) dma_pro(0);  // lands during the LN prologue (the loaders take no part in it)
    if (loader && HPA_RG_PRO < 1) dma_pro(1);

    // prologue loads, all in flight together: LNf statistics partials, the
    // wave's raw activations, LNf gamma / beta (into LDS)
    if (threadIdx.x < 4 * R) {
        // the same partial-sum order as gemm16_body: thread (row, q) sums
        // tiles q, q + 4, ..., q + 44 in order (K = 768: 48 tiles)
        const int rr = threadIdx.x >> 2, q = threadIdx.x & 3;
        float s1 = 0.f, s2 = 0.f;
        if (rr < p.M) {
            float2 xs[kRgK16 / 4];
            const float2* ls = reinterpret_cast<const float2*>(p.ln_stats) + rr;
#pragma unroll
            for (int j = 0; j < kRgK16 / 4; ++j) xs[j] = ls[(size_t)(q + 4 * j) * p.Mp];
#pragma unroll
            for (int j = 0; j < kRgK16 / 4; ++j) {
                s1 += xs[j].x;
                s2 += xs[j].y;
            }
        }
        lnscr[2 * threadIdx.x] = s1;
        lnscr[2 * threadIdx.x + 1] = s2;
    }
    if (threadIdx.x < 2 * kRgK16 * 4) {  // 192 float4 of gamma, then 192 of beta
        const float4* src = reinterpret_cast<const float4*>(threadIdx.x < kRgK16 * 4 ? p.ln_w : p.ln_b);
        reinterpret_cast<float4*>(lngb)[threadIdx.x] = src[threadIdx.x % (kRgK16 * 4)];
    }
    float4 a[NPW][kRgPart];
    {
        const float4* xf = reinterpret_cast<const float4*>(p.x) + (size_t)r * kRgK16 * 64 + lane;
        if (rvalid) {
#pragma unroll
            for (int j = 0; j < NPW; ++j)
#pragma unroll
                for (int i = 0; i < kRgPart; ++i) a[j][i] = xf[((h * NPW + j) * kRgPart + i) * 64];
        } else {
#pragma unroll
            for (int j = 0; j < NPW; ++j)
#pragma unroll
                for (int i = 0; i < kRgPart; ++i) a[j][i] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }
    __syncthreads();
    if (loader && HPA_RG_PRO >= 2) dma_pro(0);  // behind the activation loads in the CU's memory queue
    if (loader && HPA_RG_PRO >= 1) dma_pro(1);
    if (threadIdx.x < R) {
        const float* tt = lnscr + 8 * threadIdx.x;
        const float s1 = (tt[0] + tt[2]) + (tt[4] + tt[6]);
        const float s2 = (tt[1] + tt[3]) + (tt[5] + tt[7]);
        const float m = s1 / p.K;
        const float v = fmaxf(s2 / p.K - m * m, 0.f);
        lnst[2 * threadIdx.x] = m;
        lnst[2 * threadIdx.x + 1] = 1.0f / sqrtf(v + 1e-5f);
    }
    __syncthreads();
    if (rvalid) {
        const float4* gw = reinterpret_cast<const float4*>(lngb);
        const float4* gb = gw + kRgK16 * 4;
        const int q4 = lane >> 4;
        const float mu = lnst[2 * (16 * r + (lane & 15))], rs = lnst[2 * (16 * r + (lane & 15)) + 1];
#pragma unroll
        for (int j = 0; j < NPW; ++j)
#pragma unroll
            for (int i = 0; i < kRgPart; ++i) {
                const int k16 = (h * NPW + j) * kRgPart + i;
                a[j][i] = ln4(a[j][i], mu, rs, gw[4 * k16 + q4], gb[4 * k16 + q4]);
            }
    }
    // the loaders' tile 0 is waited for by iteration 0's counted vmcnt (tile
    // 1's 12 DMAs still in flight), tile 1 by iteration 1's.  Stage 2 (gamma,
    // beta) is first overwritten by iteration 0's DMA, after its barrier.
    RG_MARK(1);

    const __amdgpu_buffer_rsrc_t out_rs =
        __builtin_amdgcn_make_buffer_rsrc(p.out, 0, (int)((size_t)p.M * p.N * 4), 0x00020000);
    constexpr int kDrop = 0x7fffff00;
    const int rbase = 16 * r + 4 * (lane >> 4);  // rows of this lane's 4 accumulator registers
    float run_v[4];  // per lane: running (max, column) of rows rbase + g over this workgroup's tiles
    int run_i[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        run_v[g] = -INFINITY;
        run_i[g] = 0x7fffffff;
    }
    f32x4 pend = f32x4{0.f, 0.f, 0.f, 0.f};  // this owner's (p0 + p1) of the previous tile
    const float* myfold = fold + (r * S::NSLOT) * 256 + lane * 4;

    // owners: epilogue of tile tp (fold buffer fb) -- the fixed-order sum,
    // the store, the per-lane running (max, column)
    auto epilogue = [&](int tp, int fb, bool any) __attribute__((always_inline)) {
        const int col = tp * 16 + (lane & 15);
        const float* fs = myfold + fb * kRgFoldF;
        f32x4 v;
        if constexpr (NPW == 2) {
            v = pend + *reinterpret_cast<const f32x4*>(fs);
        } else {
            const f32x4 o1 = *reinterpret_cast<const f32x4*>(fs);
            const f32x4 o2 = *reinterpret_cast<const f32x4*>(fs + 256);
            const f32x4 o3 = *reinterpret_cast<const f32x4*>(fs + 512);
            v = (pend + o1) + (o2 + o3);
        }
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int row = rbase + g;
            const bool live = any && row < p.M && col < p.N;
            int off = live ? (row * p.N + col) * 4 : kDrop + 16 * g;  // dropped past num_records
            asm volatile("" : "+v"(off));                     // a select, not a branch around the store
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v[g]), out_rs, off, 0, 0);
            const bool up = live && v[g] > run_v[g];  // tiles in increasing column order: first max stays
            run_v[g] = up ? v[g] : run_v[g];
            run_i[g] = up ? col : run_i[g];
        }
    };

    int stage = 0;  // ring stage of tile t
    int it = 0;
#ifdef HPA_RG_TRACE
    unsigned long long tr_vm = 0, tr_bar = 0, tr_mf[2] = {0, 0};
#endif
    for (; t < tend; t += TS, ++it) {
        // loaders: their DMA of tile t landed (issued two iterations ago;
        // after it, the previous iteration's kRgDma); the barrier makes every
        // loader's landed and frees the stage read in the previous iteration
#ifdef HPA_RG_TRACE
        const unsigned long long tr_w0 = __builtin_amdgcn_s_memrealtime();
#endif
        if (loader) {
            if (t + TS < tend)  // tile t + TS's kRgDma DMAs may stay in flight
                __builtin_amdgcn_s_waitcnt((kRgDma & 15) | ((kRgDma >> 4) << 14) | (7 << 4));  // vmcnt(kRgDma) lgkmcnt(0)
            else
                __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0) lgkmcnt(0)
#ifdef HPA_RG_TRACE
            if (w == kRgNC) tr_vm += __builtin_amdgcn_s_memrealtime() - tr_w0;
#endif
        } else {
            __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0) only
        }
        asm volatile("" ::: "memory");
#ifdef HPA_RG_TRACE
        const unsigned long long tr_b0 = __builtin_amdgcn_s_memrealtime();
#endif
        __builtin_amdgcn_s_barrier();
#ifdef HPA_RG_TRACE
        if (it < 14) RG_MARK(2 + it);
        const unsigned long long tr_b1 = __builtin_amdgcn_s_memrealtime();
        if (w == 0) tr_bar += tr_b1 - tr_b0;
#endif
        if (loader) {
            // tile t + 2G into the stage freed by the barrier: the loader
            // waves do nothing else, so the stalls of a saturated per-CU
            // memory queue never hold up an MFMA
            const int st2 = stage == 0 ? 2 : stage - 1;
            if (t + 2 * TS < tend) {
                const float* dsrc = dma_src(t + 2 * TS);
                const unsigned ddst = dma_dst(st2);
#pragma unroll
                for (int j = 0; j < kRgDma; ++j) rg_dma(dsrc + kRgLoaders * j * 256, ddst + kRgLoaders * j * 1024);
            }
        } else {
            // (waves of a missing row block compute on zeros)
            const float* rb = ring + stage * kRgTileF + lane * 4 + h * NPW * kRgPart * 256;
            if (owner) epilogue(t - TS, (it + 1) & 1, it > 0);
            f32x4 acc[NPW];
#pragma unroll
            for (int j = 0; j < NPW; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int i = 0; i < kRgPart; ++i) {
                float4 b[NPW];
#pragma unroll
                for (int j = 0; j < NPW; ++j) b[j] = *reinterpret_cast<const float4*>(rb + (j * kRgPart + i) * 256);
#pragma unroll
                for (int q = 0; q < 4; ++q)
#pragma unroll
                    for (int j = 0; j < NPW; ++j) {
                        const float xs = q == 0 ? a[j][i].x : q == 1 ? a[j][i].y : q == 2 ? a[j][i].z : a[j][i].w;
                        const float ws = q == 0 ? b[j].x : q == 1 ? b[j].y : q == 2 ? b[j].z : b[j].w;
                        acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(xs, ws, acc[j], 0, 0, 0);
                    }
            }
            f32x4 s = acc[0];
            if constexpr (NPW == 2) s = acc[0] + acc[1];
            if (owner) {
                pend = s;
            } else if (rvalid) {
                *reinterpret_cast<f32x4*>(fold + (it & 1) * kRgFoldF + (r * S::NSLOT + h - 1) * 256 + lane * 4) = s;
            }
        }
        stage = stage == kRgStages - 1 ? 0 : stage + 1;
#ifdef HPA_RG_TRACE
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (w == 0 || w == kRgNC) tr_mf[w == kRgNC] += __builtin_amdgcn_s_memrealtime() - tr_b1;
#endif
    }
    RG_MARK(16);
#ifdef HPA_RG_TRACE
    if (lane == 0 && w == kRgNC) {
        g_rg_trace[0][blockIdx.x][18] = tr_vm;
        g_rg_trace[0][blockIdx.x][21] = tr_mf[1];
    }
    if (lane == 0 && w == 0) {
        g_rg_trace[0][blockIdx.x][19] = tr_bar;
        g_rg_trace[0][blockIdx.x][20] = tr_mf[0];
    }
#endif
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (owner) epilogue(t - TS, (it + 1) & 1, it > 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA outlives the workgroup
    RG_MARK(17);
    // one partial per row: slot blockIdx.x of part_out ([G][Mp][2]); the
    // 16 columns' running maxima of a row sit in 16 adjacent lanes
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        rg_argmax<0x140>(run_v[g], run_i[g]);  // row_mirror
        rg_argmax<0x141>(run_v[g], run_i[g]);  // row_half_mirror
        rg_argmax<0x4E>(run_v[g], run_i[g]);   // quad_perm [2,3,0,1]
        rg_argmax<0xB1>(run_v[g], run_i[g]);   // quad_perm [1,0,3,2]
    }
    if (owner && (lane & 15) == 0) {
        const __amdgpu_buffer_rsrc_t part_rs =
            __builtin_amdgcn_make_buffer_rsrc(p.part_out, 0, (int)((size_t)G * p.Mp * 8), 0x00020000);
        typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const u32x2 pv = {__float_as_uint(run_v[g]), (unsigned int)run_i[g]};
            __builtin_amdgcn_raw_buffer_store_b64(pv, part_rs, ((int)blockIdx.x * p.Mp + rbase + g) * 8, 0,
                                                  hpa::kCpolSc1);
        }
    }
    if (p.pick_next) final_pick<kRgNW>(p, ring);  // the ring is idle now (every DMA drained)
}

int g_num_cus = 0;

// A/B builds: HPA_LOGITS_FORM=16 / ring forces a form; else 0 = the caller's
int logits_form() {
#ifdef HPA_AB
    static const int f = [] {
        const char* e = getenv("HPA_LOGITS_FORM");
        return (e && e[0] == '1' && e[1] == '6') ? 16 : (e && e[0] == 'r') ? 12 : 0;
    }();
    return f;
#else
    return 0;
#endif
}


template <int MT>
int launch_resident_mt(const FG& p, int form) {
    if (form == 16)
        logits_resident_kernel<MT><<<(unsigned)logits_resident_grid(p), kResNW * 64, 0, hpa_stream()>>>(p);
    else
        logits_ring_kernel<MT><<<(unsigned)logits_resident_grid(p), kRgNW * 64, 0, hpa_stream()>>>(p);
    HPA_LAUNCH_CHECK();
    return 0;
}

}  // namespace

// one workgroup per CU of the current stream (CU-masked streams: their
// budget); also the number of argmax partials per row the kernel writes
int logits_resident_grid(const FG& p) {
    if (!g_num_cus) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&g_num_cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            g_num_cus <= 0)
            return hpa_fail(__FILE__, __LINE__, "logits: CU count"), 1;
    }
    const int cus = g_num_cus;
    return min(p.ntn, cus);
}

bool logits_resident_eligible(const FG& p, int epi) {
    return epi == HPA_FEPI_LOGITS && p.ln_stats && p.K16 == kResNW * kResS && p.Mp <= 64 && p.M <= p.Mp &&
           (logits_form() == 16 || p.ln_ntiles == kRgK16);
}

// form: 16 = the 16-wave K-split form, 12 = the ring form, else by the rows
// (the ring at 48-64 rows, 57.5 vs 58.7-59.8 us at 64; the 16-wave form at
// 8-32 rows: 28.0 vs 35.3 us at 8, where the kernel streams wte with one
// computing wave per SIMD).  The two forms sum a row's K in different orders:
// callers that must match another batch size bit for bit (sharded decode)
// pass the form of the GLOBAL batch.  HPA_LOGITS_FORM=16 / ring overrides.
int launch_logits_resident(const FG& p, int form) {
    if (logits_form() == 16 || logits_form() == 12) form = logits_form();
    if (form != 16 && form != 12) form = p.Mp >= 48 ? 12 : 16;
    switch (p.Mp / 16) {
        case 1: return launch_resident_mt<1>(p, form);
        case 2: return launch_resident_mt<2>(p, form);
        case 3: return launch_resident_mt<3>(p, form);
        case 4: return launch_resident_mt<4>(p, form);
        default: return hpa_fail(__FILE__, __LINE__, "logits: rows must be <= 64");
    }
}

// trace build only: the ring logits kernel's per-workgroup stamps of the
// last launch ([2][256][24] u64: s_memrealtime 10 ns ticks, s_memtime).  Returns 1 in
// the product build.
extern "C" int hpa_logits_trace(unsigned long long* host) {
#ifdef HPA_RG_TRACE
    HPA_CHECK(hipMemcpyFromSymbol(host, HIP_SYMBOL(g_rg_trace), sizeof(g_rg_trace)));
    return 0;
#else
    (void)host;
    return 1;
#endif
}

}  // namespace hpa_gemm
