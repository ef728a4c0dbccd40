// hpa_gemm_sk.hip -- stream-K fused GEMM for the decode rows (M <= 64),
// variant 6 of hpa_gemm_fused; the engine's logits GEMM where the resident
// kernel does not fit (GPT-2 XL).  On the layer GEMMs it measured slower than
// the looped / one-shot kernels (the slab hand-off), so they keep
// those.
//
// Why (measured, profiles/r2/mfma_xl.txt): the tile-per-workgroup kernels
// keep the XL GEMMs at 19-48 % of the fp32 MFMA peak.  Their grids are one
// wave of 100-400 column tiles over 256 CUs, so either CUs idle (150-200
// workgroups) or a second partial round runs; and each workgroup's pipeline
// is short next to the first-load latency.  The weights (123 MB per XL layer)
// must stream from HBM once at <= ~25 GB/s per CU (MI355X_MICROARCH.md), so
// the work has to be spread evenly over EVERY CU, each streaming its own
// contiguous share of the weights for the whole kernel.
//
// How:
//  * work = (32-column super-tile, 16-deep k-step) pairs in super-tile-major
//    order; one 8-wave workgroup per CU takes an equal contiguous range of
//    them, its waves equal contiguous sub-ranges.  A step loads the two
//    weight fragments of the super-tile (1 KiB each, streamed in order) and
//    the <= 4 activation fragments of all M rows (L2-resident), and issues
//    32 v_mfma_f32_16x16x4_f32 into 8 accumulators (4 row blocks x 2 column
//    tiles): every weight byte is fetched from HBM exactly once.  Loads run
//    SK_D steps ahead in a register ring.
//  * a wave's sub-range covers at most 2 super-tiles (it is shorter than
//    K/16 steps); it leaves each one's partial tile in LDS.  The workgroup
//    then folds, per super-tile it touched, the partials of its waves in wave
//    order.  A super-tile wholly inside the workgroup's range goes straight
//    to the epilogue; one split between workgroups is published as a
//    write-through slab (sc1 stores, drained) with an arrival ticket
//    (agent-scope atomic add), and the last of its workgroups to arrive sums
//    the slabs in workgroup order (sc1 loads: MI355X_MICROARCH.md "Valid
//    forms", row 1) and runs the epilogue, then rewinds the counter.
//    Summation order: k in order within a wave, waves in order, workgroups in
//    order -- fixed by the shape and the CU count, never by M or timing.
//  * epilogues are the shared Epi (QKV + KV append, RESID + statistics, GELU,
//    LOGITS + argmax partials).  A LayerNorm is either folded into the weights
//    (qkv / fc: row statistics from the producer's 16-column partials, since
//    no workgroup sees a whole row's K) or applied to the A fragments on load
//    (logits' LNf: the looped kernel's prologue, weights staged in LDS).
#include <math.h>

#include "hpa_gemm_body.h"

namespace {
using namespace hpa_gemm;

constexpr int SK_NW = 8;           // waves per workgroup (2 per SIMD)
constexpr int SK_MT = 4;           // row blocks: all M <= 64 rows
constexpr int SK_NTW = 2;          // column tiles per super-tile
constexpr int SK_TE = SK_MT * 256;  // elements per column tile (64 rows x 16 cols)
constexpr int SK_STE = SK_NTW * SK_TE;  // elements per super-tile
constexpr int SK_D = 4;            // steps in flight per wave
constexpr int SK_NT = SK_NW * 64;
constexpr int SK_MAXG = 1024;      // workgroups (one per CU)
// LayerNorm applied on load (ln_stats without a fold): its weight / bias
// [2][HPA_FUSED_LN_KMAX] overlay the row-statistics and epilogue-scratch areas
// (dead during the steps) plus SK_LNX_GB more floats, then ln_prologue's
// statistics [64][2] and scratch [256][2]
constexpr int SK_LNX_GB = 2 * HPA_FUSED_LN_KMAX - (SK_NW * 64 * 2 + SK_NTW * 64 * 17);
constexpr int SK_LNX = SK_LNX_GB + 2 * 64 + 8 * 64;
// LDS: [wave][2 slots][super-tile] partials, then row statistics [NW][64][2],
// the epilogue's row-statistics scratch [NTW * 64][17], the LN area, a
// broadcast word (+3 pad), the per-wave super-tile span [NW][2] and the range
// table [SK_MAXG + 1]
constexpr int SK_LDS_FLOATS =
    SK_NW * 2 * SK_STE + SK_NW * 64 * 2 + SK_NTW * 64 * 17 + SK_LNX + 4 + 2 * SK_NW + SK_MAXG + 4;
static_assert(SK_LNX_GB >= 0 && SK_LDS_FLOATS * 4 <= 160 * 1024, "stream-K LDS");

// workgroup g owns steps [F*g/G, F*(g+1)/G); all index math is 32-bit
// (F*G < 2^31, checked on the host): the 64-bit divisions this replaced cost
// ~15 us per launch (tools/sk_trace.py)
__device__ __forceinline__ int sk_start(int F, int G, int g) { return (int)((unsigned)(F * g) / (unsigned)G); }

#ifdef HPA_SK_TRACE  // phase timestamps per workgroup (tools/sk_trace.py; A/B build only)
__device__ unsigned long long sk_tr[1024 * 16];
#define SK_T(i) \
    do { if (threadIdx.x == 0) sk_tr[blockIdx.x * 16 + (i)] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define SK_T(i) do {} while (0)
#endif

// MT: row blocks computed (1, 2 or 4; compile-time, so the step body has no
// branches -- a runtime row-block test put one around every MFMA); LN: the
// LayerNorm applied to the A fragments on load (the logits' LNf)
template <int EPI, int MT, bool LN>
__global__ __launch_bounds__(SK_NT) void gemm_sk_kernel(FG p) {
    extern __shared__ __attribute__((aligned(16))) float sk_smem[];
    float* part = sk_smem;                         // [NW][2][STE]
    float* wsum = part + SK_NW * 2 * SK_STE;       // [NW][64][2] (slot 0 = row totals, others 0)
    float* tile = wsum + SK_NW * 64 * 2;           // [NTW*64][17]
    float* lnx = tile + SK_NTW * 64 * 17;          // LN area (with wsum and tile)
    int* bcast = reinterpret_cast<int*>(lnx + SK_LNX);
    int* wst = bcast + 4;  // [NW][2]: first and last super-tile of each wave's steps (-1: none)
    int* bnd = wst + 2 * SK_NW;  // [G + 1]: sk_start of every workgroup

    SK_T(0);
    const int G = gridDim.x, g = blockIdx.x;
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // uniform: scalar step bounds and branches
    const int K16 = p.K16, MTv = p.Mp >> 4;
    const int nst = (p.ntn + SK_NTW - 1) / SK_NTW;
    const int F = nst * K16;
    for (int i = threadIdx.x; i <= G; i += SK_NT) bnd[i] = sk_start(F, G, i);
    const int g_lo = sk_start(F, G, g), g_hi = sk_start(F, G, g + 1);
    const int n_g = g_hi - g_lo;
    const int a = g_lo + n_g * w / SK_NW, b = g_lo + n_g * (w + 1) / SK_NW;  // this wave's steps
    // folded LayerNorm: wsum slot 0 gets the row totals (below), the other slots 0
    if (p.fold_c1)
        for (int i = 128 + threadIdx.x; i < SK_NW * 64 * 2; i += SK_NT) wsum[i] = 0.f;
    // LayerNorm on load: weight / bias into LDS over wsum.., mean / rstd of the
    // rows (l & 15) + 16 r of lane l (the looped kernel's prologue)
    float mu[MT], rs[MT];
#pragma unroll
    for (int r = 0; r < MT; ++r) mu[r] = rs[r] = 0.f;
    if (LN) ln_prologue<SK_NW, MT>(p, wsum, lnx + SK_LNX_GB, lnx + SK_LNX_GB + 128, 0, true, mu, rs);
    const float4* lng4 = reinterpret_cast<const float4*>(wsum) + (lane >> 4);
    const float4* lnb4 = reinterpret_cast<const float4*>(wsum + HPA_FUSED_LN_KMAX) + (lane >> 4);

    // ---- the wave's steps: a register ring SK_D steps deep
    const float4* __restrict__ W4 = reinterpret_cast<const float4*>(p.w);
    const float4* __restrict__ X4 = reinterpret_cast<const float4*>(p.x);
    struct Step {
        float4 w[SK_NTW], x[MT];
        int k;  // k-step within the super-tile
    };
    auto load = [&](Step& s, int u) {
        u = u < b ? u : b - 1;  // clamped, unconditional
        const int st = (int)((unsigned)u / (unsigned)K16), k = u - st * K16;
        s.k = k;
#pragma unroll
        for (int j = 0; j < SK_NTW; ++j) {
            const int t = min(st * SK_NTW + j, p.ntn - 1);  // tail tile past ntn: re-read, never stored
            const f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(W4 + ((size_t)t * K16 + k) * 64 + lane));
            s.w[j] = make_float4(v.x, v.y, v.z, v.w);
        }
#pragma unroll
        for (int r = 0; r < MT; ++r) s.x[r] = X4[((size_t)min(r, MTv - 1) * K16 + k) * 64 + lane];
    };
    f32x4 acc[SK_NTW * SK_MT];
#pragma unroll
    for (int i = 0; i < SK_NTW * SK_MT; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int st_first = b > a ? (int)((unsigned)a / (unsigned)K16) : 0;
    int st_cur = st_first;
    auto flush = [&](int slot) {  // accumulators -> part[w][slot] in the epilogue's element order
        float* d = part + ((size_t)w * 2 + slot) * SK_STE;
#pragma unroll
        for (int j = 0; j < SK_NTW; ++j)
#pragma unroll
            for (int r = 0; r < SK_MT; ++r)
#pragma unroll
                for (int q = 0; q < 4; ++q) d[j * SK_TE + (r * 4 + q) * 64 + lane] = acc[j * SK_MT + r][q];
#pragma unroll
        for (int i = 0; i < SK_NTW * SK_MT; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    };
    if (b > a) {
        // Branch-free body: every ring slot is consumed by its step's MFMAs
        // and only then reloaded (same registers, no copies).  A load inside a
        // conditional, or one issued before its slot's old value was used,
        // made the compiler move the new data into the ring at the join,
        // i.e. wait for it within the same step (measured: half the MFMA rate).
        // Steps past b (the last group's tail) run with zero weights.
        Step ring[SK_D];
#pragma unroll
        for (int d = 0; d < SK_D; ++d) load(ring[d], a + d);
        int next_st = (st_first + 1) * K16;  // first step of the next super-tile
        for (int u0 = a; u0 < b; u0 += SK_D) {
#pragma unroll
            for (int d = 0; d < SK_D; ++d) {
                const int u = u0 + d;
                const bool live = u < b;  // uniform
                if (live && u == next_st) {  // at most once per wave: its first super-tile is done
                    flush(0);
                    ++st_cur;
                    next_st += K16;
                }
                if (LN) {  // compile-time
                    const float4 gg = lng4[4 * ring[d].k], bb = lnb4[4 * ring[d].k];
#pragma unroll
                    for (int r = 0; r < MT; ++r) ring[d].x[r] = ln4(ring[d].x[r], mu[r], rs[r], gg, bb);
                }
                const float wm = live ? 1.f : 0.f;  // select, not a branch
#pragma unroll
                for (int j = 0; j < SK_NTW; ++j) {
                    ring[d].w[j].x *= wm;
                    ring[d].w[j].y *= wm;
                    ring[d].w[j].z *= wm;
                    ring[d].w[j].w *= wm;
                }
#pragma unroll
                for (int q = 0; q < 4; ++q)
#pragma unroll
                    for (int j = 0; j < SK_NTW; ++j)
#pragma unroll
                        for (int r = 0; r < MT; ++r) {
                            const Step& s = ring[d];
                            const float xs = q == 0 ? s.x[r].x : q == 1 ? s.x[r].y : q == 2 ? s.x[r].z : s.x[r].w;
                            const float ws = q == 0 ? s.w[j].x : q == 1 ? s.w[j].y : q == 2 ? s.w[j].z : s.w[j].w;
                            acc[j * SK_MT + r] =
                                __builtin_amdgcn_mfma_f32_16x16x4f32(xs, ws, acc[j * SK_MT + r], 0, 0, 0);
                        }
                load(ring[d], u + SK_D);
            }
        }
        flush(st_cur == st_first ? 0 : 1);
    }
    if (lane == 0) {
        wst[2 * w] = b > a ? st_first : -1;
        wst[2 * w + 1] = st_cur;
    }
    // the folded LayerNorm's row totals: the producer's 16-column partials
    // summed in tile order, by the last wave after its steps
    if (p.fold_c1 && w == SK_NW - 1) {
        float s1 = 0.f, s2 = 0.f;
        if (lane < p.M) {
            const float2* ls2 = reinterpret_cast<const float2*>(p.ln_stats);
#pragma unroll 8
            for (int t = 0; t < p.ln_ntiles; ++t) {
                const float2 v = ls2[(size_t)t * p.Mp + lane];
                s1 += v.x;
                s2 += v.y;
            }
        }
        wsum[2 * lane] = s1;
        wsum[2 * lane + 1] = s2;
    }
    SK_T(1);
    __syncthreads();
    SK_T(2);

    // ---- per super-tile this workgroup touched: fold its waves, finish or hand off
    if (n_g <= 0) return;
    const int st_lo = g_lo / K16, st_hi = (g_hi - 1) / K16;
    Epi<SK_NW, EPI, SK_MT, SK_NTW> epi;
    constexpr int EPT = Epi<SK_NW, EPI, SK_MT, SK_NTW>::EPT;
    for (int st = st_lo; st <= st_hi; ++st) {
        epi.prefetch(p, st * SK_NTW, 0);
        float vals[EPT];
#pragma unroll
        for (int i = 0; i < EPT; ++i) vals[i] = 0.f;
        for (int ww = 0; ww < SK_NW; ++ww) {  // waves in order
            const int fs = wst[2 * ww], ls = wst[2 * ww + 1];
            if (fs < 0 || st < fs || st > ls) continue;
            const float* src = part + ((size_t)ww * 2 + (st == fs ? 0 : 1)) * SK_STE;
#pragma unroll
            for (int i = 0; i < EPT; ++i) {
                const int e = threadIdx.x + i * SK_NT;
                if (e < SK_STE) vals[i] += src[e];
            }
        }
        SK_T(3 + 4 * (st - st_lo));
        const int t_lo = st * K16, t_hi = t_lo + K16;
        if (t_lo < g_lo || t_hi > g_hi) {  // split between workgroups: hand off
            static_assert(EPT == 4, "slab rows: one float4 per thread");
            const int slot = st == st_lo ? 0 : 1;
            // thread-major slab: thread t's four elements as one 16-B write-through store
            hpa::store_wt16(p.sk_slab + ((size_t)g * 2 + slot) * SK_STE, (int)threadIdx.x * 16,
                            make_float4(vals[0], vals[1], vals[2], vals[3]));
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every slab store drained before the ticket
            __syncthreads();
            // the workgroups whose ranges meet this tile: g0 owns t_lo, g1 owns t_hi - 1
            int g0 = g, g1 = g;
            while (g0 > 0 && bnd[g0] > t_lo) --g0;
            while (g1 + 1 < G && bnd[g1 + 1] <= t_hi - 1) ++g1;
            if (threadIdx.x == 0)
                bcast[0] = __hip_atomic_fetch_add(p.sk_cnt + st, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __syncthreads();
            const int ticket = bcast[0];
            SK_T(4 + 4 * (st - st_lo));
            __syncthreads();
            int arrivals = 0;  // workgroups with steps in this tile (with fewer steps than
            for (int gg = g0; gg <= g1; ++gg)  // workgroups, some ranges are empty)
                arrivals += bnd[gg + 1] > bnd[gg];
            if (ticket != arrivals - 1) continue;  // not the last: the last arriver finishes this tile
            if (threadIdx.x == 0) __hip_atomic_store(p.sk_cnt + st, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
            for (int i = 0; i < EPT; ++i) vals[i] = 0.f;
            // workgroups in order, 8 slabs in flight at a time (each load is a
            // cross-XCD round trip: issued one after another they serialise)
            for (int gb = g0; gb <= g1; gb += 8) {
                float4 v[8];
                bool has[8];
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const int gg = min(gb + q, g1);
                    has[q] = gb + q <= g1 && bnd[gg + 1] > bnd[gg];  // empty range: no slab
                    const int s_slot = bnd[gg] >= t_lo ? 0 : 1;  // its first tile, or its second
                    v[q] = hpa::load_wt16(p.sk_slab + ((size_t)gg * 2 + s_slot) * SK_STE, (int)threadIdx.x * 16);
                }
#pragma unroll
                for (int q = 0; q < 8; ++q)
                    if (has[q]) {
                        vals[0] += v[q].x;
                        vals[1] += v[q].y;
                        vals[2] += v[q].z;
                        vals[3] += v[q].w;
                    }
            }
        }
        SK_T(5 + 4 * (st - st_lo));
        epi.apply(p, vals, tile, st * SK_NTW, 0, wsum);
        __syncthreads();  // tile scratch reuse by the next super-tile
        SK_T(6 + 4 * (st - st_lo));
    }
}

template <int EPI, int MT, bool LN>
int launch_sk_mt(const FG& p, int G) {
    const size_t lds = (size_t)SK_LDS_FLOATS * sizeof(float);
    static bool attr_set = false;
    if (!attr_set) {
        HPA_CHECK(hipFuncSetAttribute((const void*)gemm_sk_kernel<EPI, MT, LN>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        attr_set = true;
    }
    gemm_sk_kernel<EPI, MT, LN><<<G, SK_NT, lds, hpa_stream()>>>(p);
    HPA_LAUNCH_CHECK();
    return 0;
}

template <int EPI, bool LN>
int launch_sk_ln(const FG& p, int G) {
    const int mtv = p.Mp >> 4;
    return mtv == 1   ? launch_sk_mt<EPI, 1, LN>(p, G)
           : mtv == 2 ? launch_sk_mt<EPI, 2, LN>(p, G)
                      : launch_sk_mt<EPI, 4, LN>(p, G);
}

template <int EPI>
int launch_sk_t(const FG& p, int G) {
    return p.ln_stats && !p.fold_c1 ? launch_sk_ln<EPI, true>(p, G) : launch_sk_ln<EPI, false>(p, G);
}

int g_sk_cus = 0;
int sk_grid() {
    if (g_sk_cus <= 0) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&g_sk_cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            g_sk_cus = 256;
    }
    return g_sk_cus;
}

}  // namespace

namespace hpa_gemm {
// the shapes launch_sk accepts (its checks, as a predicate for the dispatch)
bool sk_eligible(int Mp, int ntn, int K16) {
    const int G = sk_grid();
    const long long nst = (ntn + SK_NTW - 1) / SK_NTW, F = nst * K16;
    return Mp <= 64 && G <= SK_MAXG && F * G < (1LL << 31) &&
           (F + (long long)G * SK_NW - 1) / ((long long)G * SK_NW) + 1 <= K16;
}

int launch_sk(const FG& p, int epi) {
    HPA_REQUIRE(p.Mp <= 64, "gemm_fused stream-K: M <= 64");
    HPA_REQUIRE(p.sk_slab && p.sk_cnt, "gemm_fused stream-K: sk_slab / sk_count workspace");
    HPA_REQUIRE(!p.ln_stats || p.fold_c1 || p.K <= HPA_FUSED_LN_KMAX, "gemm_fused stream-K: LayerNorm K too large");
    HPA_REQUIRE(!p.fold_c1 || p.ln_stats, "gemm_fused stream-K: folded LayerNorm needs ln_stats");
    const int G = sk_grid();
    const long long nst = (p.ntn + SK_NTW - 1) / SK_NTW, F = nst * p.K16;
    HPA_REQUIRE(G <= SK_MAXG && F * G < (1LL << 31), "gemm_fused stream-K: grid or step count too large");
    // a wave's sub-range must span at most two super-tiles
    HPA_REQUIRE((F + (long long)G * SK_NW - 1) / ((long long)G * SK_NW) + 1 <= p.K16,
                "gemm_fused stream-K: too few steps per super-tile for this grid");
    switch (epi) {
        case HPA_FEPI_QKV: return launch_sk_t<HPA_FEPI_QKV>(p, G);
        case HPA_FEPI_RESID: return launch_sk_t<HPA_FEPI_RESID>(p, G);
        case HPA_FEPI_GELU: return launch_sk_t<HPA_FEPI_GELU>(p, G);
        case HPA_FEPI_LOGITS: return launch_sk_t<HPA_FEPI_LOGITS>(p, G);
        default: return hpa_fail(__FILE__, __LINE__, "gemm_fused stream-K: unknown epilogue");
    }
}
}  // namespace hpa_gemm

#ifdef HPA_SK_TRACE
extern "C" int hpa_sk_trace_read(unsigned long long* host) {
    HPA_CHECK(hipDeviceSynchronize());
    HPA_CHECK(hipMemcpyFromSymbol(host, HIP_SYMBOL(sk_tr), sizeof(sk_tr)));
    void* d = nullptr;
    HPA_CHECK(hipGetSymbolAddress(&d, HIP_SYMBOL(sk_tr)));
    HPA_CHECK(hipMemset(d, 0, sizeof(sk_tr)));
    return 0;
}
#endif

extern "C" int hpa_gemm_sk_workspace(int N, size_t* slab_floats, size_t* counters) {
    HPA_REQUIRE(N > 0 && slab_floats && counters, "gemm_sk_workspace: arguments");
    *slab_floats = (size_t)sk_grid() * 2 * SK_STE;
    *counters = (size_t)((N + 15) / 16 + SK_NTW - 1) / SK_NTW;
    return 0;
}
