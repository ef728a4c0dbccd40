// hpa_gemm_ring.hip -- the 64-row fp32 layer GEMM with a loader / MFMA-wave
// split over an LDS ring (variant 3 of hpa_gemm_fused; GPT-2 XL's decode
// qkv and fc, matmul_forward paged_infer.c:92-114 / matmul_cached :117-160).
//
// Why (DESIGN.md "Where an XL layer GEMM's time goes"):
// in the looped kernel every wave both loads its operands and runs the
// MFMAs, and the two barely overlap (XL fc: loads alone 10.9 us, MFMAs alone
// 14.1, both 21.8).  Here one workgroup of 12 waves takes 64 rows x 32
// columns over the whole K (rows past Mp: a repeated row block, never stored):
//   * 4 loader waves move each 8-deep k16 stage -- the 4 row blocks' A
//     fragments (16 KiB, default cache policy: every workgroup re-reads A
//     from its XCD's L2) and the 2 column tiles' W fragments (8 KiB,
//     non-temporal: read once) -- into a 3-stage LDS ring by LDS-DMA
//     (global_load_lds_dwordx4), two stages ahead, and do nothing else;
//   * 8 MFMA waves (2 per SIMD): wave w owns row block w & 3 and half h =
//     w >> 2 of every stage's steps (4h .. 4h + 3) for BOTH column tiles --
//     two independent accumulator chains, each A fragment read once for two
//     W fragments (ds_read_b128 from the ring); the two halves are added in
//     the epilogue (h = 0 + h = 1);
//   * one workgroup barrier per stage (the loaders' counted vmcnt makes the
//     stage's bytes visible; the barrier also frees the stage read before).
// Measured (tools/ring_tune.py, profiles/r3/experiments/xl_ring_gemm.txt,
// B = 64): XL qkv 21.7 vs 23.8 us, fc 22.4 vs 24.7 (the engine's default
// for them; XL step 10.23 vs 10.38 ms).  The ring traffic alone takes 12.6 /
// 13.8 us, the MFMA waves alone 19.1 / 19.7 (against 12.4 at the fp32 issue
// rate): the MFMA side bounds it.  attproj (50 workgroups) and fcproj (K =
// 6400 on 50 workgroups) stay on the looped kernel.
// The row statistics of a folded LayerNorm come from the A fragments the
// waves read (each half's partial sums in its own slot); the epilogue is the shared
// Epi::apply (QKV with the K/V append, GELU, RESID with LN partial sums).
// A row's summation order depends only on K (two fixed chains per tile),
// never on M or the grid: bit-identical rows across launch shapes.
#include "hpa_gemm_body.h"

namespace hpa_gemm {
namespace {

constexpr int kRnNW = 12;                   // waves per workgroup
constexpr int kRnNC = 8;                    // MFMA waves (row block w & 3, stage half w >> 2)
constexpr int kRnLd = kRnNW - kRnNC;        // loader waves
constexpr int kRnStages = 3;
// per stage of KS k16 steps: 1 KiB fragments A[4][KS], W[2][KS]
template <int KS>
struct RnShape {
    static constexpr int Chunks = 6 * KS;
    static constexpr int PerLd = Chunks / kRnLd;  // LDS-DMA wave-instructions per loader per stage
    static constexpr int StageF = Chunks * 256;   // floats per stage
    static constexpr int LdsF = kRnStages * StageF;
    static_assert(LdsF * 4 <= 160 * 1024, "LDS");
    static_assert(Chunks % kRnLd == 0 && KS % 2 == 0, "chunks per loader, stage halves");
};
// epilogue scratch over the ring (dead after the loop)
constexpr int kRnRedF = 2 * 2 * 4 * 256;    // [2 halves][2 tiles][4 row blocks][4 regs][64 lanes]
constexpr int kRnTileF = 2 * 64 * 17;       // Epi::apply's row-statistics tile
constexpr int kRnWsumF = kRnNW * 64 * 2;    // [NW][64 rows][2] LN row partials (slots 0, 1 used)
static_assert(kRnRedF + kRnTileF + kRnWsumF <= RnShape<4>::LdsF, "epilogue scratch");
// K-split workspace per (column pair, K part): the folded 64 x 32 tile, then
// the rows' (sum, sum of squares)
constexpr int kRnPartF = 2048 + 128;

// LDS-DMA of one 1 KiB fragment (16 B per lane to lds_addr + 16 * lane).
// Inline asm (as hpa_logits.hip's ring): the compiler does not count these
// loads, the loader waves wait for them themselves.
template <bool NT>
__device__ __forceinline__ void rn_dma(const float* src, unsigned lds_addr) {
    unsigned keep;
    if constexpr (NT)
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep)
                     : "v"(src), "s"(lds_addr)
                     : "memory");
    else
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep)
                     : "v"(src), "s"(lds_addr)
                     : "memory");
}

// MODE (diagnostics, tools/ring_tune.py): 0 the product; 1 no MFMAs (the
// ring runs, the MFMA waves only read it); 2 no LDS-DMA (MFMAs on whatever
// the ring holds); 3 as 2 without the per-stage barriers; 4 as 3 on
// register operands (no LDS reads)
// KS: k16 steps per stage (8: one 12-wave workgroup per CU, 144 KiB of ring;
// 4: two per CU, 72 KiB).  SPLIT: the grid is column pairs x p.gy K parts
// (contiguous stage ranges); each part publishes its folded tile and row
// sums to p.sk_slab (write-through), draws a ticket on p.sk_cnt[pair], and
// the last of the pair sums the parts in part order (results independent of
// arrival order and of M), rewinds the counter and runs the epilogue.
template <int EPI, int MODE, int KS, bool SPLIT>
__global__ __launch_bounds__(kRnNW * 64, KS == 4 ? 2 : 1) void gemm_ring_kernel(FG p) {
    using S = RnShape<KS>;
    __shared__ __attribute__((aligned(16))) float ring[S::LdsF];
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const bool loader = w >= kRnNC;
    const int r = w & 3, h = (w >> 2) & 1;
    const int npairs = (p.ntn + 1) / 2;
    const int nparts = SPLIT ? p.gy : 1;
    const int pair = SPLIT ? (int)(blockIdx.x % (unsigned)npairs) : (int)blockIdx.x;
    const int part = SPLIT ? (int)(blockIdx.x / (unsigned)npairs) : 0;
    const int nt0 = pair * 2;
    const int K16 = p.K16;
    const int nst_all = (K16 + KS - 1) / KS;
    const int st_b = part * nst_all / nparts;
    const int nst = (part + 1) * nst_all / nparts - st_b;  // this part's stages
    auto phys = [&](int st) __attribute__((always_inline)) {  // the part's stage st -> k stage
        return st_b + st;
    };
    const bool fold = p.fold_c1 != nullptr;

    Epi<kRnNW, EPI, 4, 2> epi;
    epi.prefetch(p, nt0, 0);  // bias / residual / c1 of the owned elements, landing during the loop

    const unsigned ring_lds =
        __builtin_amdgcn_readfirstlane((unsigned)(size_t)(__attribute__((address_space(3))) float*)ring);
    // loader wave L = w - 8 moves chunks q = L + 4 i of every stage: q < 4 KS
    // -> A (row block q / KS, step q % KS), else W (tile (q - 4 KS) / KS)
    const int L = w - kRnNC;
    const int nrb = p.Mp >> 4;
    const float* xa = p.x + (size_t)lane * 4;
    const float* wa0 = p.w + (size_t)min(nt0, p.ntn - 1) * K16 * 256 + lane * 4;
    const float* wa1 = p.w + (size_t)min(nt0 + 1, p.ntn - 1) * K16 * 256 + lane * 4;
    auto issue = [&](int st) __attribute__((always_inline)) {
        const unsigned base = ring_lds + (unsigned)((st % kRnStages) * S::StageF) * 4;
        const int kst = st < nst ? phys(st) : phys(nst - 1);  // past the part's end: a harmless re-read
#pragma unroll
        for (int i = 0; i < S::PerLd; ++i) {
            const int q = L + kRnLd * i;
            const int s = q % KS;
            const int k = min(kst * KS + s, K16 - 1);
            const unsigned dst = base + (unsigned)q * 1024;
            if (i < KS) {  // A chunk (compile-time: q < 4 KS for every loader); row
                // blocks past Mp re-read the last one (their rows are never stored)
                rn_dma<false>(xa + ((size_t)min(q / KS, nrb - 1) * K16 + k) * 256, dst);
            } else {
                rn_dma<true>((((q - 4 * KS) / KS) ? wa1 : wa0) + (size_t)k * 256, dst);
            }
        }
    };
    if (loader && MODE < 2) {
        issue(0);
        issue(1);
    }

    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
    float fs1 = 0.f, fs2 = 0.f;
    constexpr int KH = KS / 2;  // steps per half-stage
    const float* ra = ring + (r * KS + h * KH) * 256 + lane * 4;   // A[r][s] of a stage
    const float* rw = ring + (4 * KS + h * KH) * 256 + lane * 4;   // W[0][s]; W[1][s] at + KS
    // iteration st: the loaders' stage st has landed -> barrier -> loaders
    // issue stage st + 2 into the slot read in iteration st - 1; the MFMA
    // waves multiply stage st.  The two roles run separate loops with the
    // same nst barriers (the loaders' address registers and the MFMA waves'
    // fragments never share a live range).  (A software-pipelined form --
    // stage st read while stage st - 1's MFMAs run, two register sets --
    // measured slower: XL qkv 23.7 vs 23.0 us, profiles/r3/experiments/.)
    if (loader) {
        for (int st = 0; st < nst; ++st) {
            if (MODE < 2)
                __builtin_amdgcn_s_waitcnt((S::PerLd & 15) | ((S::PerLd >> 4) << 14) | (7 << 4));  // vmcnt(PerLd) lgkmcnt(0)
            if (MODE < 3) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
            if (MODE < 2) issue(st + 2);
        }
    } else {
        for (int st = 0; st < nst; ++st) {
            if (MODE < 3) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
            const int so = (st % kRnStages) * S::StageF;
            const int ns = min(KH, K16 - phys(st) * KS - h * KH);  // may be <= 0 in the last stage
#pragma unroll
            for (int s = 0; s < KH; ++s) {
                if (s < ns) {
                    float4 xv, w0, w1;
                    if (MODE == 4) {  // register operands only
                        const float f = (float)(lane + s + st);
                        xv = make_float4(f, f + 1.f, f + 2.f, f + 3.f);
                        w0 = make_float4(f * 0.5f, f, f, f);
                        w1 = make_float4(f, f * 0.25f, f, f);
                    } else {
                        xv = *reinterpret_cast<const float4*>(ra + so + s * 256);
                        w0 = *reinterpret_cast<const float4*>(rw + so + s * 256);
                        w1 = *reinterpret_cast<const float4*>(rw + so + (KS + s) * 256);
                    }
                    if (fold) row_sums_add(xv, fs1, fs2);
                    if (MODE == 1) {
                        acc0[0] += (xv.x + w0.x) + (xv.y + w0.y);
                        acc1[1] += (xv.z + w1.z) + (xv.w + w1.w);
                    } else {
                        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(xv.x, w0.x, acc0, 0, 0, 0);
                        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(xv.x, w1.x, acc1, 0, 0, 0);
                        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(xv.y, w0.y, acc0, 0, 0, 0);
                        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(xv.y, w1.y, acc1, 0, 0, 0);
                        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(xv.z, w0.z, acc0, 0, 0, 0);
                        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(xv.z, w1.z, acc1, 0, 0, 0);
                        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(xv.w, w0.w, acc0, 0, 0, 0);
                        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(xv.w, w1.w, acc1, 0, 0, 0);
                    }
                }
            }
        }
    }
    // no LDS-DMA outlives the loop: the scratch below overlays the ring
    if (loader) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");

    float* red = ring;                       // [2 halves][2 tiles][4][4][64]
    float* tile = ring + kRnRedF;            // Epi::apply row statistics
    float* wsum = tile + kRnTileF;           // [NW][64][2]: slots 0, 1 = the halves' row sums, the rest 0
    if (!loader) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            red[h * 2048 + r * 256 + g * 64 + lane] = acc0[g];
            red[h * 2048 + 1024 + r * 256 + g * 64 + lane] = acc1[g];
        }
        if (fold) row_sums_publish(fs1, fs2, wsum + h * 128 + 32 * r);
    } else if (fold) {
        for (int i = (w - kRnNC) * 64 + lane; i < kRnWsumF - 256; i += kRnLd * 64) wsum[256 + i] = 0.f;
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    constexpr int EPT = (2 * 1024 + kRnNW * 64 - 1) / (kRnNW * 64);
    float vals[EPT];
#pragma unroll
    for (int i = 0; i < EPT; ++i) {
        const int e = threadIdx.x + i * kRnNW * 64;
        vals[i] = e < 2 * 1024 ? red[e] + red[2048 + e] : 0.f;  // half 0 + half 1
    }
    if constexpr (SPLIT) {
        float* slab = p.sk_slab;
        const int own = (pair * nparts + part) * kRnPartF;
#pragma unroll
        for (int i = 0; i < EPT; ++i) {
            const int e = threadIdx.x + i * kRnNW * 64;
            if (e < 2048) hpa::store_wt4(slab, (own + e) * 4, vals[i]);
        }
        float rsum = 0.f;  // thread t < 128: row t / 2's sum (t even) or sum of squares
        if (fold && threadIdx.x < 128) {
            rsum = wsum[threadIdx.x] + wsum[128 + threadIdx.x];
            hpa::store_wt4(slab, (own + 2048 + threadIdx.x) * 4, rsum);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drained
        __shared__ int s_last;
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        if (threadIdx.x == 0) {
            const int t = __hip_atomic_fetch_add(p.sk_cnt + pair, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_last = t == nparts - 1;
            if (t == nparts - 1) __hip_atomic_store(p.sk_cnt + pair, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        if (!s_last) return;
        // the last part: every part's value in part order (own from registers)
        const int pb = pair * nparts * kRnPartF;
#pragma unroll
        for (int i = 0; i < EPT; ++i) {
            const int e = threadIdx.x + i * kRnNW * 64;
            if (e < 2048) {
                float v = 0.f;
                for (int q = 0; q < nparts; ++q) v += q == part ? vals[i] : hpa::load_wt4(slab, (pb + q * kRnPartF + e) * 4);
                vals[i] = v;
            }
        }
        if (fold && threadIdx.x < 128) {
            float v = 0.f;
            for (int q = 0; q < nparts; ++q) v += q == part ? rsum : hpa::load_wt4(slab, (pb + q * kRnPartF + 2048 + threadIdx.x) * 4);
            wsum[threadIdx.x] = v;  // slot 0: the whole K; slot 1 emptied
            wsum[128 + threadIdx.x] = 0.f;
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
    epi.apply(p, vals, tile, nt0, 0, wsum);
}

template <int EPI>
int launch_ring_epi(const FG& p, int mode, int parts) {
    const unsigned npairs = (unsigned)((p.ntn + 1) / 2);
    if (parts > 1) {
        gemm_ring_kernel<EPI, 0, 4, true><<<npairs * (unsigned)parts, kRnNW * 64, 0, hpa_stream()>>>(p);
    } else {
#ifdef HPA_RING_DIAG  // diagnostic build only (tools/ring_modes.sh): never in the product library
        switch (mode) {
            case 0: gemm_ring_kernel<EPI, 0, 8, false><<<npairs, kRnNW * 64, 0, hpa_stream()>>>(p); break;
            case 1: gemm_ring_kernel<EPI, 1, 8, false><<<npairs, kRnNW * 64, 0, hpa_stream()>>>(p); break;
            case 2: gemm_ring_kernel<EPI, 2, 8, false><<<npairs, kRnNW * 64, 0, hpa_stream()>>>(p); break;
            case 3: gemm_ring_kernel<EPI, 3, 8, false><<<npairs, kRnNW * 64, 0, hpa_stream()>>>(p); break;
            default: gemm_ring_kernel<EPI, 4, 8, false><<<npairs, kRnNW * 64, 0, hpa_stream()>>>(p); break;
        }
#else
        (void)mode;
        gemm_ring_kernel<EPI, 0, 8, false><<<npairs, kRnNW * 64, 0, hpa_stream()>>>(p);
#endif
    }
    HPA_LAUNCH_CHECK();
    return 0;
}

}  // namespace

// at most 64 padded rows (4 row blocks; fewer compute on a repeated block
// and store nothing), an even or odd tile count, LN folded or absent (no LN
// applied on load), an epilogue other than LOGITS
bool ring_eligible(const FG& p, int epi) {
    return p.Mp <= 64 && p.M <= 64 && p.K16 >= 1 && (!p.ln_stats || p.fold_c1) &&
           (epi == HPA_FEPI_QKV || epi == HPA_FEPI_GELU || epi == HPA_FEPI_RESID);
}

// parts: K parts (1 = no split; 2..4 with p.sk_slab / p.sk_cnt from
// hpa_gemm_ring_workspace).  HPA_RING_MODE=1..4 in a -DHPA_RING_DIAG build
// only: the unsplit kernel's diagnostic forms (no MFMAs / no LDS-DMA / no
// barriers / register operands); the product library has none of them
int launch_ring(const FG& p_in, int epi, int parts) {
    HPA_REQUIRE(ring_eligible(p_in, epi), "gemm_fused ring (variant 3): <= 64 padded rows, LN folded or none, "
                                          "QKV / GELU / RESID");
    HPA_REQUIRE(parts >= 1 && parts <= 4, "gemm_fused ring: K parts 1..4");
    HPA_REQUIRE(parts == 1 || (p_in.sk_slab && p_in.sk_cnt), "gemm_fused ring: K split needs sk_slab / sk_count");
    HPA_REQUIRE(parts == 1 || (p_in.K16 + 3) / 4 >= parts, "gemm_fused ring: fewer 4-step stages than K parts");
#ifdef HPA_RING_DIAG
    static const int mode = [] {
        const char* e = getenv("HPA_RING_MODE");
        return e ? atoi(e) : 0;
    }();
#else
    constexpr int mode = 0;
#endif
    FG p = p_in;
    p.gy = parts;
    switch (epi) {
        case HPA_FEPI_QKV: return launch_ring_epi<HPA_FEPI_QKV>(p, mode, parts);
        case HPA_FEPI_GELU: return launch_ring_epi<HPA_FEPI_GELU>(p, mode, parts);
        default: return launch_ring_epi<HPA_FEPI_RESID>(p, mode, parts);
    }
}

}  // namespace hpa_gemm

// K-split workspace of the ring kernel (variant 3, waves = K parts) for an
// (N) GEMM: slab floats and counters (zero before the first launch; every
// launch leaves them zero)
extern "C" int hpa_gemm_ring_workspace(int N, int parts, size_t* slab_floats, size_t* counters) {
    if (N <= 0 || parts < 1 || parts > 4 || !slab_floats || !counters) return 1;
    const size_t npairs = (size_t)((N + 15) / 16 + 1) / 2;
    *slab_floats = npairs * (size_t)parts * hpa_gemm::kRnPartF;
    *counters = npairs;
    return 0;
}
