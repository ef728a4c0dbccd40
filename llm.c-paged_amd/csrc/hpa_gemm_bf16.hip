// hpa_gemm_bf16.hip -- the fused decode GEMMs on bf16 weights (BASELINE
// config 5, "GPT-2 124M bf16 decode"; SURVEY.md §8f rank 3: "bf16 weights
// kept bf16 in HBM").
//
// Same launches, epilogues and XCD-aware grid as the fp32 looped kernel
// (hpa_fused.hip / hpa_gemm_body.h gemm16_body), with two differences:
//  * weights live in HBM as bf16 (half the bytes of the fp32 pack) in the
//    "bf16 frag" layout below, and the A operand (LN'ed activations, still
//    fp32 in HBM) is rounded to bf16 (round to nearest even) in registers;
//  * the contraction is v_mfma_f32_16x16x32_bf16 (16x the fp32 MFMA rate,
//    MI355X_MICROARCH.md), fp32 accumulation; bf16 x bf16 products are exact
//    in fp32, so the only rounding beyond fp32 is the operands' own.
// The numerics are "bf16 storage of weights and GEMM inputs, fp32 arithmetic"
// (train_gpt2.cu's bf16 mode); the oracle restates them
// (oracle_paged_set_w_bf16).
//
// bf16 frag layout of a [rows][K] matrix (rows padded to 16, K % 32 == 0): the
// v_mfma_f32_16x16x32_bf16 operand fragment of (16-row block, 32-deep k-step
// s) is 1 KiB contiguous, 16 bytes per lane.  Lane l = (row l & 15, group
// g = l >> 4) holds k = 32s + 4g + {0..3} in elements 0..3 and
// k = 32s + 16 + 4g + {0..3} in elements 4..7 -- exactly the two float4s the
// same lane loads from the fp32 frag layout at k16-steps 2s and 2s+1, so the
// A operand is built from fp32 frag activations with no data movement.  The
// MFMA sums over the k slots of a lane group in any order as long as A and B
// agree, which they do by construction (cdna_hip_programming.md "A/B operand
// lane maps, bf16").
#include <math.h>

#include "hpa_gemm_body.h"

namespace hpa_gemm {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));

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

// k-steps (32 deep) per trip, two trips in flight: by the registers one step
// holds (NTW weight fragments + 2*MT activation float4s per lane)
template <int MT, int NTW>
constexpr int b16_trip() {
    return (2 * MT + NTW) <= 3 ? 4 : (2 * MT + NTW) <= 6 ? 2 : 1;
}

// MT = 16-row blocks, NTW = 16-column tiles per workgroup, NW = waves sharing
// the K range (contiguous runs of 32-deep steps, folded in wave order in the
// epilogue): a row's summation order depends on NW only, never on MT, NTW, M.
template <int NW, int EPI, int MT, int NTW>
__global__ __launch_bounds__(NW * 64) void gemm_b16_kernel(FG p) {
    constexpr int U = b16_trip<MT, NTW>();
    __shared__ __attribute__((aligned(16))) float smem[gemm16_lds_floats<NW, MT, NTW>()];
    constexpr int R = MT * 16;
    float* lngb = smem;                         // LN weight [K], bias [K]
    float* red = smem + 2 * HPA_FUSED_LN_KMAX;  // [NW][NTW][MT x 4][64]
    float* tile = red + NW * MT * NTW * 256;    // [NTW][R][17]
    float* lnst = tile + NTW * R * 17;          // [R][2]
    float* lnscr = lnst + 2 * R;                // [4R][2]

    int cx, ry;
    if (!xcd_tile(p, blockIdx.x, cx, ry)) return;
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const int nt0 = cx * NTW;
    const int row0 = ry * MT * 16;
    const int q4 = lane >> 4;

    const int K32 = p.K >> 5;
    const int per = (K32 + NW - 1) / NW;
    const int kb0 = w * per;
    const int nsteps = max(0, min(K32, kb0 + per) - kb0);
    const uint4* __restrict__ wf[NTW];
#pragma unroll
    for (int j = 0; j < NTW; ++j)  // tail tiles past ntn re-read the last tile (never stored)
        wf[j] = reinterpret_cast<const uint4*>(p.w) + (size_t)min(nt0 + j, p.ntn - 1) * K32 * 64 + lane;
    const float4* __restrict__ xf = reinterpret_cast<const float4*>(p.x) + (size_t)ry * MT * p.K16 * 64 + lane;
    const size_t rbs = (size_t)p.K16 * 64;  // float4 stride between row blocks
    const bool ln_apply = p.ln_stats != nullptr;
    const float4* sg = reinterpret_cast<const float4*>(lngb) + q4;
    const float4* sb = reinterpret_cast<const float4*>(lngb + HPA_FUSED_LN_KMAX) + q4;

    struct Buf {
        uint4 w[U][NTW];
        float4 x[U][MT][2];
    };
    Buf A, Bb;
    auto load = [&](Buf& f, int t) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int k = kb0 + min(t * U + u, max(nsteps - 1, 0));  // clamped, unconditional
#pragma unroll
            for (int j = 0; j < NTW; ++j) f.w[u][j] = wf[j][(size_t)k * 64];
#pragma unroll
            for (int r = 0; r < MT; ++r) {
                f.x[u][r][0] = xf[r * rbs + (size_t)(2 * k) * 64];
                f.x[u][r][1] = xf[r * rbs + (size_t)(2 * k + 1) * 64];
            }
        }
    };
    const int trips = (nsteps + U - 1) / U;
    if (trips > 0) load(A, 0);  // first operands in flight during the LN prologue

    float mu[MT], rs[MT];
#pragma unroll
    for (int r = 0; r < MT; ++r) mu[r] = rs[r] = 0.f;
    if (ln_apply) ln_prologue<NW, MT>(p, lngb, lnst, lnscr, row0, true, mu, rs);

    f32x4 acc[MT * NTW];
#pragma unroll
    for (int i = 0; i < MT * NTW; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto comp = [&](Buf& f, int t) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (t * U + u < nsteps) {
                const int k = kb0 + t * U + u;
                float4 g0, b0, g1, b1;
                if (ln_apply) {
                    g0 = sg[4 * (2 * k)];
                    b0 = sb[4 * (2 * k)];
                    g1 = sg[4 * (2 * k + 1)];
                    b1 = sb[4 * (2 * k + 1)];
                }
                bf16x8 xa[MT];
#pragma unroll
                for (int r = 0; r < MT; ++r) {
                    float4 x0 = f.x[u][r][0], x1 = f.x[u][r][1];
                    if (ln_apply) {
                        x0 = ln4(x0, mu[r], rs[r], g0, b0);
                        x1 = ln4(x1, mu[r], rs[r], g1, b1);
                    }
                    xa[r] = pack_bf16(x0, x1);
                }
#pragma unroll
                for (int j = 0; j < NTW; ++j) {
                    const bf16x8 wb = __builtin_bit_cast(bf16x8, f.w[u][j]);
#pragma unroll
                    for (int r = 0; r < MT; ++r)
                        acc[j * MT + r] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xa[r], wb, acc[j * MT + r], 0, 0, 0);
                }
            }
        }
    };
    for (int t = 0; t < trips; t += 2) {
        if (t + 1 < trips) load(Bb, t + 1);
        comp(A, t);
        if (t + 1 >= trips) break;
        if (t + 2 < trips) load(A, t + 2);
        comp(Bb, t + 1);
    }

    Epi<NW, EPI, MT, NTW> epi;
    epi.prefetch(p, nt0, row0);
    epi.finish(p, acc, red, tile, nt0, row0, lngb);
}

// ---- A-resident variant (variant 5): the workgroup's MT*16 rows of A are
// LayerNorm'ed and rounded to bf16 ONCE into LDS (bf16 frag layout), then its
// waves walk the workgroup's chunk of column tiles in rounds -- wave w takes
// tile c0 + round*NW + w over the whole K (no K split, no fold), streaming
// its weight fragments U steps ahead and reading A fragments from LDS.  The
// looped kernel instead re-reads (and re-normalises) the fp32 A rows for
// every column-tile group: at M = 256 that A traffic, not the MFMA, bounds
// it.  A row's sum is one in-order k chain per wave (differs from the looped
// kernel's per-wave ranges; equal for every launch shape of this variant).
// KC = A capacity in 32-deep steps (24: K <= 768, 50: 1600, 100: 3200), MT*KC <= 100
// (100 KiB of bf16): the LDS, hence the workgroups per CU, follows K
// The LN weights (staging only) and the epilogue's fold / row-statistics
// scratch (rounds only) share one region, so the K = 768 / MT = 2 instance
// fits two workgroups per CU.
template <int NW, int MT>
constexpr int ares_union_floats() {
    constexpr int red = NW * MT * 256 > NW * MT * 16 * 17 ? NW * MT * 256 : NW * MT * 16 * 17;
    return red > 2 * HPA_FUSED_LN_KMAX ? red : 2 * HPA_FUSED_LN_KMAX;
}
template <int NW, int MT, int KC>
constexpr int ares_lds_floats() {
    return ares_union_floats<NW, MT>() + 10 * MT * 16 + MT * KC * 64 * 4;
}

template <int NW, int EPI, int MT, int KC, int U>
__global__ __launch_bounds__(NW * 64) void gemm_b16_ares_kernel(FG p, int cpw) {
    constexpr int NT = NW * 64;
    constexpr int R = MT * 16;
    constexpr int TE = MT * 256;
    constexpr int EPT = TE / 64;  // elements per thread of one round (NW tiles x TE over NT)
    __shared__ __attribute__((aligned(16))) float smem[ares_lds_floats<NW, MT, KC>()];
    float* lngb = smem;                       // LN weight [K], bias [K] (staging only)
    float* red = smem;                        // [NW][TE] fold / tile scratch (rounds only)
    float* lnst = smem + ares_union_floats<NW, MT>();  // [R][2]
    float* lnscr = lnst + 2 * R;              // [4R][2]
    uint4* As = reinterpret_cast<uint4*>(lnscr + 8 * R);  // [MT][K32][64 lanes] bf16x8

    int cx, ry;
    if (!xcd_tile(p, blockIdx.x, cx, ry)) return;
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const int row0 = ry * R;
    const int K32 = p.K >> 5;
    const int t_begin = cx * cpw, t_end = min(p.ntn, t_begin + cpw);

    // 1. A: LN'ed, rounded, into LDS
    const bool ln_apply = p.ln_stats != nullptr;
    float mu[MT], rs[MT];
    if (ln_apply) ln_prologue<NW, MT>(p, lngb, lnst, lnscr, row0, true, mu, rs);
    {
        const float4* xf = reinterpret_cast<const float4*>(p.x) + (size_t)ry * MT * p.K16 * 64 + lane;
        const float4* sg = reinterpret_cast<const float4*>(lngb) + (lane >> 4);
        const float4* sb = reinterpret_cast<const float4*>(lngb + HPA_FUSED_LN_KMAX) + (lane >> 4);
        const int nst = MT * K32;
        for (int i = w; i < nst; i += NW) {  // (row block, step) pairs, one per wave
            const int r = i / K32, st = i - r * K32;
            float4 x0 = xf[(size_t)r * p.K16 * 64 + (size_t)(2 * st) * 64];
            float4 x1 = xf[(size_t)r * p.K16 * 64 + (size_t)(2 * st + 1) * 64];
            if (ln_apply) {
                const float m = lnst[2 * (16 * r + (lane & 15))], q = lnst[2 * (16 * r + (lane & 15)) + 1];
                x0 = ln4(x0, m, q, sg[4 * (2 * st)], sb[4 * (2 * st)]);
                x1 = ln4(x1, m, q, sg[4 * (2 * st + 1)], sb[4 * (2 * st + 1)]);
            }
            As[(size_t)(r * K32 + st) * 64 + lane] = __builtin_bit_cast(uint4, pack_bf16(x0, x1));
        }
    }
    __syncthreads();

    // 2. rounds of NW column tiles
    for (int tb = t_begin; tb < t_end; tb += NW) {
        Epi<NW, EPI, MT, NW> epi;
        epi.prefetch(p, tb, row0);
        const int t = min(tb + w, p.ntn - 1);  // past the chunk: computed, never stored (col >= N or next round)
        const uint4* wp = reinterpret_cast<const uint4*>(p.w) + (size_t)t * K32 * 64 + lane;
        f32x4 acc[MT];
#pragma unroll
        for (int r = 0; r < MT; ++r) acc[r] = f32x4{0.f, 0.f, 0.f, 0.f};
        uint4 wq[U];
#pragma unroll
        for (int u = 0; u < U; ++u) wq[u] = wp[(size_t)min(u, K32 - 1) * 64];
        for (int s0 = 0; s0 < K32; s0 += U) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int st = s0 + u;
                const uint4 wc = wq[u];
                wq[u] = wp[(size_t)min(st + U, K32 - 1) * 64];  // U steps ahead, clamped (unconditional)
                if (st < K32) {
                    const bf16x8 wb = __builtin_bit_cast(bf16x8, wc);
#pragma unroll
                    for (int r = 0; r < MT; ++r) {
                        const bf16x8 a = __builtin_bit_cast(bf16x8, As[(size_t)(r * K32 + st) * 64 + lane]);
                        acc[r] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, wb, acc[r], 0, 0, 0);
                    }
                }
            }
        }
        // wave w's tile is column tile j = w of the round's Epi<.., NTW = NW>
#pragma unroll
        for (int r = 0; r < MT; ++r)
#pragma unroll
            for (int g = 0; g < 4; ++g) red[w * TE + (r * 4 + g) * 64 + lane] = acc[r][g];
        __syncthreads();
        float vals[EPT];
#pragma unroll
        for (int i = 0; i < EPT; ++i) vals[i] = red[threadIdx.x + i * NT];
        __syncthreads();  // tile (the row statistics' scratch) aliases red
        epi.apply(p, vals, red, tb, row0, nullptr);
        __syncthreads();
    }
}

template <int NW, int MT, int KC>
static int launch_ares_t(FG p, int epi, int rounds) {
    constexpr int U = 8;
    const int gy = p.Mp / 16 / MT;
    if (rounds <= 0) {  // auto: one pass of workgroups over the CUs at this LDS footprint
        constexpr int lds = ares_lds_floats<NW, MT, KC>() * 4;
        const int per_cu = (160 * 1024) / lds > 0 ? (160 * 1024) / lds : 1;
        const int slots = 256 * per_cu;
        rounds = (p.ntn * gy + NW * slots - 1) / (NW * slots);
        if (rounds < 1) rounds = 1;
    }
    const int cpw = NW * rounds;
    const int gx = (p.ntn + cpw - 1) / cpw;
    p.gx = gx;
    p.gy = gy;
    dim3 grid((unsigned)(((gx + 7) / 8) * 8 * gy)), block(NW * 64);
    switch (epi) {
        case HPA_FEPI_QKV: gemm_b16_ares_kernel<NW, HPA_FEPI_QKV, MT, KC, U><<<grid, block, 0, hpa_stream()>>>(p, cpw); break;
        case HPA_FEPI_RESID: gemm_b16_ares_kernel<NW, HPA_FEPI_RESID, MT, KC, U><<<grid, block, 0, hpa_stream()>>>(p, cpw); break;
        case HPA_FEPI_GELU: gemm_b16_ares_kernel<NW, HPA_FEPI_GELU, MT, KC, U><<<grid, block, 0, hpa_stream()>>>(p, cpw); break;
        case HPA_FEPI_LOGITS: gemm_b16_ares_kernel<NW, HPA_FEPI_LOGITS, MT, KC, U><<<grid, block, 0, hpa_stream()>>>(p, cpw); break;
        default: return hpa_fail(__FILE__, __LINE__, "gemm_fused bf16: unknown epilogue");
    }
    HPA_LAUNCH_CHECK();
    return 0;
}

int launch_b16_ares(const FG& p, int epi, int nw, int mt, int rounds) {
    HPA_REQUIRE(rounds >= 0 && (p.Mp / 16) % mt == 0, "gemm_fused bf16 A-resident: rounds >= 0 (0: auto), row blocks of M");
    HPA_REQUIRE((mt == 4 && p.K <= 768) || (mt == 2 && p.K <= 1600) || (mt == 1 && p.K <= 3200),
                "gemm_fused bf16 A-resident: row_blocks * K <= 3200 (4: K <= 768, 2: 1600, 1: 3200)");
    const int k32 = p.K / 32;
    const int kc = k32 <= 24 ? 24 : k32 <= 50 ? 50 : 100;
    switch (nw * 1000 + mt * 100 + kc) {  // kc in {24, 50, 100}: keys unique
        case 4424: return launch_ares_t<4, 4, 24>(p, epi, rounds);
        case 4224: return launch_ares_t<4, 2, 24>(p, epi, rounds);
        case 4250: return launch_ares_t<4, 2, 50>(p, epi, rounds);
        case 4124: return launch_ares_t<4, 1, 24>(p, epi, rounds);
        case 4150: return launch_ares_t<4, 1, 50>(p, epi, rounds);
        case 4200: return launch_ares_t<4, 1, 100>(p, epi, rounds);  // mt 1, kc 100
        case 8424: return launch_ares_t<8, 4, 24>(p, epi, rounds);
        case 8224: return launch_ares_t<8, 2, 24>(p, epi, rounds);
        case 8250: return launch_ares_t<8, 2, 50>(p, epi, rounds);
        case 8124: return launch_ares_t<8, 1, 24>(p, epi, rounds);
        case 8150: return launch_ares_t<8, 1, 50>(p, epi, rounds);
        case 8200: return launch_ares_t<8, 1, 100>(p, epi, rounds);
        default: return hpa_fail(__FILE__, __LINE__, "gemm_fused bf16 A-resident: waves 4/8, row_blocks 1/2/4");
    }
}

template <int NW, int MT, int NTW>
static int launch_b16_t(FG p, int epi) {
    const int gx = (p.ntn + NTW - 1) / NTW, gy = p.Mp / 16 / MT;
    p.gx = gx;
    p.gy = gy;
    dim3 grid((unsigned)(((gx + 7) / 8) * 8 * gy)), block(NW * 64);
    switch (epi) {
        case HPA_FEPI_QKV: gemm_b16_kernel<NW, HPA_FEPI_QKV, MT, NTW><<<grid, block, 0, hpa_stream()>>>(p); break;
        case HPA_FEPI_RESID: gemm_b16_kernel<NW, HPA_FEPI_RESID, MT, NTW><<<grid, block, 0, hpa_stream()>>>(p); break;
        case HPA_FEPI_GELU: gemm_b16_kernel<NW, HPA_FEPI_GELU, MT, NTW><<<grid, block, 0, hpa_stream()>>>(p); break;
        case HPA_FEPI_LOGITS: gemm_b16_kernel<NW, HPA_FEPI_LOGITS, MT, NTW><<<grid, block, 0, hpa_stream()>>>(p); break;
        default: return hpa_fail(__FILE__, __LINE__, "gemm_fused bf16: unknown epilogue");
    }
    HPA_LAUNCH_CHECK();
    return 0;
}

template <int NW>
static int launch_b16_nw(const FG& p, int epi, int mt, int ntw) {
    switch (mt * 10 + ntw) {
        case 11: return launch_b16_t<NW, 1, 1>(p, epi);
        case 21: return launch_b16_t<NW, 2, 1>(p, epi);
        case 41: return launch_b16_t<NW, 4, 1>(p, epi);
        case 22: return launch_b16_t<NW, 2, 2>(p, epi);
        case 42: return launch_b16_t<NW, 4, 2>(p, epi);
        default:
            return hpa_fail(__FILE__, __LINE__,
                            "gemm_fused bf16: (row_blocks, col_tiles) in {(1,1), (2,1), (4,1), (2,2), (4,2)}");
    }
}

int launch_b16(const FG& p, int epi, int nw, int mt, int ntw) {
    switch (nw) {
        case 4: return launch_b16_nw<4>(p, epi, mt, ntw);
        case 8: return launch_b16_nw<8>(p, epi, mt, ntw);
        default: return hpa_fail(__FILE__, __LINE__, "gemm_fused bf16: waves must be 4 or 8");
    }
}

}  // namespace hpa_gemm

namespace {
// one thread per (fragment, lane): 8 bf16 (RNE) from two float4 of row m
__global__ void pack_frag_bf16_kernel(const float* __restrict__ src, int rows, int K, int ld,
                                      uint4* __restrict__ dst, size_t n8) {
    const size_t o = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (o >= n8) return;
    const int lane = (int)(o & 63);
    const size_t blk = o >> 6;  // rb * K32 + s
    const int K32 = K >> 5;
    const int s = (int)(blk % K32);
    const int rb = (int)(blk / K32);
    const int m = rb * 16 + (lane & 15);
    const int k0 = s * 32 + 4 * (lane >> 4);
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
    if (m < rows) {
        a = *reinterpret_cast<const float4*>(src + (size_t)m * ld + k0);
        b = *reinterpret_cast<const float4*>(src + (size_t)m * ld + k0 + 16);
    }
    dst[o] = __builtin_bit_cast(uint4, hpa_gemm::pack_bf16(a, b));
}
}  // namespace

extern "C" {

size_t hpa_frag_bf16_elems(int rows, int K) { return (size_t)((rows + 15) / 16) * 16 * (size_t)K; }

int hpa_pack_frag_bf16(const float* src, int rows, int K, int ld, void* dst) {
    HPA_REQUIRE(src && dst && rows > 0 && K > 0 && K % 32 == 0 && ld >= K && ld % 4 == 0,
                "pack_frag_bf16: bad shape (K % 32, ld % 4)");
    const size_t n8 = hpa_frag_bf16_elems(rows, K) / 8;
    pack_frag_bf16_kernel<<<(unsigned)((n8 + 255) / 256), 256, 0, hpa_stream()>>>(src, rows, K, ld,
                                                                                 reinterpret_cast<uint4*>(dst), n8);
    HPA_LAUNCH_CHECK();
    return 0;
}

}  // extern "C"
