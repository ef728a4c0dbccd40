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
#include "hpa_gemm_body.h"
#ifndef HPA_RES_EXP
#define HPA_RES_EXP 0  // timing experiments (tools/logits_exp.sh); 0 in the product
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
            __builtin_amdgcn_raw_buffer_store_b64(pv, part_rs, ((int)blockIdx.x * p.Mp + frow) * 8, 0, 0);
        }
    }
}

int g_num_cus = 0;

template <int MT>
int launch_resident_mt(const FG& p) {
    logits_resident_kernel<MT><<<(unsigned)logits_resident_grid(p), kResNW * 64, 0, hpa_stream()>>>(p);
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
    return epi == HPA_FEPI_LOGITS && p.ln_stats && p.K16 == kResNW * kResS && p.Mp <= 64 && p.M <= p.Mp;
}

int launch_logits_resident(const FG& p) {
    switch (p.Mp / 16) {
        case 1: return launch_resident_mt<1>(p);
        case 2: return launch_resident_mt<2>(p);
        case 3: return launch_resident_mt<3>(p);
        case 4: return launch_resident_mt<4>(p);
        default: return hpa_fail(__FILE__, __LINE__, "logits: rows must be <= 64");
    }
}

}  // namespace hpa_gemm
