// hpa_gemm_ares.hip -- the A-resident fp32 decode GEMM (variant 5 with fp32
// weights): the bf16 A-resident structure (hpa_gemm_bf16.hip) on exact fp32
// v_mfma_f32_16x16x4_f32.  The workgroup's 16*MT rows of A are LayerNorm'ed
// once into LDS (fp32 frag layout, MT*K <= 1600 floats per row block column:
// <= 100 KiB), then wave w takes column tile c0 + round*NW + w over the
// whole K, streaming its weight fragments U k16-steps ahead and reading A
// fragments from LDS.  No K split, no fold: each output is one in-order k
// chain per wave, the same for every launch shape of this kernel (it differs
// from the looped kernel's wave-range fold, so a GEMM uses one or the other
// by (N, K), never by M -- hpa_fused_pick_f32_ares).
// Meant for the MFMA-bound GEMMs whose looped grid leaves CUs idle or whose
// A re-reads per column-tile group cost more than the MFMA (GPT-2 XL layer
// GEMMs, logits).
#include <math.h>

#include "hpa_gemm_body.h"

namespace hpa_gemm {

// KC = A capacity in 16-deep steps (48: K <= 768, 100: K <= 1600), MT*KC <= 100
template <int NW, int MT, int KC>
constexpr int ares32_lds_floats() {
    return 2 * HPA_FUSED_LN_KMAX + 10 * MT * 16 + MT * KC * 64 * 4 +
           (NW * MT * 256 > NW * MT * 16 * 17 ? NW * MT * 256 : NW * MT * 16 * 17);
}

template <int NW, int EPI, int MT, int KC, int U>
__global__ __launch_bounds__(NW * 64) void gemm_f32_ares_kernel(FG p, int cpw) {
    constexpr int NT = NW * 64;
    constexpr int R = MT * 16;
    constexpr int TE = MT * 256;
    constexpr int EPT = TE / 64;
    __shared__ __attribute__((aligned(16))) float smem[ares32_lds_floats<NW, MT, KC>()];
    float* lngb = smem;
    float* lnst = lngb + 2 * HPA_FUSED_LN_KMAX;
    float* lnscr = lnst + 2 * R;
    float4* As = reinterpret_cast<float4*>(lnscr + 8 * R);  // [MT][K16][64 lanes]
    float* red = reinterpret_cast<float*>(As + MT * KC * 64);  // [NW][TE]; aliased by tile

    int cx, ry, slice;
    if (!xcd_tile(p, blockIdx.x, cx, ry, slice)) return;
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const int row0 = ry * R;
    const int K16 = p.K16;
    const int t_begin = cx * cpw, t_end = min(p.ntn, t_begin + cpw);

    const bool ln_apply = p.ln_stats != nullptr;
    float mu[MT], rs[MT];
    if (ln_apply) ln_prologue<NW, MT>(p, lngb, lnst, lnscr, row0, true, mu, rs);
    {
        const float4* xf = reinterpret_cast<const float4*>(p.x) + (size_t)ry * MT * K16 * 64 + lane;
        const float4* sg = reinterpret_cast<const float4*>(lngb) + (lane >> 4);
        const float4* sb = reinterpret_cast<const float4*>(lngb + HPA_FUSED_LN_KMAX) + (lane >> 4);
        for (int i = w; i < MT * K16; i += NW) {
            const int r = i / K16, st = i - r * K16;
            float4 x = xf[(size_t)r * K16 * 64 + (size_t)st * 64];
            if (ln_apply)
                x = ln4(x, lnst[2 * (16 * r + (lane & 15))], lnst[2 * (16 * r + (lane & 15)) + 1], sg[4 * st],
                        sb[4 * st]);
            As[(size_t)(r * K16 + st) * 64 + lane] = x;
        }
    }
    __syncthreads();

    for (int tb = t_begin; tb < t_end; tb += NW) {
        Epi<NW, EPI, MT, NW> epi;
        epi.prefetch(p, tb, row0);
        const int t = min(tb + w, p.ntn - 1);
        const float4* wp = reinterpret_cast<const float4*>(p.w) + (size_t)t * K16 * 64 + lane;
        f32x4 acc[MT];
#pragma unroll
        for (int r = 0; r < MT; ++r) acc[r] = f32x4{0.f, 0.f, 0.f, 0.f};
        float4 wq[U];
#pragma unroll
        for (int u = 0; u < U; ++u) wq[u] = wp[(size_t)min(u, K16 - 1) * 64];
        for (int s0 = 0; s0 < K16; s0 += U) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int st = s0 + u;
                const float4 wc = wq[u];
                wq[u] = wp[(size_t)min(st + U, K16 - 1) * 64];
                if (st < K16) {
                    float4 a[MT];
#pragma unroll
                    for (int r = 0; r < MT; ++r) a[r] = As[(size_t)(r * K16 + st) * 64 + lane];
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const float ws = q == 0 ? wc.x : q == 1 ? wc.y : q == 2 ? wc.z : wc.w;
#pragma unroll
                        for (int r = 0; r < MT; ++r) {
                            const float xs = q == 0 ? a[r].x : q == 1 ? a[r].y : q == 2 ? a[r].z : a[r].w;
                            acc[r] = __builtin_amdgcn_mfma_f32_16x16x4f32(xs, ws, acc[r], 0, 0, 0);
                        }
                    }
                }
            }
        }
#pragma unroll
        for (int r = 0; r < MT; ++r)
#pragma unroll
            for (int g = 0; g < 4; ++g) red[w * TE + (r * 4 + g) * 64 + lane] = acc[r][g];
        __syncthreads();
        float vals[EPT];
#pragma unroll
        for (int i = 0; i < EPT; ++i) vals[i] = red[threadIdx.x + i * NT];
        __syncthreads();
        epi.apply(p, vals, red, red, tb, row0, nullptr, false);
        __syncthreads();
    }
}

template <int NW, int MT, int KC>
static int launch_f32_ares_t(FG p, int epi, int rounds) {
    constexpr int U = 8;
    const int cpw = NW * rounds;
    const int gx = (p.ntn + cpw - 1) / cpw, gy = p.Mp / 16 / MT;
    p.gx = gx;
    p.gy = gy;
    dim3 grid((unsigned)(((gx + 7) / 8) * 8 * gy)), block(NW * 64);
    switch (epi) {
        case HPA_FEPI_QKV: gemm_f32_ares_kernel<NW, HPA_FEPI_QKV, MT, KC, U><<<grid, block, 0, hpa_stream()>>>(p, cpw); break;
        case HPA_FEPI_RESID: gemm_f32_ares_kernel<NW, HPA_FEPI_RESID, MT, KC, U><<<grid, block, 0, hpa_stream()>>>(p, cpw); break;
        case HPA_FEPI_GELU: gemm_f32_ares_kernel<NW, HPA_FEPI_GELU, MT, KC, U><<<grid, block, 0, hpa_stream()>>>(p, cpw); break;
        case HPA_FEPI_LOGITS: gemm_f32_ares_kernel<NW, HPA_FEPI_LOGITS, MT, KC, U><<<grid, block, 0, hpa_stream()>>>(p, cpw); break;
        default: return hpa_fail(__FILE__, __LINE__, "gemm_fused A-resident: unknown epilogue");
    }
    HPA_LAUNCH_CHECK();
    return 0;
}

int launch_f32_ares(const FG& p, int epi, int nw, int mt, int rounds) {
    HPA_REQUIRE(rounds >= 1 && (p.Mp / 16) % mt == 0, "gemm_fused A-resident: rounds >= 1, row blocks of M");
    HPA_REQUIRE((mt == 2 && p.K <= 768) || (mt == 1 && p.K <= 1600),
                "gemm_fused A-resident fp32: row_blocks 2 (K <= 768) or 1 (K <= 1600)");
    const int kc = p.K16 <= 48 ? 48 : 100;
    switch (nw * 1000 + mt * 100 + kc) {
        case 4248: return launch_f32_ares_t<4, 2, 48>(p, epi, rounds);
        case 4148: return launch_f32_ares_t<4, 1, 48>(p, epi, rounds);
        case 4200: return launch_f32_ares_t<4, 1, 100>(p, epi, rounds);  // mt 1, kc 100
        case 8248: return launch_f32_ares_t<8, 2, 48>(p, epi, rounds);
        case 8148: return launch_f32_ares_t<8, 1, 48>(p, epi, rounds);
        case 8200: return launch_f32_ares_t<8, 1, 100>(p, epi, rounds);
        default: return hpa_fail(__FILE__, __LINE__, "gemm_fused A-resident fp32: waves 4/8, row_blocks 1/2");
    }
}

}  // namespace hpa_gemm
