// hpa_gemm.hip -- decode-row GEMM on gfx950 fp32 MFMA.
//
// out[M][N] = x[M][K] . W[N][K]^T  (W row-major [out][in], the PyTorch Linear
// layout of the llm.c checkpoint, train_gpt2.py:179-188).  Replaces
// matmul_forward / matmul_cached for the decode rows (reference
// paged_infer.c:92-160): at decode M = batch (<= 64 per row block) and the
// weights are streamed once per step.
//
// At M = 64 fp32 the weight GEMMs sit at ~32 FLOP/B, above the fp32 ridge
// (157 TF / 8 TB/s = 19.7), so the roof is the fp32 MFMA rate (exact f32
// v_mfma_f32_32x32x2_f32, 64 FLOP/clk/SIMD, MI355X_MICROARCH.md "Matrix
// cores"): the kernel's job is to keep every SIMD issuing MFMAs, which at
// N = 768..3072 needs a K split.
//
// Tiling: a workgroup owns a 64-row x 32-column output tile and a K range
// (blockIdx.z of `splitk`); its NW waves take interleaved 8-deep k-steps of
// that range, each into its own 2 x (32x32) f32 accumulators, and fold them in
// LDS in a fixed order (deterministic).  Per 8-deep k-step a lane issues one
// float4 load of W (row n0 + lane%32, k + 4*(lane/32)) and one float4 of each
// of the two x rows -- the A/B fragments of four 32x32x2 MFMAs each:
//   A[i][kk] = x[m0 + i][k + 4*(lane/32) + j],  B[kk][c] = W[n0 + c][same k]
// with j = 0..3 the float4 element.  Operands go straight to VGPRs (the
// "GEMV / M <= 16" row of the staging table: a weight operand streamed once
// gains nothing from an LDS round trip); x rows are L2-resident.
// splitk > 1 writes fp32 partial slabs [splitk][M][N] that the following row
// epilogue kernel sums (hpa_rows.hip), fusing bias / residual / LN / GELU /
// KV-append there.
#include "hpa_internal.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int NW, int EPI>
__global__ __launch_bounds__(NW * 64) void gemm_f32_m64n32(
    const float* __restrict__ x, int ldx, const float* __restrict__ W, const float* __restrict__ bias,
    float* __restrict__ out, int ldo, int M, int N, int K, int kchunk, size_t slab) {
    __shared__ float red[NW > 1 ? NW : 1][32][64];
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const int c = lane & 31;
    const int h = lane >> 5;
    const int n0 = blockIdx.x * 32;
    const int m0 = blockIdx.y * 64;
    const int kbeg = blockIdx.z * kchunk;
    const int kend = min(K, kbeg + kchunk);
    const int n = min(n0 + c, N - 1);
    const int r0 = min(m0 + c, M - 1);
    const int r1 = min(m0 + 32 + c, M - 1);
    const float* __restrict__ wp = W + (size_t)n * K + 4 * h;
    const float* __restrict__ xp0 = x + (size_t)r0 * ldx + 4 * h;
    const float* __restrict__ xp1 = x + (size_t)r1 * ldx + 4 * h;

    f32x16 acc0, acc1;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        acc0[i] = 0.f;
        acc1[i] = 0.f;
    }

    // this wave's k-steps: k = k0 + j*NW*8, j < nk.  Trips of U k-steps,
    // register double buffer: the loads of trip t+1 are in flight while the
    // MFMAs of trip t issue (the operand latency is otherwise exposed on
    // every trip: a wave has only a few trips at decode sizes).
    constexpr int U = 4;
    const int k0 = kbeg + w * 8;
    const int nk = k0 < kend ? (kend - k0 + NW * 8 - 1) / (NW * 8) : 0;
    float4 wa[U], xa0[U], xa1[U], wb[U], xb0[U], xb1[U];
    auto load = [&](float4 (&wv)[U], float4 (&a0)[U], float4 (&a1)[U], int t) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int j = t * U + u;
            if (j < nk) {
                const int kk = k0 + j * NW * 8;
                wv[u] = *reinterpret_cast<const float4*>(wp + kk);
                a0[u] = *reinterpret_cast<const float4*>(xp0 + kk);
                a1[u] = *reinterpret_cast<const float4*>(xp1 + kk);
            }
        }
    };
    auto compute = [&](const float4 (&wv)[U], const float4 (&a0)[U], const float4 (&a1)[U], int t) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (t * U + u < nk) {
                acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[u].x, wv[u].x, acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[u].x, wv[u].x, acc1, 0, 0, 0);
                acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[u].y, wv[u].y, acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[u].y, wv[u].y, acc1, 0, 0, 0);
                acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[u].z, wv[u].z, acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[u].z, wv[u].z, acc1, 0, 0, 0);
                acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[u].w, wv[u].w, acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[u].w, wv[u].w, acc1, 0, 0, 0);
            }
        }
    };
    const int trips = (nk + U - 1) / U;
    if (trips > 0) load(wa, xa0, xa1, 0);
    for (int t = 0; t < trips; t += 2) {
        if (t + 1 < trips) load(wb, xb0, xb1, t + 1);
        compute(wa, xa0, xa1, t);
        if (t + 1 >= trips) break;
        if (t + 2 < trips) load(wa, xa0, xa1, t + 2);
        compute(wb, xb0, xb1, t + 1);
    }

    // fold the NW waves' accumulators in LDS ([wave][reg][lane]: conflict-free)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        red[w][r][lane] = acc0[r];
        red[w][16 + r][lane] = acc1[r];
    }
    __syncthreads();
    float* __restrict__ o = out + (EPI == HPA_EPI_PARTIAL ? (size_t)blockIdx.z * slab : 0);
#pragma unroll
    for (int e = threadIdx.x; e < 2048; e += NW * 64) {
        const int reg = e >> 6;
        const int ln = e & 63;
        float s = red[0][reg][ln];
#pragma unroll
        for (int ww = 1; ww < NW; ++ww) s += red[ww][reg][ln];
        const int rr = reg & 15;
        // 32x32 C/D map: col = lane & 31, row = (reg&3) + 8*(reg>>2) + 4*(lane>>5)
        const int row = m0 + (reg >> 4) * 32 + (rr & 3) + 8 * (rr >> 2) + 4 * (ln >> 5);
        const int col = n0 + (ln & 31);
        if (row < M && col < N) {
            if (EPI == HPA_EPI_PARTIAL) {
                o[(size_t)row * ldo + col] = s;
            } else {
                float v = bias ? s + bias[col] : s;
                if (EPI == HPA_EPI_BIAS_GELU) v = hpa::gelu_ref(v);
                o[(size_t)row * ldo + col] = v;
            }
        }
    }
}

template <int NW>
int launch(dim3 grid, const float* x, int ldx, const float* W, const float* bias, float* out, int ldo,
           int M, int N, int K, int kchunk, size_t slab, int epilogue) {
    dim3 block(NW * 64);
    switch (epilogue) {
        case HPA_EPI_PARTIAL:
            gemm_f32_m64n32<NW, HPA_EPI_PARTIAL><<<grid, block, 0, hpa_stream()>>>(
                x, ldx, W, bias, out, ldo, M, N, K, kchunk, slab);
            break;
        case HPA_EPI_BIAS:
            gemm_f32_m64n32<NW, HPA_EPI_BIAS><<<grid, block, 0, hpa_stream()>>>(
                x, ldx, W, bias, out, ldo, M, N, K, kchunk, slab);
            break;
        case HPA_EPI_BIAS_GELU:
            gemm_f32_m64n32<NW, HPA_EPI_BIAS_GELU><<<grid, block, 0, hpa_stream()>>>(
                x, ldx, W, bias, out, ldo, M, N, K, kchunk, slab);
            break;
        default:
            return hpa_fail(__FILE__, __LINE__, "gemm: unknown epilogue");
    }
    HPA_LAUNCH_CHECK();
    return 0;
}

// waves per workgroup: 8 when there are few column tiles (the K split then
// stays inside the workgroup, reduced in LDS, instead of in HBM slabs)
int pick_waves(int M, int N) {
    const int ntiles = ((N + 31) / 32) * ((M + 63) / 64);
    return ntiles < 64 ? 8 : 4;
}

}  // namespace

extern "C" {

int hpa_gemm_pick_splitk(int M, int N, int K) {
    const int nblk = ((N + 31) / 32) * ((M + 63) / 64);
    const int nw = pick_waves(M, N);
    // aim for ~2048 waves (2 per SIMD) while every wave keeps >= 4 k-steps
    const int target_blocks = 2048 / nw;
    int s = (target_blocks + nblk - 1) / nblk;
    int smax = K / (nw * 8 * 4);
    if (smax < 1) smax = 1;
    if (s > smax) s = smax;
    if (s < 1) s = 1;
    return s;
}

int hpa_gemm_f32(const float* x, int ldx, const float* W, const float* bias, float* out, int ldo,
                 int M, int N, int K, int splitk, int epilogue) {
    HPA_REQUIRE(x && W && out, "gemm: null pointer");
    HPA_REQUIRE(M > 0 && N > 0 && K > 0, "gemm: empty shape");
    HPA_REQUIRE(K % 8 == 0 && ldx % 4 == 0 && ldx >= K, "gemm: K must be a multiple of 8, ldx of 4");
    HPA_REQUIRE(ldo >= N, "gemm: ldo < N");
    HPA_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)W & 15) == 0, "gemm: x/W must be 16-byte aligned");
    HPA_REQUIRE(splitk >= 1, "gemm: splitk >= 1");
    HPA_REQUIRE(splitk == 1 || epilogue == HPA_EPI_PARTIAL, "gemm: splitk > 1 needs the partial epilogue");
    int kchunk = (K + splitk - 1) / splitk;
    kchunk = (kchunk + 7) / 8 * 8;
    const int zs = (K + kchunk - 1) / kchunk;
    HPA_REQUIRE(zs == splitk || epilogue != HPA_EPI_PARTIAL, "gemm: splitk does not divide K into 8-multiples");
    dim3 grid((N + 31) / 32, (M + 63) / 64, zs);
    const size_t slab = (size_t)M * ldo;
    if (pick_waves(M, N) == 8)
        return launch<8>(grid, x, ldx, W, bias, out, ldo, M, N, K, kchunk, slab, epilogue);
    return launch<4>(grid, x, ldx, W, bias, out, ldo, M, N, K, kchunk, slab, epilogue);
}

}  // extern "C"
