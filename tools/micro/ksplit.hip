// Microbenchmark for the next-round K-split of the decode layer GEMMs
// (DESIGN.md section 7): M = 64 rows, fp32 v_mfma_f32_16x16x4_f32 on frag-layout
// operands as the product kernels (hpa_gemm_body.h), one workgroup = all 4
// row blocks x NTW column tiles x one of S K-ranges, NW waves splitting the
// range.  MODE 0 writes each range's partial tile (no combine: the load-side
// floor of the tiling); MODE 1 (S = 2) publishes the partial, takes an
// agent-scope ticket and the second arriver adds the first's partial (exact
// in either order: fp32 a + b == b + a) -- the combine's cost.  MODE 2: the
// same loads, no MFMAs (one VALU add per fragment keeps them live); MODE 3:
// the MFMAs on operands loaded once (no loads in the loop); MODE 4: MODE 0
// with s_setprio(1) around each MFMA cluster; MODE 5: MODE 0 with the
// younger half of the waves at priority 1 (cdna_hip_programming.md T5).
// Build: hipcc --offload-arch=gfx950 -O3 -o ksplit tools/micro/ksplit.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void init_kernel(float* p, size_t n, unsigned seed) {
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) p[i] = (float)((i * 2654435761u + seed) % 2001u) * 1e-3f - 1.0f;
}

template <int NTW, int NW, int MODE>
__global__ __launch_bounds__(NW * 64) void ks_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                     float* __restrict__ slab, float* __restrict__ out,
                                                     int* __restrict__ cnt, int K16, int S) {
    constexpr int MT = 4;
    constexpr int E = MT * NTW * 256;  // outputs of the workgroup
    constexpr int NT = NW * 64;
    __shared__ float red[NW * E];
    const int bid = blockIdx.x;
    const int cg = bid / S, kz = bid - cg * S;
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int kper = (K16 + S - 1) / S;
    const int k0 = kz * kper, k1 = min(K16, k0 + kper);
    const int per = (k1 - k0 + NW - 1) / NW;
    const int kb = k0 + wv * per, ke = min(k1, kb + per);
    const float4* x4 = reinterpret_cast<const float4*>(x) + lane;
    const float4* w4 = reinterpret_cast<const float4*>(w) + (size_t)cg * NTW * K16 * 64 + lane;
    f32x4 acc[MT * NTW];
#pragma unroll
    for (int i = 0; i < MT * NTW; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int n = max(0, ke - kb);
    float4 wa[NTW], xa[MT], wb[NTW], xb[MT];
    auto load = [&](float4* wr, float4* xr, int s) {
        if (MODE == 3 && s > 0) return;
        const int k = kb + min(s, max(n - 1, 0));
#pragma unroll
        for (int j = 0; j < NTW; ++j) wr[j] = w4[((size_t)j * K16 + k) * 64];
#pragma unroll
        for (int r = 0; r < MT; ++r) xr[r] = x4[((size_t)r * K16 + k) * 64];
    };
    auto comp = [&](const float4* wr, const float4* xr, int s) {
        if (MODE == 2) {
            if (s < n)
#pragma unroll
                for (int j = 0; j < NTW; ++j)
#pragma unroll
                    for (int r = 0; r < MT; ++r) acc[j * MT + r][0] += xr[r].x + wr[j].y;
            return;
        }
        if (s < n) {
            if (MODE == 4) __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int j = 0; j < NTW; ++j)
#pragma unroll
                    for (int r = 0; r < MT; ++r) {
                        const float xs = q == 0 ? xr[r].x : q == 1 ? xr[r].y : q == 2 ? xr[r].z : xr[r].w;
                        const float ws = q == 0 ? wr[j].x : q == 1 ? wr[j].y : q == 2 ? wr[j].z : wr[j].w;
                        acc[j * MT + r] = __builtin_amdgcn_mfma_f32_16x16x4f32(xs, ws, acc[j * MT + r], 0, 0, 0);
                    }
            if (MODE == 4) __builtin_amdgcn_s_setprio(0);
        }
    };
    if (MODE == 5 && wv >= NW / 2) __builtin_amdgcn_s_setprio(1);
    if (n > 0) load(wa, xa, 0);
    if (MODE == 3) {
#pragma unroll
        for (int j = 0; j < NTW; ++j) wb[j] = wa[j];
#pragma unroll
        for (int r = 0; r < MT; ++r) xb[r] = xa[r];
    }
    for (int s = 0; s < n; s += 2) {
        load(wb, xb, s + 1);
        comp(wa, xa, s);
        load(wa, xa, s + 2);
        comp(wb, xb, s + 1);
    }
#pragma unroll
    for (int i = 0; i < MT * NTW; ++i)
#pragma unroll
        for (int g = 0; g < 4; ++g) red[(wv * MT * NTW * 4 + i * 4 + g) * 64 + lane] = acc[i][g];
    __syncthreads();
    float v[E / NT];
#pragma unroll
    for (int i = 0; i < E / NT; ++i) {
        const int e = threadIdx.x + i * NT;
        float a = red[e];
#pragma unroll
        for (int ww = 1; ww < NW; ++ww) a += red[ww * E + e];
        v[i] = a;
    }
    float* mine = slab + (size_t)bid * E;
    if (MODE != 1 || S == 1) {
#pragma unroll
        for (int i = 0; i < E / NT; ++i) mine[threadIdx.x + i * NT] = v[i];
        return;
    }
    // MODE 1, S = 2: publish, ticket, the second arriver sums
#pragma unroll
    for (int i = 0; i < E / NT; ++i)
        __hip_atomic_store(mine + threadIdx.x + i * NT, v[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __threadfence();
    __syncthreads();
    __shared__ int s_ticket;
    if (threadIdx.x == 0) s_ticket = __hip_atomic_fetch_add(cnt + cg, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (s_ticket != 1) return;
    if (threadIdx.x == 0) __hip_atomic_store(cnt + cg, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const float* other = slab + (size_t)(cg * S + (1 - kz)) * E;
    float* o = out + (size_t)cg * E;
#pragma unroll
    for (int i = 0; i < E / NT; ++i) {
        const float b = __hip_atomic_load(other + threadIdx.x + i * NT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        o[threadIdx.x + i * NT] = v[i] + b;
    }
}

template <int NTW, int NW, int MODE>
static void run(const char* name, int K, int N, int S, float* x, float* w, float* slab, float* out, int* cnt) {
    const int K16 = K / 16, ntg = N / 16 / NTW;
    const int grid = ntg * S;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int i = 0; i < 5; ++i) ks_kernel<NTW, NW, MODE><<<grid, NW * 64>>>(x, w, slab, out, cnt, K16, S);
    const int it = 50;
    hipEventRecord(e0);
    for (int i = 0; i < it; ++i) ks_kernel<NTW, NW, MODE><<<grid, NW * 64>>>(x, w, slab, out, cnt, K16, S);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    const double wg_bytes = (4.0 + NTW) * 16.0 * ((K16 + S - 1) / S) * 16.0 * 4.0;
    const double per_cu = wg_bytes * ((grid + 255) / 256);
    printf("%-8s K=%5d N=%5d MT=4 NTW=%d NW=%2d S=%d mode=%d  WGs=%4d  %7.2f us  KB/WG=%6.1f  KB/CU(max)=%6.1f\n", name, K,
           N, NTW, NW, S, MODE, grid, 1000.0 * ms / it, wg_bytes / 1024, per_cu / 1024);
}

int main() {
    const size_t xe = 64ull * 6400, we = 6400ull * 6400;
    float *x, *w, *slab, *out;
    int* cnt;
    if (hipMalloc(&x, xe * 4) || hipMalloc(&w, we * 4) || hipMalloc(&slab, 64ull << 20) || hipMalloc(&out, 64ull << 20) ||
        hipMalloc(&cnt, 1 << 20))
        return 1;
    init_kernel<<<(xe + 255) / 256, 256>>>(x, xe, 1);
    init_kernel<<<(we + 255) / 256, 256>>>(w, we, 2);
    hipMemset(cnt, 0, 1 << 20);
    hipDeviceSynchronize();
    // GPT-2 124M, B = 64 (product one-shot: qkv 9.0, attproj 5.0, fc 9.0, fcproj 10.3 us in the step)
    run<1, 4, 0>("qkv", 768, 2304, 1, x, w, slab, out, cnt);
    run<1, 4, 0>("qkv", 768, 2304, 2, x, w, slab, out, cnt);
    run<1, 4, 1>("qkv", 768, 2304, 2, x, w, slab, out, cnt);
    run<2, 4, 0>("qkv", 768, 2304, 2, x, w, slab, out, cnt);
    run<2, 4, 1>("qkv", 768, 2304, 2, x, w, slab, out, cnt);
    run<2, 4, 0>("qkv", 768, 2304, 4, x, w, slab, out, cnt);
    run<1, 4, 0>("attproj", 768, 768, 2, x, w, slab, out, cnt);
    run<1, 4, 1>("attproj", 768, 768, 2, x, w, slab, out, cnt);
    run<1, 4, 0>("attproj", 768, 768, 4, x, w, slab, out, cnt);
    run<1, 4, 0>("fc", 768, 3072, 1, x, w, slab, out, cnt);
    run<1, 4, 1>("fc", 768, 3072, 2, x, w, slab, out, cnt);
    run<2, 4, 1>("fc", 768, 3072, 2, x, w, slab, out, cnt);
    run<1, 4, 0>("fcproj", 3072, 768, 4, x, w, slab, out, cnt);
    run<1, 4, 1>("fcproj", 3072, 768, 2, x, w, slab, out, cnt);
    run<1, 8, 1>("fcproj", 3072, 768, 2, x, w, slab, out, cnt);
    run<1, 4, 0>("fcproj", 3072, 768, 8, x, w, slab, out, cnt);
    // GPT-2 XL, B = 64 (product looped: qkv 24.8, attproj 8.8, fc 25.4, fcproj 23.2 us isolated)
    run<2, 8, 0>("xl_fc", 1600, 6400, 1, x, w, slab, out, cnt);
    run<2, 8, 2>("xl_fc", 1600, 6400, 1, x, w, slab, out, cnt);
    run<2, 8, 3>("xl_fc", 1600, 6400, 1, x, w, slab, out, cnt);
    run<2, 8, 4>("xl_fc", 1600, 6400, 1, x, w, slab, out, cnt);
    run<2, 8, 5>("xl_fc", 1600, 6400, 1, x, w, slab, out, cnt);
    run<2, 4, 0>("xl_fc", 1600, 6400, 1, x, w, slab, out, cnt);
    run<2, 4, 4>("xl_fc", 1600, 6400, 1, x, w, slab, out, cnt);
    run<1, 4, 4>("qkv", 768, 2304, 1, x, w, slab, out, cnt);
    run<1, 4, 2>("qkv", 768, 2304, 1, x, w, slab, out, cnt);
    run<1, 4, 3>("qkv", 768, 2304, 1, x, w, slab, out, cnt);
    run<1, 4, 0>("xl_fcproj", 6400, 1600, 1, x, w, slab, out, cnt);
    run<1, 4, 2>("xl_fcproj", 6400, 1600, 1, x, w, slab, out, cnt);
    run<1, 4, 3>("xl_fcproj", 6400, 1600, 1, x, w, slab, out, cnt);
    run<2, 4, 0>("xl_fc", 1600, 6400, 2, x, w, slab, out, cnt);
    run<2, 4, 1>("xl_fc", 1600, 6400, 2, x, w, slab, out, cnt);
    run<1, 4, 1>("xl_fc", 1600, 6400, 2, x, w, slab, out, cnt);
    run<2, 4, 1>("xl_qkv", 1600, 4800, 2, x, w, slab, out, cnt);
    run<1, 4, 1>("xl_fcproj", 6400, 1600, 2, x, w, slab, out, cnt);
    run<1, 4, 0>("xl_fcproj", 6400, 1600, 4, x, w, slab, out, cnt);
    return hipDeviceSynchronize() != hipSuccess;
}
