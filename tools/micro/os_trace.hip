// Phase timeline of the one-shot fused GEMM body (hpa_gemm_body.h) at the
// 124M decode shapes: per wave, s_memrealtime (100 MHz) at entry (0), after
// every load is issued (1), after the LN prologue (2), after the MFMA chain
// (3, operand loads landed), after the epilogue's stores drained (4); plus
// XCC / CU ids.  Prints per-phase distributions over the grid.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I llm.c-paged_amd/csrc \
//        tools/micro/os_trace.hip -o tools/micro/os_trace
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>

__device__ unsigned long long* g_trace;
#ifdef NO_TS  // timing-only build: the body exactly as in the library
#define HPA_TS(i, bid)
#else
#define HPA_TS(i, bid)                                                                   \
    do {                                                                                 \
        if ((i) == 1 || (i) == 4) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");       \
        if ((threadIdx.x & 63) == 0) {                                                   \
            unsigned long long t_ = __builtin_amdgcn_s_memrealtime();                    \
            unsigned long long* r_ = g_trace + ((size_t)(bid) * 16 + (threadIdx.x >> 6)) * 8; \
            r_[i] = t_;                                                                  \
            if ((i) == 0) {                                                              \
                unsigned xcc_ = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11)); \
                unsigned hw_ = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11)); \
                r_[6] = xcc_;                                                            \
                r_[7] = hw_;                                                             \
            }                                                                            \
        }                                                                                \
    } while (0)
#define HPA_TS_ACC(a) asm volatile("v_mov_b32 %0, %0" : "+v"(a[0]))
#endif
#include "hpa_gemm_body.h"

int hpa_fail(const char* file, int line, const char* what) {
    fprintf(stderr, "[os_trace] %s:%d %s\n", file, line, what);
    exit(1);
}

template <int NW, int EPI, int S>
__global__ __launch_bounds__(NW * 64) void os_kernel(hpa_gemm::FG p) {
    __shared__ __attribute__((aligned(16))) float smem[hpa_gemm::gemm16_os_lds_floats<NW>()];
    hpa_gemm::gemm16_os_body<NW, EPI, S>(p, blockIdx.x, smem);
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

static float* dev_rand(size_t n, float scale, unsigned seed) {
    std::vector<float> h(n);
    unsigned long long s = seed * 0x9E3779B97F4A7C15ull + 1;
    for (auto& v : h) { s ^= s >> 12; s ^= s << 25; s ^= s >> 27; v = scale * (((s * 0x2545F4914F6CDD1Dull) >> 40) / 16777216.f - 0.5f); }
    float* d; CK(hipMalloc(&d, n * 4)); CK(hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice));
    return d;
}

template <int NW, int S>
void run(const char* name, int M, int N, int K, bool ln, bool cold) {
    using namespace hpa_gemm;
    FG p{};
    p.M = M; p.Mp = (M + 15) / 16 * 16; p.K = K; p.K16 = K / 16; p.N = N; p.ntn = N / 16;
    p.x = dev_rand((size_t)p.Mp * K, 2.f, 1);
    p.w = dev_rand((size_t)N * K, 0.07f, 2);
    p.bias = dev_rand(N, 0.1f, 3);
    float* out; CK(hipMalloc(&out, (size_t)p.Mp * N * 4)); p.out = out;
    if (ln) {
        p.ln_ntiles = K / 16;
        std::vector<float> st((size_t)p.ln_ntiles * p.Mp * 2);
        for (size_t i = 0; i < st.size(); i += 2) { st[i] = 0.1f; st[i + 1] = 16.f; }
        float* d; CK(hipMalloc(&d, st.size() * 4)); CK(hipMemcpy(d, st.data(), st.size() * 4, hipMemcpyHostToDevice));
        p.ln_stats = d; p.ln_w = dev_rand(K, 1.f, 4); p.ln_b = dev_rand(K, 0.1f, 5);
    }
    p.gx = p.ntn; p.gy = p.Mp / 16;
    const int grid = (p.gx + 7) / 8 * 8 * p.gy;
    unsigned long long* tr; CK(hipMalloc(&tr, (size_t)grid * 16 * 8 * 8));
    CK(hipMemset(tr, 0, (size_t)grid * 16 * 8 * 8));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_trace), &tr, sizeof(tr)));
    char* junk = nullptr; const size_t JB = 512ull << 20;
    if (cold) CK(hipMalloc(&junk, JB));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    float tot = 0; int n = 0;
    for (int it = 0; it < 30; it++) {
        if (cold) CK(hipMemsetAsync(junk, it, JB, 0));
        CK(hipEventRecord(e0, 0));
        os_kernel<NW, HPA_FEPI_GELU, S><<<grid, NW * 64>>>(p);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        if (it >= 5) { tot += ms; n++; }
    }
#ifdef NO_TS
    printf("%-8s M=%d N=%d K=%d NW=%d grid=%d ln=%d %s: event %.2f us/launch\n", name, M, N, K, NW, grid, ln,
           cold ? "cold" : "warm", 1000 * tot / n);
    return;
#endif
    std::vector<unsigned long long> h((size_t)grid * 16 * 8);
    CK(hipMemcpy(h.data(), tr, h.size() * 8, hipMemcpyDeviceToHost));
    unsigned long long t0 = ~0ull;
    for (int b = 0; b < grid; b++) for (int w = 0; w < NW; w++) { auto v = h[((size_t)b * 16 + w) * 8]; if (v) t0 = std::min(t0, v); }
    std::vector<double> ph[6];
    std::vector<int> percu(2048, 0);
    for (int b = 0; b < grid; b++) for (int w = 0; w < NW; w++) {
        const unsigned long long* r = &h[((size_t)b * 16 + w) * 8];
        if (!r[0]) continue;
        ph[0].push_back((r[0] - t0) * 0.01);
        ph[1].push_back((r[1] - r[0]) * 0.01);
        ph[2].push_back((r[2] - r[1]) * 0.01);
        ph[3].push_back((r[3] - r[2]) * 0.01);
        ph[4].push_back((r[4] - r[3]) * 0.01);
        ph[5].push_back((r[4] - t0) * 0.01);
        if (w == 0) { int xcc = r[6] & 15, cu = (r[7] >> 8) & 15, se = (r[7] >> 13) & 7; percu[(xcc * 8 + se) * 16 + cu]++; }
    }
    int mx = 0, used = 0; for (int c : percu) { mx = std::max(mx, c); used += c > 0; }
    printf("%-8s M=%d N=%d K=%d NW=%d grid=%d ln=%d %s: event %.2f us/launch; CUs used %d, max WGs/CU %d\n", name, M, N, K,
           NW, grid, ln, cold ? "cold" : "warm", 1000 * tot / n, used, mx);
    const char* nm[6] = {"start", "issue+loads(1)", "LN(2)", "mfma(3)", "epi(4)", "end"};
    for (int i = 0; i < 6; i++) {
        auto v = ph[i]; std::sort(v.begin(), v.end());
        printf("   %-16s min %6.2f p10 %6.2f p50 %6.2f p90 %6.2f max %6.2f us\n", nm[i], v[0], v[v.size() / 10],
               v[v.size() / 2], v[v.size() * 9 / 10], v.back());
    }
    CK(hipFree(tr)); if (junk) CK(hipFree(junk));
}

int main() {
    for (int cold = 0; cold < 2; cold++) {
        run<4, 12>("qkv", 64, 2304, 768, true, cold);
        run<4, 12>("attproj", 64, 768, 768, false, cold);
        run<4, 12>("fc", 64, 3072, 768, true, cold);
        run<8, 24>("fcproj", 64, 768, 3072, false, cold);
    }
    return 0;
}
