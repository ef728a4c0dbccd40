// Workgroup timeline of the paged decode attention (fp32 pool, page 16,
// GPT-2 124M heads, B sequences at ctx 1024, scattered pages): per
// workgroup, s_memrealtime (100 MHz) at entry, after its K/V stream, and at
// exit, plus XCC id.  Shows the launch ramp and the tail that the marginal
// bandwidth (attn_scan.py: 7.1 TB/s between B = 64 and 128) does not.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I llm.c-paged_amd/csrc \
//        tools/micro/attn_trace.hip -o tools/micro/attn_trace
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "hpa_attn_body.h"

int hpa_fail(const char* file, int line, const char* what) {
    fprintf(stderr, "[attn_trace] %s:%d %s\n", file, line, what);
    exit(1);
}

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e = (x);                                                                    \
        if (e != hipSuccess) {                                                                 \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                             \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

using namespace hpa_attn;

template <int P, int NW>
__global__ __launch_bounds__(NW * 64, 3) void attn_traced(const float* __restrict__ q, const float* __restrict__ base,
                                                          size_t page_elems, int NH, const int* __restrict__ bt_all,
                                                          int bt_stride, const int* __restrict__ pos, float* out,
                                                          float qscale, float m_init, unsigned long long* tr) {
    constexpr int TILE = P * HS;
    __shared__ float s_m[NW];
    __shared__ float s_l[NW];
    __shared__ float4 s_acc[NW * 16];
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    const int bh = blockIdx.x;
    const int b = bh / NH, h = bh - b * NH;
    const int lane = threadIdx.x & 63;
    const int ctx = pos[b] + 1;
    const float* qh = q + ((size_t)b * NH + h) * HS;
    const int* bt = bt_all + (size_t)b * bt_stride;
    float m = m_init, l = 0.f;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    attn_tiles<P, NW>(qh, base + (size_t)h * TILE, base + (size_t)(NH + h) * TILE, page_elems, bt, ctx, 0,
                      (ctx + 63) >> 6, qscale, m, l, acc);
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if (!attn_fold<NW>(m, l, acc, s_m, s_l, s_acc)) return;
    const float inv = l == 0.f ? 0.f : 1.f / l;
    *reinterpret_cast<float4*>(out + hpa::frag_index(b, h * HS + 4 * lane, NH * HS)) =
        make_float4(acc.x * inv, acc.y * inv, acc.z * inv, acc.w * inv);
    if (lane == 0) {
        tr[bh * 4 + 0] = t0;
        tr[bh * 4 + 1] = t1;
        tr[bh * 4 + 2] = __builtin_amdgcn_s_memrealtime();
        tr[bh * 4 + 3] = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11));
    }
}

static void pct(const char* name, std::vector<double> v) {
    std::sort(v.begin(), v.end());
    printf("  %-22s min %6.2f p10 %6.2f p50 %6.2f p90 %6.2f max %6.2f us\n", name, v[0], v[v.size() / 10],
           v[v.size() / 2], v[v.size() * 9 / 10], v.back());
}

int main(int argc, char** argv) {
    const int B = argc > 1 ? atoi(argv[1]) : 64;
    constexpr int P = 16, NW = 4;
    const int NH = 12, ctx = 1024, pages_per_seq = ctx / P, npages = B * pages_per_seq;
    const size_t page_elems = (size_t)2 * NH * P * HS;
    float* pool;
    CK(hipMalloc(&pool, npages * page_elems * 4));
    CK(hipMemset(pool, 0x3c, npages * page_elems * 4));  // ~0.012 everywhere
    std::vector<int> perm(npages);
    for (int i = 0; i < npages; i++) perm[i] = i;
    unsigned long long s = 0x9E3779B97F4A7C15ull;
    for (int i = npages - 1; i > 0; i--) {
        s ^= s >> 12; s ^= s << 25; s ^= s >> 27;
        std::swap(perm[i], perm[(s * 0x2545F4914F6CDD1Dull >> 33) % (i + 1)]);
    }
    int *bt, *pos;
    CK(hipMalloc(&bt, npages * 4));
    CK(hipMemcpy(bt, perm.data(), npages * 4, hipMemcpyHostToDevice));
    std::vector<int> hp(B, ctx - 1);
    CK(hipMalloc(&pos, B * 4));
    CK(hipMemcpy(pos, hp.data(), B * 4, hipMemcpyHostToDevice));
    float *q, *out;
    CK(hipMalloc(&q, (size_t)B * NH * HS * 4));
    CK(hipMemset(q, 0, (size_t)B * NH * HS * 4));
    CK(hipMalloc(&out, (size_t)((B + 15) / 16 * 16) * NH * HS * 4));
    unsigned long long* tr;
    const int nb = B * NH;
    CK(hipMalloc(&tr, (size_t)nb * 4 * 8));
    const float log2e = 1.4426950408889634f;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float tot = 0;
    const int iters = 40;
    for (int it = 0; it < iters; it++) {
        CK(hipEventRecord(e0, 0));
        attn_traced<P, NW><<<nb, NW * 64>>>(q, pool, page_elems, NH, bt, pages_per_seq, pos, out, 0.125f * log2e,
                                            -10000.f * log2e, tr);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (it >= 5) tot += ms;
    }
    std::vector<unsigned long long> h((size_t)nb * 4);
    CK(hipMemcpy(h.data(), tr, h.size() * 8, hipMemcpyDeviceToHost));
    unsigned long long t0 = ~0ull, tend = 0;
    for (int i = 0; i < nb; i++) {
        t0 = std::min(t0, h[i * 4]);
        tend = std::max(tend, h[i * 4 + 2]);
    }
    std::vector<double> st, dur, fold, en;
    for (int i = 0; i < nb; i++) {
        st.push_back((h[i * 4] - t0) * 0.01);
        dur.push_back((h[i * 4 + 1] - h[i * 4]) * 0.01);
        fold.push_back((h[i * 4 + 2] - h[i * 4 + 1]) * 0.01);
        en.push_back((h[i * 4 + 2] - t0) * 0.01);
    }
    const double bytes = (double)B * NH * ctx * HS * 2 * 4;
    printf("B=%d: event %.2f us/launch (%.0f GB/s), first start -> last end %.2f us\n", B, 1000 * tot / (iters - 5),
           bytes / (tot / (iters - 5)) / 1e6, (tend - t0) * 0.01);
    pct("start", st);
    pct("stream", dur);
    pct("fold+store", fold);
    pct("end", en);
    // by XCC: is the spread systematic (placement) or per workgroup?
    double sx[8] = {0}, ex[8] = {0};
    int nx[8] = {0};
    for (int i = 0; i < nb; i++) {
        const int x = (int)(h[i * 4 + 3] & 7);
        sx[x] += dur[i];
        ex[x] += en[i];
        nx[x]++;
    }
    printf("  per XCC mean stream / end (us):");
    for (int x = 0; x < 8; x++) printf(" [%d] %.1f/%.1f n=%d", x, nx[x] ? sx[x] / nx[x] : 0, nx[x] ? ex[x] / nx[x] : 0, nx[x]);
    printf("\n");
    // by launch order within an XCC (bid / 8): early vs late dispatched
    double sq[4] = {0};
    int nq[4] = {0};
    for (int i = 0; i < nb; i++) {
        const int qd = std::min(3, (int)((long long)i * 4 / nb));
        sq[qd] += dur[i];
        nq[qd]++;
    }
    printf("  mean stream by block-index quarter: %.1f %.1f %.1f %.1f\n", sq[0] / nq[0], sq[1] / nq[1], sq[2] / nq[2],
           sq[3] / nq[3]);
    return 0;
}
