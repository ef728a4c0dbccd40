// Microbenchmark: how fast can ONE CU ingest a stream, and does it depend on
// how many CUs stream at once?  (The small-batch decode step -- attention at
// B = 8 runs 50 MB on 192 workgroups in 12.8 us, the chain's phases move
// ~100 KB per CU -- looks bound by a per-CU rate, not by HBM.)
//
// N workgroups, one per CU (dynamic LDS of 96 KiB keeps a second one out),
// W waves each; every workgroup streams `per_wg` bytes of its own contiguous
// region: rounds of D float4 loads per lane in flight (D KiB per wave), summed
// after each round.  Modes: cold (regions rotate through 4 GiB, so every
// launch reads HBM), mall (a 96 MiB buffer re-read: Infinity-Cache resident),
// l2 (every workgroup re-reads the same 32 KiB per XCD slot: L2 resident).
// Time per launch from hipEvents around a graph of back-to-back launches.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e = (x);                                                            \
        if (e != hipSuccess) {                                                         \
            printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));            \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

typedef float v4 __attribute__((ext_vector_type(4)));

template <int D, bool NT>
__global__ void stream_cu(const v4* __restrict__ base, size_t wg_stride_f4, size_t per_wg_f4, size_t wrap_f4,
                          float* out) {
    extern __shared__ float pad[];
    const size_t start = ((size_t)blockIdx.x * wg_stride_f4) % wrap_f4;
    const v4* p = base + start + threadIdx.x;
    const size_t step = (size_t)blockDim.x * D;
    v4 acc = {0.f, 0.f, 0.f, 0.f};
    for (size_t i = 0; i + step <= per_wg_f4; i += step) {
        v4 r[D];
#pragma unroll
        for (int d = 0; d < D; ++d) r[d] = NT ? __builtin_nontemporal_load(p + i + (size_t)d * blockDim.x)
                                             : p[i + (size_t)d * blockDim.x];
#pragma unroll
        for (int d = 0; d < D; ++d) acc += r[d];
    }
    if (acc.x + acc.y + acc.z + acc.w == 1234.5f) {
        pad[threadIdx.x] = acc.x;
        out[threadIdx.x] = pad[(threadIdx.x + 1) % blockDim.x];
    }
}

template <int D>
int run(const char* mode, int N, int W, size_t per_wg, v4* buf, size_t buf_bytes, float* out, hipStream_t s,
        hipEvent_t e0, hipEvent_t e1) {
    const int iters = 40;
    const size_t per_f4 = per_wg / 16;
    size_t wrap = buf_bytes / 16, stride = per_f4;
    if (!strcmp(mode, "mall")) wrap = (96ull << 20) / 16;
    if (!strcmp(mode, "l2")) stride = 0, wrap = per_f4 + 1;  // every workgroup the same bytes
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int it = 0; it < iters; ++it) {
        // cold: each launch starts its regions further along (never re-read within 4 GiB)
        const size_t shift = !strcmp(mode, "cold") ? ((size_t)it * N * per_f4) % (wrap - (size_t)N * per_f4) : 0;
        stream_cu<D, true><<<N, W * 64, 96 * 1024, s>>>(buf + shift, stride, per_f4, wrap, out);
    }
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
        CK(hipEventRecord(e0, s));
        CK(hipGraphLaunch(ge, s));
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
    }
    const double us = best * 1e3 / iters;
    const double bytes = (double)N * (per_f4 / (W * 64 * D)) * (W * 64 * D) * 16;
    printf("%-5s N=%3d W=%2d D=%2d per_wg=%7zu KiB  %8.2f us/launch  %7.1f GB/s per CU  %7.1f GB/s chip\n", mode, N,
           W, D, per_wg >> 10, us, bytes / N / (us * 1e-6) / 1e9, bytes / (us * 1e-6) / 1e9);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    return 0;
}

int main(int argc, char** argv) {
    const size_t buf_bytes = 4096ull << 20;
    v4* buf;
    float* out;
    CK(hipMalloc(&buf, buf_bytes));
    CK(hipMemset(buf, 0, buf_bytes));
    CK(hipMalloc(&out, 1 << 16));
    CK(hipFuncSetAttribute((const void*)stream_cu<8, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024));
    CK(hipFuncSetAttribute((const void*)stream_cu<16, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024));
    CK(hipFuncSetAttribute((const void*)stream_cu<32, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char* modes[] = {"cold", "mall", "l2"};
    for (const char* mode : modes) {
        const int Ns[] = {32, 96, 192, 256};
        for (int N : Ns)
            for (int W : {4, 8, 16})
                for (int D : {8, 16, 32}) {
                    size_t per_wg = !strcmp(mode, "l2") ? (32u << 10) * 8 : (1u << 20);
                    if (!strcmp(mode, "l2") && N != 256) continue;
                    int rc = D == 8    ? run<8>(mode, N, W, per_wg, buf, buf_bytes, out, s, e0, e1)
                             : D == 16 ? run<16>(mode, N, W, per_wg, buf, buf_bytes, out, s, e0, e1)
                                       : run<32>(mode, N, W, per_wg, buf, buf_bytes, out, s, e0, e1);
                    if (rc) return rc;
                }
        fflush(stdout);
    }
    // small per-workgroup volumes (a chain phase's unit: 48-96 KiB; the B = 8
    // attention's 256 KiB): latency + volume, cold
    CK(hipFuncSetAttribute((const void*)stream_cu<4, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024));
    for (int N : {48, 192, 256}) {  // one round per workgroup: W waves x D KiB = the volume
        if (run<4>("cold", N, 12, 48 << 10, buf, buf_bytes, out, s, e0, e1)) return 1;
        if (run<8>("cold", N, 12, 96 << 10, buf, buf_bytes, out, s, e0, e1)) return 1;
        if (run<16>("cold", N, 16, 256 << 10, buf, buf_bytes, out, s, e0, e1)) return 1;
        if (run<8>("cold", N, 8, 256 << 10, buf, buf_bytes, out, s, e0, e1)) return 1;  // 4 rounds
    }
    return 0;
}
