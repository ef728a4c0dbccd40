// Microbenchmark: per-kernel cost of a serial chain of small kernels replayed
// from a hipGraph (the decode step's shape): empty kernels, and kernels that
// stream a weight-sized buffer (7.08 MB = QKV, 2.36 MB = attproj) once.
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); return 1; } } while (0)

__global__ void empty_k(float* out) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && out[0] == 12345.f) out[1] = 1.f;
}

// each workgroup streams `per` float4 per thread, contiguous per workgroup
__global__ void stream_k(const float4* __restrict__ w, float* out, int per) {
    const float4* p = w + (size_t)blockIdx.x * blockDim.x * per + threadIdx.x;
    float4 a = {0, 0, 0, 0};
    float4 r[16];
#pragma unroll
    for (int i = 0; i < 16; ++i)
        if (i < per) { typedef float v4 __attribute__((ext_vector_type(4))); v4 t = __builtin_nontemporal_load(reinterpret_cast<const v4*>(p + i * blockDim.x)); r[i] = make_float4(t.x, t.y, t.z, t.w); }
#pragma unroll
    for (int i = 0; i < 16; ++i)
        if (i < per) { a.x += r[i].x; a.y += r[i].y; a.z += r[i].z; a.w += r[i].w; }
    if (a.x + a.y + a.z + a.w == 12345.f) out[threadIdx.x] = a.x;
}

int main() {
    float* out; CK(hipMalloc(&out, 1 << 20)); CK(hipMemset(out, 0, 1 << 20));
    float4* w; const size_t wbytes = 2048ull << 20;  // > MALL (256 MB): rotating offsets read cold CK(hipMalloc(&w, wbytes)); CK(hipMemset(w, 0, wbytes));
    hipStream_t s; CK(hipStreamCreate(&s));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const int N = 200;
    struct Cfg { const char* name; int grid, block, per; int hot; } cfgs[] = {
        {"empty 576x256", 576, 256, 0, 0},
        {"empty 2304x64", 2304, 64, 0, 0},
        {"cold 7.08MB 576x256 (12 f4/thr)", 576, 256, 12, 0},
        {"cold 7.08MB 1152x256 (6 f4/thr)", 1152, 256, 6, 0},
        {"hot  7.08MB 576x256 (12 f4/thr)", 576, 256, 12, 1},
        {"cold 2.36MB 576x256 (4 f4/thr)", 576, 256, 4, 0},
        {"hot  2.36MB 576x256 (4 f4/thr)", 576, 256, 4, 1},
        {"cold 28.3MB 2304x256 (12 f4/thr)", 2304, 256, 12, 0},
        {"hot  28.3MB 2304x256 (12 f4/thr)", 2304, 256, 12, 1},
    };
    for (auto& c : cfgs) {
        hipGraph_t g; hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
        for (int i = 0; i < N; ++i) {
            // rotate through the 64 MB buffer so consecutive kernels do not hit in L2/MALL
            const size_t span = (size_t)c.grid * c.block * c.per;
            const size_t nf4 = wbytes / 16;
            if (span > nf4 / 4) { printf("config too large\n"); return 1; }
            const size_t off = (span && !c.hot) ? ((size_t)i * span) % (nf4 - span) : 0;
            if (c.per) stream_k<<<c.grid, c.block, 0, s>>>(w + off, out, c.per);
            else empty_k<<<c.grid, c.block, 0, s>>>(out);
        }
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        CK(hipGraphLaunch(ge, s)); CK(hipStreamSynchronize(s));
        float best = 1e30f;
        for (int rep = 0; rep < 5; ++rep) {
            CK(hipEventRecord(e0, s)); CK(hipGraphLaunch(ge, s)); CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1)); if (ms < best) best = ms;
        }
        const double us = best * 1e3 / N;
        const double mb = (double)c.grid * c.block * c.per * 16 / 1e6;
        printf("%-40s %7.2f us/kernel  %7.1f GB/s\n", c.name, us, mb ? mb * 1e3 / us : 0.0);
        CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(g));
    }
    return 0;
}
