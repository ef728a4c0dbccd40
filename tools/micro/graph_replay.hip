// graph_replay.hip -- a profiler probe with none of libpaged_hip.so in it:
// capture a hipGraph of K trivial kernels (plus one 16-byte async copy, as
// the decode step's block-table upload) and replay it N times in batches of
// 16 with a stream sync after each batch -- the shape of bench.py's spin-up
// loop (bench.py, "spinup").  Used to tell a fault of the profiler's
// graph-replay path from one of the library.
//   graph_replay K N [e]      (e: the same K kernels launched eagerly, no graph)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                           \
        }                                                                       \
    } while (0)

__global__ void bump(float* p, int i) {
    if (threadIdx.x == 0) p[blockIdx.x] += (float)i;
}

int main(int argc, char** argv) {
    const int K = argc > 1 ? atoi(argv[1]) : 40;
    const long N = argc > 2 ? atol(argv[2]) : 1000;
    const bool eager = argc > 3 && argv[3][0] == 'e';
    float* d = nullptr;
    int* h = nullptr;
    int* dh = nullptr;
    CK(hipMalloc(&d, 256 * sizeof(float)));
    CK(hipMemset(d, 0, 256 * sizeof(float)));
    CK(hipHostMalloc(&h, 16, hipHostMallocDefault));
    CK(hipMalloc(&dh, 16));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    CK(hipMemcpyAsync(dh, h, 16, hipMemcpyHostToDevice, s));
    for (int i = 0; i < K; ++i) bump<<<256, 64, 0, s>>>(d, i);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    long done = 0;
    while (done < N) {
        for (int j = 0; j < 16 && done < N; ++j, ++done) {
            if (eager) {
                CK(hipMemcpyAsync(dh, h, 16, hipMemcpyHostToDevice, s));
                for (int i = 0; i < K; ++i) bump<<<256, 64, 0, s>>>(d, i);
            } else {
                CK(hipGraphLaunch(ge, s));
            }
        }
        CK(hipStreamSynchronize(s));
        if (done % 256 == 0) {
            printf("replays %ld\n", done);
            fflush(stdout);
        }
    }
    float out = 0.f;
    CK(hipMemcpy(&out, d, sizeof(float), hipMemcpyDeviceToHost));
    printf("graph_replay K=%d N=%ld %s ok (d[0] = %.0f)\n", K, N, eager ? "eager" : "graph", out);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    return 0;
}
