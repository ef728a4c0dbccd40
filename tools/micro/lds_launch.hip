// Empty-kernel launch cost against dynamic LDS size (256 / 512 workgroups x 512 threads, back to back,
// HIP events): 2.4-3.6 us per launch from 4 KiB to 160 KiB -- LDS size does not set the fixed cost.
// build: hipcc --offload-arch=gfx950 -O3 tools/micro/lds_launch.hip -o tools/micro/lds_launch
// launch cost of an (almost) empty kernel vs its dynamic LDS size and grid:
// the stream-K GEMM showed ~20 us of fixed cost per launch.
// hipcc --offload-arch=gfx950 -O3 tools/micro/lds_launch.hip -o /tmp/lds_launch
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void k_dyn(float* out) {
    extern __shared__ float sm[];
    sm[threadIdx.x] = threadIdx.x;
    __syncthreads();
    if (threadIdx.x == 0 && sm[5] == 12345.f) out[blockIdx.x] = sm[7];
}

int main() {
    float* out;
    hipMalloc(&out, 1 << 20);
    hipStream_t s;
    hipStreamCreate(&s);
    hipFuncSetAttribute((const void*)k_dyn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int grids[] = {256, 512};
    const int ldss[] = {4096, 32768, 65536, 98304, 131072, 144384, 163840};
    for (int gi = 0; gi < 2; ++gi)
        for (int li = 0; li < 7; ++li) {
            for (int w = 0; w < 5; ++w) k_dyn<<<grids[gi], 512, ldss[li], s>>>(out);
            hipEventRecord(a, s);
            for (int i = 0; i < 100; ++i) k_dyn<<<grids[gi], 512, ldss[li], s>>>(out);
            hipEventRecord(b, s);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            printf("grid %4d x 512 threads, dynamic LDS %6d B: %7.2f us per launch\n", grids[gi], ldss[li], ms * 10);
        }
    return 0;
}
