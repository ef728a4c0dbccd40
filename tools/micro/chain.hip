// Microbenchmark: cost of a dependent fp32 add chain on one lane of a wave
// (the sampler's serial core), from registers and from LDS.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void chain_reg(float* out, int n, float x) {
    float a = 0.f, v0 = x, v1 = x * 1.5f, v2 = x * 0.5f, v3 = x * 0.25f;
    if (threadIdx.x == 0) {
        for (int i = 0; i < n; i += 4) {
            a += v0; a += v1; a += v2; a += v3;
        }
    }
    out[threadIdx.x] = a;
}

template <int MODE>
__global__ void chain_lds(float* out, int n) {
    __shared__ __attribute__((aligned(16))) float sh[1024];
    for (int i = threadIdx.x; i < 1024; i += blockDim.x) sh[i] = 1e-6f * i;
    __syncthreads();
    float a = 0.f;
    if (threadIdx.x == 0) {
        const float4* s4 = reinterpret_cast<const float4*>(sh);
        for (int rep = 0; rep < n / 1024; ++rep) {
            for (int q0 = 0; q0 < 256; q0 += 16) {
                float4 r[16];
#pragma unroll
                for (int q = 0; q < 16; ++q) r[q] = s4[q0 + q];
#pragma unroll
                for (int q = 0; q < 16; ++q) { a += r[q].x; a += r[q].y; a += r[q].z; a += r[q].w; }
            }
        }
    }
    out[threadIdx.x] = a;
}

int main() {
    float* d; hipMalloc(&d, 4096);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    const int n = 1 << 20;
    float ms;
    for (int wv = 1; wv <= 2; ++wv) {
        chain_reg<<<1, 64 * wv>>>(d, n, 1e-7f);
        hipEventRecord(e0); chain_reg<<<64, 64 * wv>>>(d, n, 1e-7f); hipEventRecord(e1); hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        printf("reg chain  waves/blk %d: %.3f ns/add\n", wv, ms * 1e6 / n);
        chain_lds<0><<<1, 64 * wv>>>(d, n);
        hipEventRecord(e0); chain_lds<0><<<64, 64 * wv>>>(d, n); hipEventRecord(e1); hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        printf("lds chain  waves/blk %d: %.3f ns/add\n", wv, ms * 1e6 / n);
    }
    return 0;
}
