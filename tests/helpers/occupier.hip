// occupier.hip -- test helper (tests/test_gpu_coresidency.py), not part of the
// library: a kernel that holds whole CUs for a bounded time on its own
// non-blocking stream, standing in for a co-running kernel (an RCCL
// collective, another process's work) beside the decode step's persistent
// launches.  Each workgroup takes 1024 threads and 160 KiB of LDS, so no
// persistent workgroup can share its CU until it exits; every workgroup
// exits after `ticks` of s_memrealtime (100 MHz) and counts itself in *done.
#include <hip/hip_runtime.h>

namespace {
__global__ __launch_bounds__(1024) void occupy_kernel(long long ticks, int* done) {
    extern __shared__ int lds[];
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    int spins = 0;
    while ((long long)__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
        __builtin_amdgcn_s_sleep(8);
        ++spins;
    }
    lds[threadIdx.x] = spins;  // keep the LDS allocation live
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(done, lds[1023] >= 0 ? 1 : 0);
}
hipStream_t g_stream = nullptr;
}  // namespace

extern "C" {
int occ_launch(int blocks, long long ticks, int lds_bytes, int* done) {
    if (blocks < 1 || blocks > 1024 || ticks < 0 || ticks > 10000000 || lds_bytes < 4096 || lds_bytes > 160 * 1024)
        return 1;  // bounded: at most 100 ms
    if (!g_stream && hipStreamCreateWithFlags(&g_stream, hipStreamNonBlocking) != hipSuccess) return 2;
    if (hipFuncSetAttribute((const void*)occupy_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes) !=
        hipSuccess)
        return 3;
    occupy_kernel<<<blocks, 1024, lds_bytes, g_stream>>>(ticks, done);
    return hipGetLastError() == hipSuccess ? 0 : 4;
}
int occ_sync(void) { return g_stream && hipStreamSynchronize(g_stream) != hipSuccess ? 1 : 0; }
}
