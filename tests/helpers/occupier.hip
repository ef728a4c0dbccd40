// occupier.hip -- test helper (tests/test_gpu_coresidency.py), not part of the
// library: a kernel that holds whole CUs for a bounded time on its own
// non-blocking stream, standing in for a co-running kernel (an RCCL
// collective, another process's work) beside the decode step's persistent
// launches.  Each workgroup takes 1024 threads and 160 KiB of LDS, so no
// persistent workgroup can share its CU until it exits; every workgroup
// exits after `ticks` of s_memrealtime (100 MHz) and counts itself in *done.
//
// recv_like_kernel (round 6) has the resources of the
// kernel RCCL 7.2 runs a grouped ncclSend/ncclRecv with on gfx950
// (ncclDevKernel_Generic_{1,2,4}, read from the code object's metadata in
// /opt/rocm/lib/librccl.so: 248-256 VGPRs, 37,664 B of LDS, up to 512
// threads): one workgroup per channel, held until `ticks` after the workgroup
// started -- a receive whose peer's data arrive that long after it was posted.
// occ_recv_after launches it behind an event recorded on `after` (the decode
// stream), so it starts when the step enqueued before it ends, exactly where
// the bench's end-of-step gather sits (gpt2_decode_gather, hpa_comm.hip).
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
__global__ __launch_bounds__(512) void recv_like_kernel(long long ticks, int* done) {
    extern __shared__ int lds[];
    // RCCL's kernel takes 256 VGPRs per lane (vgpr_count 248-256): claim the
    // same so this workgroup leaves the CU the registers RCCL's would
    asm volatile("" ::: "v255");
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    int spins = 0;
    while ((long long)__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
        __builtin_amdgcn_s_sleep(4);
        ++spins;
    }
    lds[threadIdx.x] = spins;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(done, lds[blockDim.x - 1] >= 0 ? 1 : 0);
}
hipStream_t g_stream = nullptr;
hipEvent_t g_evs[4] = {nullptr, nullptr, nullptr, nullptr};
hipEvent_t g_ring[4] = {nullptr, nullptr, nullptr, nullptr};
unsigned* g_flag = nullptr;
unsigned g_count = 0;
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
// mode (what to isolate, tools/recv_coresidency.py): bit 0 record the event on
// `after`, bit 1 make the helper stream wait for it, bit 2 launch the kernel;
// 7 = the gather's pattern; bits 3-4 pick the event: 0 timing disabled (the
// library's hpa_event_create_sync), 1 + hipEventDisableSystemFence, 2 +
// hipEventReleaseToDevice, 3 both; bit 5: instead of the event, `after` writes a
// step counter to device memory (hipStreamWriteValue32) and the helper stream
// waits for it (hipStreamWaitValue32)
int occ_recv_after(void* after, int blocks, int threads, long long ticks, int lds_bytes, int* done, int mode) {
    if (blocks < 1 || blocks > 256 || (threads != 256 && threads != 512) || ticks < 0 || ticks > 1000000 ||
        lds_bytes < 2048 || lds_bytes > 64 * 1024)
        return 1;  // bounded: at most 10 ms
    if (!g_stream && hipStreamCreateWithFlags(&g_stream, hipStreamNonBlocking) != hipSuccess) return 2;
    const unsigned evf[4] = {hipEventDisableTiming, hipEventDisableTiming | hipEventDisableSystemFence,
                             hipEventDisableTiming | hipEventReleaseToDevice,
                             hipEventDisableTiming | hipEventDisableSystemFence | hipEventReleaseToDevice};
    const int ek = (mode >> 3) & 3;
    if (!g_evs[ek] && hipEventCreateWithFlags(&g_evs[ek], evf[ek]) != hipSuccess) return 2;
    hipEvent_t g_ev = g_evs[ek];
    if (hipFuncSetAttribute((const void*)recv_like_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes) !=
        hipSuccess)
        return 3;
    if (mode & 32) {
        if (!g_flag && hipMalloc(&g_flag, 64) != hipSuccess) return 2;
        if (!g_count && hipMemset(g_flag, 0, 64) != hipSuccess) return 2;
        ++g_count;
        if ((mode & 1) && hipStreamWriteValue32((hipStream_t)after, g_flag, g_count, 0) != hipSuccess) return 5;
        if ((mode & 2) && hipStreamWaitValue32(g_stream, g_flag, g_count, hipStreamWaitValueGte, 0xffffffffu) !=
                              hipSuccess)
            return 5;
    } else {
        if ((mode & 1) && hipEventRecord(g_ev, (hipStream_t)after) != hipSuccess) return 5;
        if ((mode & 2) && hipStreamWaitEvent(g_stream, g_ev, 0) != hipSuccess) return 5;
    }
    if (mode & 4) recv_like_kernel<<<blocks, threads, lds_bytes, g_stream>>>(ticks, done);
    return hipGetLastError() == hipSuccess ? 0 : 4;
}
// host-deferred posting: record a ring event on `after` / block the host on an
// earlier one (then occ_recv_after(mode 4) posts with no device dependency)
int occ_ring_record(void* after, int slot) {
    if (slot < 0 || slot > 3) return 1;
    if (!g_ring[slot] && hipEventCreateWithFlags(&g_ring[slot], hipEventDisableTiming) != hipSuccess) return 2;
    return hipEventRecord(g_ring[slot], (hipStream_t)after) == hipSuccess ? 0 : 3;
}
int occ_ring_wait(int slot) {
    if (slot < 0 || slot > 3 || !g_ring[slot]) return 1;
    return hipEventSynchronize(g_ring[slot]) == hipSuccess ? 0 : 3;
}
int occ_sync(void) { return g_stream && hipStreamSynchronize(g_stream) != hipSuccess ? 1 : 0; }
}
