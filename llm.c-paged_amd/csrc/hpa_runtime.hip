// hpa_runtime.hip -- device selection, stream, memory, events, page pool.
#include <stdlib.h>
#include <string.h>

#include "hpa_internal.h"

static hipStream_t g_default_stream = nullptr;
static hipStream_t g_stream = nullptr;  // current (default or external)
static int g_device = -1;
static char g_last_error[512] = "";

int hpa_fail(const char* file, int line, const char* what) {
    snprintf(g_last_error, sizeof(g_last_error), "%s:%d %s", file, line, what);
    fprintf(stderr, "[hpa] %s\n", g_last_error);
    const char* f = getenv("HPA_FATAL");
    if (f && f[0] == '1') exit(1);
    return 1;
}

int hpa_build_flags(void) {
#ifdef HPA_AB
    return 1;
#else
    return 0;
#endif
}

constexpr int kMaxDevices = 64;
hipStream_t g_dev_streams[kMaxDevices];
hipStream_t hpa_stream() { return g_stream; }

// Infinity-Cache warm-up (hpa_l3_prefetch): read [p, p + n float4) with the
// default cache policy and drop it.  The 256 MiB die-level cache keeps those
// lines for a later kernel while the bytes loaded or stored in between stay
// under its size (MI355X_MICROARCH.md "Infinity Cache").  4 float4 per thread
// per trip in flight; every component summed so the loads stay whole.
__global__ __launch_bounds__(256) void l3_prefetch_kernel(const float4* __restrict__ p, size_t n, float* sink) {
    float acc = 0.f;
    const size_t stride = (size_t)gridDim.x * 1024;
    for (size_t i = (size_t)blockIdx.x * 1024 + threadIdx.x; i < n; i += stride) {
        float4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const size_t j = i + (size_t)u * 256;
            v[u] = j < n ? p[j] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) acc += (v[u].x + v[u].y) + (v[u].z + v[u].w);
    }
    if (acc == 1.2345e-38f && sink) *sink = acc;  // keeps the sum (never true for pool data in practice)
}

extern "C" {

const char* hpa_last_error(void) { return g_last_error; }

int hpa_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int hpa_init(int device) {
    int n = 0;
    HPA_CHECK(hipGetDeviceCount(&n));
    HPA_REQUIRE(n > 0, "no HIP device visible");
    HPA_REQUIRE(device >= 0 && device < n, "device index out of range");
    HPA_REQUIRE(device < kMaxDevices, "device index beyond the library's table");
    HPA_CHECK(hipSetDevice(device));
    // one default stream per device (the single-process multi-GPU form,
    // hpa_comm_use, switches devices); a current stream that was the old
    // device's default follows the switch
    if (!g_dev_streams[device]) HPA_CHECK(hipStreamCreateWithFlags(&g_dev_streams[device], hipStreamNonBlocking));
    const bool follow = !g_stream || g_stream == g_default_stream;
    g_default_stream = g_dev_streams[device];
    g_device = device;
    if (follow) g_stream = g_default_stream;
    return 0;
}

int hpa_get_device(void) { return g_device; }

int hpa_set_stream(void* s) {
    g_stream = s ? (hipStream_t)s : g_default_stream;
    return 0;
}

void* hpa_get_stream(void) { return (void*)g_stream; }

int hpa_synchronize(void) {
    HPA_CHECK(hipStreamSynchronize(g_stream));
    return 0;
}

int hpa_device_synchronize(void) {
    HPA_CHECK(hipDeviceSynchronize());
    return 0;
}

void* hpa_malloc(size_t bytes) {
    void* p = nullptr;
    if (hipMalloc(&p, bytes ? bytes : 1) != hipSuccess) {
        hpa_fail(__FILE__, __LINE__, "hipMalloc failed");
        return nullptr;
    }
    return p;
}

void* hpa_malloc_managed(size_t bytes) {
    void* p = nullptr;
    if (hipMallocManaged(&p, bytes ? bytes : 1, hipMemAttachGlobal) != hipSuccess) {
        hpa_fail(__FILE__, __LINE__, "hipMallocManaged failed");
        return nullptr;
    }
    return p;
}

void* hpa_host_alloc(size_t bytes) {
    void* p = nullptr;
    if (hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess) {
        hpa_fail(__FILE__, __LINE__, "hipHostMalloc failed");
        return nullptr;
    }
    return p;
}

int hpa_free(void* p) {
    if (p) HPA_CHECK(hipFree(p));
    return 0;
}

int hpa_host_free(void* p) {
    if (p) HPA_CHECK(hipHostFree(p));
    return 0;
}

int hpa_memcpy(void* dst, const void* src, size_t bytes) {
    if (!bytes) return 0;
    HPA_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, g_stream));
    HPA_CHECK(hipStreamSynchronize(g_stream));
    return 0;
}

int hpa_memcpy_async(void* dst, const void* src, size_t bytes) {
    if (!bytes) return 0;
    HPA_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, g_stream));
    return 0;
}

int hpa_l3_prefetch(const void* p, size_t bytes, int grid) {
    if (!bytes) return 0;
    HPA_REQUIRE(p && grid > 0, "l3_prefetch: pointer, grid");
    l3_prefetch_kernel<<<(unsigned)grid, 256, 0, g_stream>>>(reinterpret_cast<const float4*>(p), bytes / 16, nullptr);
    HPA_LAUNCH_CHECK();
    return 0;
}

int hpa_memset_async(void* dst, int value, size_t bytes) {
    if (!bytes) return 0;
    HPA_CHECK(hipMemsetAsync(dst, value, bytes, g_stream));
    return 0;
}

int hpa_is_device_accessible(const void* p) {
    if (!p) return 0;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    switch (a.type) {
        case hipMemoryTypeDevice:
        case hipMemoryTypeManaged:
        case hipMemoryTypeUnified:
            return 1;
        case hipMemoryTypeHost:
            return a.devicePointer != nullptr;  // pinned / registered host memory
        default:
            return 0;
    }
}

void* hpa_event_create(void) {
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) {
        hpa_fail(__FILE__, __LINE__, "hipEventCreate failed");
        return nullptr;
    }
    return (void*)e;
}

void* hpa_event_create_nt(void) {
    hipEvent_t e = nullptr;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
        hpa_fail(__FILE__, __LINE__, "hipEventCreateWithFlags failed");
        return nullptr;
    }
    return (void*)e;
}

void* hpa_stream_create(void) {
    hipStream_t s = nullptr;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) {
        hpa_fail(__FILE__, __LINE__, "hipStreamCreateWithFlags failed");
        return nullptr;
    }
    return (void*)s;
}

int hpa_stream_destroy(void* s) {
    if (s) HPA_CHECK(hipStreamDestroy((hipStream_t)s));
    return 0;
}
int hpa_stream_wait_event(void* ev) {
    HPA_CHECK(hipStreamWaitEvent(g_stream, (hipEvent_t)ev, 0));
    return 0;
}

/* a cross-stream dependency through a device word instead of an event: the
 * current stream writes `value` to *flag once its earlier work is done, and
 * the current stream of the waiter blocks until *flag >= value.  Measured
 * (profiles/r6/recv_coresidency.txt): a stream waiting on an EVENT of the
 * decode stream slows the decode stream's own kernels by ~25 us per step
 * while the wait is pending; a pending wait-value costs 5-9 us. */
/* 1 if the current device runs hipStreamWaitValue32 (the gather's hand-off;
 * else the caller falls back to an event) */
int hpa_stream_value_ops(void) {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeCanUseStreamWaitValue, dev) != hipSuccess) return 0;
    return v != 0;
}

int hpa_stream_write_value32(unsigned* flag, unsigned value) {
    HPA_CHECK(hipStreamWriteValue32(g_stream, flag, value, 0));
    return 0;
}

int hpa_stream_wait_value32(unsigned* flag, unsigned value) {
    HPA_CHECK(hipStreamWaitValue32(g_stream, flag, value, hipStreamWaitValueGte, 0xffffffffu));
    return 0;
}

int hpa_event_record(void* ev) {
    HPA_CHECK(hipEventRecord((hipEvent_t)ev, g_stream));
    return 0;
}

float hpa_event_elapsed_ms(void* start, void* stop) {
    float ms = -1.f;
    if (hipEventSynchronize((hipEvent_t)stop) != hipSuccess) return -1.f;
    if (hipEventElapsedTime(&ms, (hipEvent_t)start, (hipEvent_t)stop) != hipSuccess) return -1.f;
    return ms;
}

int hpa_event_synchronize(void* ev) {
    if (ev) HPA_CHECK(hipEventSynchronize((hipEvent_t)ev));
    return 0;
}

int hpa_event_destroy(void* ev) {
    if (ev) HPA_CHECK(hipEventDestroy((hipEvent_t)ev));
    return 0;
}

int hpa_device_info(char* name, int name_len, int* num_cus, size_t* total_mem) {
    hipDeviceProp_t p;
    int dev = g_device >= 0 ? g_device : 0;
    HPA_CHECK(hipGetDeviceProperties(&p, dev));
    if (name && name_len > 0) {
        snprintf(name, name_len, "%s (%s)", p.name, p.gcnArchName);
    }
    if (num_cus) *num_cus = p.multiProcessorCount;
    if (total_mem) *total_mem = p.totalGlobalMem;
    return 0;
}

// ---------------- hipGraph capture ----------------
int hpa_graph_begin(void) {
    HPA_REQUIRE(g_stream, "hpa_init first");
    HPA_CHECK(hipStreamBeginCapture(g_stream, hipStreamCaptureModeThreadLocal));
    return 0;
}

void* hpa_graph_end(void) {
    hipGraph_t graph = nullptr;
    if (hipStreamEndCapture(g_stream, &graph) != hipSuccess || !graph) {
        hpa_fail(__FILE__, __LINE__, "hipStreamEndCapture failed");
        return nullptr;
    }
    hipGraphExec_t exec = nullptr;
    hipError_t e = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
    (void)hipGraphDestroy(graph);
    if (e != hipSuccess) {
        hpa_fail(__FILE__, __LINE__, hipGetErrorString(e));
        return nullptr;
    }
    return (void*)exec;
}

int hpa_graph_launch(void* exec) {
    HPA_REQUIRE(exec, "null graph");
    HPA_CHECK(hipGraphLaunch((hipGraphExec_t)exec, g_stream));
    return 0;
}

int hpa_graph_destroy(void* exec) {
    if (exec) HPA_CHECK(hipGraphExecDestroy((hipGraphExec_t)exec));
    return 0;
}

// ---------------- page pool ----------------
int hpa_pool_create(HpaKVPool* pool, int num_layers, int num_heads, int head_size, int page_size,
                    int num_pages, int dtype, int managed) {
    HPA_REQUIRE(pool, "pool is NULL");
    memset(pool, 0, sizeof(*pool));
    HPA_REQUIRE(dtype == HPA_F32 || dtype == HPA_BF16, "pool dtype must be HPA_F32 or HPA_BF16");
    HPA_REQUIRE(head_size % 8 == 0, "head_size must be a multiple of 8");
    HPA_REQUIRE(dtype == HPA_F32 || page_size % 8 == 0, "bf16 pages need a page size multiple of 8");
    HPA_REQUIRE(page_size > 0 && num_pages > 0 && num_layers > 0 && num_heads > 0, "bad pool shape");
    pool->num_layers = num_layers;
    pool->num_heads = num_heads;
    pool->head_size = head_size;
    pool->page_size = page_size;
    pool->num_pages = num_pages;
    pool->dtype = dtype;
    pool->elem_bytes = dtype == HPA_BF16 ? 2 : 4;
    pool->page_elems = (size_t)2 * num_heads * page_size * head_size;
    pool->layer_elems = (size_t)num_pages * pool->page_elems;
    pool->bytes = (size_t)num_layers * pool->layer_elems * pool->elem_bytes;
    pool->managed = managed;
    pool->base = managed ? hpa_malloc_managed(pool->bytes) : hpa_malloc(pool->bytes);
    HPA_REQUIRE(pool->base, "page pool allocation failed");
    // defined contents: a masked-out lane never multiplies garbage (NaN) pages
    HPA_CHECK(hipMemsetAsync(pool->base, 0, pool->bytes, g_stream));
    HPA_CHECK(hipStreamSynchronize(g_stream));
    return 0;
}

void hpa_pool_destroy(HpaKVPool* pool) {
    if (pool && pool->base) {
        hpa_free(pool->base);
        pool->base = nullptr;
    }
}

void* hpa_pool_tile(const HpaKVPool* p, int layer, int page, int kv, int head) {
    size_t tile = (size_t)p->page_size * p->head_size;
    size_t e = (size_t)layer * p->layer_elems + (size_t)page * p->page_elems +
               ((size_t)kv * p->num_heads + head) * tile;
    return (char*)p->base + e * p->elem_bytes;
}

size_t hpa_pool_k_index(const HpaKVPool* p, int layer, int page, int head, int slot, int d) {
    size_t tile = (size_t)p->page_size * p->head_size;
    size_t base = (size_t)layer * p->layer_elems + (size_t)page * p->page_elems + (size_t)head * tile;
    if (p->dtype == HPA_BF16) return base + ((size_t)(d >> 3) * p->page_size + slot) * 8 + (d & 7);
    return base + ((size_t)(d >> 2) * p->page_size + slot) * 4 + (d & 3);
}

size_t hpa_pool_v_index(const HpaKVPool* p, int layer, int page, int head, int slot, int d) {
    size_t tile = (size_t)p->page_size * p->head_size;
    size_t base = (size_t)layer * p->layer_elems + (size_t)page * p->page_elems +
                  ((size_t)p->num_heads + head) * tile;
    return base + (size_t)slot * p->head_size + d;
}

}  // extern "C"
