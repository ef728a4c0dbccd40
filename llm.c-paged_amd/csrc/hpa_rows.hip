// hpa_rows.hip -- synthetic K/V fill of the page pool (the bench's
// synthetic prefill and the attention microbench): every (layer, sequence,
// position) token row of K and V gets U(-1, 1) from a counter-based hash, in
// the pool's fp32 or bf16 layout (hip_paged_attn.h).
#include "hpa_internal.h"

namespace {

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// grid (ctx, B, L): every (layer, sequence, position) token row of K and V
__global__ __launch_bounds__(256) void pool_fill_random_kernel(void* __restrict__ base_v, int bf16,
                                                               size_t layer_elems, size_t page_elems,
                                                               int NH, int P, const int* __restrict__ bt,
                                                               int bt_stride, uint64_t seed, int seq0) {
    const int p = blockIdx.x, b = blockIdx.y, l = blockIdx.z;
    const int bg = seq0 + b;  // the hash follows the global sequence index (shards fill what the whole batch would)
    const int C = NH * 64;
    const int page = bt[(size_t)b * bt_stride + p / P];
    const int slot = p % P;
    const size_t off = (size_t)l * layer_elems + (size_t)page * page_elems;
    const uint64_t key = (((uint64_t)l * 4096u + bg) * 1048576u + p) * 4u;
    for (int i = threadIdx.x; i < 2 * C; i += 256) {
        const int kv = i >= C;
        const int c = i - kv * C;
        const int hh = c >> 6, d = c & 63;
        const uint64_t r = splitmix64(seed ^ (key * 2654435761ull + (uint64_t)i));
        const float u = (float)(r >> 40) * (1.0f / 16777216.0f) * 2.0f - 1.0f;
        const size_t tile = off + ((size_t)kv * NH + hh) * P * 64;
        if (bf16) {
            unsigned short* t = reinterpret_cast<unsigned short*>(base_v) + tile;
            t[kv == 0 ? ((d >> 3) * P + slot) * 8 + (d & 7) : slot * 64 + d] = hpa::f32_to_bf16(u);
        } else {
            float* t = reinterpret_cast<float*>(base_v) + tile;
            t[kv == 0 ? ((d >> 2) * P + slot) * 4 + (d & 3) : slot * 64 + d] = u;
        }
    }
}

}  // namespace

extern "C" {

int hpa_pool_fill_random_ex(const HpaKVPool* pool, const int* block_table, int bt_stride, int B, int ctx,
                            uint64_t seed, int seq_offset) {
    HPA_REQUIRE(pool && pool->base && (pool->dtype == HPA_F32 || pool->dtype == HPA_BF16) && pool->head_size == 64,
                "fill_random: fp32/bf16 pool with head_size 64 expected");
    HPA_REQUIRE(B > 0 && seq_offset >= 0 && seq_offset + B <= 4096 && ctx >= 0 && ctx < 1048576,
                "fill_random: bad shape");
    if (ctx == 0) return 0;
    dim3 grid(ctx, B, pool->num_layers);
    pool_fill_random_kernel<<<grid, 256, 0, hpa_stream()>>>(pool->base, pool->dtype == HPA_BF16, pool->layer_elems,
                                                            pool->page_elems, pool->num_heads,
                                                            pool->page_size, block_table, bt_stride,
                                                            seed, seq_offset);
    HPA_LAUNCH_CHECK();
    return 0;
}

int hpa_pool_fill_random(const HpaKVPool* pool, const int* block_table, int bt_stride, int B, int ctx,
                         uint64_t seed) {
    return hpa_pool_fill_random_ex(pool, block_table, bt_stride, B, ctx, seed, 0);
}

}  // extern "C"
