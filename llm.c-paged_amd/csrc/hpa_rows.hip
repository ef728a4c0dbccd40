// hpa_rows.hip -- row-wise decode kernels: embedding+LN, split-K reduction
// epilogues (bias, residual, LN, GELU, KV append into pages), greedy argmax.
// All HBM-light (a few hundred KB per launch at B = 64); their job is to fuse
// what the reference does in separate passes (paged_infer.c:24-89, :243-257,
// :505-573, :937-951) so each decode-step tensor is written once.
#include "hpa_internal.h"

namespace {

constexpr int kRowThreads = 256;
constexpr int kMaxPerThread = 8;  // C <= 2048 (GPT-2 XL: 1600)

// block-wide sum over kRowThreads threads (4 waves); fixed order -> deterministic
__device__ __forceinline__ float block_sum(float v, float* scratch) {
    v = hpa::wave_sum(v);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) scratch[w] = v;
    __syncthreads();
    float t = scratch[0] + scratch[1] + scratch[2] + scratch[3];
    __syncthreads();
    return t;
}

// LN of x[0..C) held as xs[i] = x[threadIdx.x + i*256] (paged_infer.c:49-89:
// mean, biased variance by the two-pass formula, rstd = 1/sqrtf(v + 1e-5))
__device__ __forceinline__ void row_layernorm(const float (&xs)[kMaxPerThread], int C,
                                              const float* __restrict__ w, const float* __restrict__ bb,
                                              float* __restrict__ out, float* scratch) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < kMaxPerThread; ++i) {
        const int c = threadIdx.x + i * kRowThreads;
        if (c < C) s += xs[i];
    }
    const float m = block_sum(s, scratch) / C;
    float v = 0.f;
#pragma unroll
    for (int i = 0; i < kMaxPerThread; ++i) {
        const int c = threadIdx.x + i * kRowThreads;
        if (c < C) {
            const float d = xs[i] - m;
            v += d * d;
        }
    }
    v = block_sum(v, scratch) / C;
    const float rs = 1.0f / sqrtf(v + 1e-5f);
#pragma unroll
    for (int i = 0; i < kMaxPerThread; ++i) {
        const int c = threadIdx.x + i * kRowThreads;
        if (c < C) out[c] = (rs * (xs[i] - m)) * w[c] + bb[c];
    }
}

__global__ __launch_bounds__(kRowThreads) void embed_ln_kernel(
    const int* __restrict__ tokens, const int* __restrict__ pos, const float* __restrict__ wte,
    const float* __restrict__ wpe, const float* __restrict__ lnw, const float* __restrict__ lnb,
    float* __restrict__ residual, float* __restrict__ ln_out, int C) {
    __shared__ float scratch[4];
    const int b = blockIdx.x;
    const float* __restrict__ te = wte + (size_t)tokens[b] * C;
    const float* __restrict__ pe = wpe + (size_t)pos[b] * C;
    float xs[kMaxPerThread];
#pragma unroll
    for (int i = 0; i < kMaxPerThread; ++i) {
        const int c = threadIdx.x + i * kRowThreads;
        xs[i] = 0.f;
        if (c < C) {
            xs[i] = te[c] + pe[c];
            residual[(size_t)b * C + c] = xs[i];
        }
    }
    row_layernorm(xs, C, lnw, lnb, ln_out + (size_t)b * C, scratch);
}

// sum_{s<S} part[s*slab + idx[e]] for E elements, slabs added in order s = 0..S-1
// (deterministic).  Loads are issued 8 slabs x E elements at a time with
// clamped, unconditional addresses so they are all in flight together; the
// split-K sum is latency-bound otherwise (one dependent HBM/L2 trip per slab).
template <int E>
__device__ __forceinline__ void sum_slabs(const float* __restrict__ part, size_t slab, int S,
                                          const size_t (&idx)[E], const bool (&ok)[E], float (&a)[E]) {
#pragma unroll
    for (int e = 0; e < E; ++e) a[e] = 0.f;
    for (int s0 = 0; s0 < S; s0 += 8) {
        float v[E][8];
#pragma unroll
        for (int e = 0; e < E; ++e)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int s = min(s0 + j, S - 1);
                v[e][j] = ok[e] ? part[(size_t)s * slab + idx[e]] : 0.f;
            }
#pragma unroll
        for (int e = 0; e < E; ++e)
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (s0 + j < S) a[e] += v[e][j];
    }
}

__global__ __launch_bounds__(kRowThreads) void residual_ln_kernel(
    const float* __restrict__ part, int splitk, size_t slab, const float* __restrict__ bias,
    const float* res_in, float* res_out, const float* __restrict__ lnw,  // may alias (in place)
    const float* __restrict__ lnb, float* __restrict__ ln_out, int C) {
    __shared__ float scratch[4];
    const int b = blockIdx.x;
    size_t idx[kMaxPerThread];
    bool ok[kMaxPerThread];
#pragma unroll
    for (int i = 0; i < kMaxPerThread; ++i) {
        const int c = threadIdx.x + i * kRowThreads;
        ok[i] = c < C;
        idx[i] = (size_t)b * C + (ok[i] ? c : 0);
    }
    float xs[kMaxPerThread];
    sum_slabs<kMaxPerThread>(part, slab, splitk, idx, ok, xs);
#pragma unroll
    for (int i = 0; i < kMaxPerThread; ++i) {
        const int c = threadIdx.x + i * kRowThreads;
        if (ok[i]) {
            float a = xs[i];
            if (bias) a += bias[c];
            xs[i] = res_in[idx[i]] + a;  // residual_forward(out, inp1, inp2)
            res_out[idx[i]] = xs[i];
        } else {
            xs[i] = 0.f;
        }
    }
    if (lnw) row_layernorm(xs, C, lnw, lnb, ln_out + (size_t)b * C, scratch);
}

// one thread per (b, o), o in [0, 3C): q -> q buffer, k/v -> page slot pos[b]
__global__ __launch_bounds__(256) void qkv_append_kernel(
    const float* __restrict__ part, int splitk, size_t slab, const float* __restrict__ bias,
    float* __restrict__ q, float* __restrict__ layer_base, size_t page_elems, int NH, int P,
    const int* __restrict__ bt, int bt_stride, const int* __restrict__ pos, int C) {
    const int b = blockIdx.y;
    const int o = blockIdx.x * 256 + threadIdx.x;
    if (o >= 3 * C) return;
    const size_t ix[1] = {(size_t)b * 3 * C + o};
    const bool ok[1] = {true};
    float sum[1];
    sum_slabs<1>(part, slab, splitk, ix, ok, sum);
    float a = sum[0];
    if (bias) a += bias[o];
    if (o < C) {
        q[(size_t)b * C + o] = a;
        return;
    }
    const int kv = o >= 2 * C;
    const int c = o - (kv ? 2 * C : C);
    const int hh = c >> 6, d = c & 63;
    const int p = pos[b];
    const int page = bt[(size_t)b * bt_stride + p / P];
    const int slot = p % P;
    float* tile = layer_base + (size_t)page * page_elems + ((size_t)kv * NH + hh) * P * 64;
    if (kv == 0)
        tile[((d >> 2) * P + slot) * 4 + (d & 3)] = a;  // K: [chunk][slot][4]
    else
        tile[slot * 64 + d] = a;  // V: [slot][64]
}

__global__ __launch_bounds__(256) void bias_gelu_kernel(const float* __restrict__ part, int splitk,
                                                        size_t slab, const float* __restrict__ bias,
                                                        float* __restrict__ out, int N, size_t total) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= total) return;
    const size_t ix[1] = {i};
    const bool ok[1] = {true};
    float sum[1];
    sum_slabs<1>(part, slab, splitk, ix, ok, sum);
    float a = sum[0];
    if (bias) a += bias[i % N];
    out[i] = hpa::gelu_ref(a);
}

// greedy: first max wins (strict > in index order, paged_infer.c:937-951)
__device__ __forceinline__ void argmax_merge(float& v, int& i, float v2, int i2) {
    if (v2 > v || (v2 == v && i2 < i)) {
        v = v2;
        i = i2;
    }
}

__global__ __launch_bounds__(1024) void argmax_advance_kernel(const float* __restrict__ logits, int V,
                                                              int* __restrict__ next,
                                                              int* __restrict__ tokens,
                                                              int* __restrict__ pos) {
    __shared__ float sv[16];
    __shared__ int si[16];
    const int b = blockIdx.x;
    const float* __restrict__ row = logits + (size_t)b * V;
    float bv = -INFINITY;
    int bi = 0x7fffffff;
    for (int i = threadIdx.x; i < V; i += 1024) {
        const float x = row[i];
        if (x > bv) {  // i increases per thread: strict > keeps the first max
            bv = x;
            bi = i;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float v2 = __shfl_xor(bv, o, 64);
        const int i2 = __shfl_xor(bi, o, 64);
        argmax_merge(bv, bi, v2, i2);
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        sv[w] = bv;
        si[w] = bi;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        float v = sv[0];
        int i = si[0];
        for (int k = 1; k < 16; ++k) argmax_merge(v, i, sv[k], si[k]);
        if (i == 0x7fffffff) i = 0;  // all-NaN row
        next[b] = i;
        if (tokens) tokens[b] = i;
        if (pos) pos[b] += 1;
    }
}

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
                                                               int bt_stride, uint64_t seed) {
    const int p = blockIdx.x, b = blockIdx.y, l = blockIdx.z;
    const int C = NH * 64;
    const int page = bt[(size_t)b * bt_stride + p / P];
    const int slot = p % P;
    const size_t off = (size_t)l * layer_elems + (size_t)page * page_elems;
    const uint64_t key = (((uint64_t)l * 4096u + b) * 1048576u + p) * 4u;
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

int hpa_embed_ln(const int* tokens, const int* pos, const float* wte, const float* wpe,
                 const float* ln_w, const float* ln_b, float* residual, float* ln_out, int B, int C) {
    HPA_REQUIRE(B > 0 && C > 0 && C <= kRowThreads * kMaxPerThread, "embed_ln: bad shape");
    embed_ln_kernel<<<B, kRowThreads, 0, hpa_stream()>>>(tokens, pos, wte, wpe, ln_w, ln_b, residual,
                                                         ln_out, C);
    HPA_LAUNCH_CHECK();
    return 0;
}

int hpa_residual_ln(const float* part, int splitk, const float* bias, const float* residual_in,
                    float* residual_out, const float* ln_w, const float* ln_b, float* ln_out, int B,
                    int C) {
    HPA_REQUIRE(B > 0 && C > 0 && C <= kRowThreads * kMaxPerThread, "residual_ln: bad shape");
    HPA_REQUIRE(splitk >= 1, "residual_ln: splitk >= 1");
    residual_ln_kernel<<<B, kRowThreads, 0, hpa_stream()>>>(part, splitk, (size_t)B * C, bias,
                                                            residual_in, residual_out, ln_w, ln_b,
                                                            ln_out, C);
    HPA_LAUNCH_CHECK();
    return 0;
}

int hpa_qkv_append(const float* part, int splitk, const float* bias, float* q, const HpaKVPool* pool,
                   int layer, const int* block_table, int bt_stride, const int* pos, int B, int C) {
    HPA_REQUIRE(pool && pool->base && pool->dtype == HPA_F32, "qkv_append: fp32 pool expected");
    HPA_REQUIRE(pool->head_size == 64 && pool->num_heads * 64 == C, "qkv_append: C != NH*64");
    HPA_REQUIRE(layer >= 0 && layer < pool->num_layers, "qkv_append: layer out of range");
    HPA_REQUIRE(B > 0 && splitk >= 1, "qkv_append: bad shape");
    float* lb = (float*)pool->base + (size_t)layer * pool->layer_elems;
    dim3 grid((3 * C + 255) / 256, B);
    qkv_append_kernel<<<grid, 256, 0, hpa_stream()>>>(part, splitk, (size_t)B * 3 * C, bias, q, lb,
                                                      pool->page_elems, pool->num_heads,
                                                      pool->page_size, block_table, bt_stride, pos, C);
    HPA_LAUNCH_CHECK();
    return 0;
}

int hpa_bias_gelu(const float* part, int splitk, const float* bias, float* out, int M, int N) {
    HPA_REQUIRE(M > 0 && N > 0 && splitk >= 1, "bias_gelu: bad shape");
    const size_t total = (size_t)M * N;
    bias_gelu_kernel<<<(unsigned)((total + 255) / 256), 256, 0, hpa_stream()>>>(part, splitk, total,
                                                                                bias, out, N, total);
    HPA_LAUNCH_CHECK();
    return 0;
}

int hpa_argmax_advance(const float* logits, int B, int V, int* next, int* tokens, int* pos) {
    HPA_REQUIRE(B > 0 && V > 0 && logits && next, "argmax: bad arguments");
    argmax_advance_kernel<<<B, 1024, 0, hpa_stream()>>>(logits, V, next, tokens, pos);
    HPA_LAUNCH_CHECK();
    return 0;
}

int hpa_pool_fill_random(const HpaKVPool* pool, const int* block_table, int bt_stride, int B, int ctx,
                         uint64_t seed) {
    HPA_REQUIRE(pool && pool->base && (pool->dtype == HPA_F32 || pool->dtype == HPA_BF16) && pool->head_size == 64,
                "fill_random: fp32/bf16 pool with head_size 64 expected");
    HPA_REQUIRE(B > 0 && B < 4096 && ctx >= 0 && ctx < 1048576, "fill_random: bad shape");
    if (ctx == 0) return 0;
    dim3 grid(ctx, B, pool->num_layers);
    pool_fill_random_kernel<<<grid, 256, 0, hpa_stream()>>>(pool->base, pool->dtype == HPA_BF16, pool->layer_elems,
                                                            pool->page_elems, pool->num_heads,
                                                            pool->page_size, block_table, bt_stride,
                                                            seed);
    HPA_LAUNCH_CHECK();
    return 0;
}

}  // extern "C"
