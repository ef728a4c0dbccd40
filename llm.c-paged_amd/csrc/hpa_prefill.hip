// hpa_prefill.hip -- multi-query (prefill) paged attention on MFMA, and the
// row gather that hands a prefill's last rows to the logits GEMM.
//
// attention_paged (reference paged_infer.c:163-240) for T query rows per
// sequence at absolute positions start[b] .. start[b]+T-1, causal over the
// sequence's pages (keys 0 .. query position).  Unlike the decode path this
// is dense: a 16-query x 16-key score tile is one v_mfma_f32_16x16x4_f32
// chain over the head dimension, and P.V another ("the step
// where head_dim x page_size is actually dense").
//
// Workgroup = (sequence, head, 64-query block), 4 waves, wave w owns queries
// 16w .. 16w+15 of the block.  Per 16-key tile:
//   * the 256 threads stage K and V rows of the tile (through the block
//     table) into LDS, rows padded to 68 floats (bank-conflict free operand
//     reads, 16-byte aligned stores); two buffers, next tile's rows already in
//     registers while the current tile computes;
//   * S = Q K^T: 16 MFMAs (d = 64 in steps of 4); the C tile gives each lane
//     4 query rows x 1 key column;
//   * online softmax per query row in the exp2 domain (running max from
//     -10000*log2(e): the reference's maxval floor, :187), causal mask;
//   * P goes through a wave-private LDS tile into MFMA A layout, O += P V:
//     16 MFMAs into 4 output tiles (16 queries x 64 dims).
// fp32 throughout (the reference's arithmetic type); summation order differs
// from the reference's sequential loops, hence the 1e-4 tolerance of the tests.
#include <math.h>

#include "hpa_attn_body.h"

namespace {

constexpr int HS = 64;
constexpr int KT = 16;    // keys per tile
constexpr int QB = 64;    // queries per workgroup
constexpr int LD = 68;    // padded LDS row (floats)
typedef float f32x4 __attribute__((ext_vector_type(4)));

struct PrefillArgs {
    const float* q;        // [rows][C] row-major (row = row0[b] + t)
    const void* layer_base;
    size_t page_elems;
    int NH, P, bf16;
    const int* bt;
    int bt_stride;
    const int* start;      // [B] position of row t = 0
    const int* row0;       // [B] first row of sequence b (nullptr: b*T)
    const int* len;        // [B] query rows of sequence b (nullptr: T); T = max
    int T;
    float* out;            // frag layout [Rp][C]
    float qscale, m_init;
};

// one K and one V element group (float4) of key `key` of the tile, dims 4c..4c+3
__device__ __forceinline__ void load_kv4(const PrefillArgs& a, const int* bt, int h, int key, int c, float4& k4,
                                         float4& v4) {
    const int page = bt[key / a.P];
    const int slot = key % a.P;
    const size_t tile = (size_t)a.P * HS;
    if (a.bf16) {
        const unsigned short* base = reinterpret_cast<const unsigned short*>(a.layer_base) + (size_t)page * a.page_elems;
        const unsigned short* kp = base + (size_t)h * tile + ((size_t)(c >> 1) * a.P + slot) * 8 + (c & 1) * 4;
        const unsigned short* vp = base + (size_t)(a.NH + h) * tile + (size_t)slot * HS + 4 * c;
        const uint2 ku = *reinterpret_cast<const uint2*>(kp);
        const uint2 vu = *reinterpret_cast<const uint2*>(vp);
        k4 = make_float4(hpa_attn::bf_lo(ku.x), hpa_attn::bf_hi(ku.x), hpa_attn::bf_lo(ku.y), hpa_attn::bf_hi(ku.y));
        v4 = make_float4(hpa_attn::bf_lo(vu.x), hpa_attn::bf_hi(vu.x), hpa_attn::bf_lo(vu.y), hpa_attn::bf_hi(vu.y));
    } else {
        const float* base = reinterpret_cast<const float*>(a.layer_base) + (size_t)page * a.page_elems;
        k4 = *reinterpret_cast<const float4*>(base + (size_t)h * tile + ((size_t)c * a.P + slot) * 4);
        v4 = *reinterpret_cast<const float4*>(base + (size_t)(a.NH + h) * tile + (size_t)slot * HS + 4 * c);
    }
}

__global__ __launch_bounds__(256) void prefill_attn_kernel(PrefillArgs a) {
    __shared__ __attribute__((aligned(16))) float sK[2][KT * LD];
    __shared__ __attribute__((aligned(16))) float sV[2][KT * LD];
    __shared__ float sP[4][16 * 17];

    const int NH = a.NH;
    const int nqb = (a.T + QB - 1) / QB;
    const int qb = blockIdx.x % nqb;
    const int bh = blockIdx.x / nqb;
    const int b = bh / NH, h = bh - b * NH;
    const int Tb = a.len ? a.len[b] : a.T;  // ragged: this sequence's query rows
    if (qb * QB >= Tb) return;              // whole workgroup past them (uniform, before any barrier)
    const int rb0 = a.row0 ? a.row0[b] : b * a.T;
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const int g = lane >> 4;     // C-layout row group: rows 4g .. 4g+3
    const int c16 = lane & 15;   // C-layout column
    const int C = NH * HS;
    const int* bt = a.bt + (size_t)b * a.bt_stride;
    const int start = a.start[b];
    const int t0 = qb * QB + 16 * w;                  // this wave's first query (row offset in the sequence)
    const int last_t = min(Tb - 1, qb * QB + QB - 1);
    const int kmax = start + last_t;                  // last key any query of the block sees
    const int ntiles = kmax / KT + 1;

    // Q operand (A layout: row m = lane & 15, k = lane >> 4 within a 4-step):
    // qa[s] = q[row t0 + (lane&15)][h*64 + 4s + (lane>>4)], pre-scaled
    float qa[16];
    {
        const int t = min(t0 + c16, Tb - 1);
        const float* qr = a.q + ((size_t)rb0 + t) * C + h * HS;
#pragma unroll
        for (int s = 0; s < 16; ++s) qa[s] = qr[4 * s + g] * a.qscale;
    }
    // per-lane softmax state of rows 4g + r (r = 0..3)
    float m[4], l[4];
    f32x4 o[4];  // output tiles: d = 16*dt + c16, rows 4g + r
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        m[r] = a.m_init;
        l[r] = 0.f;
        o[r] = f32x4{0.f, 0.f, 0.f, 0.f};
    }

    // staging: thread -> (key = tid & 15, chunk c = tid >> 4): one float4 of K, one of V
    const int skey = threadIdx.x & 15, sc = threadIdx.x >> 4;
    float4 rk, rv;
    load_kv4(a, bt, h, min(skey, kmax), sc, rk, rv);

    for (int it = 0; it < ntiles; ++it) {
        const int buf = it & 1;
        *reinterpret_cast<float4*>(&sK[buf][skey * LD + 4 * sc]) = rk;
        *reinterpret_cast<float4*>(&sV[buf][skey * LD + 4 * sc]) = rv;
        __syncthreads();
        if (it + 1 < ntiles) load_kv4(a, bt, h, min((it + 1) * KT + skey, kmax), sc, rk, rv);
        const int k0 = it * KT;
        if (k0 <= start + min(t0 + 15, Tb - 1)) {  // any key of the tile visible to this wave's queries
            // S = Q K^T  (B operand: B[k = lane>>4][n = key lane&15] = K[key][4s + k])
            f32x4 s4 = f32x4{0.f, 0.f, 0.f, 0.f};
            const float* kr = &sK[buf][c16 * LD + g];
#pragma unroll
            for (int s = 0; s < 16; ++s) s4 = __builtin_amdgcn_mfma_f32_16x16x4f32(qa[s], kr[4 * s], s4, 0, 0, 0);
            // online softmax per query row 4g + r over this tile's 16 keys (lanes c16)
            const int key = k0 + c16;
            float p[4], alpha[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int qpos = start + t0 + 4 * g + r;
                const float sv = key <= qpos ? s4[r] : -INFINITY;
                float mt = sv;
#pragma unroll
                for (int x = 1; x < 16; x <<= 1) mt = fmaxf(mt, __shfl_xor(mt, x, 64));
                const float mn = fmaxf(m[r], mt);
                alpha[r] = exp2f(m[r] - mn);
                p[r] = exp2f(sv - mn);
                float ps = p[r];
#pragma unroll
                for (int x = 1; x < 16; x <<= 1) ps += __shfl_xor(ps, x, 64);
                l[r] = fmaf(l[r], alpha[r], ps);
                m[r] = mn;
            }
            // rescale: register r of every output tile is query row 4g + r
#pragma unroll
            for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                for (int r = 0; r < 4; ++r) o[dt][r] *= alpha[r];
            // P -> wave-private LDS tile (C layout in: row 4g+r, col c16; read back
            // in A layout: row lane&15, k = lane>>4); wavefront-scope ordering
            // only (waves skip tiles independently: no workgroup barrier here)
            float* pw = sP[w];
#pragma unroll
            for (int r = 0; r < 4; ++r) pw[(4 * g + r) * 17 + c16] = p[r];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            // O += P V: A[m = q = lane&15][k = key 4j + lane>>4], B[k][n = d] = V[key][16dt + c16]
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float pa = pw[c16 * 17 + 4 * j + g];
                const float* vr = &sV[buf][(4 * j + g) * LD + c16];
#pragma unroll
                for (int dt = 0; dt < 4; ++dt)
                    o[dt] = __builtin_amdgcn_mfma_f32_16x16x4f32(pa, vr[16 * dt], o[dt], 0, 0, 0);
            }
            __builtin_amdgcn_wave_barrier();  // P reads done before the next tile's P stores
        }
    }
    // normalise and write: tile dt, reg r -> row t0 + 4g + r, col h*64 + 16dt + c16
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int t = t0 + 4 * g + r;
        if (t < Tb) {
            const float inv = l[r] == 0.f ? 0.f : 1.f / l[r];
            const int row = rb0 + t;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt) a.out[hpa::frag_index(row, h * HS + 16 * dt + c16, C)] = o[dt][r] * inv;
        }
    }
}

}  // namespace

namespace {

// rows idx[i] of a frag-layout [*][C] matrix and its LN statistics
// ([ct][src_Mp][2]) -> rows i of another ([*][C], [ct][dst_Mp][2])
__global__ __launch_bounds__(256) void gather_rows_kernel(const float* __restrict__ src, const float* __restrict__ sst,
                                                          int src_Mp, const int* __restrict__ idx, float* __restrict__ dst,
                                                          float* __restrict__ dst_st, int dst_Mp, int C, int ct) {
    const int i = blockIdx.x, r = idx[i];
    if (r < 0) return;  // row i left as it is
    for (int c = threadIdx.x * 4; c < C; c += 1024)
        *reinterpret_cast<float4*>(dst + hpa::frag_index(i, c, C)) =
            *reinterpret_cast<const float4*>(src + hpa::frag_index(r, c, C));
    for (int t = threadIdx.x; t < ct; t += 256) {
        dst_st[((size_t)t * dst_Mp + i) * 2] = sst[((size_t)t * src_Mp + r) * 2];
        dst_st[((size_t)t * dst_Mp + i) * 2 + 1] = sst[((size_t)t * src_Mp + r) * 2 + 1];
    }
}

}  // namespace

extern "C" {

int hpa_paged_attention_prefill_ragged(const float* q, const HpaKVPool* pool, int layer, const int* block_table,
                                       int bt_stride, const int* start, const int* row0, const int* len, int B,
                                       int T, float* out_frag) {
    HPA_REQUIRE(pool && pool->base && pool->head_size == HS, "prefill attention: pool with head_size 64");
    HPA_REQUIRE(pool->dtype == HPA_F32 || pool->dtype == HPA_BF16, "prefill attention: fp32 or bf16 pool");
    HPA_REQUIRE(pool->dtype == HPA_F32 || pool->page_size % 8 == 0, "prefill attention: bf16 pages need P % 8");
    HPA_REQUIRE(layer >= 0 && layer < pool->num_layers, "prefill attention: layer out of range");
    HPA_REQUIRE(q && block_table && start && out_frag && B > 0 && T > 0, "prefill attention: bad arguments");
    HPA_REQUIRE(!row0 == !len, "prefill attention: row0 and len go together");
    PrefillArgs a;
    a.q = q;
    a.layer_base = (const char*)pool->base + (size_t)layer * pool->layer_elems * pool->elem_bytes;
    a.page_elems = pool->page_elems;
    a.NH = pool->num_heads;
    a.P = pool->page_size;
    a.bf16 = pool->dtype == HPA_BF16;
    a.bt = block_table;
    a.bt_stride = bt_stride;
    a.start = start;
    a.row0 = row0;
    a.len = len;
    a.T = T;
    a.out = out_frag;
    const float log2e = 1.4426950408889634f;
    a.qscale = (float)(1.0 / sqrt((double)HS)) * log2e;  // the reference's 1/sqrtf(hs) (:197), log2 domain
    a.m_init = -10000.0f * log2e;                         // the reference's maxval = -10000 (:187)
    const int nqb = (T + QB - 1) / QB;
    prefill_attn_kernel<<<(unsigned)(B * a.NH * nqb), 256, 0, hpa_stream()>>>(a);
    HPA_LAUNCH_CHECK();
    return 0;
}

int hpa_paged_attention_prefill(const float* q, const HpaKVPool* pool, int layer, const int* block_table,
                                int bt_stride, const int* start, int B, int T, float* out_frag) {
    return hpa_paged_attention_prefill_ragged(q, pool, layer, block_table, bt_stride, start, nullptr, nullptr, B, T,
                                              out_frag);
}

int hpa_gather_rows_frag(const float* src, const float* src_stats, int src_Mp, const int* rows, int n,
                         float* dst, float* dst_stats, int dst_Mp, int C) {
    HPA_REQUIRE(src && src_stats && rows && dst && dst_stats && n > 0 && C % 16 == 0 && n <= dst_Mp,
                "gather_rows_frag: bad arguments");
    gather_rows_kernel<<<n, 256, 0, hpa_stream()>>>(src, src_stats, src_Mp, rows, dst, dst_stats, dst_Mp, C, C / 16);
    HPA_LAUNCH_CHECK();
    return 0;
}

}  // extern "C"
