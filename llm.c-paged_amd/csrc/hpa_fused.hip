// hpa_fused.hip -- the decode layer's GEMMs with everything around them fused.
//
// One launch per weight GEMM of a GPT-2 block (reference gpt2_forward,
// paged_infer.c:696-722, for one decode row per sequence):
//   QKV     : LN1(x) . Wqkv^T + b -> q (row-major) and K/V appended into the
//             sequence's page at pos[b]        (layernorm_forward :696,
//             matmul_cached :706, add_to_cache :710 fused)
//   ATTPROJ : res2 = res + att . Wap^T + b, LN2 row statistics   (:716-718)
//   FC      : gelu(LN2(res2) . Wfc^T + b)                        (:718-720)
//   FCPROJ  : res = res2 + fch . Wfp^T + b, next-LN row statistics (:721-722)
//   LOGITS  : LNf(res) . wte^T, per-tile (max, argmax) for greedy (:725-727)
//
// Shape of the kernel (measured on MI355X, see DESIGN.md "GEMMs"):
//  * At decode M = batch <= 64, each layer GEMM is 75..300 MFLOP.  fp32 MFMA
//    runs at 256 FLOP/clk per CU, so a GEMM spread over only N/16 = 48 CUs
//    is MFMA-bound per CU (fcproj: ~10 us) while 200 CUs idle.  The grid is
//    therefore (16-column tile) x (16-row block): 4x the workgroups at
//    M = 64, with no inter-workgroup reduction (an agent-scope hand-off costs
//    an L2 writeback on this multi-XCD part); the K range is split over the
//    workgroup's 4..16 waves and folded in LDS in a fixed order.
//  * v_mfma_f32_16x16x4_f32 (exact fp32) on operands in the "frag" layout
//    (hpa_internal.h frag_index): every fragment load is one 1 KiB
//    contiguous dwordx4 burst; two trips of U k-steps in flight per wave;
//    one accumulator chain per row block (summation order independent of
//    the row split), MFMA dependency latency hidden by 4+ waves per SIMD.
//  * LayerNorm is applied to the A fragments on load from per-row partial
//    sums written by the previous kernel's epilogue; the epilogue's own
//    operands (bias, residual) are loaded before the LDS fold so their
//    latency overlaps it.
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "hpa_gemm_body.h"

namespace {
using namespace hpa_gemm;

// ---------------------------------------------------------------- frag packing
__global__ void pack_frag_kernel(const float* __restrict__ src, int rows, int K, int ld,
                                 float4* __restrict__ dst, size_t n4) {
    const size_t o = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (o >= n4) return;
    const int lane = (int)(o & 63);
    const size_t blk = o >> 6;  // rb * K16 + kb
    const int K16 = K >> 4;
    const int kb = (int)(blk % K16);
    const int rb = (int)(blk / K16);
    const int m = rb * 16 + (lane & 15);
    const int k = kb * 16 + 4 * (lane >> 4);
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (m < rows) v = *reinterpret_cast<const float4*>(src + (size_t)m * ld + k);
    dst[o] = v;
}

// LayerNorm folding (hpa_ln_fold_pack): one wave per output column n
__global__ __launch_bounds__(64) void ln_fold_kernel(const float* __restrict__ W, int K,
                                                     const float* __restrict__ g, const float* __restrict__ b,
                                                     const float* __restrict__ bias, float* __restrict__ Wg,
                                                     float* __restrict__ c1, float* __restrict__ c2) {
    const int n = blockIdx.x, lane = threadIdx.x;
    const float* wr = W + (size_t)n * K;
    float* wgr = Wg + (size_t)n * K;
    double s1 = 0.0, s2 = 0.0;
    for (int k = lane; k < K; k += 64) {
        const float wg = wr[k] * g[k];  // the packed weight, rounded once
        wgr[k] = wg;
        s1 += (double)wg;
        s2 += (double)b[k] * (double)wr[k];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        s1 += __shfl_xor(s1, o, 64);
        s2 += __shfl_xor(s2, o, 64);
    }
    if (lane == 0) {
        c1[n] = (float)s1;
        c2[n] = (float)(s2 + (bias ? (double)bias[n] : 0.0));
    }
}

__global__ void unpack_frag_kernel(const float4* __restrict__ src, int rows, int K,
                                   float* __restrict__ dst, int ld, size_t n4) {
    const size_t o = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (o >= n4) return;
    const int lane = (int)(o & 63);
    const size_t blk = o >> 6;
    const int K16 = K >> 4;
    const int kb = (int)(blk % K16);
    const int rb = (int)(blk / K16);
    const int m = rb * 16 + (lane & 15);
    const int k = kb * 16 + 4 * (lane >> 4);
    if (m < rows) *reinterpret_cast<float4*>(dst + (size_t)m * ld + k) = src[o];
}

// ---------------------------------------------------------------- embedding
__global__ __launch_bounds__(256) void embed_frag_kernel(const int* __restrict__ tokens,
                                                         const int* __restrict__ pos,
                                                         const float* __restrict__ wte,
                                                         const float* __restrict__ wpe,
                                                         float* __restrict__ res, float* __restrict__ stats,
                                                         int C, int4* __restrict__ zero, int zero_n4) {
    __shared__ float sc[8];
    const int b = blockIdx.x;
    // the step's counter block (persistent layer hand-offs), zeroed here
    // instead of by a memset node of its own
    for (int i = b * 256 + threadIdx.x; i < zero_n4; i += gridDim.x * 256) zero[i] = make_int4(0, 0, 0, 0);
    const float* te = wte + (size_t)tokens[b] * C;
    const float* pe = wpe + (size_t)pos[b] * C;
    float s1 = 0.f, s2 = 0.f;
    for (int c = threadIdx.x; c < C; c += 256) {
        const float x = te[c] + pe[c];  // encoder_forward (paged_infer.c:43), absolute position
        res[hpa::frag_index(b, c, C)] = x;
        s1 += x;
        s2 += x * x;
    }
    s1 = hpa::wave_sum(s1);
    s2 = hpa::wave_sum(s2);
    if ((threadIdx.x & 63) == 0) {
        sc[threadIdx.x >> 6] = s1;
        sc[4 + (threadIdx.x >> 6)] = s2;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        stats[(size_t)b * 2] = (sc[0] + sc[1]) + (sc[2] + sc[3]);
        stats[(size_t)b * 2 + 1] = (sc[4] + sc[5]) + (sc[6] + sc[7]);
    }
}

// ---------------------------------------------------------------- greedy
__global__ __launch_bounds__(256) void argmax_final_kernel(const float* __restrict__ part, int ntiles,
                                                           int Mp, int* __restrict__ next,
                                                           int* __restrict__ tokens,
                                                           int* __restrict__ pos,
                                                           const int* __restrict__ active) {
    __shared__ float sv[4];
    __shared__ int si[4];
    const int b = blockIdx.x;
    if (active && active[b] <= 0) return;  // row left as it is
    float bv = -INFINITY;
    int bi = 0x7fffffff;
    for (int t = threadIdx.x; t < ntiles; t += 256) {
        const float v = part[((size_t)t * Mp + b) * 2];
        const int i = __float_as_int(part[((size_t)t * Mp + b) * 2 + 1]);
        if (v > bv) {  // tiles visited in increasing index order per thread
            bv = v;
            bi = i;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float v2 = __shfl_xor(bv, o, 64);
        const int i2 = __shfl_xor(bi, o, 64);
        if (v2 > bv || (v2 == bv && i2 < bi)) {
            bv = v2;
            bi = i2;
        }
    }
    if ((threadIdx.x & 63) == 0) {
        sv[threadIdx.x >> 6] = bv;
        si[threadIdx.x >> 6] = bi;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        float v = sv[0];
        int i = si[0];
        for (int k = 1; k < 4; ++k)
            if (sv[k] > v || (sv[k] == v && si[k] < i)) {
                v = sv[k];
                i = si[k];
            }
        if (i == 0x7fffffff) i = 0;
        next[b] = i;
        if (tokens) tokens[b] = i;
        if (pos) pos[b] += 1;
    }
}

// ---------------------------------------------------------------- sampling
// Multinomial draw from softmax(logits[b]) in the REFERENCE's arithmetic
// order (softmax_forward paged_infer.c:259-286, sample_mult :837-848, coin =
// random_f32 :826-835), so draws match it: the fp32 running sums over ~50k
// probabilities drift by more than one probability's width, so any other
// summation order picks neighbouring ids near CDF boundaries.  The additions
// stay sequential (one lane), everything else is parallel (see the kernel).
// Each sequence has its own xorshift state, advanced once per draw on the
// device.
__device__ __forceinline__ unsigned int xorshift_u32(unsigned long long& s) {
    s ^= s >> 12;
    s ^= s << 25;
    s ^= s >> 27;
    return (unsigned int)((s * 0x2545F4914F6CDD1Dull) >> 32);
}

constexpr int kSampPer = 16;                 // elements per lane per block
constexpr int kSampBlk = 64 * kSampPer;     // 1024 elements per block

// a block of logits, coalesced: element base + j*64 + lane -> v[j]
__device__ __forceinline__ void samp_load(const float* lg, int V, int base, int lane, float* v) {
#pragma unroll
    for (int j = 0; j < kSampPer; ++j) {
        const int i = base + j * 64 + lane;
        v[j] = i < V ? lg[i] : -INFINITY;
    }
}

// lane 0 of the consumer wave: acc += v[k] for nb*64 values of an LDS
// buffer, in index order, branch-free (batches of 16 x 16-B LDS reads).
// Pads beyond V hold +0 and leave the sum unchanged.  The chain runs at the
// dependent-add latency (~4 ns per add, tools/micro/chain.hip); prefetching
// the next batch's LDS reads measured slower (465 vs 416 us per launch).
__device__ __forceinline__ float samp_chain(const float* buf, int nb, float acc) {
    const float4* s4 = reinterpret_cast<const float4*>(buf);
    for (int q0 = 0; q0 < nb * 16; q0 += 16) {
        float4 r[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) r[q] = s4[q0 + q];
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            acc += r[q].x;
            acc += r[q].y;
            acc += r[q].z;
            acc += r[q].w;
        }
    }
    return acc;
}

// Two waves per row.  Wave 1 produces: it streams the logits (one block of
// 1024 ahead) and writes expf(x - max) (pass 1) or expf(x - max) / sum
// (pass 2) into one of two LDS buffers.  Wave 0's lane 0 consumes the other
// buffer with the order-dependent additions, so the serial chain never waits
// for a load or an exp.  Pass 2 checks coin < cdf once per 64 values: cdf is
// non-decreasing, so when the batch-end cdf exceeds the coin the batch is
// replayed from its start with the per-element test (same additions, same
// roundings), which yields the first index where coin < cdf.
__global__ __launch_bounds__(128) void sample_final_kernel(const float* __restrict__ logits, int V,
                                                           unsigned long long* __restrict__ state,
                                                           int* __restrict__ next, int* __restrict__ tokens,
                                                           int* __restrict__ pos, const int* __restrict__ active) {
    __shared__ __attribute__((aligned(16))) float sh[2][kSampBlk];
    __shared__ float s_red[2];
    __shared__ int s_found;
    const int b = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (active && active[b] <= 0) return;  // row left as it is (its RNG state too)
    const float* lg = logits + (size_t)b * V;
    // maxval = -10000; if (x > maxval) maxval = x  (exact in any order)
    float mx = -10000.0f;
    for (int i = threadIdx.x; i < V; i += 128) mx = fmaxf(mx, lg[i]);
    mx = hpa::wave_max(mx);
    if (lane == 0) s_red[w] = mx;
    __syncthreads();
    mx = fmaxf(s_red[0], s_red[1]);
    const int nblk = (V + kSampBlk - 1) / kSampBlk;
    float cur[kSampPer], nxt[kSampPer];
    // pass 1: sum += expf(x - maxval) in index order
    float sum = 0.f;
    if (w == 1) samp_load(lg, V, 0, lane, cur);
    for (int it = 0; it <= nblk; ++it) {
        if (w == 1 && it < nblk) {
            if (it + 1 < nblk) samp_load(lg, V, (it + 1) * kSampBlk, lane, nxt);
            float* dst = sh[it & 1];
#pragma unroll
            for (int j = 0; j < kSampPer; ++j) dst[j * 64 + lane] = expf(cur[j] - mx);  // expf(-inf) = +0 pads
#pragma unroll
            for (int j = 0; j < kSampPer; ++j) cur[j] = nxt[j];
        }
        if (w == 0 && lane == 0 && it > 0) {
            const int blk = it - 1;
            sum = samp_chain(sh[blk & 1], (min(kSampBlk, V - blk * kSampBlk) + 63) / 64, sum);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) s_red[0] = sum;
    if (threadIdx.x == 0) s_found = -1;
    __syncthreads();
    sum = s_red[0];
    // pass 2: coin; cdf += expf(x - maxval) / sum; if (coin < cdf) return i
    // (the exps recomputed: expf is deterministic)
    unsigned long long st = state[b];
    const float coin = (xorshift_u32(st) >> 8) / 16777216.0f;
    int pick = V - 1;
    float cdf = 0.f;
    if (w == 1) samp_load(lg, V, 0, lane, cur);
    for (int it = 0; it <= nblk; ++it) {
        if (w == 1 && it < nblk) {
            if (it + 1 < nblk) samp_load(lg, V, (it + 1) * kSampBlk, lane, nxt);
            float* dst = sh[it & 1];
#pragma unroll
            for (int j = 0; j < kSampPer; ++j) dst[j * 64 + lane] = expf(cur[j] - mx) / sum;
#pragma unroll
            for (int j = 0; j < kSampPer; ++j) cur[j] = nxt[j];
        }
        if (w == 0 && lane == 0 && it > 0) {
            const int blk = it - 1;
            const int n = min(kSampBlk, V - blk * kSampBlk);
            const float* buf = sh[blk & 1];
            for (int q0 = 0; q0 < n; q0 += 64) {
                // cdf is non-decreasing: test once per 64 values, and replay
                // the batch that crosses the coin from its start with the
                // per-element test (same additions, same roundings)
                const float4* s4 = reinterpret_cast<const float4*>(buf + q0);
                float4 r[16];
#pragma unroll
                for (int q = 0; q < 16; ++q) r[q] = s4[q];
                const float c0 = cdf;
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    cdf += r[q].x;
                    cdf += r[q].y;
                    cdf += r[q].z;
                    cdf += r[q].w;
                }
                if (coin < cdf) {
                    float c = c0;
                    int k = q0;
                    for (; k < q0 + 63; ++k) {
                        c += buf[k];
                        if (coin < c) break;
                    }
                    s_found = min(blk * kSampBlk + k, V - 1);
                    break;
                }
            }
        }
        __syncthreads();
        if (s_found >= 0) {
            pick = s_found;
            break;
        }
    }
    if (threadIdx.x == 0) {
        state[b] = st;
        next[b] = pick;
        if (tokens) tokens[b] = pick;
        if (pos) pos[b] += 1;
    }
}

// ---------------------------------------------------- order-exact scan sampling
// The same draw as sample_final_kernel (bit-equal sum, cdf and pick), without
// the serial chain.  While the running fp32 sum S stays in one binade
// [2^e, 2^(e+1)) (or below 2^-125, where the grid is the denormal one), every
// fl(S + a) equals S + RN_u(a), with u = ulp(S) and RN_u rounding a term onto
// the multiples of u.  The ordered sum is then an integer prefix sum of
// k_i = RN_u(a_i) / u, which is associative and runs as a block scan.  A term
// breaks the segment when its rounding is a tie (the result's parity decides
// it), when it is too large for the grid, or when the sum leaves the binade;
// that one addition is done in fp32 on the exact S before it, and the scan
// resumes with the new grid.  Breaks are rare past the first chunk (which one
// lane sums in order, ss_serial): about one per binade of the sum
// plus ties, whose odds fall as 1/i.  (softmax_forward :259-286, sample_mult
// :837-848 order.)
// 16 waves x 4 terms per 4096-term chunk (measured per launch at B = 64,
// V = 50257: 16 x 4 251 us with __syncthreads, 4 x 4 295 us, 4 x 16 668 us):
// a round's latency is set by the per-thread serial work and the barriers,
// so many threads with few terms each and few rounds per pass win
constexpr int kSsThreads = 1024, kSsPer = 4, kSsChunk = kSsThreads * kSsPer;
constexpr unsigned kSsSat = 1u << 30;  // saturation of the integer prefix
constexpr int kSsNone = 0x7fffffff;

struct SsShared {
    unsigned tot[kSsThreads / 64];
    int jmin[kSsThreads / 64];
    int fmin[kSsThreads / 64];
    float red[kSsThreads / 64];
    float S;
    int found;
    __attribute__((aligned(16))) float buf[kSsChunk];  // the first chunk's terms for the serial lane
};

// workgroup barrier that orders LDS only: the next chunk's global loads stay
// in flight across it (__syncthreads would wait for them)
__device__ __forceinline__ void ss_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ unsigned ss_add(unsigned a, unsigned b) { return min(a + b, kSsSat); }

// x >= 0 as M * 2^E (M with the hidden bit; E of the denormal grid below 2^-126)
__device__ __forceinline__ void ss_split(float x, unsigned& M, int& E) {
    const unsigned bits = __float_as_uint(x), e8 = bits >> 23;
    M = (bits & 0x7fffffu) | (e8 ? 0x800000u : 0u);
    E = (int)max(e8, 1u) - 150;
}

// a rounded to the multiples of 2^gexp, in units of 2^gexp; brk on a tie or a
// term of 2^8 units or more (it leaves the binade anyway)
__device__ __forceinline__ unsigned ss_quant(float a, int gexp, bool& brk) {
    unsigned M;
    int E;
    ss_split(a, M, E);
    if (M == 0) return 0;
    const int s = E - gexp;
    if (s >= 0) {
        if (s >= 8) {
            brk = true;
            return 0;
        }
        return M << s;
    }
    const int sh = -s;
    if (sh >= 25) return 0;  // a < u/2
    const unsigned half = 1u << (sh - 1), r = M & ((1u << sh) - 1u);
    unsigned k = M >> sh;
    if (r > half) k += 1;
    else if (r == half) brk = true;
    return k;
}

// the first lane's value among lanes with v != kSsNone (lanes run in index
// order, so this is the wave's minimum index): a ballot and a scalar read
__device__ __forceinline__ int ss_wave_first(int v) {
    const unsigned long long bal = __ballot(v != kSsNone);
    return bal ? __builtin_amdgcn_readlane(v, __ffsll((long long)bal) - 1) : kSsNone;
}

// inclusive saturating wave64 scan on DPP (row_shr 1/2/4/8, row_bcast 15/31):
// VALU lane moves, no LDS round trips
template <int CTRL, int ROWS>
__device__ __forceinline__ unsigned ss_dpp(unsigned v) {
    return (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWS, 0xf, false);
}
__device__ __forceinline__ unsigned ss_wave_scan(unsigned v) {
    v = ss_add(v, ss_dpp<0x111, 0xf>(v));
    v = ss_add(v, ss_dpp<0x112, 0xf>(v));
    v = ss_add(v, ss_dpp<0x114, 0xf>(v));
    v = ss_add(v, ss_dpp<0x118, 0xf>(v));
    v = ss_add(v, ss_dpp<0x142, 0xa>(v));
    v = ss_add(v, ss_dpp<0x143, 0xc>(v));
    return v;
}

// One chunk of kSsChunk terms a[] (thread t holds terms 4t..4t+3) added to S
// in index order.  CDF: also stop at the first term whose running sum exceeds
// coin (returns true, pick = its index).  Uniform over the block.
template <bool CDF>
__device__ bool ss_chunk(const float (&a)[kSsPer], int base, int n, float coin, float& S, int& pick, SsShared& sh) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    int start = 0;
    while (start < n) {
        unsigned M;
        int gexp;
        ss_split(S, M, gexp);
        unsigned inc[kSsPer];
        bool brk[kSsPer];
        unsigned run = 0;
#pragma unroll
        for (int j = 0; j < kSsPer; ++j) {
            const int l = t * kSsPer + j;
            brk[j] = false;
            const unsigned k = l >= start ? ss_quant(a[j], gexp, brk[j]) : 0u;
            run = ss_add(run, k);
            inc[j] = run;
        }
        const unsigned wsc = ss_wave_scan(run);                  // inclusive over the wave's threads
        unsigned pre = ss_dpp<0x138, 0xf>(wsc);                    // wave_shr:1 -> exclusive (lane 0: 0)
        if (lane == 63) sh.tot[w] = wsc;
        ss_sync();
        unsigned tv[kSsThreads / 64];
#pragma unroll
        for (int v = 0; v < kSsThreads / 64; ++v) tv[v] = sh.tot[v];
#pragma unroll
        for (int v = 0; v < kSsThreads / 64; ++v) pre = ss_add(pre, v < w ? tv[v] : 0u);
        int myj = kSsNone, myf = kSsNone;
#pragma unroll
        for (int j = kSsPer - 1; j >= 0; --j) {
            const int l = t * kSsPer + j;
            if (l < start) continue;
            const unsigned P = M + ss_add(pre, inc[j]);  // < 2^31
            if (brk[j] || P >= (1u << 24)) myj = l;
            else if (CDF && l < n && coin < ldexpf((float)P, gexp)) myf = l;
        }
        myj = ss_wave_first(myj);
        myf = ss_wave_first(myf);
        if (lane == 0) {
            sh.jmin[w] = myj;
            sh.fmin[w] = myf;
        }
        ss_sync();
        int jb = kSsNone, fb = kSsNone;
#pragma unroll
        for (int v = 0; v < kSsThreads / 64; ++v) {
            jb = min(jb, sh.jmin[v]);
            fb = min(fb, sh.fmin[v]);
        }
        if (CDF && fb < jb) {  // the cdf crossed the coin inside the exact run
            pick = base + fb;
            return true;
        }
        const int last = jb == kSsNone ? n - 1 : jb;
        if (t == last / kSsPer) {
            const int j = last % kSsPer;
            if (jb == kSsNone) {
                sh.S = ldexpf((float)(M + ss_add(pre, inc[j])), gexp);
                sh.found = 0;
            } else {  // the breaking term: one fp32 addition on the exact sum before it
                const unsigned Pb = M + (j ? ss_add(pre, inc[j - 1]) : pre);
                const float Sn = ldexpf((float)Pb, gexp) + a[j];
                sh.S = Sn;
                sh.found = CDF && coin < Sn;
            }
        }
        ss_sync();
        S = sh.S;
        if (CDF && sh.found) {
            pick = base + jb;
            return true;
        }
        start = last + 1;
    }
    return false;
}

// The first chunk holds most breaks (tie odds fall as 1/i, the sum crosses
// binades at i ~ 2^k), so one lane adds it in order, as the serial kernel
// does (64 adds per cdf test, the crossing batch replayed).
template <bool CDF>
__device__ bool ss_serial(const float (&a)[kSsPer], int n, float coin, float& S, int& pick, SsShared& sh) {
    const int t = threadIdx.x;
#pragma unroll
    for (int j = 0; j < kSsPer; ++j) sh.buf[t * kSsPer + j] = a[j];  // +0 beyond n
    ss_sync();
    if (t == 0) {
        float s = S;
        int f = -1;
        if (!CDF) s = samp_chain(sh.buf, (n + 63) / 64, s);
        else
            for (int q0 = 0; q0 < n; q0 += 64) {
                const float c0 = s;
                s = samp_chain(sh.buf + q0, 1, s);
                if (coin < s) {
                    float c = c0;
                    int k = q0;
                    for (; k < q0 + 63; ++k) {
                        c += sh.buf[k];
                        if (coin < c) break;
                    }
                    f = k;
                    break;
                }
            }
        sh.S = s;
        sh.found = f;
    }
    ss_sync();
    S = sh.S;
    if (CDF && sh.found >= 0) {
        pick = sh.found;
        return true;
    }
    return false;
}

__device__ __forceinline__ void ss_load(const float* lg, int V, int base, float (&x)[kSsPer]) {
#pragma unroll
    for (int j = 0; j < kSsPer; ++j) {
        const int i = base + threadIdx.x * kSsPer + j;
        x[j] = i < V ? lg[i] : 0.f;
    }
}

__global__ __launch_bounds__(kSsThreads) void sample_scan_kernel(const float* __restrict__ logits, int V,
                                                                 unsigned long long* __restrict__ state,
                                                                 int* __restrict__ next, int* __restrict__ tokens,
                                                                 int* __restrict__ pos, const int* __restrict__ active) {
    __shared__ SsShared sh;
    const int b = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6;
    if (active && active[b] <= 0) return;  // row left as it is (its RNG state too)
    const float* lg = logits + (size_t)b * V;
    float mx = -10000.0f;  // maxval as the reference (exact in any order)
    for (int i = t; i < V; i += kSsThreads) mx = fmaxf(mx, lg[i]);
    mx = hpa::wave_max(mx);
    if (lane == 0) sh.red[w] = mx;
    __syncthreads();
#pragma unroll
    for (int v = 0; v < kSsThreads / 64; ++v) mx = fmaxf(mx, sh.red[v]);
    float a[kSsPer];
    int pick = -1;
    // pass 1: sum += expf(x - maxval)
    float S = 0.f, x[kSsPer];
    ss_load(lg, V, 0, x);
    for (int base = 0; base < V; base += kSsChunk) {
#pragma unroll
        for (int j = 0; j < kSsPer; ++j) a[j] = base + t * kSsPer + j < V ? expf(x[j] - mx) : 0.f;
        ss_load(lg, V, base + kSsChunk, x);  // next chunk in flight during this one's scan
        if (base == 0) ss_serial<false>(a, min(kSsChunk, V), 0.f, S, pick, sh);
        else ss_chunk<false>(a, base, min(kSsChunk, V - base), 0.f, S, pick, sh);
    }
    const float sum = S;
    // pass 2: cdf += expf(x - maxval) / sum; first i with coin < cdf
    unsigned long long st = state[b];
    const float coin = (xorshift_u32(st) >> 8) / 16777216.0f;
    S = 0.f;
    ss_load(lg, V, 0, x);
    for (int base = 0; base < V; base += kSsChunk) {
#pragma unroll
        for (int j = 0; j < kSsPer; ++j) a[j] = base + t * kSsPer + j < V ? expf(x[j] - mx) / sum : 0.f;
        ss_load(lg, V, base + kSsChunk, x);
        if (base == 0 ? ss_serial<true>(a, min(kSsChunk, V), coin, S, pick, sh)
                      : ss_chunk<true>(a, base, min(kSsChunk, V - base), coin, S, pick, sh))
            break;
    }
    if (pick < 0) pick = V - 1;  // sample_mult's "rounding errors" return
    if (t == 0) {
        state[b] = st;
        next[b] = pick;
        if (tokens) tokens[b] = pick;
        if (pos) pos[b] += 1;
    }
}

inline dim3 xcd_grid(FG& p, int gx, int gy) {
    p.gx = gx;
    p.gy = gy;
    return dim3((unsigned)(((gx + 7) / 8) * 8 * gy));
}

template <int NW, int MT, int NTW = 1>
int launch16(FG p, int epi) {
    dim3 grid = xcd_grid(p, (p.ntn + NTW - 1) / NTW, p.Mp / 16 / MT), block(NW * 64);
    switch (epi) {
        case HPA_FEPI_QKV: gemm16_kernel<NW, HPA_FEPI_QKV, MT, NTW><<<grid, block, 0, hpa_stream()>>>(p); break;
        case HPA_FEPI_RESID: gemm16_kernel<NW, HPA_FEPI_RESID, MT, NTW><<<grid, block, 0, hpa_stream()>>>(p); break;
        case HPA_FEPI_GELU: gemm16_kernel<NW, HPA_FEPI_GELU, MT, NTW><<<grid, block, 0, hpa_stream()>>>(p); break;
        case HPA_FEPI_LOGITS: gemm16_kernel<NW, HPA_FEPI_LOGITS, MT, NTW><<<grid, block, 0, hpa_stream()>>>(p); break;
        default: return hpa_fail(__FILE__, __LINE__, "gemm_fused: unknown epilogue");
    }
    HPA_LAUNCH_CHECK();
    return 0;
}

template <int NW, int S, bool NT>
int launch16_os_nt(const FG& p, int epi, dim3 grid, dim3 block) {
    switch (epi) {
        case HPA_FEPI_QKV: gemm16_os_kernel<NW, HPA_FEPI_QKV, S, NT><<<grid, block, 0, hpa_stream()>>>(p); break;
        case HPA_FEPI_RESID: gemm16_os_kernel<NW, HPA_FEPI_RESID, S, NT><<<grid, block, 0, hpa_stream()>>>(p); break;
        case HPA_FEPI_GELU: gemm16_os_kernel<NW, HPA_FEPI_GELU, S, NT><<<grid, block, 0, hpa_stream()>>>(p); break;
        case HPA_FEPI_LOGITS: gemm16_os_kernel<NW, HPA_FEPI_LOGITS, S, NT><<<grid, block, 0, hpa_stream()>>>(p); break;
        default: return hpa_fail(__FILE__, __LINE__, "gemm_fused: unknown epilogue");
    }
    HPA_LAUNCH_CHECK();
    return 0;
}

// weights non-temporal where each tile has one reader (one 16-row block)
template <int NW, int S>
int launch16_os(FG p, int epi) {
    dim3 grid = xcd_grid(p, p.ntn, p.Mp / 16), block(NW * 64);
    return p.Mp == 16 ? launch16_os_nt<NW, S, true>(p, epi, grid, block)
                      : launch16_os_nt<NW, S, false>(p, epi, grid, block);
}

// one-shot instances: (NW, S) with K16 = NW * S for K = 768 (K16 = 48) and 3072 (192)
int launch_os(const FG& p, int epi, int nw) {
    const int S = p.K16 / nw;
    if (p.K16 % nw) return -1;
    switch (nw * 100 + S) {
        case 4 * 100 + 12: return launch16_os<4, 12>(p, epi);
        case 8 * 100 + 6: return launch16_os<8, 6>(p, epi);
        case 16 * 100 + 3: return launch16_os<16, 3>(p, epi);
        case 8 * 100 + 24: return launch16_os<8, 24>(p, epi);
        case 16 * 100 + 12: return launch16_os<16, 12>(p, epi);
        case 10 * 100 + 10: return launch16_os<10, 10>(p, epi);  // GPT-2 XL (K = 1600)
        default: return -1;
    }
}

// multi-column-tile instances: (waves, row_blocks, col_tiles) in
// {(4|8, 4, 2), (4|8, 2, 2), (4, 4, 4)} -- the rest exceed LDS or registers
template <int NW>
int launch16_mt(const FG& p, int epi, int mt, int ntw) {
    if constexpr (NW <= 8) {
        if (ntw == 2 && mt == 4) return launch16<NW, 4, 2>(p, epi);
        if (ntw == 2 && mt == 2) return launch16<NW, 2, 2>(p, epi);
    }
    if constexpr (NW == 4) {
        if (ntw == 4 && mt == 4) return launch16<NW, 4, 4>(p, epi);
    }
    if (ntw != 1)
        return hpa_fail(__FILE__, __LINE__,
                        "gemm_fused: col_tiles 2 needs waves 4/8 and row_blocks 2/4; 4 needs waves 4, row_blocks 4");
    switch (mt) {
        case 1: return launch16<NW, 1>(p, epi);
        case 2: return launch16<NW, 2>(p, epi);
        case 4: return launch16<NW, 4>(p, epi);
        default: return hpa_fail(__FILE__, __LINE__, "gemm_fused: row_blocks must be 1, 2 or 4");
    }
}

}  // namespace

extern "C" {

size_t hpa_frag_elems(int rows, int K) { return (size_t)((rows + 15) / 16) * 16 * (size_t)K; }

int hpa_pack_frag(const float* src, int rows, int K, int ld, float* dst) {
    HPA_REQUIRE(src && dst && rows > 0 && K > 0 && K % 16 == 0 && ld >= K && ld % 4 == 0,
                "pack_frag: bad shape (K % 16, ld % 4)");
    const size_t n4 = hpa_frag_elems(rows, K) / 4;
    pack_frag_kernel<<<(unsigned)((n4 + 255) / 256), 256, 0, hpa_stream()>>>(
        src, rows, K, ld, reinterpret_cast<float4*>(dst), n4);
    HPA_LAUNCH_CHECK();
    return 0;
}

int hpa_ln_fold_pack(const float* W, int N, int K, const float* ln_w, const float* ln_b, const float* bias,
                     float* dst_frag, float* c1, float* c2) {
    HPA_REQUIRE(W && ln_w && ln_b && dst_frag && c1 && c2 && N > 0 && K > 0 && K % 16 == 0,
                "ln_fold_pack: bad arguments (K % 16)");
    float* tmp = nullptr;
    HPA_CHECK(hipMalloc(&tmp, (size_t)N * K * sizeof(float)));
    ln_fold_kernel<<<N, 64, 0, hpa_stream()>>>(W, K, ln_w, ln_b, bias, tmp, c1, c2);
    int rc = hipGetLastError() != hipSuccess ? hpa_fail(__FILE__, __LINE__, "ln_fold_kernel launch") : 0;
    if (!rc) rc = hpa_pack_frag(tmp, N, K, K, dst_frag);
    const hipError_t e = hipStreamSynchronize(hpa_stream());
    (void)hipFree(tmp);
    if (!rc && e != hipSuccess) rc = hpa_fail(__FILE__, __LINE__, hipGetErrorString(e));
    return rc;
}

int hpa_unpack_frag(const float* src, int rows, int K, float* dst, int ld) {
    HPA_REQUIRE(src && dst && rows > 0 && K > 0 && K % 16 == 0 && ld >= K && ld % 4 == 0,
                "unpack_frag: bad shape");
    const size_t n4 = hpa_frag_elems(rows, K) / 4;
    unpack_frag_kernel<<<(unsigned)((n4 + 255) / 256), 256, 0, hpa_stream()>>>(
        reinterpret_cast<const float4*>(src), rows, K, dst, ld, n4);
    HPA_LAUNCH_CHECK();
    return 0;
}

// launch shape by GEMM shape: one 16-row block per workgroup for the layer
// GEMMs (spreads the fp32 MFMA work over >= 4 * N/16 workgroups), four for
// logits (3142 column tiles already fill the chip; amortises the A reads);
// waves sharing the K range: enough k-steps per wave to amortise the fold
void hpa_fused_pick(int M, int N, int K, int* out3) {
    (void)M;  // never by M: a row's summation order must not depend on the batch
    const int ntn = (N + 15) / 16;
    const int k16 = K / 16;
    if (ntn >= 1024) {  // logits (profiles/r1/gemm_tune_b64_*.log)
        out3[0] = 4;
        out3[1] = 2;
        out3[2] = 2;
    } else if (ntn >= 256 && k16 >= 96) {  // GPT-2 XL qkv / fc: MFMA-bound, reuse A over 2 tiles
        out3[0] = 8;
        out3[1] = 4;
        out3[2] = 2;
    } else if (ntn >= 96 && k16 >= 96) {  // GPT-2 XL attproj / fcproj (round 2 sweep: 4 waves
        out3[0] = 4;                        // 8.8 / 23.4 us vs 9.4 / 24.5 at 8, profiles/r2/gemm_tune_xl.log)
        out3[1] = 2;
        out3[2] = 1;
    } else {  // GPT-2 124M layer GEMMs: one row block per workgroup (one-shot where K allows)
        out3[0] = k16 >= 96 ? 8 : 4;
        out3[1] = 1;
        out3[2] = 1;
    }
}

// bf16 weights (profiles/r1/gemm_tune_bf16_b256.log, _b64.log; bf16 MFMA is
// 16x the fp32 rate, so operand delivery bounds these GEMMs):
//  * A-resident kernel (variant 5) for the logits at every M and for the
//    K = 768 / N >= 2304 GEMMs (qkv, fc) from M > 112: the looped kernel
//    re-reads and re-normalises the fp32 A rows per column-tile group
//    (B = 256 logits 184 -> 56 us, qkv 15.8 -> 10.8, fc 16.1 -> 11.2);
//  * looped kernel otherwise (8 waves, 2 row blocks x 2 column tiles;
//    1 x 1 for the N <= 1024 GEMMs at M <= 112).
// A row's summation order follows the kernel (one k chain per wave in
// variant 5, 8 wave ranges folded in order in the looped one), so in bf16
// mode it may depend on M; both are held to the oracle's bf16 bound.
// A-resident shape: out3 = {waves, row_blocks, rounds}; returns 1 where
// variant 0 uses it.
int hpa_fused_pick_bf16_ares(int M, int N, int K, int* out3) {
    const int ntn = (N + 15) / 16;
    const int big = (M + 15) / 16 >= 8;
    out3[0] = 8;
    out3[1] = K <= 768 ? (big && ntn >= 1024 ? 4 : 2) : K <= 1600 ? 2 : 1;
    out3[2] = 0;  // rounds: auto (one pass of workgroups over the CUs, hpa_gemm_bf16.hip)
    if (K > 3200) return 0;
    return ntn >= 1024 || (big && ntn >= 144);
}

void hpa_fused_pick_bf16(int M, int N, int K, int* out3) {
    (void)K;
    const int small = (M + 15) / 16 < 8 && N <= 1024;
    out3[0] = 8;
    out3[1] = small ? 1 : 2;
    out3[2] = small ? 1 : 2;
}

int hpa_fused_pick_waves(int M, int N, int K) {
    int p[3];
    hpa_fused_pick(M, N, K, p);
    return p[0];
}

// the looped kernel's launch shape for g (as hpa_gemm_fused resolves it)
static void looped_shape(const HpaFusedGemm* g, int Mp, int* nw, int* mt, int* ntw) {
    int pick[3];
    hpa_fused_pick(g->M, g->N, g->K, pick);
    *nw = g->waves ? g->waves : pick[0];
    *mt = g->row_blocks ? g->row_blocks : pick[1];
    while (*mt > 1 && (Mp / 16) % *mt) *mt >>= 1;  // row blocks of this M
    *ntw = g->col_tiles ? g->col_tiles : pick[2];
    // a launch-shape hint: where this M's row blocks (or the waves) cannot
    // carry it, fall back to one column tile (results are identical)
    if ((*ntw == 2 && (*mt == 1 || *nw == 16)) || (*ntw == 4 && (*mt != 4 || *nw != 4))) *ntw = 1;
}

static int gemm_fused_launch(const HpaFusedGemm* g, FG& p);

// the resident logits kernel takes the final pick into its launch (its last
// workgroup reduces the partials); any other LOGITS path picks afterwards with
// hpa_argmax_final, so pick_next means the same on every path
int hpa_gemm_fused(const HpaFusedGemm* g) {
    FG p;
    if (fused_prepare(g, &p)) return 1;
    const bool pick = g->pick_next != nullptr;
    HPA_REQUIRE(!pick || (g->epilogue == HPA_FEPI_LOGITS && g->part_out), "gemm_fused: pick_next needs a LOGITS GEMM");
    const bool fused = pick && g->pick_count && g->w_dtype == HPA_F32 && g->variant == 4 &&
                       logits_resident_eligible(p, g->epilogue) && logits_resident_grid(p) <= 256;
    if (!fused) p.pick_next = p.pick_tokens = p.pick_pos = p.pick_count = nullptr;
    const int rc = gemm_fused_launch(g, p);
    if (rc || !pick || fused) return rc;
    const int npart = hpa_logits_partials(g);
    HPA_REQUIRE(npart > 0, "gemm_fused: logits partials");
    return hpa_argmax_final(p.part_out, npart, p.Mp, p.M, g->pick_next, g->pick_tokens, g->pick_pos, nullptr);
}

static int gemm_fused_launch(const HpaFusedGemm* g, FG& p) {
    int nw, mt, ntw;
    if (g->w_dtype == HPA_BF16) {  // bf16 weights: hpa_gemm_bf16.hip
        HPA_REQUIRE(g->K % 32 == 0 && !g->ln_fold_c1 &&
                        (g->variant == 0 || g->variant == 4 || g->variant == 5 || g->variant == 1),
                    "gemm_fused bf16: K % 32, no ln_fold_c1, variant 0/1/5");
        int pk[3];
        // A/B builds: HPA_BF16_ARES=0 = no A-resident default (variant 5 still honoured)
#ifdef HPA_AB
        static const int ares_default = [] {
            const char* e = getenv("HPA_BF16_ARES");
            return !(e && e[0] == '0');
        }();
#else
        constexpr int ares_default = 1;
#endif
        if (g->variant == 5 ||
            (g->variant != 1 && ares_default && hpa_fused_pick_bf16_ares(g->M, g->N, g->K, pk))) {
            if (g->variant == 5) hpa_fused_pick_bf16_ares(g->M, g->N, g->K, pk);
            nw = g->waves ? g->waves : pk[0];
            mt = g->row_blocks ? g->row_blocks : pk[1];
            while (mt > 1 && ((p.Mp / 16) % mt || mt * g->K > 3200 || (mt == 4 && g->K > 768))) mt >>= 1;
            return launch_b16_ares(p, g->epilogue, nw, mt, g->col_tiles ? g->col_tiles : pk[2]);
        }
        hpa_fused_pick_bf16(g->M, g->N, g->K, pk);
        nw = g->waves ? g->waves : pk[0];
        mt = g->row_blocks ? g->row_blocks : pk[1];
        ntw = g->col_tiles ? g->col_tiles : pk[2];
        while (mt > 1 && (p.Mp / 16) % mt) mt >>= 1;  // row blocks of this M
        if (ntw == 2 && mt == 1) ntw = 1;
        return launch_b16(p, g->epilogue, nw, mt, ntw);
    }
    HPA_REQUIRE(g->w_dtype == HPA_F32, "gemm_fused: w_dtype must be HPA_F32 or HPA_BF16");
    if (g->variant == 6) return launch_sk(p, g->epilogue);  // stream-K (hpa_gemm_sk.hip)
    HPA_REQUIRE(g->row_blocks == 0 || g->row_blocks == 1 || g->row_blocks == 2 || g->row_blocks == 4,
                "gemm_fused: row_blocks must be 1, 2 or 4");
    looped_shape(g, p.Mp, &nw, &mt, &ntw);
    HPA_REQUIRE(g->variant >= 0 && g->variant <= 4, "gemm_fused: variant must be 0, 1, 2, 3 or 4");
    if (g->variant == 3)  // loader / MFMA-wave ring (hpa_gemm_ring.hip); waves = K parts
        return launch_ring(p, g->epilogue, g->waves > 0 ? g->waves : 1);
    // (waves 16 / 12: the resident kernel's 16-wave or ring form; else by M)
    if (g->variant == 4 && logits_resident_eligible(p, g->epilogue)) return launch_logits_resident(p, g->waves);
    // variant 4 elsewhere (GPT-2 XL logits, K = 1600): stream-K when the caller
    // gave its workspace (120 vs 143 us at M = 64, profiles/r2/sk_tune_xl.txt)
    if (g->variant == 4 && g->epilogue == HPA_FEPI_LOGITS && p.sk_slab && p.sk_cnt && sk_eligible(p.Mp, p.ntn, p.K16))
        return launch_sk(p, g->epilogue);  // else the looped kernel below
    HPA_REQUIRE(g->col_tiles == 0 || g->col_tiles == 1 || g->col_tiles == 2 || g->col_tiles == 4,
                "gemm_fused: col_tiles must be 1, 2 or 4");
    if (g->variant == 2 || (g->variant == 0 && mt == 1 && p.ntn < 1024 && g->col_tiles <= 1)) {
        const int rc = launch_os(p, g->epilogue, nw);
        if (rc >= 0) return rc;
        HPA_REQUIRE(g->variant == 0, "gemm_fused: one-shot needs (waves, K/16) in {(4,48), (8,48), (16,48), (8,192), (16,192), (10,100)}");
    }
    switch (nw) {
        case 4: return launch16_mt<4>(p, g->epilogue, mt, ntw);
        case 8: return launch16_mt<8>(p, g->epilogue, mt, ntw);
        case 16:
            HPA_REQUIRE(ntw == 1, "gemm_fused: col_tiles > 1 needs waves 4 or 8");
            return launch16_mt<16>(p, g->epilogue, mt, ntw);
        default: return hpa_fail(__FILE__, __LINE__, "gemm_fused: waves must be 4, 8 or 16");
    }
}

int hpa_logits_kernel(int M, int N, int K) {
    if (M <= 0 || N <= 0 || K <= 0 || K % 16) return -1;
    const int Mp = (M + 15) / 16 * 16, K16 = K / 16, ntn = (N + 15) / 16;
    FG p;
    memset(&p, 0, sizeof(p));
    p.M = M;
    p.Mp = Mp;
    p.K = K;
    p.K16 = K16;
    p.N = N;
    p.ntn = ntn;
    p.ln_stats = reinterpret_cast<const float*>(16);  // "LN present": only its presence is read
    p.ln_ntiles = K16;                                 // the engine's statistics: one per 16 columns
    if (logits_resident_eligible(p, HPA_FEPI_LOGITS)) return 4;
    return sk_eligible(Mp, ntn, K16) ? 6 : 1;
}

int hpa_logits_partials(const HpaFusedGemm* g) {
    FG p;
    if (!g || g->epilogue != HPA_FEPI_LOGITS || fused_prepare(g, &p)) return -1;
    if (g->w_dtype == HPA_F32 && g->variant == 4 && logits_resident_eligible(p, g->epilogue))
        return logits_resident_grid(p);
    return p.ntn;  // one partial per 16-column tile
}

int hpa_embed_frag(const int* tokens, const int* pos, const float* wte, const float* wpe,
                   float* res_frag, float* stats, int B, int C) {
    HPA_REQUIRE(B > 0 && C > 0 && C % 16 == 0, "embed_frag: bad shape");
    embed_frag_kernel<<<B, 256, 0, hpa_stream()>>>(tokens, pos, wte, wpe, res_frag, stats, C, nullptr, 0);
    HPA_LAUNCH_CHECK();
    return 0;
}

int hpa_embed_frag_zero(const int* tokens, const int* pos, const float* wte, const float* wpe, float* res_frag,
                        float* stats, int B, int C, void* zero, size_t zero_bytes) {
    HPA_REQUIRE(B > 0 && C > 0 && C % 16 == 0, "embed_frag_zero: bad shape");
    HPA_REQUIRE(zero_bytes % 16 == 0 && zero_bytes / 16 <= 0x7fffffff && ((size_t)zero & 15) == 0,
                "embed_frag_zero: the zeroed block must be whole 16-byte granules");
    embed_frag_kernel<<<B, 256, 0, hpa_stream()>>>(tokens, pos, wte, wpe, res_frag, stats, C,
                                                   reinterpret_cast<int4*>(zero), (int)(zero_bytes / 16));
    HPA_LAUNCH_CHECK();
    return 0;
}

int hpa_sample_final(const float* logits, int B, int V, unsigned long long* state, int* next, int* tokens,
                     int* pos, const int* active) {
    HPA_REQUIRE(logits && state && next && B > 0 && V > 0, "sample_final: bad arguments");
    sample_scan_kernel<<<B, kSsThreads, 0, hpa_stream()>>>(logits, V, state, next, tokens, pos, active);
    HPA_LAUNCH_CHECK();
    return 0;
}

int hpa_sample_final_serial(const float* logits, int B, int V, unsigned long long* state, int* next, int* tokens,
                            int* pos, const int* active) {
    HPA_REQUIRE(logits && state && next && B > 0 && V > 0, "sample_final_serial: bad arguments");
    sample_final_kernel<<<B, 128, 0, hpa_stream()>>>(logits, V, state, next, tokens, pos, active);
    HPA_LAUNCH_CHECK();
    return 0;
}

int hpa_argmax_final(const float* part, int ntiles, int Mp, int B, int* next, int* tokens, int* pos,
                     const int* active) {
    HPA_REQUIRE(part && next && B > 0 && ntiles > 0 && Mp >= B, "argmax_final: bad arguments");
    argmax_final_kernel<<<B, 256, 0, hpa_stream()>>>(part, ntiles, Mp, next, tokens, pos, active);
    HPA_LAUNCH_CHECK();
    return 0;
}

}  // extern "C"
