// hpa_gemm_body.h -- the fused decode GEMM workgroup bodies (see
// hpa_fused.hip for the design notes), shared by the fp32 launchers
// (hpa_fused.hip), the bf16-weight kernels (hpa_gemm_bf16.hip) and the
// resident logits kernel (hpa_logits.hip).
#pragma once
#include <math.h>

#include "hpa_internal.h"

namespace hpa_gemm {

typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int HPA_FUSED_LN_KMAX = 2048;  // LN'ed A operands: K <= 2048 (GPT-2 C <= 1600)

struct FG {
    const float* x;
    int M, Mp, K, K16;
    const float* ln_stats;
    int ln_ntiles;
    const float* ln_w;
    const float* ln_b;
    const float* w;
    int N, ntn;
    const float* bias;
    float* out;
    const float* res_in;
    float* stats_out;
    float* part_out;
    float* kv_base;  // layer base of the KV pool (bf16 pools: reinterpreted)
    int kv_bf16;
    size_t page_elems;
    int NH, P;
    const int* bt;
    int bt_stride;
    const int* pos;
    const int* row_seq;  // QKV: block-table row per GEMM row; LOGITS: output row per GEMM row (NULL: the row)
    const float* fold_c1;  // LN folded into w: out = rstd*(acc - mean*c1) + bias (bias = c2)
    int gx, gy;  // column-tile groups x row groups of the launch
    float* sk_slab;  // stream-K (variant 6): [workgroup][2][super-tile] partials
    int* sk_cnt;     // stream-K: [super-tile] arrival counters (zero between launches)
    int* pick_next;  // resident logits: the last workgroup's final pick (HpaFusedGemm.pick_*)
    int* pick_tokens;
    int* pick_pos;
    int* pick_count;
};

// XCD-aware workgroup order (MI355X_MICROARCH.md "Workgroup dispatch":
// blocks b and b+8 share an XCD -- used for L2 affinity only).  The 1-D grid
// of ceil(gx/8)*8*gy blocks is dealt so that the gy row groups of one column
// group run back to back on ONE XCD: its weight tile is fetched from HBM once
// and re-read from that XCD's L2.  Returns false for the padding blocks.
__device__ __forceinline__ bool xcd_tile(const FG& p, int bid, int& cx, int& ry) {
    const int xg = bid & 7;
    const int s = bid >> 3;
    const int q = s / p.gy;
    ry = s - q * p.gy;
    cx = q * 8 + xg;
    return cx < p.gx;
}

__device__ __forceinline__ float4 ln4(float4 a, float mu, float rs, float4 g, float4 b) {
    // paged_infer.c:80-81: n = s * (x - m); o = n * w + b
    a.x = (rs * (a.x - mu)) * g.x + b.x;
    a.y = (rs * (a.y - mu)) * g.y + b.y;
    a.z = (rs * (a.z - mu)) * g.z + b.z;
    a.w = (rs * (a.w - mu)) * g.w + b.w;
    return a;
}

// ---- folded LayerNorm: row statistics from the A fragments themselves ----
// (no statistics loads: measured, they cost more than the operand loads they
// precede).  A lane holds 4 consecutive k of row (lane & 15) per k-step; the
// per-lane sums run over the wave's k-steps in order, then the 4 lanes of a
// row combine (xor 16, xor 32: the same value on all four), then the waves in
// wave order in the epilogue -- the same order in every body and launch shape.
__device__ __forceinline__ void row_sums_add(float4 x, float& s1, float& s2) {
    s1 = (((s1 + x.x) + x.y) + x.z) + x.w;
    s2 = __fmaf_rn(x.w, x.w, __fmaf_rn(x.z, x.z, __fmaf_rn(x.y, x.y, __fmaf_rn(x.x, x.x, s2))));
}
// lanes 0..15 store the wave's (sum, sum of squares) of rows row_base + lane
__device__ __forceinline__ void row_sums_publish(float s1, float s2, float* wsum_wave_rows) {
    const int lane = threadIdx.x & 63;
    s1 += __shfl_xor(s1, 16, 64);
    s2 += __shfl_xor(s2, 16, 64);
    s1 += __shfl_xor(s1, 32, 64);
    s2 += __shfl_xor(s2, 32, 64);
    if (lane < 16) {
        wsum_wave_rows[2 * lane] = s1;
        wsum_wave_rows[2 * lane + 1] = s2;
    }
}

// ---- shared epilogue ---------------------------------------------------
// A workgroup's output is NTW 16-column tiles x MT 16-row blocks.  Element e
// (0 .. NTW*MT*256-1): column tile j = e / (MT*256); within it e' = e % (MT*256):
// rb = e'>>8, reg = (e'>>6)&3, l = e'&63 -> row rb*16 + (l>>4)*4 + reg,
// col l&15 (16x16 C/D map: col = lane & 15, row = 4*(lane >> 4) + reg).
// Thread t owns e = t + i*NT.  Accumulator acc[j*MT + r] holds (tile j, block r).
template <int NW, int EPI, int MT, int NTW = 1>
struct Epi {
    static constexpr int NT = NW * 64;
    static constexpr int R = MT * 16;
    static constexpr int TE = MT * 256;                    // elements per column tile
    static constexpr int EPT = (NTW * TE + NT - 1) / NT;   // elements per thread
    float pre_bias[EPT], pre_res[EPT], pre_c1[EPT];

    __device__ __forceinline__ static void where(int e, int nt0, int row0, int& j, int& lrow, int& lcol,
                                                 int& row, int& col) {
        j = e / TE;
        const int e2 = e - j * TE;
        const int l = e2 & 63;
        lrow = (e2 >> 8) * 16 + (l >> 4) * 4 + ((e2 >> 6) & 3);
        lcol = l & 15;
        row = row0 + lrow;
        col = (nt0 + j) * 16 + lcol;
    }

    // bias / residual operands of the owned elements: issued early so their
    // latency hides under the main loop
    __device__ __forceinline__ void prefetch(const FG& p, int nt0, int row0) {
#pragma unroll
        for (int i = 0; i < EPT; ++i) {
            const int e = threadIdx.x + i * NT;
            int j, lrow, lcol, row, col;
            where(e, nt0, row0, j, lrow, lcol, row, col);
            const bool in = e < NTW * TE;
            pre_bias[i] = (EPI != HPA_FEPI_LOGITS && in && p.bias && col < p.N) ? p.bias[col] : 0.f;
            pre_res[i] = 0.f;
            pre_c1[i] = (EPI != HPA_FEPI_LOGITS && in && p.fold_c1 && col < p.N) ? p.fold_c1[col] : 0.f;
            if (EPI == HPA_FEPI_RESID && in && row < p.M && col < p.N)
                pre_res[i] = p.res_in[hpa::frag_index(row, col, p.N)];
        }
    }

    // fold the waves' accumulators through LDS (fixed order) and apply the
    // epilogue; wsum = the waves' row partial statistics [NW][R][2] in LDS,
    // read when p.fold_c1 (LN folded into w; written before the fold's barrier)
    __device__ __forceinline__ void finish(const FG& p, const f32x4* acc, float* red, float* tile, int nt0,
                                           int row0, const float* wsum) {
        const int lane = threadIdx.x & 63;
        const int w = threadIdx.x >> 6;
#pragma unroll
        for (int j = 0; j < NTW; ++j)
#pragma unroll
            for (int r = 0; r < MT; ++r)
#pragma unroll
                for (int g = 0; g < 4; ++g)
                    red[w * NTW * TE + j * TE + (r * 4 + g) * 64 + lane] = acc[j * MT + r][g];
        __syncthreads();

        float vals[EPT];
#pragma unroll
        for (int i = 0; i < EPT; ++i) {
            const int e = threadIdx.x + i * NT;
            float val = 0.f;
            if (e < NTW * TE) {
                val = red[e];
#pragma unroll
                for (int ww = 1; ww < NW; ++ww) val += red[ww * NTW * TE + e];
            }
            vals[i] = val;
        }
        apply(p, vals, tile, nt0, row0, wsum);
    }

    // the epilogue proper on the folded values of the owned elements (vals[i]
    // = element threadIdx.x + i*NT); tile = LDS scratch for the row statistics
    __device__ __forceinline__ void apply(const FG& p, const float* vals, float* tile, int nt0, int row0,
                                          const float* wsum) {
        const bool rowstat = EPI == HPA_FEPI_LOGITS || (EPI == HPA_FEPI_RESID && p.stats_out);  // uniform
#pragma unroll
        for (int i = 0; i < EPT; ++i) {
            const int e = threadIdx.x + i * NT;
            if (e < NTW * TE) {
                float val = vals[i];
                int j, lrow, lcol, row, col;
                where(e, nt0, row0, j, lrow, lcol, row, col);
                const bool live = row < p.M && col < p.N;
                if (EPI != HPA_FEPI_LOGITS && p.fold_c1) {  // sum_k LN(x)_k W_nk = rstd*(sum_k x_k W'_nk - mean*c1_n)
                    float S1 = wsum[2 * lrow], S2 = wsum[2 * lrow + 1];
#pragma unroll
                    for (int ww = 1; ww < NW; ++ww) {
                        S1 += wsum[(ww * R + lrow) * 2];
                        S2 += wsum[(ww * R + lrow) * 2 + 1];
                    }
                    const float m = S1 / p.K;  // layernorm_forward statistics, one-pass form
                    const float rstd = 1.0f / sqrtf(fmaxf(S2 / p.K - m * m, 0.f) + 1e-5f);
                    val = rstd * (val - m * pre_c1[i]);
                }
                val += pre_bias[i];
                if (EPI == HPA_FEPI_QKV) {
                    if (live) {
                        const int C = p.N / 3;
                        if (col < C) {
                            p.out[(size_t)row * C + col] = val;
                        } else {
                            const int kv = col >= 2 * C;
                            const int c = col - (kv ? 2 * C : C);
                            const int hh = c >> 6, d = c & 63;
                            const int ps = p.pos[row];
                            const int seq = p.row_seq ? p.row_seq[row] : row;
                            const int page = p.bt[(size_t)seq * p.bt_stride + ps / p.P];
                            if (page < 0) continue;  // no page (host bug): never write below the pool
                            const int slot = ps % p.P;
                            const size_t toff = (size_t)page * p.page_elems + ((size_t)kv * p.NH + hh) * p.P * 64;
                            if (p.kv_bf16) {  // bf16 pool: K [chunk of 8][slot][8], V [slot][64], RNE
                                unsigned short* kvt = reinterpret_cast<unsigned short*>(p.kv_base) + toff;
                                kvt[kv == 0 ? ((d >> 3) * p.P + slot) * 8 + (d & 7) : slot * 64 + d] =
                                    hpa::f32_to_bf16(val);
                            } else {
                                float* kvt = p.kv_base + toff;
                                if (kv == 0)
                                    kvt[((d >> 2) * p.P + slot) * 4 + (d & 3)] = val;  // K: [chunk][slot][4]
                                else
                                    kvt[slot * 64 + d] = val;  // V: [slot][64]
                            }
                        }
                    }
                } else if (EPI == HPA_FEPI_GELU) {
                    if (row < p.Mp && col < p.N)
                        p.out[hpa::frag_index(row, col, p.N)] = live ? hpa::gelu_ref(val) : 0.f;
                } else if (EPI == HPA_FEPI_RESID) {
                    val = live ? pre_res[i] + val : 0.f;  // residual_forward(out, res, proj)
                    if (row < p.Mp && col < p.N) p.out[hpa::frag_index(row, col, p.N)] = val;
                    tile[(j * R + lrow) * 17 + lcol] = val;
                } else {  // LOGITS (row_seq: the output row of each GEMM row)
                    if (live) p.out[(size_t)(p.row_seq ? p.row_seq[row] : row) * p.N + col] = val;
                    tile[(j * R + lrow) * 17 + lcol] = live ? val : -INFINITY;
                }
            }
        }
        if (rowstat) {
            __syncthreads();
            for (int t = threadIdx.x; t < NTW * R; t += NT) {
                const int j = t / R, lr = t - j * R;
                const int row = row0 + lr, nt = nt0 + j;
                const float* tr = tile + t * 17;
                if (row < p.Mp && nt < p.ntn) {
                    if (EPI == HPA_FEPI_RESID) {
                        float s1 = 0.f, s2 = 0.f;
#pragma unroll
                        for (int c = 0; c < 16; ++c) {
                            s1 += tr[c];
                            s2 += tr[c] * tr[c];
                        }
                        p.stats_out[((size_t)nt * p.Mp + row) * 2] = s1;
                        p.stats_out[((size_t)nt * p.Mp + row) * 2 + 1] = s2;
                    } else {
                        float bv = tr[0];
                        int bi = 0;
#pragma unroll
                        for (int c = 1; c < 16; ++c)
                            if (tr[c] > bv) {  // first max wins (paged_infer.c:937-951)
                                bv = tr[c];
                                bi = c;
                            }
                        p.part_out[((size_t)nt * p.Mp + row) * 2] = bv;
                        p.part_out[((size_t)nt * p.Mp + row) * 2 + 1] = __int_as_float(nt * 16 + bi);
                    }
                }
            }
        }
    }
};

// ---- LayerNorm prologue: the LN weight / bias of K into LDS (lngb) and the
// mean / rstd of the workgroup's R = 16*MT rows from the producer's 16-column
// partial sums (4 threads per row, partials summed in tile order); lane l gets
// the statistics of row (l & 15) of each row block.  Every thread calls it.
template <int NW, int MT>
__device__ __forceinline__ void ln_prologue(const FG& p, float* lngb, float* lnst, float* lnscr, int row0,
                                            bool ln_apply, float* mu, float* rs) {
    constexpr int NT = NW * 64;
    constexpr int R = MT * 16;
    const int lane = threadIdx.x & 63;
    for (int i = threadIdx.x; ln_apply && i < p.K / 4; i += NT) {
        reinterpret_cast<float4*>(lngb)[i] = reinterpret_cast<const float4*>(p.ln_w)[i];
        reinterpret_cast<float4*>(lngb + HPA_FUSED_LN_KMAX)[i] = reinterpret_cast<const float4*>(p.ln_b)[i];
    }
    if (threadIdx.x < 4 * R) {
        const int r = threadIdx.x >> 2, q = threadIdx.x & 3;
        const int row = row0 + r;
        float s1 = 0.f, s2 = 0.f;
        if (row < p.M) {
            for (int t0 = q; t0 < p.ln_ntiles; t0 += 32) {
                float a[8], b[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int t = min(t0 + 4 * j, p.ln_ntiles - 1);
                    a[j] = p.ln_stats[((size_t)t * p.Mp + row) * 2];
                    b[j] = p.ln_stats[((size_t)t * p.Mp + row) * 2 + 1];
                }
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    if (t0 + 4 * j < p.ln_ntiles) {
                        s1 += a[j];
                        s2 += b[j];
                    }
            }
        }
        lnscr[2 * threadIdx.x] = s1;
        lnscr[2 * threadIdx.x + 1] = s2;
    }
    __syncthreads();
    if (threadIdx.x < R) {
        const float* t = lnscr + 8 * threadIdx.x;
        const float s1 = (t[0] + t[2]) + (t[4] + t[6]);
        const float s2 = (t[1] + t[3]) + (t[5] + t[7]);
        const float m = s1 / p.K;
        const float v = fmaxf(s2 / p.K - m * m, 0.f);
        lnst[2 * threadIdx.x] = m;
        lnst[2 * threadIdx.x + 1] = 1.0f / sqrtf(v + 1e-5f);
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < MT; ++r) {
        mu[r] = lnst[2 * (16 * r + (lane & 15))];
        rs[r] = lnst[2 * (16 * r + (lane & 15)) + 1];
    }
}

// MT = 16-row blocks per workgroup (1, 2 or 4), NTW = 16-column tiles per
// workgroup (every wave computes all of them over its K range), NW = waves
// sharing the K range.  Grid (ceil(ntn/NTW), Mp/16/MT).  MT = 1 spreads the
// MFMA work of a 64-row GEMM over 4x the workgroups -- the per-CU fp32 MFMA
// rate, not bandwidth, bounds these GEMMs when only N/16 CUs are busy.  NTW > 1
// (logits) reuses every activation fragment for NTW weight fragments: with
// NTW = 1 a k-step loads 5 KiB for 16 MFMAs, more than the CU's L2->L1 port
// feeds at three waves per SIMD.
// LDS floats of one looped-GEMM workgroup
template <int NW, int MT, int NTW>
constexpr int gemm16_lds_floats() {
    return 2 * HPA_FUSED_LN_KMAX + NW * MT * NTW * 256 + NTW * MT * 16 * 17 + 10 * MT * 16;
}

// body of the looped GEMM workgroup `bid` of the XCD-ordered 1-D grid
// (gemm16_kernel, and the GEMM role of the pipelined combo launches)
template <int NW, int EPI, int MT, int NTW>
__device__ __forceinline__ void gemm16_body(const FG& p, int bid, float* smem) {
    constexpr int R = MT * 16;  // rows per workgroup
    // k-steps per trip (two trips in flight; register budget)
    constexpr int U = NTW > 1 ? 1 : (NW >= 16 ? (MT == 4 ? 1 : 2) : (MT == 4 ? 2 : 4));
    float* lngb = smem;                              // LN weight [K], bias [K]
    float* red = smem + 2 * HPA_FUSED_LN_KMAX;       // [NW][NTW][MT rb x 4 reg][64 lanes]
    float* tile = red + NW * MT * NTW * 256;         // [NTW][R rows][17]
    float* lnst = tile + NTW * R * 17;               // [R][2] mean, rstd
    float* lnscr = lnst + 2 * R;                     // [4R][2]

    int cx, ry;
    if (!xcd_tile(p, bid, cx, ry)) return;
    const int lane = threadIdx.x & 63;
    // uniform wave index: the step bounds below live in SGPRs and every
    // per-step test is a scalar branch (with a VGPR index the compiler made
    // them divergent and waited for loads at each join)
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nt0 = cx * NTW;
    const int rb0 = ry * MT;
    const int row0 = rb0 * 16;
    const int q4 = lane >> 4;  // which 4-k group of the 16-k step

    // ---- this wave's contiguous k-step range
    const int per = (p.K16 + NW - 1) / NW;
    const int kb0 = w * per;
    const int nsteps = max(0, min(p.K16, kb0 + per) - kb0);
    const float4* __restrict__ wf[NTW];
#pragma unroll
    for (int j = 0; j < NTW; ++j)  // tail tiles past ntn re-read the last tile (never stored)
        wf[j] = reinterpret_cast<const float4*>(p.w) + (size_t)min(nt0 + j, p.ntn - 1) * p.K16 * 64 + lane;
    const float4* __restrict__ xf = reinterpret_cast<const float4*>(p.x) + (size_t)rb0 * p.K16 * 64 + lane;
    const size_t rbs = (size_t)p.K16 * 64;  // float4 stride between row blocks
    const bool ln_apply = p.ln_stats != nullptr && !p.fold_c1;  // folded LN: raw A, statistics in the epilogue
    const bool use_ln = ln_apply;
    const float4* sg = reinterpret_cast<const float4*>(lngb) + q4;
    const float4* sb = reinterpret_cast<const float4*>(lngb + HPA_FUSED_LN_KMAX) + q4;

    struct Buf {
        float4 w[U][NTW], x[U][MT];
    };
    Buf A, Bb;
    auto load = [&](Buf& f, int t) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int k = kb0 + min(t * U + u, max(nsteps - 1, 0));  // clamped, unconditional
#pragma unroll
            for (int j = 0; j < NTW; ++j) f.w[u][j] = wf[j][(size_t)k * 64];
#pragma unroll
            for (int r = 0; r < MT; ++r) f.x[u][r] = xf[r * rbs + (size_t)k * 64];
        }
    };
    const int trips = (nsteps + U - 1) / U;
    if (trips > 0) load(A, 0);  // first operands in flight during the LN prologue

    // ---- LayerNorm statistics of this workgroup's R rows (4 threads per row)
    float mu[MT], rs[MT];
#pragma unroll
    for (int r = 0; r < MT; ++r) mu[r] = rs[r] = 0.f;
    if (use_ln) ln_prologue<NW, MT>(p, lngb, lnst, lnscr, row0, ln_apply, mu, rs);

    // one accumulator chain per (column tile, row block): a row's summation
    // order depends only on NW (the per-wave K ranges), never on MT, NTW or M
    // -- results are bit-identical across launch shapes and micro-batch lanes.
    // The dependent MFMA latency is covered by the other chains / waves.
    f32x4 acc[MT * NTW];
#pragma unroll
    for (int i = 0; i < MT * NTW; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    const bool fold = p.fold_c1 != nullptr;  // row statistics from the A fragments (row_sums_add)
    float fs1[MT], fs2[MT];
#pragma unroll
    for (int r = 0; r < MT; ++r) fs1[r] = fs2[r] = 0.f;
    auto comp = [&](Buf& f, int t) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (t * U + u < nsteps) {
                float4 xa[MT];
                float4 g, b;
                if (ln_apply) {
                    const int k = kb0 + t * U + u;
                    g = sg[4 * k];
                    b = sb[4 * k];
                }
#pragma unroll
                for (int r = 0; r < MT; ++r) {
                    xa[r] = f.x[u][r];
                    if (fold) row_sums_add(xa[r], fs1[r], fs2[r]);
                    if (ln_apply) xa[r] = ln4(xa[r], mu[r], rs[r], g, b);
                }
#pragma unroll
                for (int q = 0; q < 4; ++q)
#pragma unroll
                    for (int j = 0; j < NTW; ++j)
#pragma unroll
                        for (int r = 0; r < MT; ++r) {
                            const float xs = q == 0 ? xa[r].x : q == 1 ? xa[r].y : q == 2 ? xa[r].z : xa[r].w;
                            const float4 wv = f.w[u][j];
                            const float ws = q == 0 ? wv.x : q == 1 ? wv.y : q == 2 ? wv.z : wv.w;
                            acc[j * MT + r] = __builtin_amdgcn_mfma_f32_16x16x4f32(xs, ws, acc[j * MT + r], 0, 0, 0);
                        }
            }
        }
    };
    // loads are unconditional (a trip past the end re-reads the last step's
    // fragments, never used): a load under a branch left its buffer to be
    // copied at the join, i.e. waited for in the same trip
    // no exit between the two halves: a mid-loop exit edge reaches the loop
    // header with the second buffer's loads still pending, and the waitcnt
    // pass then drains every load (vmcnt(0)) before each trip's issue; an odd
    // trip count runs one empty half instead (comp skips steps >= nsteps)
    for (int t = 0; t < trips; t += 2) {
        load(Bb, t + 1);
        comp(A, t);
        load(A, t + 2);
        comp(Bb, t + 1);
    }

    if (fold)  // [NW][R][2] over the LN weight area (unused when folded)
#pragma unroll
        for (int r = 0; r < MT; ++r) row_sums_publish(fs1[r], fs2[r], lngb + (w * R + 16 * r) * 2);
    Epi<NW, EPI, MT, NTW> epi;
    epi.prefetch(p, nt0, row0);
    epi.finish(p, acc, red, tile, nt0, row0, lngb);
}

template <int NW, int EPI, int MT, int NTW>
__global__ __launch_bounds__(NW * 64) void gemm16_kernel(FG p) {
    __shared__ __attribute__((aligned(16))) float smem[gemm16_lds_floats<NW, MT, NTW>()];
    gemm16_body<NW, EPI, MT, NTW>(p, blockIdx.x, smem);
}

// One-shot variant for the layer GEMMs (one 16-row block per workgroup,
// K16 = NW * S): every k-step operand of the wave -- S weight fragments and S
// activation fragments, 2 KiB per step -- is issued up front together with
// the LayerNorm statistics and the epilogue's bias/residual, so the kernel
// pays ONE dependent memory round trip instead of one per trip.  These GEMMs
// run <= 2 waves per SIMD, so the registers are there.
template <int NW>
constexpr int gemm16_os_lds_floats() {
    return 2 * HPA_FUSED_LN_KMAX + NW * 256 + 16 * 17 + 2 * 16;
}

// WNT: the weight loads non-temporal -- where every weight tile is read by ONE
// workgroup (a single 16-row block, B <= 16: MI355X_MICROARCH.md nt-weights;
// B = 8 decode step 0.522 -> 0.506 ms); with several row blocks the tile is
// re-read from L2 by its row-block neighbours and the default policy is faster
template <int NW, int EPI, int S, bool WNT = false>
__device__ __forceinline__ void gemm16_os_body(const FG& p, int bid, float* smem) {
    constexpr int NT = NW * 64;
    float* lngb = smem;                         // LN weight [K], bias [K]
    float* red = smem + 2 * HPA_FUSED_LN_KMAX;  // [NW][4 reg][64 lanes]
    float* tile = red + NW * 256;               // [16 rows][17]
    float* lnst = tile + 16 * 17;               // [16][2] mean, rstd

    int nt, ry;
    if (!xcd_tile(p, bid, nt, ry)) return;
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const int row0 = ry * 16;
    const int q4 = lane >> 4;
    const bool fold = p.fold_c1 != nullptr;  // LN folded into w: row sums from xv
    const bool ln_apply = p.ln_stats != nullptr && !fold;

    // 1. LN statistics partials of the 16 rows: 4 threads per row, issued first
    constexpr int SPT = 12;  // partial tiles per thread: ln_ntiles <= 48 (C <= 768); else looped
    float s1 = 0.f, s2 = 0.f;
    float sa[SPT], sb[SPT];
    const int srow = row0 + (threadIdx.x >> 2), sq = threadIdx.x & 3;
    const bool stat_thread = ln_apply && threadIdx.x < 64 && srow < p.M;
    if (stat_thread) {
#pragma unroll
        for (int j = 0; j < SPT; ++j) {
            const int t = min(sq + 4 * j, p.ln_ntiles - 1);
            sa[j] = p.ln_stats[((size_t)t * p.Mp + srow) * 2];
            sb[j] = p.ln_stats[((size_t)t * p.Mp + srow) * 2 + 1];
        }
    }
    // 2. LN weight / bias -> registers (stored to LDS below)
    float4 lw4 = make_float4(0.f, 0.f, 0.f, 0.f), lb4 = lw4;
    const int K4 = p.K / 4;
    if (ln_apply && (int)threadIdx.x < K4) {
        lw4 = reinterpret_cast<const float4*>(p.ln_w)[threadIdx.x];
        lb4 = reinterpret_cast<const float4*>(p.ln_b)[threadIdx.x];
    }
    // 3. all operand fragments of this wave's k range [w*S, w*S+S)
    const float4* __restrict__ wf = reinterpret_cast<const float4*>(p.w) + ((size_t)nt * p.K16 + w * S) * 64 + lane;
    const float4* __restrict__ xf = reinterpret_cast<const float4*>(p.x) + ((size_t)ry * p.K16 + w * S) * 64 + lane;
    // issued strictly in k-step order (a scheduling barrier per step): the
    // chain below then waits for each step's pair with a descending vmcnt and
    // the MFMAs of early steps overlap the arrival of later ones (left to
    // itself the scheduler grouped the loads by base register, and step 4
    // waited for nearly every load of the wave)
    float4 wv[S], xv[S];
#pragma unroll
    for (int s = 0; s < S; ++s) {
        if (WNT) {  // compile-time
            const f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(wf + s * 64));
            wv[s] = make_float4(v.x, v.y, v.z, v.w);
        } else {
            wv[s] = wf[s * 64];
        }
        xv[s] = xf[s * 64];
        __builtin_amdgcn_sched_barrier(0);
    }
    // 4. epilogue operands
    Epi<NW, EPI, 1, 1> epi;
    epi.prefetch(p, nt, row0);

    // LN: reduce the statistics (waits only for the loads of step 1) into
    // lnst; the 4 threads of a row are adjacent lanes of wave 0
    auto reduce_stats = [&]() {
        if (stat_thread) {
#pragma unroll
            for (int j = 0; j < SPT; ++j)
                if (sq + 4 * j < p.ln_ntiles) {
                    s1 += sa[j];
                    s2 += sb[j];
                }
            for (int t0 = sq + 4 * SPT; t0 < p.ln_ntiles; t0 += 4) {  // wider C
                s1 += p.ln_stats[((size_t)t0 * p.Mp + srow) * 2];
                s2 += p.ln_stats[((size_t)t0 * p.Mp + srow) * 2 + 1];
            }
        }
        // 4 threads of a row are adjacent lanes of wave 0: combine in a fixed order
        if (threadIdx.x < 64) {
            const float a1 = __shfl_xor(s1, 1, 64), a2 = __shfl_xor(s2, 1, 64);
            const float t1 = (sq & 1) ? a1 + s1 : s1 + a1;
            const float t2 = (sq & 1) ? a2 + s2 : s2 + a2;
            const float b1 = __shfl_xor(t1, 2, 64), b2 = __shfl_xor(t2, 2, 64);
            const float S1 = (sq & 2) ? b1 + t1 : t1 + b1;
            const float S2 = (sq & 2) ? b2 + t2 : t2 + b2;
            if (sq == 0) {
                const float m = S1 / p.K;
                const float v = fmaxf(S2 / p.K - m * m, 0.f);
                lnst[2 * (threadIdx.x >> 2)] = m;
                lnst[2 * (threadIdx.x >> 2) + 1] = 1.0f / sqrtf(v + 1e-5f);
            }
        }
    };
    float mu = 0.f, rs = 0.f;
    if (ln_apply) {
        reduce_stats();
        if ((int)threadIdx.x < K4) {
            reinterpret_cast<float4*>(lngb)[threadIdx.x] = lw4;
            reinterpret_cast<float4*>(lngb + HPA_FUSED_LN_KMAX)[threadIdx.x] = lb4;
        }
        for (int i = threadIdx.x + NT; i < K4; i += NT) {  // K > 4*NT
            reinterpret_cast<float4*>(lngb)[i] = reinterpret_cast<const float4*>(p.ln_w)[i];
            reinterpret_cast<float4*>(lngb + HPA_FUSED_LN_KMAX)[i] = reinterpret_cast<const float4*>(p.ln_b)[i];
        }
        __syncthreads();
        mu = lnst[2 * (lane & 15)];
        rs = lnst[2 * (lane & 15) + 1];
    }

    // one accumulator chain: the same k order as gemm16_kernel with NW waves
    f32x4 acc[1];
    acc[0] = f32x4{0.f, 0.f, 0.f, 0.f};
    const float4* sg = reinterpret_cast<const float4*>(lngb) + q4;
    const float4* sbv = reinterpret_cast<const float4*>(lngb + HPA_FUSED_LN_KMAX) + q4;
#pragma unroll
    for (int s = 0; s < S; ++s) {
        float4 xa = xv[s];
        if (ln_apply) xa = ln4(xa, mu, rs, sg[4 * (w * S + s)], sbv[4 * (w * S + s)]);
        acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa.x, wv[s].x, acc[0], 0, 0, 0);
        acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa.y, wv[s].y, acc[0], 0, 0, 0);
        acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa.z, wv[s].z, acc[0], 0, 0, 0);
        acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa.w, wv[s].w, acc[0], 0, 0, 0);
    }
    if (fold) {  // published by the fold's barrier in finish(): [NW][16][2] over the LN weight area
        float fs1 = 0.f, fs2 = 0.f;
#pragma unroll
        for (int s = 0; s < S; ++s) row_sums_add(xv[s], fs1, fs2);
        row_sums_publish(fs1, fs2, lngb + w * 32);
    }
    epi.finish(p, acc, red, tile, nt, row0, lngb);
}

template <int NW, int EPI, int S, bool WNT>
__global__ __launch_bounds__(NW * 64) void gemm16_os_kernel(FG p) {
    __shared__ __attribute__((aligned(16))) float smem[gemm16_os_lds_floats<NW>()];
    gemm16_os_body<NW, EPI, S, WNT>(p, blockIdx.x, smem);
}


// validate a HpaFusedGemm and build the kernel argument block (gx/gy are
// set by the launcher); nonzero (with hpa_last_error) on a bad description
// the activation-resident logits kernel (hpa_logits.hip, variant 4)
bool logits_resident_eligible(const FG& p, int epi);
int launch_logits_resident(const FG& p, int form);  // form: 16 / 12 (ring) / 0 by rows
int logits_resident_grid(const FG& p);  // workgroups = argmax partials per row it writes

// bf16-weight GEMM launch (hpa_gemm_bf16.hip): waves 4/8, (row_blocks,
// col_tiles) in {(1,1), (2,1), (4,1), (2,2), (4,2)}
int launch_b16(const FG& p, int epi, int nw, int mt, int ntw);
// A-resident bf16 variant (variant 5): waves 4/8, row_blocks (mt) 1/2/4 with
// mt*K <= 3200; each workgroup takes waves*rounds column tiles
int launch_b16_ares(const FG& p, int epi, int nw, int mt, int rounds);
// loader / MFMA-wave ring kernel (hpa_gemm_ring.hip, variant 3): <= 64
// padded rows, LN folded or absent, QKV / GELU / RESID; parts = K parts
// (> 1: sk_slab / sk_cnt workspace, hpa_gemm_ring_workspace)
bool ring_eligible(const FG& p, int epi);
int launch_ring(const FG& p, int epi, int parts);
// stream-K fp32 kernel (hpa_gemm_sk.hip, variant 6): M <= 64
int launch_sk(const FG& p, int epi);
bool sk_eligible(int Mp, int ntn, int K16);

static inline int fused_prepare(const HpaFusedGemm* g, FG* p) {
    HPA_REQUIRE(g && g->x && g->w && g->out, "gemm_fused: null operand");
    HPA_REQUIRE(g->M > 0 && g->N > 0 && g->K > 0 && g->K % 16 == 0, "gemm_fused: K % 16 != 0");
    HPA_REQUIRE(!g->ln_stats || (g->ln_w && g->ln_b && g->ln_ntiles > 0), "gemm_fused: LN params");
    HPA_REQUIRE(!g->ln_stats || g->K <= HPA_FUSED_LN_KMAX, "gemm_fused: LN over K > 2048");
    p->x = g->x;
    p->M = g->M;
    p->Mp = (g->M + 15) / 16 * 16;
    p->K = g->K;
    p->K16 = g->K / 16;
    p->ln_stats = g->ln_stats;
    p->ln_ntiles = g->ln_ntiles;
    p->ln_w = g->ln_w;
    p->ln_b = g->ln_b;
    p->w = g->w;
    p->N = g->N;
    p->ntn = (g->N + 15) / 16;
    p->bias = g->bias;
    p->out = g->out;
    p->res_in = g->res_in;
    p->stats_out = g->stats_out;
    p->part_out = g->part_out;
    p->kv_base = nullptr;
    p->kv_bf16 = 0;
    p->page_elems = 0;
    p->NH = 0;
    p->P = 1;
    p->bt = g->block_table;
    p->bt_stride = g->bt_stride;
    p->pos = g->pos;
    p->row_seq = g->row_seq;
    p->fold_c1 = g->ln_fold_c1;
    p->sk_slab = g->sk_slab;
    p->sk_cnt = g->sk_count;
    p->pick_next = g->pick_next;
    p->pick_tokens = g->pick_tokens;
    p->pick_pos = g->pick_pos;
    p->pick_count = g->pick_count;
    HPA_REQUIRE(!g->ln_fold_c1 || g->epilogue != HPA_FEPI_LOGITS, "gemm_fused: ln_fold_c1 with LOGITS");
    if (g->epilogue == HPA_FEPI_QKV) {
        const HpaKVPool* pool = g->pool;
        HPA_REQUIRE(pool && pool->base && (pool->dtype == HPA_F32 || pool->dtype == HPA_BF16) &&
                        pool->head_size == 64,
                    "gemm_fused QKV: fp32/bf16 pool with head_size 64");
        HPA_REQUIRE(g->N == 3 * pool->num_heads * 64, "gemm_fused QKV: N != 3*C");
        HPA_REQUIRE(g->layer >= 0 && g->layer < pool->num_layers, "gemm_fused QKV: layer");
        HPA_REQUIRE(g->block_table && g->pos, "gemm_fused QKV: block table / positions");
        p->kv_base = (float*)((char*)pool->base + (size_t)g->layer * pool->layer_elems * pool->elem_bytes);
        p->kv_bf16 = pool->dtype == HPA_BF16;
        p->page_elems = pool->page_elems;
        p->NH = pool->num_heads;
        p->P = pool->page_size;
    }
    if (g->epilogue == HPA_FEPI_RESID) HPA_REQUIRE(g->res_in, "gemm_fused RESID: res_in");
    if (g->epilogue == HPA_FEPI_LOGITS) HPA_REQUIRE(g->part_out, "gemm_fused LOGITS: part_out");
    p->gx = p->gy = 0;
    return 0;
}

}  // namespace hpa_gemm
