// hpa_compat.hip -- reference-layout, reference-order kernels behind the
// drop-in paged_infer.c API (attention_paged, matmul_forward, matmul_cached,
// layernorm_forward, encoder_forward, gelu_forward, residual_forward,
// softmax_forward).  They keep the reference's page layout (token-major
// [block_size][C] pages, block_manager.c:145-146) and its sequential
// arithmetic with no FMA contraction (__fmul_rn/__fadd_rn), so a caller that
// swaps the reference functions for these gets the reference's numbers
// (bit-identical up to expf/tanhf ulps), computed on the GPU.  They are the
// compatibility surface, not the decode hot path (that is hpa_attn.hip /
// hpa_gemm.hip / hpa_rows.hip).
#include "hpa_internal.h"

// The reference is built without FMA contraction (x86-64 SSE: separate
// mul and add); keep every product and sum separately rounded here too.
#pragma clang fp contract(off)

namespace {

// one thread per (b, t, h): the 4 passes of paged_infer.c:186-236
__global__ void ref_attention_paged_kernel(float* __restrict__ out, float* __restrict__ preatt,
                                           float* __restrict__ att, const float* __restrict__ inp,
                                           float* const* __restrict__ kb, float* const* __restrict__ vb,
                                           int B, int T, int C, int NH, int offset, int bs) {
    const int id = blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= B * T * NH) return;
    const int h = id % NH;
    const int t = (id / NH) % T;
    const int b = id / (NH * T);
    const int C3 = 3 * C, hs = C / NH;
    const float scale = (float)(1.0 / (double)sqrtf((float)hs));
    const float* q = inp + (size_t)b * T * C3 + (size_t)t * C3 + h * hs;
    float* pre = preatt + (size_t)b * NH * T * T + (size_t)h * T * T + (size_t)t * T;
    float* a = att + (size_t)b * NH * T * T + (size_t)h * T * T + (size_t)t * T;
    float maxval = -10000.0f;
    for (int t2 = 0; t2 <= t; t2++) {
        const int p = t2 + offset;
        const float* k = kb[p / bs] + (size_t)(p % bs) * C + h * hs;
        float val = 0.0f;
        for (int i = 0; i < hs; i++) val = __fadd_rn(val, __fmul_rn(q[i], k[i]));
        val = __fmul_rn(val, scale);
        if (val > maxval) maxval = val;
        pre[t2] = val;
    }
    float expsum = 0.0f;
    for (int t2 = 0; t2 <= t; t2++) {
        const float e = expf(__fsub_rn(pre[t2], maxval));
        expsum = __fadd_rn(expsum, e);
        a[t2] = e;
    }
    const float inv = expsum == 0.0f ? 0.0f : __fdiv_rn(1.0f, expsum);
    for (int t2 = 0; t2 < T; t2++) a[t2] = t2 <= t ? __fmul_rn(a[t2], inv) : 0.0f;
    float* o = out + (size_t)b * T * C + (size_t)t * C + h * hs;
    for (int i = 0; i < hs; i++) o[i] = 0.0f;
    for (int t2 = 0; t2 <= t; t2++) {
        const int p = t2 + offset;
        const float* v = vb[p / bs] + (size_t)(p % bs) * C + h * hs;
        const float w = a[t2];
        for (int i = 0; i < hs; i++) o[i] = __fadd_rn(o[i], __fmul_rn(w, v[i]));
    }
}

// one thread per (row, o): paged_infer.c:92-114 / :117-160
__global__ void ref_matmul_kernel(float* __restrict__ out, const float* __restrict__ inp,
                                  const float* __restrict__ w, const float* __restrict__ bias, int B,
                                  int T, int C, int OC, int cached) {
    const size_t id = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= (size_t)B * T * OC) return;
    const int o = (int)(id % OC);
    const size_t r = id / OC;
    const int t = (int)(r % T);
    if (cached && t < T - 1 && o >= C) return;  // matmul_cached: K/V only for the last row
    const float* x = inp + r * C;
    const float* wr = w + (size_t)o * C;
    float val = bias ? bias[o] : 0.0f;
    for (int i = 0; i < C; i++) val = __fadd_rn(val, __fmul_rn(x[i], wr[i]));
    out[r * OC + o] = val;
}

// one thread per row: paged_infer.c:49-89
__global__ void ref_layernorm_kernel(float* __restrict__ out, float* __restrict__ mean,
                                     float* __restrict__ rstd, const float* __restrict__ inp,
                                     const float* __restrict__ w, const float* __restrict__ bb, int N,
                                     int C) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= N) return;
    const float* x = inp + (size_t)r * C;
    float m = 0.0f;
    for (int i = 0; i < C; i++) m = __fadd_rn(m, x[i]);
    m = __fdiv_rn(m, (float)C);
    float v = 0.0f;
    for (int i = 0; i < C; i++) {
        const float d = __fsub_rn(x[i], m);
        v = __fadd_rn(v, __fmul_rn(d, d));
    }
    v = __fdiv_rn(v, (float)C);
    const float s = __fdiv_rn(1.0f, sqrtf(__fadd_rn(v, 1e-5f)));
    float* o = out + (size_t)r * C;
    for (int i = 0; i < C; i++) {
        const float n = __fmul_rn(s, __fsub_rn(x[i], m));
        o[i] = __fadd_rn(__fmul_rn(n, w[i]), bb[i]);
    }
    if (mean) mean[r] = m;
    if (rstd) rstd[r] = s;
}

// paged_infer.c:24-47 (wpe row t + pos_offset)
__global__ void ref_encoder_kernel(float* __restrict__ out, const int* __restrict__ inp,
                                   const float* __restrict__ wte, const float* __restrict__ wpe, int B,
                                   int T, int C, int pos_offset) {
    const size_t id = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= (size_t)B * T * C) return;
    const int i = (int)(id % C);
    const size_t bt = id / C;
    const int t = (int)(bt % T);
    out[id] = __fadd_rn(wte[(size_t)inp[bt] * C + i], wpe[(size_t)(t + pos_offset) * C + i]);
}

__global__ void ref_gelu_kernel(float* __restrict__ out, const float* __restrict__ inp, int N) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < N) out[i] = hpa::gelu_ref(inp[i]);
}

__global__ void ref_residual_kernel(float* out, const float* a, const float* b, int N) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < N) out[i] = __fadd_rn(a[i], b[i]);
}

// one thread per row: paged_infer.c:259-286
__global__ void ref_softmax_kernel(float* __restrict__ probs, const float* __restrict__ logits, int N,
                                   int V) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= N) return;
    const float* l = logits + (size_t)r * V;
    float* p = probs + (size_t)r * V;
    float maxval = -10000.0f;
    for (int i = 0; i < V; i++)
        if (l[i] > maxval) maxval = l[i];
    float sum = 0.0f;
    for (int i = 0; i < V; i++) {
        p[i] = expf(__fsub_rn(l[i], maxval));
        sum = __fadd_rn(sum, p[i]);
    }
    for (int i = 0; i < V; i++) p[i] = __fdiv_rn(p[i], sum);
}

inline unsigned nblocks(size_t n, int t) { return (unsigned)((n + t - 1) / t); }

}  // namespace

extern "C" {

int hpa_ref_attention_paged(float* out, float* preatt, float* att, const float* inp,
                            float* const* key_blocks, float* const* value_blocks, int B, int T, int C,
                            int NH, int offset, int block_size) {
    HPA_REQUIRE(B > 0 && T > 0 && NH > 0 && C % NH == 0 && block_size > 0 && offset >= 0,
                "attention_paged: bad shape");
    const int n = B * T * NH;
    ref_attention_paged_kernel<<<nblocks(n, 64), 64, 0, hpa_stream()>>>(
        out, preatt, att, inp, key_blocks, value_blocks, B, T, C, NH, offset, block_size);
    HPA_LAUNCH_CHECK();
    return 0;
}

int hpa_ref_matmul(float* out, const float* inp, const float* weight, const float* bias, int B, int T,
                   int C, int OC, int cached) {
    HPA_REQUIRE(B > 0 && T > 0 && C > 0 && OC > 0, "matmul: bad shape");
    HPA_REQUIRE(!cached || OC >= 3 * C, "matmul_cached: OC must be >= 3C");
    const size_t n = (size_t)B * T * OC;
    ref_matmul_kernel<<<nblocks(n, 256), 256, 0, hpa_stream()>>>(out, inp, weight, bias, B, T, C, OC,
                                                                  cached);
    HPA_LAUNCH_CHECK();
    return 0;
}

int hpa_ref_layernorm(float* out, float* mean, float* rstd, const float* inp, const float* weight,
                      const float* bias, int N, int C) {
    HPA_REQUIRE(N > 0 && C > 0, "layernorm: bad shape");
    ref_layernorm_kernel<<<nblocks(N, 64), 64, 0, hpa_stream()>>>(out, mean, rstd, inp, weight, bias,
                                                                  N, C);
    HPA_LAUNCH_CHECK();
    return 0;
}

int hpa_ref_encoder(float* out, const int* inp, const float* wte, const float* wpe, int B, int T, int C,
                    int pos_offset) {
    HPA_REQUIRE(B > 0 && T > 0 && C > 0 && pos_offset >= 0, "encoder: bad shape");
    const size_t n = (size_t)B * T * C;
    ref_encoder_kernel<<<nblocks(n, 256), 256, 0, hpa_stream()>>>(out, inp, wte, wpe, B, T, C,
                                                                   pos_offset);
    HPA_LAUNCH_CHECK();
    return 0;
}

int hpa_ref_gelu(float* out, const float* inp, int N) {
    HPA_REQUIRE(N >= 0, "gelu: bad shape");
    if (!N) return 0;
    ref_gelu_kernel<<<nblocks(N, 256), 256, 0, hpa_stream()>>>(out, inp, N);
    HPA_LAUNCH_CHECK();
    return 0;
}

int hpa_ref_residual(float* out, const float* a, const float* b, int N) {
    HPA_REQUIRE(N >= 0, "residual: bad shape");
    if (!N) return 0;
    ref_residual_kernel<<<nblocks(N, 256), 256, 0, hpa_stream()>>>(out, a, b, N);
    HPA_LAUNCH_CHECK();
    return 0;
}

int hpa_ref_softmax(float* probs, const float* logits, int N, int V) {
    HPA_REQUIRE(N > 0 && V > 0, "softmax: bad shape");
    ref_softmax_kernel<<<nblocks(N, 64), 64, 0, hpa_stream()>>>(probs, logits, N, V);
    HPA_LAUNCH_CHECK();
    return 0;
}

}  // extern "C"
