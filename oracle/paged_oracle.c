/*
 * paged_oracle.c -- CPU restatement of the reference paged decode path.
 * TEST INFRASTRUCTURE ONLY (see paged_oracle.h).  Not part of the product.
 *
 * Parity pinning: tests/test_oracle.py checks these functions against the
 * golden vectors in tests/golden/, which tests/golden/gen_golden.py produced
 * by running the reference sources themselves (compiled where they lie under
 * /root/reference into oracle/_ref by oracle/Makefile).
 */
#include "paged_oracle.h"
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* threads of the OpenMP regions from now on (n <= 0: leave as is); returns
 * the count in effect.  The timed CPU baseline sets it per run (bench.py). */
int oracle_set_threads(int n) {
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
    return omp_get_max_threads();
#else
    (void)n;
    return 1;
#endif
}

size_t oracle_num_params(OracleConfig c) {
    size_t off[16];
    oracle_param_offsets(c, off);
    size_t C = (size_t)c.channels;
    return off[15] + C;
}

/* paged_infer.c:461-476 (sizes) and :329-348 (consecutive placement) */
void oracle_param_offsets(OracleConfig c, size_t off[16]) {
    size_t V = c.vocab_size, maxT = c.max_seq_len, L = c.num_layers, C = c.channels;
    size_t sz[16] = {V * C, maxT * C, L * C, L * C, L * 3 * C * C, L * 3 * C, L * C * C, L * C,
                     L * C, L * C, L * 4 * C * C, L * 4 * C, L * C * 4 * C, L * C, C, C};
    size_t o = 0;
    for (int i = 0; i < 16; i++) { off[i] = o; o += sz[i]; }
}

/* paged_infer.c:24-47 */
void oracle_encoder_forward(float* out, const int* inp, const float* wte, const float* wpe,
                            int B, int T, int C) {
    for (int b = 0; b < B; b++)
        for (int t = 0; t < T; t++) {
            float* o = out + (size_t)b * T * C + (size_t)t * C;
            const float* we = wte + (size_t)inp[b * T + t] * C;
            const float* wp = wpe + (size_t)t * C;
            for (int i = 0; i < C; i++) o[i] = we[i] + wp[i];
        }
}

/* paged_infer.c:24-47 with an explicit absolute position per row */
void oracle_encoder_forward_pos(float* out, const int* inp, const int* pos, const float* wte,
                                const float* wpe, int N, int C) {
    for (int n = 0; n < N; n++) {
        const float* we = wte + (size_t)inp[n] * C;
        const float* wp = wpe + (size_t)pos[n] * C;
        for (int i = 0; i < C; i++) out[(size_t)n * C + i] = we[i] + wp[i];
    }
}

/* paged_infer.c:49-89 */
void oracle_layernorm_forward(float* out, float* mean, float* rstd, const float* inp,
                              const float* weight, const float* bias, int B, int T, int C) {
    float eps = 1e-5f;
    for (int b = 0; b < B; b++)
        for (int t = 0; t < T; t++) {
            const float* x = inp + (size_t)b * T * C + (size_t)t * C;
            float m = 0.0f;
            for (int i = 0; i < C; i++) m += x[i];
            m = m / C;
            float v = 0.0f;
            for (int i = 0; i < C; i++) { float xs = x[i] - m; v += xs * xs; }
            v = v / C;
            float s = 1.0f / sqrtf(v + eps);
            float* o = out + (size_t)b * T * C + (size_t)t * C;
            for (int i = 0; i < C; i++) { float n = (s * (x[i] - m)); o[i] = n * weight[i] + bias[i]; }
            if (mean) mean[b * T + t] = m;
            if (rstd) rstd[b * T + t] = s;
        }
}

/* paged_infer.c:92-114 (OpenMP over (b,t) like :99; each output is one
 * sequential-i dot so results do not depend on the thread count) */
void oracle_matmul_forward(float* out, const float* inp, const float* weight, const float* bias,
                           int B, int T, int C, int OC) {
    #pragma omp parallel for collapse(2)
    for (int b = 0; b < B; b++)
        for (int t = 0; t < T; t++) {
            float* ob = out + (size_t)b * T * OC + (size_t)t * OC;
            const float* ib = inp + (size_t)b * T * C + (size_t)t * C;
            for (int o = 0; o < OC; o++) {
                float val = (bias != NULL) ? bias[o] : 0.0f;
                const float* w = weight + (size_t)o * C;
                for (int i = 0; i < C; i++) val += ib[i] * w[i];
                ob[o] = val;
            }
        }
}

/* OC-parallel variant used by the decode oracle when B*T is small (logits):
 * same per-output arithmetic as :92-114, only the work split differs. */
static void matmul_rows_ocpar(float* out, const float* inp, const float* weight, const float* bias,
                              int N, int C, int OC) {
    #pragma omp parallel for schedule(static)
    for (int o = 0; o < OC; o++) {
        const float* w = weight + (size_t)o * C;
        for (int n = 0; n < N; n++) {
            const float* ib = inp + (size_t)n * C;
            float val = (bias != NULL) ? bias[o] : 0.0f;
            for (int i = 0; i < C; i++) val += ib[i] * w[i];
            out[(size_t)n * OC + o] = val;
        }
    }
}

/* paged_infer.c:117-160: Q for every row, K and V for the last row only
 * (OC is the full 3C; the reference's inner loops use C as the Q width). */
void oracle_matmul_cached(float* out, const float* inp, const float* weight, const float* bias,
                          int B, int T, int C, int OC) {
    #pragma omp parallel for
    for (int b = 0; b < B; b++) {
        for (int t = 0; t < T; t++) {
            float* ob = out + (size_t)b * T * OC + (size_t)t * OC;
            const float* ib = inp + (size_t)b * T * C + (size_t)t * C;
            for (int o = 0; o < C; o++) {
                float val = (bias != NULL) ? bias[o] : 0.0f;
                const float* w = weight + (size_t)o * C;
                for (int i = 0; i < C; i++) val += ib[i] * w[i];
                ob[o] = val;
            }
        }
        float* ok = out + (size_t)b * T * OC + (size_t)(T - 1) * OC + C;
        float* ov = out + (size_t)b * T * OC + (size_t)(T - 1) * OC + 2 * C;
        const float* ib = inp + (size_t)b * T * C + (size_t)(T - 1) * C;
        for (int o = 0; o < C; o++) {
            float vk = (bias != NULL) ? bias[o + C] : 0.0f;
            const float* wk = weight + (size_t)(o + C) * C;
            for (int i = 0; i < C; i++) vk += ib[i] * wk[i];
            ok[o] = vk;
            float vv = (bias != NULL) ? bias[o + 2 * C] : 0.0f;
            const float* wv = weight + (size_t)(o + 2 * C) * C;
            for (int i = 0; i < C; i++) vv += ib[i] * wv[i];
            ov[o] = vv;
        }
    }
}

/* paged_infer.c:243-251 */
#define ORACLE_GELU_SCALING_FACTOR sqrtf(2.0f / M_PI)
void oracle_gelu_forward(float* out, const float* inp, int N) {
    for (int i = 0; i < N; i++) {
        float x = inp[i];
        float cube = 0.044715f * x * x * x;
        out[i] = 0.5f * x * (1.0f + tanhf(ORACLE_GELU_SCALING_FACTOR * (x + cube)));
    }
}

/* paged_infer.c:253-257 */
void oracle_residual_forward(float* out, const float* inp1, const float* inp2, int N) {
    for (int i = 0; i < N; i++) out[i] = inp1[i] + inp2[i];
}

/* paged_infer.c:259-286 */
void oracle_softmax_forward(float* probs, const float* logits, int B, int T, int V) {
    #pragma omp parallel for collapse(2)
    for (int b = 0; b < B; b++)
        for (int t = 0; t < T; t++) {
            const float* l = logits + (size_t)b * T * V + (size_t)t * V;
            float* p = probs + (size_t)b * T * V + (size_t)t * V;
            float maxval = -10000.0f;
            for (int i = 0; i < V; i++) if (l[i] > maxval) maxval = l[i];
            float sum = 0.0f;
            for (int i = 0; i < V; i++) { p[i] = expf(l[i] - maxval); sum += p[i]; }
            for (int i = 0; i < V; i++) p[i] /= sum;
        }
}

/* generate_tokens_from_logits, paged_infer.c:937-951: strict '>' so the
 * lowest index wins a tie. */
int oracle_argmax(const float* x, int n) {
    int mi = 0;
    float mv = x[0];
    for (int v = 1; v < n; v++) if (x[v] > mv) { mv = x[v]; mi = v; }
    return mi;
}

/* paged_infer.c:826-835 */
unsigned int oracle_random_u32(unsigned long long* state) {
    *state ^= *state >> 12;
    *state ^= *state << 25;
    *state ^= *state >> 27;
    return (*state * 0x2545F4914F6CDD1Dull) >> 32;
}
float oracle_random_f32(unsigned long long* state) {
    return (oracle_random_u32(state) >> 8) / 16777216.0f;
}

/* paged_infer.c:837-848 */
int oracle_sample_mult(const float* probabilities, int n, float coin) {
    float cdf = 0.0f;
    for (int i = 0; i < n; i++) {
        cdf += probabilities[i];
        if (coin < cdf) return i;
    }
    return n - 1;
}

/* The per-(row, head) body shared by attention_forward (train_scratch.c:232-287)
 * and attention_paged (paged_infer.c:186-236): keys for logical positions
 * p in [start, start+n) come from kfetch(p); 4 passes exactly as there. */
typedef const float* (*row_fetch_fn)(const void* ctx, int p);

static void attn_row(float* out_bth, float* preatt_bth, float* att_bth, int T, const float* query_t,
                     row_fetch_fn kfetch, row_fetch_fn vfetch, const void* fctx, int start, int n,
                     int hs) {
    float scale = 1.0 / sqrtf(hs);
    /* pass 1 (paged_infer.c:186-203) */
    float maxval = -10000.0f;
    for (int t2 = 0; t2 < n; t2++) {
        const float* key_t2 = kfetch(fctx, start + t2);
        float val = 0.0f;
        for (int i = 0; i < hs; i++) val += query_t[i] * key_t2[i];
        val *= scale;
        if (val > maxval) maxval = val;
        preatt_bth[t2] = val;
    }
    /* pass 2 (:205-212) */
    float expsum = 0.0f;
    for (int t2 = 0; t2 < n; t2++) {
        float expv = expf(preatt_bth[t2] - maxval);
        expsum += expv;
        att_bth[t2] = expv;
    }
    float expsum_inv = expsum == 0.0f ? 0.0f : 1.0f / expsum;
    /* pass 3 (:215-224); T is the row length of att (zero tail) */
    for (int t2 = 0; t2 < T; t2++) {
        if (t2 < n) att_bth[t2] *= expsum_inv;
        else att_bth[t2] = 0.0f;
    }
    /* pass 4 (:226-236) */
    for (int i = 0; i < hs; i++) out_bth[i] = 0.0f;
    for (int t2 = 0; t2 < n; t2++) {
        const float* value_t2 = vfetch(fctx, start + t2);
        float a = att_bth[t2];
        for (int i = 0; i < hs; i++) out_bth[i] += a * value_t2[i];
    }
}

typedef struct { const float* inp; int T, C, b, h, hs; } contig_ctx;
static const float* contig_k(const void* c, int p) {
    const contig_ctx* x = (const contig_ctx*)c;
    return x->inp + (size_t)x->b * x->T * 3 * x->C + (size_t)p * 3 * x->C + x->h * x->hs + x->C;
}
static const float* contig_v(const void* c, int p) {
    const contig_ctx* x = (const contig_ctx*)c;
    return x->inp + (size_t)x->b * x->T * 3 * x->C + (size_t)p * 3 * x->C + x->h * x->hs + 2 * x->C;
}

/* train_scratch.c:218-291 */
void oracle_attention_forward(float* out, float* preatt, float* att, const float* inp,
                              int B, int T, int C, int NH) {
    int C3 = C * 3, hs = C / NH;
    #pragma omp parallel for collapse(3)
    for (int b = 0; b < B; b++)
        for (int t = 0; t < T; t++)
            for (int h = 0; h < NH; h++) {
                contig_ctx cx = {inp, T, C, b, h, hs};
                const float* q = inp + (size_t)b * T * C3 + (size_t)t * C3 + h * hs;
                size_t r = (size_t)b * NH * T * T + (size_t)h * T * T + (size_t)t * T;
                attn_row(out + (size_t)b * T * C + (size_t)t * C + h * hs, preatt + r, att + r, T, q,
                         contig_k, contig_v, &cx, 0, t + 1, hs);
            }
}

typedef struct { float* const* kb; float* const* vb; int bs, C, h, hs; } paged_ctx;
static const float* paged_k(const void* c, int p) {
    const paged_ctx* x = (const paged_ctx*)c;
    return x->kb[p / x->bs] + (size_t)(p % x->bs) * x->C + x->h * x->hs;
}
static const float* paged_v(const void* c, int p) {
    const paged_ctx* x = (const paged_ctx*)c;
    return x->vb[p / x->bs] + (size_t)(p % x->bs) * x->C + x->h * x->hs;
}

/* paged_infer.c:163-240 (same block lists for every b, as in the reference) */
void oracle_attention_paged(float* out, float* preatt, float* att, const float* inp,
                            float* const* key_blocks, float* const* value_blocks,
                            int B, int T, int C, int NH, int offset, int block_size) {
    int C3 = C * 3, hs = C / NH;
    #pragma omp parallel for collapse(3)
    for (int b = 0; b < B; b++)
        for (int t = 0; t < T; t++)
            for (int h = 0; h < NH; h++) {
                paged_ctx px = {key_blocks, value_blocks, block_size, C, h, hs};
                const float* q = inp + (size_t)b * T * C3 + (size_t)t * C3 + h * hs;
                size_t r = (size_t)b * NH * T * T + (size_t)h * T * T + (size_t)t * T;
                attn_row(out + (size_t)b * T * C + (size_t)t * C + h * hs, preatt + r, att + r, T, q,
                         paged_k, paged_v, &px, offset, t + 1, hs);
            }
}

/* ---------------- full-recompute forward, train_scratch.c:658-798 ---------------- */
void oracle_gpt2_forward(const float* params, OracleConfig cfg, const int* tokens, int B, int T,
                         float* logits) {
    int V = cfg.vocab_size, L = cfg.num_layers, NH = cfg.num_heads, C = cfg.channels;
    size_t off[16];
    oracle_param_offsets(cfg, off);
    const float *wte = params + off[0], *wpe = params + off[1];
    size_t BTC = (size_t)B * T * C;
    float* residual = malloc(BTC * 4);
    float* ln = malloc(BTC * 4);
    float* qkv = malloc(BTC * 3 * 4);
    float* atty = malloc(BTC * 4);
    float* tmp = malloc(BTC * 4);
    float* res2 = malloc(BTC * 4);
    float* fch = malloc(BTC * 4 * 4);
    float* fchg = malloc(BTC * 4 * 4);
    size_t natt = (size_t)B * NH * T * T;
    float* preatt = malloc(natt * 4);
    float* att = malloc(natt * 4);
    oracle_encoder_forward(residual, tokens, wte, wpe, B, T, C);
    for (int l = 0; l < L; l++) {
        const float* ln1w = params + off[2] + (size_t)l * C;
        const float* ln1b = params + off[3] + (size_t)l * C;
        const float* qkvw = params + off[4] + (size_t)l * 3 * C * C;
        const float* qkvb = params + off[5] + (size_t)l * 3 * C;
        const float* apw = params + off[6] + (size_t)l * C * C;
        const float* apb = params + off[7] + (size_t)l * C;
        const float* ln2w = params + off[8] + (size_t)l * C;
        const float* ln2b = params + off[9] + (size_t)l * C;
        const float* fcw = params + off[10] + (size_t)l * 4 * C * C;
        const float* fcb = params + off[11] + (size_t)l * 4 * C;
        const float* fpw = params + off[12] + (size_t)l * C * 4 * C;
        const float* fpb = params + off[13] + (size_t)l * C;
        oracle_layernorm_forward(ln, NULL, NULL, residual, ln1w, ln1b, B, T, C);
        oracle_matmul_forward(qkv, ln, qkvw, qkvb, B, T, C, 3 * C);
        oracle_attention_forward(atty, preatt, att, qkv, B, T, C, NH);
        oracle_matmul_forward(tmp, atty, apw, apb, B, T, C, C);
        oracle_residual_forward(res2, residual, tmp, (int)BTC);
        oracle_layernorm_forward(ln, NULL, NULL, res2, ln2w, ln2b, B, T, C);
        oracle_matmul_forward(fch, ln, fcw, fcb, B, T, C, 4 * C);
        oracle_gelu_forward(fchg, fch, (int)(BTC * 4));
        oracle_matmul_forward(tmp, fchg, fpw, fpb, B, T, 4 * C, C);
        oracle_residual_forward(residual, res2, tmp, (int)BTC);
    }
    oracle_layernorm_forward(ln, NULL, NULL, residual, params + off[14], params + off[15], B, T, C);
    oracle_matmul_forward(logits, ln, wte, NULL, B, T, C, V);
    free(residual); free(ln); free(qkv); free(atty); free(tmp); free(res2);
    free(fch); free(fchg); free(preatt); free(att);
}

/* ---------------- paged incremental decode ---------------- */
struct OraclePaged {
    OracleConfig cfg;
    const float* params;
    size_t off[16];
    int B, P, max_pages, num_pages;
    float* kpool;  /* [L][num_pages][P][C] */
    float* vpool;
    int* block_table; /* [B][max_pages] */
    int* pos;         /* [B] */
    int* free_perm;   /* page ids in hand-out order */
    int next_free;
    int kv_bf16;      /* round appended K/V to bf16 (round to nearest even) */
    float* pw_bf16;   /* bf16 weights mode: params with qkvw/attprojw/fcw/fcprojw rounded */
    float* wte_bf16;  /* ... and the logits' wte rounded (the embedding keeps fp32 wte) */
    float *x, *ln, *qkv, *atty, *tmp, *res2, *fch, *fchg, *logits;
};

OraclePaged* oracle_paged_create(const float* params, OracleConfig cfg, int B, int page_size,
                                 int max_ctx, unsigned long long page_seed) {
    OraclePaged* o = calloc(1, sizeof(OraclePaged));
    o->cfg = cfg;
    o->params = params;
    oracle_param_offsets(cfg, o->off);
    o->B = B;
    o->P = page_size;
    o->max_pages = (max_ctx + page_size - 1) / page_size;
    o->num_pages = B * o->max_pages;
    size_t C = cfg.channels, L = cfg.num_layers;
    size_t pool = L * (size_t)o->num_pages * page_size * C;
    o->kpool = malloc(pool * 4);
    o->vpool = malloc(pool * 4);
    if (!o->kpool || !o->vpool) { free(o->kpool); free(o->vpool); free(o); return NULL; }
    o->block_table = malloc((size_t)B * o->max_pages * sizeof(int));
    for (size_t i = 0; i < (size_t)B * o->max_pages; i++) o->block_table[i] = -1;
    o->pos = calloc(B, sizeof(int));
    o->free_perm = malloc(o->num_pages * sizeof(int));
    for (int i = 0; i < o->num_pages; i++) o->free_perm[i] = i;
    unsigned long long st = page_seed ? page_seed : 1;
    for (int i = o->num_pages - 1; i > 0; i--) { /* Fisher-Yates with the reference xorshift */
        int j = (int)(oracle_random_u32(&st) % (unsigned)(i + 1));
        int t = o->free_perm[i]; o->free_perm[i] = o->free_perm[j]; o->free_perm[j] = t;
    }
    int V = cfg.vocab_size;
    o->x = malloc(B * C * 4); o->ln = malloc(B * C * 4); o->qkv = malloc(B * 3 * C * 4);
    o->atty = malloc(B * C * 4); o->tmp = malloc(B * C * 4); o->res2 = malloc(B * C * 4);
    o->fch = malloc(B * 4 * C * 4); o->fchg = malloc(B * 4 * C * 4);
    o->logits = malloc((size_t)B * V * 4);
    return o;
}

void oracle_paged_free(OraclePaged* o) {
    if (!o) return;
    free(o->kpool); free(o->vpool); free(o->block_table); free(o->pos); free(o->free_perm);
    free(o->x); free(o->ln); free(o->qkv); free(o->atty); free(o->tmp); free(o->res2);
    free(o->fch); free(o->fchg); free(o->logits); free(o->pw_bf16); free(o->wte_bf16); free(o);
}

int oracle_paged_pos(const OraclePaged* o, int b) { return o->pos[b]; }

void oracle_paged_set_kv_bf16(OraclePaged* o, int on) { o->kv_bf16 = on ? 1 : 0; }

/* fp32 -> the value a bf16 store keeps: round to nearest even on the upper
 * 16 bits (finite inputs), returned as fp32 */
float oracle_round_bf16(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    u += 0x7fffu + ((u >> 16) & 1u);
    u &= 0xffff0000u;
    memcpy(&f, &u, 4);
    return f;
}

/* "bf16 decode" (gpt2_decode_init_w with HPA_BF16 weights): every GEMM's
 * weights and its input rows (after LayerNorm / attention / GELU) are
 * rounded to bf16 (nearest even), the products summed in fp32; everything
 * else stays fp32.  Restates hpa_gemm_bf16.hip's numerics for parity tests. */
int oracle_paged_set_w_bf16(OraclePaged* o, int on) {
    free(o->pw_bf16); free(o->wte_bf16);
    o->pw_bf16 = o->wte_bf16 = NULL;
    if (!on) return 0;
    size_t n = oracle_num_params(o->cfg);
    size_t nwte = (size_t)o->cfg.vocab_size * o->cfg.channels;
    o->pw_bf16 = malloc(n * 4);
    o->wte_bf16 = malloc(nwte * 4);
    if (!o->pw_bf16 || !o->wte_bf16) return -1;
    memcpy(o->pw_bf16, o->params, n * 4);
    const int mats[4] = {4, 6, 10, 12}; /* qkvw, attprojw, fcw, fcprojw (paged_infer.c:308-326) */
    size_t sz[16];
    for (int i = 0; i < 15; i++) sz[i] = o->off[i + 1] - o->off[i];
    sz[15] = n - o->off[15];
    for (int m = 0; m < 4; m++)
        for (size_t i = 0; i < sz[mats[m]]; i++) {
            float* x = o->pw_bf16 + o->off[mats[m]] + i;
            *x = oracle_round_bf16(*x);
        }
    for (size_t i = 0; i < nwte; i++) o->wte_bf16[i] = oracle_round_bf16(o->params[o->off[0] + i]);
    return 0;
}

static void round_bf16_n(OraclePaged* o, float* x, size_t n) {
    if (!o->pw_bf16) return;
    for (size_t i = 0; i < n; i++) x[i] = oracle_round_bf16(x[i]);
}

static float* page_ptr(OraclePaged* o, float* pool, int layer, int page) {
    return pool + ((size_t)layer * o->num_pages + page) * o->P * o->cfg.channels;
}

static int ensure_page(OraclePaged* o, int b, int p) {
    int lp = p / o->P;
    if (lp >= o->max_pages) return -1;
    int* bt = o->block_table + (size_t)b * o->max_pages;
    if (bt[lp] < 0) {
        if (o->next_free >= o->num_pages) return -1;
        bt[lp] = o->free_perm[o->next_free++];  /* request_block, block_manager.c:115-162 */
    }
    return 0;
}

void oracle_paged_fill_random(OraclePaged* o, int ctx, unsigned long long seed) {
    unsigned long long st = seed ? seed : 1;
    int C = o->cfg.channels, L = o->cfg.num_layers;
    for (int b = 0; b < o->B; b++) {
        for (int p = 0; p < ctx; p++) ensure_page(o, b, p);
        o->pos[b] = ctx;
    }
    for (int l = 0; l < L; l++)
        for (int b = 0; b < o->B; b++)
            for (int p = 0; p < ctx; p++) {
                int page = o->block_table[(size_t)b * o->max_pages + p / o->P];
                float* k = page_ptr(o, o->kpool, l, page) + (size_t)(p % o->P) * C;
                float* v = page_ptr(o, o->vpool, l, page) + (size_t)(p % o->P) * C;
                for (int i = 0; i < C; i++) {
                    k[i] = 2.0f * oracle_random_f32(&st) - 1.0f;
                    v[i] = 2.0f * oracle_random_f32(&st) - 1.0f;
                }
            }
}

/* parity tests: positions [0, n) of sequence b at layer l take the given
 * K/V rows (token-major [n][C], the cache the GPU engine holds, so both
 * sides decode from identical pages); the sequence's position becomes n */
int oracle_paged_set_kv(OraclePaged* o, int layer, int b, int n, const float* k, const float* v) {
    const int C = o->cfg.channels;
    if (layer < 0 || layer >= o->cfg.num_layers || b < 0 || b >= o->B || n < 0) return -1;
    for (int p = 0; p < n; p++) {
        if (ensure_page(o, b, p) != 0) return -1;
        const int page = o->block_table[(size_t)b * o->max_pages + p / o->P];
        memcpy(page_ptr(o, o->kpool, layer, page) + (size_t)(p % o->P) * C, k + (size_t)p * C, (size_t)C * 4);
        memcpy(page_ptr(o, o->vpool, layer, page) + (size_t)(p % o->P) * C, v + (size_t)p * C, (size_t)C * 4);
    }
    o->pos[b] = n;
    return 0;
}

int oracle_paged_step(OraclePaged* o, const int* tokens, float* logits, int* next) {
    return oracle_paged_step_ex(o, tokens, NULL, NULL, logits, next);
}

/* forced_x (nullable, [L+1][B][C]): the residual stream entering layer l is
 * taken from forced_x[l] (and the final one, LNf's input, from forced_x[L])
 * instead of this decoder's own previous layer -- each layer then runs on the
 * GPU engine's input (gpt2_decode_step_traced), so a per-layer comparison is
 * not compounded over layers; layer_out (nullable, [L][B][C]) receives every
 * layer's output.  The K/V appended are those computed from the forced input. */
int oracle_paged_step_ex(OraclePaged* o, const int* tokens, const float* forced_x, float* layer_out,
                         float* logits, int* next) {
    OracleConfig cfg = o->cfg;
    int B = o->B, C = cfg.channels, NH = cfg.num_heads, L = cfg.num_layers, V = cfg.vocab_size;
    int hs = C / NH;
    const float* P = o->params;
    const float* PW = o->pw_bf16 ? o->pw_bf16 : o->params; /* GEMM weights */
    for (int b = 0; b < B; b++) {
        if (o->pos[b] >= cfg.max_seq_len) return -1;
        if (ensure_page(o, b, o->pos[b]) != 0) return -1;
    }
    /* encoder_forward at absolute positions (paged_infer.c:24-47) */
    oracle_encoder_forward_pos(o->x, tokens, o->pos, P + o->off[0], P + o->off[1], B, C);
    for (int l = 0; l < L; l++) {
        const float* ln1w = P + o->off[2] + (size_t)l * C;
        const float* ln1b = P + o->off[3] + (size_t)l * C;
        const float* qkvw = PW + o->off[4] + (size_t)l * 3 * C * C;
        const float* qkvb = P + o->off[5] + (size_t)l * 3 * C;
        const float* apw = PW + o->off[6] + (size_t)l * C * C;
        const float* apb = P + o->off[7] + (size_t)l * C;
        const float* ln2w = P + o->off[8] + (size_t)l * C;
        const float* ln2b = P + o->off[9] + (size_t)l * C;
        const float* fcw = PW + o->off[10] + (size_t)l * 4 * C * C;
        const float* fcb = P + o->off[11] + (size_t)l * 4 * C;
        const float* fpw = PW + o->off[12] + (size_t)l * C * 4 * C;
        const float* fpb = P + o->off[13] + (size_t)l * C;
        if (forced_x) memcpy(o->x, forced_x + (size_t)l * B * C, (size_t)B * C * 4);
        oracle_layernorm_forward(o->ln, NULL, NULL, o->x, ln1w, ln1b, B, 1, C);
        round_bf16_n(o, o->ln, (size_t)B * C);
        /* decode QKV = matmul_cached's last row (paged_infer.c:117-160) */
        matmul_rows_ocpar(o->qkv, o->ln, qkvw, qkvb, B, C, 3 * C);
        /* add_to_cache (paged_infer.c:548-566): K,V of this token into its page slot */
        for (int b = 0; b < B; b++) {
            int p = o->pos[b];
            int page = o->block_table[(size_t)b * o->max_pages + p / o->P];
            float* k = page_ptr(o, o->kpool, l, page) + (size_t)(p % o->P) * C;
            float* v = page_ptr(o, o->vpool, l, page) + (size_t)(p % o->P) * C;
            memcpy(k, o->qkv + (size_t)b * 3 * C + C, C * 4);
            memcpy(v, o->qkv + (size_t)b * 3 * C + 2 * C, C * 4);
            if (o->kv_bf16)
                for (int i = 0; i < C; i++) {
                    k[i] = oracle_round_bf16(k[i]);
                    v[i] = oracle_round_bf16(v[i]);
                }
        }
        /* attention_paged arithmetic (paged_infer.c:163-240), keys 0..pos[b] */
        #pragma omp parallel for collapse(2) schedule(dynamic)
        for (int b = 0; b < B; b++)
            for (int h = 0; h < NH; h++) {
                int n = o->pos[b] + 1;
                float* pre = malloc((size_t)n * 4);
                float* att = malloc((size_t)n * 4);
                float** kptr = malloc(sizeof(float*) * o->max_pages);
                float** vptr = malloc(sizeof(float*) * o->max_pages);
                int np = (n + o->P - 1) / o->P;
                for (int i = 0; i < np; i++) {
                    int page = o->block_table[(size_t)b * o->max_pages + i];
                    kptr[i] = page_ptr(o, o->kpool, l, page);
                    vptr[i] = page_ptr(o, o->vpool, l, page);
                }
                paged_ctx px = {kptr, vptr, o->P, C, h, hs};
                attn_row(o->atty + (size_t)b * C + h * hs, pre, att, n,
                         o->qkv + (size_t)b * 3 * C + h * hs, paged_k, paged_v, &px, 0, n, hs);
                free(pre); free(att); free(kptr); free(vptr);
            }
        round_bf16_n(o, o->atty, (size_t)B * C);
        matmul_rows_ocpar(o->tmp, o->atty, apw, apb, B, C, C);
        oracle_residual_forward(o->res2, o->x, o->tmp, B * C);
        oracle_layernorm_forward(o->ln, NULL, NULL, o->res2, ln2w, ln2b, B, 1, C);
        round_bf16_n(o, o->ln, (size_t)B * C);
        matmul_rows_ocpar(o->fch, o->ln, fcw, fcb, B, C, 4 * C);
        oracle_gelu_forward(o->fchg, o->fch, B * 4 * C);
        round_bf16_n(o, o->fchg, (size_t)B * 4 * C);
        matmul_rows_ocpar(o->tmp, o->fchg, fpw, fpb, B, 4 * C, C);
        oracle_residual_forward(o->x, o->res2, o->tmp, B * C);
        if (layer_out) memcpy(layer_out + (size_t)l * B * C, o->x, (size_t)B * C * 4);
    }
    if (forced_x) memcpy(o->x, forced_x + (size_t)L * B * C, (size_t)B * C * 4);
    oracle_layernorm_forward(o->ln, NULL, NULL, o->x, P + o->off[14], P + o->off[15], B, 1, C);
    round_bf16_n(o, o->ln, (size_t)B * C);
    float* lg = logits ? logits : o->logits;
    matmul_rows_ocpar(lg, o->ln, o->wte_bf16 ? o->wte_bf16 : P + o->off[0], NULL, B, C, V);
    for (int b = 0; b < B; b++) {
        if (next) next[b] = oracle_argmax(lg + (size_t)b * V, V);
        o->pos[b]++;
    }
    return 0;
}

/* one decode query row per sequence: q (C) attends logical positions
 * 0..ctx-1 through key_blocks/value_blocks (pages of block_size tokens,
 * token-major [block_size][C]) with attention_paged's per-row arithmetic
 * (paged_infer.c:186-236); out (C). */
void oracle_attention_decode(float* out, const float* q, float* const* key_blocks,
                             float* const* value_blocks, int ctx, int C, int NH, int block_size) {
    int hs = C / NH;
    float* pre = malloc((size_t)(ctx > 0 ? ctx : 1) * 4);
    float* att = malloc((size_t)(ctx > 0 ? ctx : 1) * 4);
    for (int h = 0; h < NH; h++) {
        paged_ctx px = {key_blocks, value_blocks, block_size, C, h, hs};
        attn_row(out + h * hs, pre, att, ctx, q + h * hs, paged_k, paged_v, &px, 0, ctx, hs);
    }
    free(pre);
    free(att);
}
