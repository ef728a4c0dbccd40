/*
 * paged_infer.c -- host side (C) of the MI355X paged-attention decode path:
 *   - drop-in versions of the reference paged_infer.c functions
 *     (mx60s/llm.c-paged paged_infer.c), computing on the GPU;
 *   - the llm.c checkpoint loader and a seeded synthetic-weights generator;
 *   - the decode engine (gpt2_decode_*): per-step orchestration of the
 *     gfx950 kernels of hip_paged_attn.h over the HBM page pool, block
 *     tables from the BlockManager, hipGraph replay.
 * No Python and no CPU compute on the product path: every tensor op is a
 * HIP kernel; the host only allocates pages and enqueues work.
 */
#include "paged_infer.h"

#include <math.h>
#include <stdint.h>
#include <ctype.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "block_manager.h"
#include "hip_paged_attn.h"

/* K parts of the ring qkv / fc at C >= 1024 (dec_gemm, hpa_gemm_ring.hip) */
#define DEC_RING_QKV_PARTS 3
#define DEC_RING_FC_PARTS 2
static int dec_ring_allowed(void);

#define PI_FATAL(...)                                         \
    do {                                                      \
        fprintf(stderr, "[paged_infer] " __VA_ARGS__);        \
        fprintf(stderr, " (%s:%d)\n", __FILE__, __LINE__);    \
        exit(1);                                              \
    } while (0)
#define PI_CHECK(call)                                                        \
    do {                                                                      \
        if ((call) != 0) PI_FATAL("%s failed: %s", #call, hpa_last_error());  \
    } while (0)

/* ------------------------------------------------------------------------ */
/* device init + host/device staging for the drop-in functions              */
/* ------------------------------------------------------------------------ */
static void ensure_device(void) {
    if (hpa_get_device() >= 0) return;
    const char* e = getenv("HPA_DEVICE");
    int dev = e ? atoi(e) : 0;
    if (hpa_init(dev) != 0) PI_FATAL("no usable HIP device (the MI355X path has no CPU fallback)");
}

typedef struct {
    void* d;
    void* h;
    size_t n;
    int owned;
} Stage;

/* device-accessible view of p (copied in when copy_in) */
static void* stage_in(Stage* s, const void* p, size_t n, int copy_in) {
    s->h = (void*)p;
    s->n = n;
    s->owned = 0;
    s->d = (void*)p;
    if (!p || n == 0 || hpa_is_device_accessible(p)) return s->d;
    s->d = hpa_malloc(n);
    if (!s->d) PI_FATAL("staging allocation of %zu bytes failed", n);
    if (copy_in) PI_CHECK(hpa_memcpy(s->d, p, n));
    s->owned = 1;
    return s->d;
}
static void stage_out(Stage* s) {
    if (s->owned) PI_CHECK(hpa_memcpy(s->h, s->d, s->n));
}
static void stage_free(Stage* s) {
    if (s->owned) hpa_free(s->d);
    s->owned = 0;
}

/* ------------------------------------------------------------------------ */
/* reference layer functions (paged_infer.c:24-302), on the GPU             */
/* ------------------------------------------------------------------------ */
void encoder_forward(float* out, int* inp, float* wte, float* wpe, int B, int T, int C) {
    ensure_device();
    Stage so, si, st, sp;
    float* d_out = stage_in(&so, out, (size_t)B * T * C * 4, 0);
    int* d_inp = stage_in(&si, inp, (size_t)B * T * 4, 1);
    /* wte/wpe sizes are not part of the signature: assume device-resident
     * model weights, or stage the rows the tokens touch when on the host */
    float* d_wte = wte;
    float* d_wpe = wpe;
    if (!hpa_is_device_accessible(wte) || !hpa_is_device_accessible(wpe)) {
        int* h = (int*)malloc((size_t)B * T * sizeof(int));
        if (hpa_is_device_accessible(inp)) PI_CHECK(hpa_memcpy(h, inp, (size_t)B * T * 4));
        else memcpy(h, inp, (size_t)B * T * 4);
        int mx = 0;
        for (int i = 0; i < B * T; i++) mx = h[i] > mx ? h[i] : mx;
        free(h);
        d_wte = stage_in(&st, wte, (size_t)(mx + 1) * C * 4, 1);
        d_wpe = stage_in(&sp, wpe, (size_t)T * C * 4, 1);
    } else {
        st.owned = sp.owned = 0;
    }
    PI_CHECK(hpa_ref_encoder(d_out, d_inp, d_wte, d_wpe, B, T, C, 0));
    PI_CHECK(hpa_synchronize());
    stage_out(&so);
    stage_free(&so); stage_free(&si); stage_free(&st); stage_free(&sp);
}

void layernorm_forward(float* out, float* mean, float* rstd, float* inp, float* weight, float* bias,
                       int B, int T, int C) {
    ensure_device();
    size_t N = (size_t)B * T;
    Stage so, sm, sr, si, sw, sb;
    float* d_out = stage_in(&so, out, N * C * 4, 0);
    float* d_mean = stage_in(&sm, mean, N * 4, 0);
    float* d_rstd = stage_in(&sr, rstd, N * 4, 0);
    float* d_inp = stage_in(&si, inp, N * C * 4, 1);
    float* d_w = stage_in(&sw, weight, (size_t)C * 4, 1);
    float* d_b = stage_in(&sb, bias, (size_t)C * 4, 1);
    PI_CHECK(hpa_ref_layernorm(d_out, d_mean, d_rstd, d_inp, d_w, d_b, (int)N, C));
    PI_CHECK(hpa_synchronize());
    stage_out(&so); stage_out(&sm); stage_out(&sr);
    stage_free(&so); stage_free(&sm); stage_free(&sr); stage_free(&si); stage_free(&sw);
    stage_free(&sb);
}

static void matmul_any(float* out, float* inp, float* weight, float* bias, int B, int T, int C, int OC,
                       int cached) {
    ensure_device();
    size_t N = (size_t)B * T;
    Stage so, si, sw, sb;
    /* matmul_cached leaves K/V of the earlier rows untouched: copy out in */
    float* d_out = stage_in(&so, out, N * OC * 4, cached);
    float* d_inp = stage_in(&si, inp, N * C * 4, 1);
    float* d_w = stage_in(&sw, weight, (size_t)OC * C * 4, 1);
    float* d_b = stage_in(&sb, bias, (size_t)OC * 4, 1);
    PI_CHECK(hpa_ref_matmul(d_out, d_inp, d_w, d_b, B, T, C, OC, cached));
    PI_CHECK(hpa_synchronize());
    stage_out(&so);
    stage_free(&so); stage_free(&si); stage_free(&sw); stage_free(&sb);
}

void matmul_forward(float* out, float* inp, float* weight, float* bias, int B, int T, int C, int OC) {
    matmul_any(out, inp, weight, bias, B, T, C, OC, 0);
}

void matmul_cached(float* out, float* inp, float* weight, float* bias, int B, int T, int C, int OC) {
    matmul_any(out, inp, weight, bias, B, T, C, OC, 1);
}

void attention_paged_bs(float* out, float* preatt, float* att, float* inp, float** key_blocks,
                        float** value_blocks, int B, int T, int C, int NH, int offset,
                        int block_size) {
    ensure_device();
    if (B <= 0 || T <= 0 || NH <= 0 || C % NH || block_size <= 0 || offset < 0)
        PI_FATAL("attention_paged: bad shape");
    int npages = (offset + T + block_size - 1) / block_size;
    size_t page_bytes = (size_t)block_size * C * 4;
    Stage so, sp, sa, si;
    float* d_out = stage_in(&so, out, (size_t)B * T * C * 4, 0);
    /* preatt rows are written only up to t (:202): keep the caller's tail */
    float* d_pre = stage_in(&sp, preatt, (size_t)B * NH * T * T * 4, 1);
    float* d_att = stage_in(&sa, att, (size_t)B * NH * T * T * 4, 0);
    float* d_inp = stage_in(&si, inp, (size_t)B * T * 3 * C * 4, 1);
    Stage* pk = (Stage*)calloc((size_t)2 * npages, sizeof(Stage));
    float** hptr = (float**)malloc(sizeof(float*) * 2 * npages);
    for (int i = 0; i < npages; i++) {
        hptr[i] = stage_in(&pk[i], key_blocks[i], page_bytes, 1);
        hptr[npages + i] = stage_in(&pk[npages + i], value_blocks[i], page_bytes, 1);
    }
    float** d_ptr = (float**)hpa_malloc(sizeof(float*) * 2 * npages);
    if (!d_ptr) PI_FATAL("attention_paged: allocation failed");
    PI_CHECK(hpa_memcpy(d_ptr, hptr, sizeof(float*) * 2 * npages));
    PI_CHECK(hpa_ref_attention_paged(d_out, d_pre, d_att, d_inp, d_ptr, d_ptr + npages, B, T, C, NH,
                                     offset, block_size));
    PI_CHECK(hpa_synchronize());
    stage_out(&so); stage_out(&sp); stage_out(&sa);
    stage_free(&so); stage_free(&sp); stage_free(&sa); stage_free(&si);
    for (int i = 0; i < 2 * npages; i++) stage_free(&pk[i]);
    free(pk);
    free(hptr);
    hpa_free(d_ptr);
}

/* paged_infer.c:163-240 (pages of BLOCK_SIZE tokens, as the reference) */
void attention_paged(float* out, float* preatt, float* att, float* inp, float** key_blocks,
                     float** value_blocks, int B, int T, int C, int NH, int offset) {
    attention_paged_bs(out, preatt, att, inp, key_blocks, value_blocks, B, T, C, NH, offset,
                       BLOCK_SIZE);
}

void gelu_forward(float* out, float* inp, int N) {
    ensure_device();
    Stage so, si;
    float* d_out = stage_in(&so, out, (size_t)N * 4, 0);
    float* d_inp = stage_in(&si, inp, (size_t)N * 4, 1);
    PI_CHECK(hpa_ref_gelu(d_out, d_inp, N));
    PI_CHECK(hpa_synchronize());
    stage_out(&so);
    stage_free(&so); stage_free(&si);
}

void residual_forward(float* out, float* inp1, float* inp2, int N) {
    ensure_device();
    Stage so, sa, sb;
    float* d_out = stage_in(&so, out, (size_t)N * 4, 0);
    float* d_a = stage_in(&sa, inp1, (size_t)N * 4, 1);
    float* d_b = stage_in(&sb, inp2, (size_t)N * 4, 1);
    PI_CHECK(hpa_ref_residual(d_out, d_a, d_b, N));
    PI_CHECK(hpa_synchronize());
    stage_out(&so);
    stage_free(&so); stage_free(&sa); stage_free(&sb);
}

void softmax_forward(float* probs, float* logits, int B, int T, int V) {
    ensure_device();
    size_t n = (size_t)B * T * V * 4;
    Stage sp, sl;
    float* d_p = stage_in(&sp, probs, n, 0);
    float* d_l = stage_in(&sl, logits, n, 1);
    PI_CHECK(hpa_ref_softmax(d_p, d_l, B * T, V));
    PI_CHECK(hpa_synchronize());
    stage_out(&sp);
    stage_free(&sp); stage_free(&sl);
}

/* add_to_cache, paged_infer.c:505-573.  Corrected semantics:
 * sequence b appends to prompt b's pages (the reference hard-codes prompt 0
 * and overwrites the same slots for every b), spilling into new pages when
 * the current one fills (the reference assumes it never does, :542-545).
 * Pages are token-major [block_size][C] as in the reference. */
void add_to_cache(BlockManager* manager, float* qkv, int B, int T, int C,
                  int how_many_tokens_to_copy_from_the_end_of_sequence) {
    ensure_device();
    int n = how_many_tokens_to_copy_from_the_end_of_sequence;
    if (n < 0 || n > T) PI_FATAL("add_to_cache: bad token count");
    int bs = manager->block_size;
    for (int b = 0; b < B; b++) {
        int t = T - n;
        while (t < T) {
            KVBlock* cur = get_current_block(manager, b);
            if (!cur || cur->filled >= bs) {
                cur = request_block(manager, b);
                if (!cur) PI_FATAL("add_to_cache: no page available for prompt %d", b);
            } else {
                cur->lru_counter = ++manager->lru_epoch; /* :524 */
            }
            int take = bs - cur->filled;
            if (take > T - t) take = T - t;
            for (int j = 0; j < take; j++) {
                const float* k = qkv + (size_t)b * T * 3 * C + (size_t)(t + j) * 3 * C + C;
                const float* v = k + C;
                PI_CHECK(hpa_memcpy(cur->keys + (size_t)(cur->filled + j) * C, k, (size_t)C * 4));
                PI_CHECK(hpa_memcpy(cur->values + (size_t)(cur->filled + j) * C, v, (size_t)C * 4));
            }
            cur->filled += take;
            t += take;
        }
    }
}

/* paged_infer.c:826-835 */
unsigned int random_u32(unsigned long long* state) {
    *state ^= *state >> 12;
    *state ^= *state << 25;
    *state ^= *state >> 27;
    return (*state * 0x2545F4914F6CDD1Dull) >> 32;
}
float random_f32(unsigned long long* state) { return (random_u32(state) >> 8) / 16777216.0f; }

/* paged_infer.c:837-848 */
int sample_mult(float* probabilities, int n, float coin) {
    float cdf = 0.0f;
    for (int i = 0; i < n; i++) {
        cdf += probabilities[i];
        if (coin < cdf) return i;
    }
    return n - 1;
}

/* paged_infer.c:937-951 (host, strict > so the lowest index wins) */
int* generate_tokens_from_logits(float* probs, int B, int T, int V) {
    int* tokens = (int*)malloc((size_t)B * T * sizeof(int));
    for (int i = 0; i < B * T; i++) {
        int mi = 0;
        float mv = probs[(size_t)i * V];
        for (int v = 1; v < V; v++)
            if (probs[(size_t)i * V + v] > mv) { mv = probs[(size_t)i * V + v]; mi = v; }
        tokens[i] = mi;
    }
    return tokens;
}

/* ------------------------------------------------------------------------ */
/* parameters: checkpoint loader, synthetic weights, writer                 */
/* ------------------------------------------------------------------------ */
static void param_sizes(GPT2Config c, size_t* s) {
    size_t V = c.vocab_size, maxT = c.max_seq_len, L = c.num_layers, C = c.channels;
    s[0] = V * C; s[1] = maxT * C; s[2] = L * C; s[3] = L * C;
    s[4] = L * 3 * C * C; s[5] = L * 3 * C; s[6] = L * C * C; s[7] = L * C;
    s[8] = L * C; s[9] = L * C; s[10] = L * 4 * C * C; s[11] = L * 4 * C;
    s[12] = L * C * 4 * C; s[13] = L * C; s[14] = C; s[15] = C;
}

size_t gpt2_num_parameters(GPT2Config c) {
    size_t s[NUM_PARAMETER_TENSORS], n = 0;
    param_sizes(c, s);
    for (int i = 0; i < NUM_PARAMETER_TENSORS; i++) n += s[i];
    return n;
}

static void model_zero(GPT2* m) {
    memset(m, 0, sizeof(*m));
    m->mean_loss = -1.0f;
}

int gpt2_build_from_params(GPT2* model, GPT2Config c, const float* host_params) {
    ensure_device();
    model_zero(model);
    if (c.channels <= 0 || c.num_heads <= 0 || c.channels % c.num_heads || c.num_layers <= 0 ||
        c.vocab_size <= 0 || c.max_seq_len <= 0) {
        fprintf(stderr, "[paged_infer] bad GPT-2 config\n");
        return 1;
    }
    model->config = c;
    param_sizes(c, model->param_sizes);
    model->num_parameters = gpt2_num_parameters(c);
    model->params_memory = (float*)hpa_malloc(model->num_parameters * sizeof(float));
    if (!model->params_memory) return 1;
    if (hpa_memcpy(model->params_memory, host_params, model->num_parameters * sizeof(float))) return 1;
    float** ptrs[NUM_PARAMETER_TENSORS] = {
        &model->params.wte, &model->params.wpe, &model->params.ln1w, &model->params.ln1b,
        &model->params.qkvw, &model->params.qkvb, &model->params.attprojw, &model->params.attprojb,
        &model->params.ln2w, &model->params.ln2b, &model->params.fcw, &model->params.fcb,
        &model->params.fcprojw, &model->params.fcprojb, &model->params.lnfw, &model->params.lnfb};
    float* it = model->params_memory;
    for (int i = 0; i < NUM_PARAMETER_TENSORS; i++) {
        *ptrs[i] = it;
        it += model->param_sizes[i];
    }
    return 0;
}

/* paged_infer.c:436-502: 256 x int32 header, magic 20240326, version 1 (fp32) */
/* Checkpoint formats (train_gpt2.py:295-320 write_model; 256-int32 header
 * magic 20240326, version, maxT, V, L, NH, C):
 *   v1: the 16 tensors in ParameterTensors order, fp32 (:242-265);
 *   v2: wte wpe qkvw qkvb attprojw attprojb fcw fcb fcprojw fcprojb as bf16,
 *       then ln1w ln1b ln2w ln2b lnfw lnfb as fp32 (:267-293).
 * The reference loader (paged_infer.c:436-502) reads v1 only; v2 loads
 * here with an exact bf16 -> fp32 widening, so compute stays fp32. */
static const int kV2Order[NUM_PARAMETER_TENSORS] = {0, 1, 4, 5, 6, 7, 10, 11, 12, 13, /* bf16 */
                                                    2, 3, 8, 9, 14, 15};               /* fp32 */
#define CKPT_V2_NBF16 10

static unsigned short f32_to_bf16_rne(float f) {
    unsigned int u;
    memcpy(&u, &f, 4);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (unsigned short)((u >> 16) | 0x40); /* quiet NaN */
    u += 0x7fffu + ((u >> 16) & 1u);
    return (unsigned short)(u >> 16);
}

int gpt2_read_checkpoint(const char* path, GPT2Config* config, float* host_params) {
    FILE* f = fopen(path, "rb");
    if (!f) { fprintf(stderr, "[paged_infer] cannot open checkpoint %s\n", path); return 1; }
    int hdr[256];
    int rc = 1;
    if (fread(hdr, sizeof(int), 256, f) != 256) { fprintf(stderr, "[paged_infer] short checkpoint header\n"); goto out; }
    if (hdr[0] != 20240326) { fprintf(stderr, "[paged_infer] bad magic in checkpoint\n"); goto out; }
    if (hdr[1] != 1 && hdr[1] != 2) { fprintf(stderr, "[paged_infer] checkpoint version %d (1 or 2)\n", hdr[1]); goto out; }
    GPT2Config c;
    c.max_seq_len = hdr[2];
    c.vocab_size = hdr[3];
    c.num_layers = hdr[4];
    c.num_heads = hdr[5];
    c.channels = hdr[6];
    if (c.max_seq_len <= 0 || c.vocab_size <= 0 || c.num_layers <= 0 || c.num_heads <= 0 || c.channels <= 0 ||
        c.channels % c.num_heads) {
        fprintf(stderr, "[paged_infer] bad checkpoint config\n");
        goto out;
    }
    if (config) *config = c;
    if (!host_params) { rc = 0; goto out; }
    size_t s[NUM_PARAMETER_TENSORS], off[NUM_PARAMETER_TENSORS], n = 0;
    param_sizes(c, s);
    for (int t = 0; t < NUM_PARAMETER_TENSORS; t++) { off[t] = n; n += s[t]; }
    if (hdr[1] == 1) {
        if (fread(host_params, sizeof(float), n, f) != n) { fprintf(stderr, "[paged_infer] truncated checkpoint\n"); goto out; }
    } else {
        for (int k = 0; k < NUM_PARAMETER_TENSORS; k++) {
            const int t = kV2Order[k];
            float* dst = host_params + off[t];
            if (k < CKPT_V2_NBF16) {
                /* read the bf16 halves into the upper half of the tensor's
                 * own fp32 slot, then widen front to back (never overtakes) */
                unsigned short* src = (unsigned short*)(dst + s[t]) - s[t];
                if (fread(src, 2, s[t], f) != s[t]) { fprintf(stderr, "[paged_infer] truncated checkpoint\n"); goto out; }
                for (size_t i = 0; i < s[t]; i++) {
                    unsigned int u = (unsigned int)src[i] << 16;
                    memcpy(dst + i, &u, 4);
                }
            } else if (fread(dst, sizeof(float), s[t], f) != s[t]) {
                fprintf(stderr, "[paged_infer] truncated checkpoint\n");
                goto out;
            }
        }
    }
    rc = 0;
out:
    fclose(f);
    return rc;
}

void gpt2_build_from_checkpoint(GPT2* model, const char* checkpoint_path) {
    GPT2Config c;
    if (gpt2_read_checkpoint(checkpoint_path, &c, NULL)) { printf("Error opening model file\n"); exit(1); }
    size_t n = gpt2_num_parameters(c);
    float* host = (float*)malloc(n * sizeof(float));
    if (!host) { printf("Out of host memory for parameters\n"); exit(1); }
    if (gpt2_read_checkpoint(checkpoint_path, &c, host)) { printf("Bad model file\n"); exit(1); }
    if (gpt2_build_from_params(model, c, host) != 0) { printf("Parameter upload failed\n"); exit(1); }
    free(host);
}

int gpt2_synthetic_params(GPT2Config c, unsigned long long seed, float* p) {
    size_t s[NUM_PARAMETER_TENSORS];
    param_sizes(c, s);
    unsigned long long st = seed ? seed : 1337;
    const float a = 0.02f * 1.7320508f; /* U(-a, a): std 0.02 */
    size_t o = 0;
    for (int t = 0; t < NUM_PARAMETER_TENSORS; t++) {
        for (size_t i = 0; i < s[t]; i++) {
            float u = 2.0f * random_f32(&st) - 1.0f; /* U(-1, 1) */
            float v;
            switch (t) {
                case 2: case 8: case 14: v = 1.0f + 0.1f * u; break;  /* LN weights */
                case 3: case 9: case 15: v = 0.05f * u; break;        /* LN biases */
                case 5: case 7: case 11: case 13: v = 0.02f * u; break; /* linear biases */
                case 1: v = 0.01f * 1.7320508f * u; break;             /* wpe */
                default: v = a * u; break;
            }
            p[o + i] = v;
        }
        o += s[t];
    }
    return 0;
}

int gpt2_build_synthetic(GPT2* model, GPT2Config c, unsigned long long seed) {
    size_t n = gpt2_num_parameters(c);
    float* host = (float*)malloc(n * sizeof(float));
    if (!host) return 1;
    gpt2_synthetic_params(c, seed, host);
    int rc = gpt2_build_from_params(model, c, host);
    free(host);
    return rc;
}

int gpt2_write_checkpoint_ex(const char* path, GPT2Config c, const float* host_params, int version) {
    if (version != 1 && version != 2) return 1;
    FILE* f = fopen(path, "wb");
    if (!f) return 1;
    int hdr[256];
    memset(hdr, 0, sizeof(hdr));
    hdr[0] = 20240326; hdr[1] = version; hdr[2] = c.max_seq_len; hdr[3] = c.vocab_size;
    hdr[4] = c.num_layers; hdr[5] = c.num_heads; hdr[6] = c.channels;
    size_t s[NUM_PARAMETER_TENSORS], off[NUM_PARAMETER_TENSORS], n = 0;
    param_sizes(c, s);
    for (int t = 0; t < NUM_PARAMETER_TENSORS; t++) { off[t] = n; n += s[t]; }
    int ok = fwrite(hdr, sizeof(int), 256, f) == 256;
    if (version == 1) {
        ok = ok && fwrite(host_params, sizeof(float), n, f) == n;
    } else {
        unsigned short buf[4096];
        for (int k = 0; k < NUM_PARAMETER_TENSORS && ok; k++) {
            const int t = kV2Order[k];
            const float* src = host_params + off[t];
            if (k >= CKPT_V2_NBF16) { ok = fwrite(src, sizeof(float), s[t], f) == s[t]; continue; }
            for (size_t i = 0; i < s[t] && ok; i += 4096) { /* torch .to(bfloat16): round to nearest even */
                const size_t m = s[t] - i < 4096 ? s[t] - i : 4096;
                for (size_t j = 0; j < m; j++) buf[j] = f32_to_bf16_rne(src[i + j]);
                ok = fwrite(buf, 2, m, f) == m;
            }
        }
    }
    fclose(f);
    return ok ? 0 : 1;
}

int gpt2_write_checkpoint(const char* path, GPT2Config c, const float* host_params) {
    return gpt2_write_checkpoint_ex(path, c, host_params, 1);
}

/* ------------------------------------------------------------------------ */
/* tokenizer (paged_infer.c:852-928): the decode-only byte table written by
 * train_gpt2.py:350-363 (header magic 20240328, version 1, vocab size; then
 * per token a length byte and the bytes)                                    */
/* ------------------------------------------------------------------------ */
void safe_printf(const char* piece) {
    if (piece == NULL || piece[0] == '\0') return;
    if (piece[1] == '\0') { /* a lone byte: printable or whitespace only */
        unsigned char b = (unsigned char)piece[0];
        if (!(isprint(b) || isspace(b))) return;
    }
    printf("%s", piece);
}

static void tokenizer_release(Tokenizer* tk, uint32_t n) {
    for (uint32_t i = 0; i < n; i++) free(tk->token_table[i]);
    free(tk->token_table);
    tk->token_table = NULL;
}

void tokenizer_init(Tokenizer* tokenizer, const char* filename) {
    tokenizer->init_ok = 0;
    tokenizer->vocab_size = 0;
    tokenizer->token_table = NULL;
    FILE* f = fopen(filename, "rb");
    if (!f) {
        printf("---\nWARNING: Failed to open the tokenizer file %s\n---\n", filename);
        return;
    }
    uint32_t hdr[256];
    if (fread(hdr, sizeof(uint32_t), 256, f) != 256 || hdr[0] != 20240328 || hdr[1] != 1) {
        fprintf(stderr, "[paged_infer] bad tokenizer file %s\n", filename);
        fclose(f);
        return;
    }
    const uint32_t n = hdr[2];
    tokenizer->token_table = (char**)calloc(n ? n : 1, sizeof(char*));
    if (!tokenizer->token_table) { fclose(f); return; }
    for (uint32_t i = 0; i < n; i++) {
        unsigned char len;
        char* piece = NULL;
        if (fread(&len, 1, 1, f) != 1 || len == 0 || !(piece = (char*)malloc(len + 1u)) ||
            fread(piece, 1, len, f) != len) {
            fprintf(stderr, "[paged_infer] truncated tokenizer file %s\n", filename);
            free(piece);
            tokenizer_release(tokenizer, i);
            fclose(f);
            return;
        }
        piece[len] = '\0';
        tokenizer->token_table[i] = piece;
    }
    fclose(f);
    tokenizer->vocab_size = n;
    tokenizer->init_ok = 1;
}

const char* tokenizer_decode(Tokenizer* tokenizer, uint32_t token_id) {
    if (!tokenizer->init_ok) return NULL;
    if (token_id >= tokenizer->vocab_size) {
        printf("invalid token id %u!\n", token_id);
        return NULL;
    }
    return tokenizer->token_table[token_id];
}

void tokenizer_free(Tokenizer* tokenizer) {
    if (tokenizer->init_ok) tokenizer_release(tokenizer, tokenizer->vocab_size);
    tokenizer->init_ok = 0;
}

/* paged_infer.c:930-935 */
void print_generated_sequence(int* tokens, int B, int T) {
    for (int i = 0; i < B * T; i++) {
        printf("%d ", tokens[i]);
        if ((i + 1) % T == 0) printf("\n");
    }
}


/* ------------------------------------------------------------------------ */
/* decode engine                                                            */
/* ------------------------------------------------------------------------ */
/* One batched decode step = embed, then per layer QKV(+LN1, +KV append) ->
 * paged attention -> attproj(+residual) -> fc(+LN2, +GELU) ->
 * fcproj(+residual), then logits(+LNf) and the token choice: 5 launches per
 * layer + 3, replayed as one hipGraph (reference gpt2_forward,
 * paged_infer.c:575-729, for one new token per sequence). */

/* manager page index -> pool slot (page_map_create) */
typedef struct {
    HpaKVPool* pool;
    int* map;
} PageView;

/* the end-of-step gather of a sequence-sharded decode (gpt2_decode_shard) */
typedef struct {
    int nranks, rank, root;
    int* rows;        /* [nranks] sequences per rank, rank order */
    size_t* bytes;    /* [nranks] bytes per rank of the current gather */
    void* stream;     /* communication stream */
    float* send[2];   /* double-buffered copies of this rank's logits [B][V] */
    float* recv[2];   /* root: [sum rows][V] */
    int* send_ids[2];
    int* recv_ids[2];
    unsigned* d_seq;  /* device word: gathers whose send copy is done (compute stream); NULL where
                         the device has no stream value ops: ev_ready then */
    void* ev_ready[2];
    unsigned seq;     /* gathers posted */
    void* ev_done[2]; /* gather from buffer k done (comm stream) */
    int k, last, pending[2];
} DecShard;

struct GPT2Decode {
    int B, P, max_ctx, max_pages, Mp;
    HpaKVPool pool;
    BlockManager* bm;
    int own_bm;
    int bt_stride;
    int* d_bt;        /* [max_prompts][bt_stride] device mirror of bm->block_table (pool slots) */
    int* d_pos;       /* [B] */
    int* d_tokens;    /* [B] */
    int* d_next;      /* [B] */
    int* h_pos;       /* host mirror of d_pos */
    char* h_evicted;  /* [B] sequences paged out by the LRU policy since the last query */
    /* pinned staging, double-buffered: a buffer is rewritten only after the
     * event recorded behind its previous upload has completed (no stream sync) */
    int* h_tok[2];
    void* ev_tok[2];
    int tok_k;
    int* h_bt[2];
    void* ev_bt[2];
    int bt_k;
    int* h_next;      /* pinned readback of the next ids */
    PageView pv;
    float* d_q;       /* [B][C] row-major */
    float* d_logits;  /* [B][V] */
    /* frag-layout activations [Mp][*] (padded rows stay zero) and LN statistics */
    float *res, *res2, *att, *fch, *st1, *st2, *part;
    float* sk_slab;   /* stream-K logits workspace (hpa_logits_kernel == 6), else NULL */
    int* sk_cnt;
    size_t sk_cnt_n;
    float* ring_slab; /* K-split workspace of the ring qkv / fc (C >= 1024, fp32), else NULL */
    int* ring_cnt;
    size_t ring_cnt_n;
    float* d_wpack;   /* packed qkvw, attprojw, fcw, fcprojw of every layer, then wte */
    int w_bf16;       /* weights packed bf16 (hpa_pack_frag_bf16; offsets in elements) */
    size_t wpack_off[5]; /* per-layer offsets (0..3) and wte offset (4) */
    float* d_fold;    /* LN folded into qkvw / fcw (hpa_ln_fold_pack): per layer c1, c2 of
                         qkv [3C] [3C] then fc [4C] [4C]; NULL: LN applied on the operand path */
    int fwaves[5];    /* waves per workgroup: qkv, attproj, fc, fcproj, logits */
    int frb[5];       /* 16-row blocks per workgroup, same order */
    int fct[5];       /* 16-column tiles per workgroup, same order */
    int attn_splits;  /* context ranges per (sequence, head) of the decode attention */
    int attn_waves;   /* waves per attention workgroup (hpa_attn_pick_waves of the global batch) */
    void* d_attn_ws;  /* split records + counters (hpa_attn_ws_bytes at HPA_ATTN_MAX_SPLITS) */
    size_t attn_ws_bytes;
    int sample;       /* 0: greedy argmax; 1: multinomial with per-sequence xorshift */
    unsigned long long* d_rng; /* [B] sampler states */
    /* prefill workspace (gpt2_decode_prefill), rows R = sum of lengths, grown on demand */
    int pf_cap;
    float *pf_res, *pf_res2, *pf_att, *pf_fch, *pf_st1, *pf_st2, *pf_q;
    int *pf_tok, *pf_pos, *pf_seq, *pf_start, *pf_last, *h_pf;
    int use_graph;
    void* graph;
    void* prof_ev[2];  /* eager profiling: events around every attention launch */
    int profiling;
    double prof_ms;
    long prof_launches;
    DecShard* shard;
    /* persistent layer (hpa_decode_layer): one launch per layer */
    int pl_want;      /* gpt2_decode_set_layer_kernel: 0 off, 1 auto, 2 full, 3 chain, 4 chain with wide units,
                         5 chain form 6 (12-wave multi-tile units), 6 chain form 8 (streamed-weight
                         units, C = 768 / 1024 / 1280 / 1600) */
    int pl_on;        /* in use: 0 five launches, 1 full persistent layer, 2 attention launch + chain,
                         3 attention launch + chain of wide units (hpa_layer.hip NWU = pl_nwu),
                         4 attention launch + the bf16-weight chain (hpa_chain_b16.hip) */
    int pl_wform;     /* wide-unit form of the chain (HpaLayerArgs.chain_only 2..6, 8), else 1 */
    int pl_splits;
    int pl_global_B;  /* gpt2_decode_set_global_batch: the batch the picks follow (<= 64); else 0 */
    float* pl_rec;
    float* pl_slab;   /* [pl_slab_n] */
    size_t pl_slab_n;
    int* pl_ctr;      /* the step's error word (DEC_ERR_INTS), then [L][pl_ctr_ints]; zeroed at the start of
                         every step */
    size_t pl_ctr_ints;
    /* pipelined halves (hpa_decode_pipe, pl_on 5): the per-layer operand
     * table on the device, the fcproj partials, the GEMM role's CUs */
    HpaPipeLayer* d_pipe_lay;
    float* pipe_slab;
    size_t pipe_slab_n;
    int pipe_g;
    /* gpt2_forward: token at every cached position [B][max_ctx] and, when it
     * fits, the logits of every position [B][max_ctx][V] (managed) */
    int* h_hist;
    float* pos_logits;
    /* gpt2_decode_step_traced: the residual stream entering every layer and
     * the final one, row-major [L+1][B][C], written during that one step */
    float* trace_x;
};

/* the manager's page index -> pool slot: a fixed pseudo-random permutation,
 * so that whatever order pages are allocated in (first-fit hands each
 * sequence a contiguous run) the K/V streams of concurrent workgroups spread
 * over the HBM channels instead of walking them in lockstep at a
 * power-of-two stride (measured: attention 68.5 us with contiguous runs of
 * 64 pages vs 62.5 us scattered, config 2).  Small page tiles (1 KiB per
 * head: bf16, page 8) stream better with 16 consecutive pages kept together
 * (config 5: 0.844 of 8 TB/s grouped by 16, 0.839 by 4, 0.833 single pages;
 * config 2: 0.813 single, 0.806 by 4, 0.787 by 16). */
static int* page_map_create(int n, int G) {
    int* map = (int*)malloc((size_t)n * sizeof(int));
    if (!map) return NULL;
    const int ng = n / G; /* groups of G consecutive pages move together; a tail stays in place */
    for (int i = 0; i < n; i++) map[i] = i;
    unsigned long long st = 0x9E3779B97F4A7C15ull;
    for (int i = ng - 1; i > 0; i--) { /* Fisher-Yates over groups with the reference's xorshift */
        const int j = (int)(random_u32(&st) % (unsigned)(i + 1));
        for (int k = 0; k < G; k++) {
            const int t = map[i * G + k];
            map[i * G + k] = map[j * G + k];
            map[j * G + k] = t;
        }
    }
    return map;
}

/* the pool view backend: page payload pointers are layer-0 tiles in HBM */
static void* pool_view_alloc(void* ctx, int page, int kv, size_t bytes) {
    (void)bytes;
    PageView* v = (PageView*)ctx;
    if (page < 0 || page >= v->pool->num_pages) return NULL;
    return hpa_pool_tile(v->pool, 0, v->map[page], kv, 0);
}
static void pool_view_release(void* ctx, int page, int kv, void* p) {
    (void)ctx; (void)page; (void)kv; (void)p;
}

static void dec_prefill_free(GPT2Decode* d) {
    hpa_free(d->pf_res); hpa_free(d->pf_res2); hpa_free(d->pf_att); hpa_free(d->pf_fch);
    hpa_free(d->pf_st1); hpa_free(d->pf_st2); hpa_free(d->pf_q);
    hpa_free(d->pf_tok); hpa_free(d->pf_pos); hpa_free(d->pf_seq); hpa_free(d->pf_start); hpa_free(d->pf_last);
    free(d->h_pf);
    d->pf_res = d->pf_res2 = d->pf_att = d->pf_fch = d->pf_st1 = d->pf_st2 = d->pf_q = NULL;
    d->pf_tok = d->pf_pos = d->pf_seq = d->pf_start = d->pf_last = d->h_pf = NULL;
    d->pf_cap = 0;
}

static void dec_shard_free(GPT2Decode* d) {
    DecShard* s = d->shard;
    if (!s) return;
    if (s->stream) {
        void* prev = hpa_get_stream();
        hpa_set_stream(s->stream);
        hpa_synchronize();
        hpa_set_stream(prev);
    }
    for (int k = 0; k < 2; k++) {
        hpa_free(s->send[k]); hpa_free(s->recv[k]); hpa_free(s->send_ids[k]); hpa_free(s->recv_ids[k]);
        hpa_event_destroy(s->ev_done[k]);
        hpa_event_destroy(s->ev_ready[k]);
    }
    hpa_free(s->d_seq);
    hpa_stream_destroy(s->stream);
    free(s->rows);
    free(s->bytes);
    free(s);
    d->shard = NULL;
}

/* every teardown and error path: a caller-owned manager gets its pages back
 * and its default backend, so it never keeps pointers into the freed pool */
static void dec_free(GPT2Decode* d) {
    if (!d) return;
    hpa_synchronize();
    if (!d->own_bm && d->bm && d->pv.map) {
        for (int p = 0; p < d->bm->max_prompts; p++)
            if (d->bm->prompt_block_count[p]) free_blocks_for_prompt(d->bm, p);
        bm_set_backend(d->bm, NULL);
    }
    dec_shard_free(d);
    dec_prefill_free(d);
    for (int k = 0; k < 2; k++) {
        hpa_event_destroy(d->prof_ev[k]);
        hpa_event_destroy(d->ev_tok[k]);
        hpa_event_destroy(d->ev_bt[k]);
        hpa_host_free(d->h_tok[k]);
        hpa_host_free(d->h_bt[k]);
    }
    if (d->graph) hpa_graph_destroy(d->graph);
    hpa_pool_destroy(&d->pool);
    hpa_free(d->d_bt); hpa_free(d->d_pos); hpa_free(d->d_tokens); hpa_free(d->d_next);
    hpa_free(d->d_q); hpa_free(d->d_logits);
    hpa_free(d->res); hpa_free(d->res2); hpa_free(d->att); hpa_free(d->fch);
    hpa_free(d->st1); hpa_free(d->st2); hpa_free(d->part);
    hpa_free(d->sk_slab); hpa_free(d->sk_cnt);
    hpa_free(d->ring_slab); hpa_free(d->ring_cnt);
    hpa_free(d->d_wpack);
    hpa_free(d->d_fold);
    hpa_free(d->d_attn_ws);
    hpa_free(d->pl_rec); hpa_free(d->pl_slab); hpa_free(d->pl_ctr);
    hpa_free(d->d_pipe_lay); hpa_free(d->pipe_slab);
    hpa_free(d->d_rng);
    hpa_free(d->pos_logits);
    hpa_host_free(d->h_next);
    free(d->pv.map);
    free(d->h_pos);
    free(d->h_evicted);
    free(d->h_hist);
    if (d->own_bm) destroy_block_manager(d->bm);
    free(d);
}

void gpt2_decode_free(GPT2* model) {
    if (model && model->decode) {
        dec_free(model->decode);
        model->decode = NULL;
    }
}

/* frag-packed weights (packed once; the weights stay also in checkpoint
 * layout for the embedding gather and the reference API), frag-layout
 * activations, LN statistics, launch shapes */
static int dec_init_weights(GPT2* model, GPT2Decode* d) {
    const GPT2Config c = model->config;
    const int B = d->B, C = c.channels, L = c.num_layers, V = c.vocab_size;
    const ParameterTensors* w = &model->params;
    const size_t e_qkv = hpa_frag_elems(3 * C, C), e_ap = hpa_frag_elems(C, C);
    const size_t e_fc = hpa_frag_elems(4 * C, C), e_fp = hpa_frag_elems(C, 4 * C);
    const size_t e_layer = e_qkv + e_ap + e_fc + e_fp;
    d->wpack_off[0] = 0;
    d->wpack_off[1] = e_qkv;
    d->wpack_off[2] = e_qkv + e_ap;
    d->wpack_off[3] = e_qkv + e_ap + e_fc;
    d->wpack_off[4] = e_layer * L; /* wte */
    const size_t total = d->wpack_off[4] + hpa_frag_elems(V, C);
    d->d_wpack = (float*)hpa_malloc(total * (d->w_bf16 ? 2 : 4));
    if (!d->d_wpack) return 1;
    if (d->w_bf16) { /* bf16 weights: same element offsets, 2 bytes each; LN on the operand path */
        unsigned short* b16 = (unsigned short*)d->d_wpack;
        for (int l = 0; l < L; l++) {
            unsigned short* base = b16 + e_layer * l;
            const size_t lc = (size_t)l * C;
            if (hpa_pack_frag_bf16(w->qkvw + lc * 3 * C, 3 * C, C, C, base + d->wpack_off[0]) ||
                hpa_pack_frag_bf16(w->attprojw + lc * C, C, C, C, base + d->wpack_off[1]) ||
                hpa_pack_frag_bf16(w->fcw + lc * 4 * C, 4 * C, C, C, base + d->wpack_off[2]) ||
                hpa_pack_frag_bf16(w->fcprojw + lc * 4 * C, C, 4 * C, 4 * C, base + d->wpack_off[3]))
                return 1;
        }
        if (hpa_pack_frag_bf16(w->wte, V, C, C, b16 + d->wpack_off[4])) return 1;
        for (int i = 0; i < 5; i++) d->fwaves[i] = d->frb[i] = d->fct[i] = 0; /* by (M, N, K) in the library */
        return 0;
    }
    /* LN1 / LN2 folded into the qkv / fc weights: the GEMM then starts on x
     * as it stands and the row statistics are needed only in its epilogue */
    d->d_fold = (float*)hpa_malloc((size_t)L * 14 * C * 4);
    if (!d->d_fold) return 1;
    for (int l = 0; l < L; l++) {
        float* base = d->d_wpack + e_layer * l;
        const size_t lc = (size_t)l * C;
        float* fl = d->d_fold + (size_t)l * 14 * C;
        if (hpa_ln_fold_pack(w->qkvw + lc * 3 * C, 3 * C, C, w->ln1w + lc, w->ln1b + lc, w->qkvb + 3 * lc,
                             base + d->wpack_off[0], fl, fl + 3 * C) ||
            hpa_pack_frag(w->attprojw + lc * C, C, C, C, base + d->wpack_off[1]) ||
            hpa_ln_fold_pack(w->fcw + lc * 4 * C, 4 * C, C, w->ln2w + lc, w->ln2b + lc, w->fcb + 4 * lc,
                             base + d->wpack_off[2], fl + 6 * C, fl + 10 * C) ||
            hpa_pack_frag(w->fcprojw + lc * 4 * C, C, 4 * C, 4 * C, base + d->wpack_off[3]))
            return 1;
    }
    if (hpa_pack_frag(w->wte, V, C, C, d->d_wpack + d->wpack_off[4])) return 1;
    const int shp[5][2] = {{3 * C, C}, {C, C}, {4 * C, C}, {C, 4 * C}, {V, C}};
    for (int i = 0; i < 5; i++) {
        int pk[3];
        hpa_fused_pick(B, shp[i][0], shp[i][1], pk);
        d->fwaves[i] = pk[0];
        d->frb[i] = pk[1];
        d->fct[i] = pk[2];
    }
    return 0;
}

/* the batch every shape pick follows: the global batch a shard was told
 * (gpt2_decode_set_global_batch, so its rows equal the unsharded engine's
 * bit for bit) where the unsharded engine has a persistent layer form for it
 * -- <= 64 rows on fp32 weights (chain forms 6 / 8), <= 256 on bf16 weights
 * (the bf16 chain) -- above that the unsharded engine runs five launches per
 * layer and a shard's own B is the better guide; else the
 * engine's own B (a shard then computes what a single-GPU engine of its rows
 * computes) */
static int dec_pick_B(const GPT2Decode* d) {
    const int lim = d->w_bf16 ? 256 : 64;
    return d->pl_global_B > 0 && d->pl_global_B <= lim ? d->pl_global_B : d->B;
}

/* ints after the per-layer counter blocks: the step's own error word (zeroed
 * with the counters, so one timed-out wait cannot make later steps bail out;
 * the first code of any step also sticks in d_next[B] for gpt2_decode_status) */
#define DEC_ERR_INTS 32

/* the attention's context ranges and their workspace (zeroed whenever the
 * split count changes: the counters sit after the records of that count) */
static int dec_set_splits(GPT2Decode* d, int splits) {
    if (splits < 1 || splits > HPA_ATTN_MAX_SPLITS) return 1;
    if (splits > 1 && !d->d_attn_ws) {
        d->attn_ws_bytes = hpa_attn_ws_bytes(d->B, d->pool.num_heads, HPA_ATTN_MAX_SPLITS);
        d->d_attn_ws = hpa_malloc(d->attn_ws_bytes);
        if (!d->d_attn_ws) return 1;
    }
    if (d->d_attn_ws && hpa_memset_async(d->d_attn_ws, 0, d->attn_ws_bytes)) return 1;
    d->attn_splits = splits;
    {   /* the waves follow the batch the picks follow (sharded: the global one) */
        int ncu = 0;
        hpa_device_info(NULL, 0, &ncu, NULL);
        d->attn_waves = hpa_attn_pick_waves(dec_pick_B(d), d->pool.num_heads, splits, ncu);
        /* bf16 pools with >= 8 (sequence, head, range) workgroups per CU: 8 waves (a workgroup
         * moves half the bytes per tile; config 5: 3.287-3.291 vs 3.298-3.305 ms per step,
         * paired runs, profiles/r5/experiments/c5_attention_waves.txt) */
        if (d->pool.dtype == HPA_BF16 && ncu > 0 &&
            (long)dec_pick_B(d) * d->pool.num_heads * splits >= 8L * ncu)
            d->attn_waves = 8;
    }
    if (d->graph) { /* recapture with the new grid */
        hpa_synchronize();
        hpa_graph_destroy(d->graph);
        d->graph = NULL;
    }
    return 0;
}

static const float* wpack_at(const GPT2Decode* d, size_t off);

/* the bf16-weight chain's workspace (hpa_chain_b16.hip: B <= 256, C = 768,
 * 12 heads): the fcproj K-part partials and the per-layer counter blocks */
static int dec_chain_b16_setup(GPT2* model, GPT2Decode* d) {
    const GPT2Config c = model->config;
    size_t sz[2];
    if (!hpa_decode_chain_b16_eligible(d->B, c.channels, c.num_heads)) return 0;
    if (hpa_decode_chain_b16_sizes(d->B, sz)) return 1;
    if (!d->pl_slab || d->pl_slab_n < sz[0]) {
        hpa_free(d->pl_slab);
        d->pl_slab_n = sz[0];
        d->pl_slab = (float*)hpa_malloc(sz[0] * sizeof(float));
    }
    if (!d->pl_ctr || d->pl_ctr_ints < sz[1]) {
        hpa_free(d->pl_ctr);
        d->pl_ctr_ints = sz[1];
        d->pl_ctr = (int*)hpa_malloc((DEC_ERR_INTS + (size_t)c.num_layers * sz[1]) * sizeof(int));
    }
    if (!d->pl_slab || !d->pl_ctr) return 1;
    d->pl_on = 4;
    return 0;
}

/* the pipelined halves (pl_on 5) where hpa_decode_pipe applies: the
 * per-layer operand table (the pointers dec_layer hands chain form 6), the
 * fcproj partials, and counter blocks of at least its size */
static int dec_pipe_setup(GPT2* model, GPT2Decode* d) {
    const GPT2Config c = model->config;
    const ParameterTensors* w = &model->params;
    const int C = c.channels, L = c.num_layers;
    if (!hpa_decode_pipe_eligible(d->B, C, c.num_heads, d->pool.dtype)) return 0; /* form 6 stays */
    size_t sz[2];
    if (hpa_decode_pipe_sizes(d->B, sz)) return 1;
    if (!d->pipe_slab || d->pipe_slab_n < sz[0]) {
        hpa_free(d->pipe_slab);
        d->pipe_slab_n = sz[0];
        d->pipe_slab = (float*)hpa_malloc(sz[0] * sizeof(float));
    }
    if (d->pl_ctr_ints < sz[1]) {
        hpa_free(d->pl_ctr);
        d->pl_ctr_ints = sz[1];
        d->pl_ctr = (int*)hpa_malloc((DEC_ERR_INTS + (size_t)L * sz[1]) * sizeof(int));
    }
    if (!d->pipe_slab || !d->pl_ctr) return 1;
    HpaPipeLayer* h = (HpaPipeLayer*)calloc((size_t)L, sizeof(HpaPipeLayer));
    if (!h) return 1;
    const size_t e_layer = d->wpack_off[3] + hpa_frag_elems(C, 4 * C);
    for (int l = 0; l < L; l++) {
        const size_t lc = (size_t)l * C;
        h[l].w_ap = wpack_at(d, e_layer * l + d->wpack_off[1]);
        h[l].b_ap = w->attprojb + lc;
        h[l].w_fc = wpack_at(d, e_layer * l + d->wpack_off[2]);
        h[l].fc_c1 = d->d_fold + 14 * lc + 6 * C;
        h[l].fc_c2 = h[l].fc_c1 + 4 * C;
        h[l].w_fp = wpack_at(d, e_layer * l + d->wpack_off[3]);
        h[l].b_fp = w->fcprojb + lc;
        if (l + 1 < L) {
            h[l].w_qkv = wpack_at(d, e_layer * (l + 1) + d->wpack_off[0]);
            h[l].qkv_c1 = d->d_fold + 14 * (lc + C);
            h[l].qkv_c2 = h[l].qkv_c1 + 3 * C;
        }
    }
    if (!d->d_pipe_lay) d->d_pipe_lay = (HpaPipeLayer*)hpa_malloc((size_t)L * sizeof(HpaPipeLayer));
    const int rc = !d->d_pipe_lay || hpa_memcpy(d->d_pipe_lay, h, (size_t)L * sizeof(HpaPipeLayer));
    free(h);
    if (rc) return 1;
    d->pl_on = 5;
    return 0;
}

static int dec_layer_setup(GPT2* model, GPT2Decode* d) {
    const GPT2Config c = model->config;
    d->pl_on = 0;
    /* bf16 weights (BASELINE config 5): the bf16 chain (hpa_chain_b16.hip),
     * B <= 256, in place of four GEMM launches per layer */
    if (d->pl_want && d->w_bf16) return dec_chain_b16_setup(model, d);
    if (!d->pl_want || d->w_bf16 || !d->d_fold) return 0;
    const int Bg = dec_pick_B(d); /* the batch the picks follow */
    if (Bg > 64) return 0;
    /* the loop's form (gpt2_decode_set_layer_kernel).  1 = auto, the form
     * measured fastest (round 4, profiles/r4/forms.txt): chain form 6 at C =
     * 768 (B = 64 / 8: 1.1106 / 0.4334 ms per step against the round-3 wide
     * units' 1.1476 / 0.4510), chain form 8 at C >= 1024 (GPT-2 XL: 9.91 vs
     * 10.29 ms for five launches), else the chain of 4-wave units.
     * mode: 1 the full persistent layer, 2 the attention launch + the chain
     * of 4-wave units, 3 the attention launch + the chain form pl_wform */
    const int Rg = (Bg + 15) / 16;
    int mode = 2;
    d->pl_wform = 1;
    switch (d->pl_want) {
        case 2: mode = 1; break;
        case 3: break;
        case 4: /* round 3's wide units, widths by row blocks: chain_only 2..5 */
            if (c.num_heads == 12) { mode = 3; d->pl_wform = 1 + Rg; }
            break;
        case 5: /* form 6 (12-wave multi-tile units) */
            if (c.num_heads == 12) { mode = 3; d->pl_wform = 6; }
            break;
        case 6: mode = 3; d->pl_wform = 8; break; /* form 8: streamed-weight units (C = 768, 1600) */
        case 7: /* the pipelined halves over chain form 6's units (form 6 where it does not apply) */
            if (c.num_heads == 12) { mode = 3; d->pl_wform = 6; }
            break;
        default: /* auto */
            if (c.num_heads == 12) { mode = 3; d->pl_wform = 6; }
            else if (c.channels >= 1024) { mode = 3; d->pl_wform = 8; }
            break;
    }
#ifndef HPA_AB
    /* the full persistent layer (2) and the wide-unit chains (4) measured
     * slower than the forms picked here: A/B builds only (hpa_build_flags) */
    if (mode == 1 || (mode == 3 && d->pl_wform >= 2 && d->pl_wform <= 5)) return 0;
#endif
    int splits = hpa_decode_layer_pick_splits(Bg, c.num_heads, d->max_ctx);
#ifdef HPA_AB
    const char* env = getenv("HPA_LAYER_SPLITS"); /* the full persistent layer's attention ranges */
    if (env && atoi(env) > 0) splits = atoi(env);
#endif
    if (mode >= 2) splits = 1; /* no attention phase: no split records */
    if (d->pl_wform >= 6 ? !hpa_decode_chain_eligible(d->B, c.channels, c.num_heads, d->pl_wform)
                         : !hpa_decode_layer_eligible(d->B, c.channels, c.num_heads, splits))
        return 0;
    size_t sz[3];
    if (hpa_decode_layer_sizes(d->B, c.channels, c.num_heads, splits, sz)) return 1;
    if (!d->pl_rec || d->pl_splits != splits) { /* records depend on the split count */
        hpa_free(d->pl_rec);
        d->pl_rec = (float*)hpa_malloc(sz[0] * sizeof(float));
    }
    if (!d->pl_slab) {
        d->pl_slab_n = sz[1];
        d->pl_slab = (float*)hpa_malloc(sz[1] * sizeof(float));
    }
    if (!d->pl_ctr) {
        d->pl_ctr_ints = sz[2];
        d->pl_ctr = (int*)hpa_malloc((DEC_ERR_INTS + (size_t)c.num_layers * sz[2]) * sizeof(int));
    }
    if (!d->pl_rec || !d->pl_slab || !d->pl_ctr) return 1;
    d->pl_splits = splits;
    d->pl_on = mode;
    if (d->pl_want == 7 && mode == 3 && d->pl_wform == 6) return dec_pipe_setup(model, d);
    return 0;
}

/* layer l's bf16 chain: attproj(l) .. fcproj(l), qkv(l+1) (pl_on 4) */
static int dec_layer_b16(GPT2* model, int l) {
    GPT2Decode* d = model->decode;
    const GPT2Config c = model->config;
    const int C = c.channels, L = c.num_layers;
    const ParameterTensors* w = &model->params;
    const size_t lc = (size_t)l * C;
    const size_t e_layer = d->wpack_off[3] + hpa_frag_elems(C, 4 * C);
    HpaChainB16Args a;
    memset(&a, 0, sizeof(a));
    a.B = d->B;
    a.layer = l;
    a.last = l + 1 == L;
    a.pool = &d->pool;
    a.block_table = d->d_bt;
    a.bt_stride = d->bt_stride;
    a.pos = d->d_pos;
    a.att = d->att;
    a.res = d->res;
    a.res2 = d->res2;
    a.fch = d->fch;
    a.w_ap = wpack_at(d, e_layer * l + d->wpack_off[1]);
    a.b_ap = w->attprojb + lc;
    a.ln2_w = w->ln2w + lc;
    a.ln2_b = w->ln2b + lc;
    a.w_fc = wpack_at(d, e_layer * l + d->wpack_off[2]);
    a.b_fc = w->fcb + 4 * lc;
    a.w_fp = wpack_at(d, e_layer * l + d->wpack_off[3]);
    a.b_fp = w->fcprojb + lc;
    if (!a.last) {
        a.w_qkv = wpack_at(d, e_layer * (l + 1) + d->wpack_off[0]);
        a.b_qkv = w->qkvb + 3 * (lc + C);
        a.ln1_w = w->ln1w + lc + C;
        a.ln1_b = w->ln1b + lc + C;
        a.q_out = d->d_q; /* every read of q(l) was the attention launch's, before this one */
    }
    a.stats_out = a.last ? d->st1 : NULL; /* LNf statistics for the logits */
    a.stats_mp = d->Mp;
    a.slab = d->pl_slab;
    a.counters = d->pl_ctr + DEC_ERR_INTS + (size_t)l * d->pl_ctr_ints;
    a.err = d->pl_ctr;
    a.err_sticky = d->d_next + d->B;
    return hpa_decode_chain_b16(&a);
}

/* layer l of the persistent path: attention(l) .. fcproj(l), qkv(l+1) */
static int dec_layer(GPT2* model, int l) {
    GPT2Decode* d = model->decode;
    const GPT2Config c = model->config;
    const int C = c.channels, L = c.num_layers;
    const ParameterTensors* w = &model->params;
    const size_t lc = (size_t)l * C;
    const size_t e_layer = d->wpack_off[3] + hpa_frag_elems(C, 4 * C);
    if (d->pl_on == 4) return dec_layer_b16(model, l);
    HpaLayerArgs a;
    memset(&a, 0, sizeof(a));
    a.B = d->B;
    a.C = C;
    a.num_heads = c.num_heads;
    a.splits = d->pl_splits;
    a.last = l + 1 == L;
    a.chain_only = d->pl_on == 3 || d->pl_on == 5 ? d->pl_wform : d->pl_on == 2;
    a.pool = &d->pool;
    a.layer = l;
    a.block_table = d->d_bt;
    a.bt_stride = d->bt_stride;
    a.pos = d->d_pos;
    a.q = d->d_q;
    a.att = d->att;
    a.res = d->res;
    a.res2 = d->res2;
    a.fch = d->fch;
    a.w_ap = wpack_at(d, e_layer * l + d->wpack_off[1]);
    a.b_ap = w->attprojb + lc;
    a.w_fc = wpack_at(d, e_layer * l + d->wpack_off[2]);
    a.fc_c1 = d->d_fold + 14 * lc + 6 * C;
    a.fc_c2 = a.fc_c1 + 4 * C;
    a.w_fp = wpack_at(d, e_layer * l + d->wpack_off[3]);
    a.b_fp = w->fcprojb + lc;
    if (!a.last) {
        a.w_qkv = wpack_at(d, e_layer * (l + 1) + d->wpack_off[0]);
        a.qkv_c1 = d->d_fold + 14 * (lc + C);
        a.qkv_c2 = a.qkv_c1 + 3 * C;
        a.q_out = d->d_q; /* every read of q(l) is done before the first qkv(l+1) store */
    }
    a.stats_out = a.last ? d->st1 : NULL; /* LNf statistics for the logits */
    a.stats_mp = d->Mp;
    a.rec = d->pl_rec;
    a.slab = d->pl_slab;
    a.counters = d->pl_ctr + DEC_ERR_INTS + (size_t)l * d->pl_ctr_ints;
    a.err = d->pl_ctr;                  /* this step's (zeroed with the counters) */
    a.err_sticky = d->d_next + d->B;    /* first code of any step, until gpt2_decode_status */
    return hpa_decode_layer(&a);
}

/* the in-launch arrival counters of the attention's split merge, of the
 * stream-K logits and of the K-split ring GEMMs back to zero: every completed launch leaves them zero, a
 * launch that failed part-way may not.  Called before a graph is
 * recaptured and after a reported failure. */
static int dec_rezero(GPT2Decode* d) {
    int rc = 0;
    if (d->d_attn_ws) rc |= hpa_memset_async(d->d_attn_ws, 0, d->attn_ws_bytes);
    if (d->sk_cnt && d->sk_cnt_n) rc |= hpa_memset_async(d->sk_cnt, 0, d->sk_cnt_n * sizeof(int));
    if (d->ring_cnt && d->ring_cnt_n) rc |= hpa_memset_async(d->ring_cnt, 0, d->ring_cnt_n * sizeof(int));
    return rc;
}

int gpt2_decode_init(GPT2* model, int B, int page_size, int max_ctx) {
    return gpt2_decode_init_ex(model, B, page_size, max_ctx, HPA_F32);
}

int gpt2_decode_init_ex(GPT2* model, int B, int page_size, int max_ctx, int kv_dtype) {
    return gpt2_decode_init_w(model, B, page_size, max_ctx, kv_dtype, HPA_F32);
}

int gpt2_decode_init_w(GPT2* model, int B, int page_size, int max_ctx, int kv_dtype, int w_dtype) {
    ensure_device();
    if (kv_dtype != HPA_F32 && kv_dtype != HPA_BF16) {
        fprintf(stderr, "[paged_infer] kv dtype must be HPA_F32 or HPA_BF16\n");
        return 1;
    }
    if (w_dtype != HPA_F32 && w_dtype != HPA_BF16) {
        fprintf(stderr, "[paged_infer] weight dtype must be HPA_F32 or HPA_BF16\n");
        return 1;
    }
    if (!model->params_memory) { fprintf(stderr, "[paged_infer] model not built\n"); return 1; }
    const GPT2Config c = model->config;
    if (c.channels != c.num_heads * 64) {
        fprintf(stderr, "[paged_infer] decode engine needs head_size 64 (C = 64*NH)\n");
        return 1;
    }
    if (B <= 0 || max_ctx <= 0 || max_ctx > c.max_seq_len) {
        fprintf(stderr, "[paged_infer] bad batch / context (max_ctx <= max_seq_len)\n");
        return 1;
    }
    gpt2_decode_free(model);
    GPT2Decode* d = (GPT2Decode*)calloc(1, sizeof(GPT2Decode));
    if (!d) return 1;
    if (model->manager) {
        d->bm = model->manager;
        page_size = d->bm->block_size;
        if (d->bm->max_prompts < B || d->bm->C != c.channels) {
            fprintf(stderr, "[paged_infer] model->manager too small for this batch\n");
            free(d);
            return 1;
        }
    }
    if (page_size != 8 && page_size != 16 && page_size != 32 && page_size != 64) {
        fprintf(stderr, "[paged_infer] page size must be 8, 16, 32 or 64\n");
        free(d);
        return 1;
    }
    d->B = B;
    d->P = page_size;
    d->max_ctx = max_ctx;
    d->max_pages = (max_ctx + page_size - 1) / page_size;
    d->Mp = (B + 15) / 16 * 16;
    int num_pages;
    if (model->manager) {
        num_pages = d->bm->max_blocks;
    } else {
        num_pages = B * d->max_pages;
        d->bm = create_block_manager_ex(c.channels, B, num_pages, page_size, d->max_pages);
        if (!d->bm) { free(d); return 1; }
        d->own_bm = 1;
    }
    if (d->bm->max_blocks_per_prompt < d->max_pages) {
        fprintf(stderr, "[paged_infer] manager's per-prompt page list shorter than max_ctx\n");
        dec_free(d);
        return 1;
    }
    if (hpa_pool_create(&d->pool, c.num_layers, c.num_heads, 64, page_size, num_pages, kv_dtype, 0)) {
        dec_free(d);
        return 1;
    }
    /* pages of this manager are views into the pool from now on */
    for (int p = 0; p < d->bm->max_prompts; p++)
        if (d->bm->prompt_block_count[p]) free_blocks_for_prompt(d->bm, p);
    d->pv.pool = &d->pool;
    {
        const size_t tile_bytes = (size_t)page_size * 64 * d->pool.elem_bytes; /* one head's K of a page */
        d->pv.map = page_map_create(num_pages, tile_bytes >= 4096 ? 1 : 16);
    }
    if (!d->pv.map) {
        dec_free(d);
        return 1;
    }
    BMPageBackend be = {pool_view_alloc, pool_view_release, &d->pv};
    bm_set_backend(d->bm, &be);
    d->bt_stride = d->bm->max_blocks_per_prompt;
    const int C = c.channels, V = c.vocab_size, ct = C / 16;
    const size_t btn = (size_t)d->bm->max_prompts * d->bt_stride, Mp = d->Mp;
    d->d_bt = (int*)hpa_malloc(btn * sizeof(int));
    d->d_pos = (int*)hpa_malloc(B * sizeof(int));
    d->d_tokens = (int*)hpa_malloc(B * sizeof(int));
    d->d_next = (int*)hpa_malloc((B + 1) * sizeof(int)); /* [B]: persistent-layer error word */
    d->h_pos = (int*)calloc(B, sizeof(int));
    d->h_evicted = (char*)calloc(B, 1);
    d->h_next = (int*)hpa_host_alloc((B + 1) * sizeof(int));
    d->d_q = (float*)hpa_malloc((size_t)B * C * 4);
    d->d_logits = (float*)hpa_malloc((size_t)B * V * 4);
    d->res = (float*)hpa_malloc(Mp * C * 4);
    d->res2 = (float*)hpa_malloc(Mp * C * 4);
    d->att = (float*)hpa_malloc(Mp * C * 4);
    d->fch = (float*)hpa_malloc(Mp * 4 * C * 4);
    d->st1 = (float*)hpa_malloc((size_t)ct * Mp * 2 * 4);
    d->st2 = (float*)hpa_malloc((size_t)ct * Mp * 2 * 4);
    d->part = (float*)hpa_malloc((size_t)((V + 15) / 16) * Mp * 2 * 4);
    int ok = d->d_bt && d->d_pos && d->d_tokens && d->d_next && d->h_pos && d->h_evicted && d->h_next && d->d_q &&
             d->d_logits && d->res && d->res2 && d->att && d->fch && d->st1 && d->st2 && d->part;
    /* logits GEMM: the activation-resident kernel where it applies (C = 768,
     * B <= 64); stream-K where its shape limits allow (XL at B <= 64), which
     * needs a slab and zeroed counters; else the looped kernel */
    if (ok && w_dtype != HPA_BF16 && hpa_logits_kernel(B, V, C) == 6) {
        size_t nf = 0, nc = 0;
        ok = hpa_gemm_sk_workspace(V, &nf, &nc) == 0;
        if (ok) {
            d->sk_slab = (float*)hpa_malloc(nf * sizeof(float));
            d->sk_cnt = (int*)hpa_malloc(nc * sizeof(int));
            d->sk_cnt_n = nc;
            ok = d->sk_slab && d->sk_cnt && hpa_memset_async(d->sk_cnt, 0, nc * sizeof(int)) == 0;
        }
    }
    /* the ring qkv / fc of wide layers (dec_gemm): K split in DEC_RING_QKV_PARTS /
     * DEC_RING_FC_PARTS parts over workgroups, one slab + counters for both */
    if (ok && w_dtype != HPA_BF16 && C >= 1024 && dec_ring_allowed() == 2) {
        size_t f1 = 0, c1 = 0, f2 = 0, c2 = 0;
        ok = hpa_gemm_ring_workspace(3 * C, DEC_RING_QKV_PARTS, &f1, &c1) == 0 &&
             hpa_gemm_ring_workspace(4 * C, DEC_RING_FC_PARTS, &f2, &c2) == 0;
        if (ok) {
            const size_t nf = f1 > f2 ? f1 : f2, nc = c1 > c2 ? c1 : c2;
            d->ring_slab = (float*)hpa_malloc(nf * sizeof(float));
            d->ring_cnt = (int*)hpa_malloc(nc * sizeof(int));
            d->ring_cnt_n = nc;
            ok = d->ring_slab && d->ring_cnt && hpa_memset_async(d->ring_cnt, 0, nc * sizeof(int)) == 0;
        }
    }
    for (int k = 0; k < 2 && ok; k++) {
        d->h_tok[k] = (int*)hpa_host_alloc(B * sizeof(int));
        d->h_bt[k] = (int*)hpa_host_alloc(btn * sizeof(int));
        d->ev_tok[k] = hpa_event_create_nt();
        d->ev_bt[k] = hpa_event_create_nt();
        d->prof_ev[k] = hpa_event_create();
        ok = d->h_tok[k] && d->h_bt[k] && d->ev_tok[k] && d->ev_bt[k] && d->prof_ev[k];
    }
    /* padded rows stay zero forever */
    if (!ok || hpa_memset_async(d->res, 0, Mp * C * 4) || hpa_memset_async(d->res2, 0, Mp * C * 4) ||
        hpa_memset_async(d->att, 0, Mp * C * 4) || hpa_memset_async(d->fch, 0, Mp * 4 * C * 4) ||
        hpa_memset_async(d->st1, 0, (size_t)ct * Mp * 2 * 4) || hpa_memset_async(d->st2, 0, (size_t)ct * Mp * 2 * 4)) {
        dec_free(d);
        return 1;
    }
    d->w_bf16 = w_dtype == HPA_BF16;
    int ncu = 0;
    hpa_device_info(NULL, 0, &ncu, NULL);
    if (dec_init_weights(model, d) || dec_set_splits(d, hpa_attn_pick_splits(B, c.num_heads, max_ctx, ncu))) {
        dec_free(d);
        return 1;
    }
    {
        const char* env = getenv("HPA_LAYER_KERNEL");
        d->pl_want = env && env[0] >= '0' && env[0] <= '7' ? env[0] - '0' : 1;
    }
    if (dec_layer_setup(model, d)) {
        dec_free(d);
        return 1;
    }
    for (size_t i = 0; i < btn; i++) d->h_bt[0][i] = -1;
    if (hpa_memcpy(d->d_bt, d->h_bt[0], btn * sizeof(int)) || hpa_memset_async(d->d_pos, 0, B * sizeof(int)) ||
        hpa_memset_async(d->d_next, 0, (B + 1) * sizeof(int)) ||
        hpa_memset_async(d->d_tokens, 0, B * sizeof(int)) || hpa_synchronize()) {
        dec_free(d);
        return 1;
    }
    bm_clear_dirty(d->bm);
    model->decode = d;
    return 0;
}

/* upload the block-table rows the manager changed since the last upload,
 * through the staging buffer whose previous upload is known to be done */
static int dec_sync_block_table(GPT2Decode* d) {
    BlockManager* m = d->bm;
    if (m->dirty_hi < m->dirty_lo) return 0;
    const size_t lo = (size_t)m->dirty_lo * d->bt_stride;
    const size_t n = (size_t)(m->dirty_hi - m->dirty_lo + 1) * d->bt_stride;
    const int k = d->bt_k;
    if (hpa_event_synchronize(d->ev_bt[k])) return 1;
    int* st = d->h_bt[k];
    for (size_t i = 0; i < n; i++) {
        const int v = m->block_table[lo + i];
        st[lo + i] = v >= 0 ? d->pv.map[v] : -1;
    }
    if (hpa_memcpy_async(d->d_bt + lo, st + lo, n * sizeof(int)) || hpa_event_record(d->ev_bt[k])) return 1;
    d->bt_k ^= 1;
    bm_clear_dirty(m);
    return 0;
}

/* host tokens -> d_tokens through the double-buffered pinned staging */
static int dec_upload_tokens(GPT2Decode* d, const int* tokens) {
    const int k = d->tok_k;
    if (hpa_event_synchronize(d->ev_tok[k])) return 1;
    memcpy(d->h_tok[k], tokens, d->B * sizeof(int));
    if (hpa_memcpy_async(d->d_tokens, d->h_tok[k], d->B * sizeof(int)) || hpa_event_record(d->ev_tok[k])) return 1;
    d->tok_k ^= 1;
    return 0;
}

/* pages for positions pos[b] .. pos[b]+n-1 of sequence b.  The reference
 * policy may evict a whole LRU sequence to make room (block_manager.c:104-162);
 * the evicted sequence restarts at position 0 and is reported by
 * gpt2_decode_evicted.  `busy` (nullable) marks the sequences of the current
 * call: evicting one of those fails the call. */
static int dec_grow(GPT2Decode* d, int b, int n, const int* busy, int* evicted) {
    for (;;) {
        const int need = (d->h_pos[b] + n - 1) / d->P + 1;
        if (d->bm->prompt_block_count[b] >= need) return 0;
        if (!request_block(d->bm, b)) return 1;
        const int ev = d->bm->last_evicted_prompt; /* may be b itself */
        if (ev < 0 || ev >= d->B) continue;
        if (evicted) ++*evicted;
        d->h_evicted[ev] = 1;
        d->h_pos[ev] = 0;
        if (hpa_memcpy(d->d_pos + ev, &d->h_pos[ev], sizeof(int))) return 1;
        if (busy && busy[ev]) {
            fprintf(stderr, "[paged_infer] sequence %d of this batch was evicted: pool too small\n", ev);
            return 1;
        }
    }
}

/* make sure every sequence owns the page its next token lands in.  An LRU
 * eviction (dec_grow) restarts the evicted sequence at position 0, which
 * needs a page again: repeat until a pass evicts nobody (bounded). */
static int dec_ensure_pages(GPT2Decode* d) {
    for (int pass = 0; pass <= d->B; pass++) {
        int evictions = 0;
        for (int b = 0; b < d->B; b++) {
            const int p = d->h_pos[b];
            if (p >= d->max_ctx) {
                fprintf(stderr, "[paged_infer] sequence %d is full (%d tokens)\n", b, p);
                return 1;
            }
            if (d->bm->prompt_block_count[b] >= p / d->P + 1) continue;
            if (dec_grow(d, b, 1, NULL, &evictions)) return 1;
        }
        if (!evictions) return 0;
    }
    fprintf(stderr, "[paged_infer] page pool thrashing: every pass evicts a sequence\n");
    return 1;
}

enum { G_QKV = 0, G_ATTPROJ = 1, G_FC = 2, G_FCPROJ = 3, G_LOGITS = 4 };

/* packed weights at element offset off (fp32 or bf16 pack) */
static const float* wpack_at(const GPT2Decode* d, size_t off) {
    return d->w_bf16 ? (const float*)((const unsigned short*)d->d_wpack + off) : d->d_wpack + off;
}

/* descriptor of fused GEMM `which` of layer l over the decode rows */
static void dec_gemm_desc(GPT2* model, int l, int which, HpaFusedGemm* g) {
    GPT2Decode* d = model->decode;
    const GPT2Config c = model->config;
    const int C = c.channels, V = c.vocab_size, ct = C / 16;
    const ParameterTensors* w = &model->params;
    const size_t lc = (size_t)l * C;
    const size_t e_layer = d->wpack_off[3] + hpa_frag_elems(C, 4 * C);
    memset(g, 0, sizeof(*g));
    g->M = d->B;
    g->w_dtype = d->w_bf16 ? HPA_BF16 : HPA_F32;
    g->epilogue = which == G_QKV ? HPA_FEPI_QKV : which == G_FC ? HPA_FEPI_GELU
                : which == G_LOGITS ? HPA_FEPI_LOGITS : HPA_FEPI_RESID;
    g->waves = d->fwaves[which];
    g->row_blocks = d->frb[which];
    g->col_tiles = d->fct[which];
    g->pool = &d->pool;
    g->layer = l;
    g->block_table = d->d_bt;
    g->bt_stride = d->bt_stride;
    g->pos = d->d_pos;
    switch (which) {
        case G_QKV: /* LN1 (stats: embedding's 1 tile at layer 0, fcproj's C/16 after) */
            g->x = d->res; g->K = C; g->ln_stats = d->st1; g->ln_ntiles = l == 0 ? 1 : ct;
            g->ln_w = w->ln1w + lc; g->ln_b = w->ln1b + lc; g->w = wpack_at(d, e_layer * l + d->wpack_off[0]);
            g->N = 3 * C; g->bias = w->qkvb + 3 * lc; g->out = d->d_q;
            if (d->d_fold) { g->ln_fold_c1 = d->d_fold + 14 * lc; g->bias = g->ln_fold_c1 + 3 * C; }
            break;
        case G_ATTPROJ: /* res2 = res + att . Wap^T + b (LN2 statistics only when fc needs them) */
            g->x = d->att; g->K = C; g->w = wpack_at(d, e_layer * l + d->wpack_off[1]); g->N = C;
            g->bias = w->attprojb + lc; g->out = d->res2; g->res_in = d->res; g->stats_out = d->d_fold ? NULL : d->st2;
            break;
        case G_FC: /* gelu(LN2(res2) . Wfc^T + b) */
            g->x = d->res2; g->K = C; g->ln_stats = d->st2; g->ln_ntiles = ct; g->ln_w = w->ln2w + lc;
            g->ln_b = w->ln2b + lc; g->w = wpack_at(d, e_layer * l + d->wpack_off[2]); g->N = 4 * C;
            g->bias = w->fcb + 4 * lc; g->out = d->fch;
            if (d->d_fold) { g->ln_fold_c1 = d->d_fold + 14 * lc + 6 * C; g->bias = g->ln_fold_c1 + 4 * C; }
            break;
        case G_FCPROJ: /* res = res2 + fch . Wfp^T + b, next-LN statistics */
            g->x = d->fch; g->K = 4 * C; g->w = wpack_at(d, e_layer * l + d->wpack_off[3]); g->N = C;
            g->bias = w->fcprojb + lc; g->out = d->res; g->res_in = d->res2;
            g->stats_out = d->d_fold && l + 1 < c.num_layers ? NULL : d->st1; /* LNf of logits: last layer */
            break;
        default: /* logits = LNf(res) . wte^T, argmax partials */
            g->x = d->res; g->K = C; g->ln_stats = d->st1; g->ln_ntiles = ct;
            g->ln_w = w->lnfw; g->ln_b = w->lnfb; g->w = wpack_at(d, d->wpack_off[4]); g->N = V;
            g->out = d->d_logits; g->part_out = d->part; g->layer = 0;
            g->variant = 4; /* activation-resident kernel where the shape allows (hpa_logits.hip), */
            g->sk_slab = d->sk_slab; g->sk_count = d->sk_cnt; /* else stream-K with this workspace */
            if (!d->w_bf16 && hpa_logits_kernel(d->B, V, C) == 4) { /* its form by the GLOBAL batch: a */
                const int Bg = dec_pick_B(d); /* row's sum order (global picks: sharded = */
                g->waves = Bg > 32 ? 12 : 16;                             /* unsharded bit for bit) */
            }
            break;
    }
}

/* GPT-2 XL's qkv / fc: 1 the ring kernel; in A/B builds HPA_GEMM_RING=0 the
 * looped kernel, =2 the ring with its K split over workgroups (XL step
 * 10.31 / 10.41 / 10.43 ms) */
static int dec_ring_allowed(void) {
#ifdef HPA_AB
    static int v = -1;
    if (v < 0) {
        const char* e = getenv("HPA_GEMM_RING");
        v = e && e[0] == '0' ? 0 : e && e[0] == '2' ? 2 : 1;
    }
    return v;
#else
    return 1;
#endif
}

static int dec_gemm(GPT2* model, int l, int which) {
    HpaFusedGemm g;
    dec_gemm_desc(model, l, which, &g);
    {   /* wide layers (C >= 1024: GPT-2 XL) at 49-64 rows of the GLOBAL batch: qkv and fc on the loader / MFMA-wave ring kernel
         * (hpa_gemm_ring.hip, variant 3; a row's sums never depend on M, so
         * shards of that batch take it too and stay bit-identical) */
        GPT2Decode* d = model->decode;
        const int Bg = dec_pick_B(d);
        const int ring = dec_ring_allowed();
        if ((which == G_QKV || which == G_FC) && !d->w_bf16 && d->d_fold && model->config.channels >= 1024 &&
            Bg > 48 && d->B <= 64 && ring) {
            g.variant = 3;
            /* HPA_GEMM_RING=2: K split over workgroups so all CUs compute (qkv
             * 150 column pairs x 3, fc 200 x 2): measured slower (qkv 22.1 vs
             * 21.9 us, fc 26.6 vs 22.9), kept as a tested option */
            g.waves = ring == 1 || !d->ring_slab ? 1 : which == G_QKV ? DEC_RING_QKV_PARTS : DEC_RING_FC_PARTS;
            g.sk_slab = d->ring_slab;
            g.sk_count = d->ring_cnt;
        }
    }
    return hpa_gemm_fused(&g);
}

/* greedy or sampled next token; active (nullable): rows with active[b] <= 0
 * are left untouched */
static int dec_pick(GPT2* model, const int* active) {
    GPT2Decode* d = model->decode;
    const int V = model->config.vocab_size;
    if (d->sample)
        return hpa_sample_final(d->d_logits, d->B, V, d->d_rng, d->d_next, d->d_tokens, d->d_pos, active);
    HpaFusedGemm g;
    dec_gemm_desc(model, 0, G_LOGITS, &g);
    const int npart = hpa_logits_partials(&g); /* per-tile or per-workgroup partials */
    if (npart <= 0) return 1;
    return hpa_argmax_final(d->part, npart, d->Mp, d->B, d->d_next, d->d_tokens, d->d_pos, active);
}

/* one decode-attention launch: the (sequence, head, context range) grid,
 * frag output */
static int dec_attn_call(GPT2Decode* d, int l, const int* pos, float* out) {
    return hpa_paged_attention_decode_split_w(d->d_q, &d->pool, l, d->d_bt, d->bt_stride, pos, out, d->B,
                                              d->attn_splits, d->d_attn_ws, 1, d->attn_waves);
}

static int dec_attention(GPT2* model, int l) {
    GPT2Decode* d = model->decode;
    int rc = 0;
    if (d->profiling) rc |= hpa_event_record(d->prof_ev[0]);
    rc |= dec_attn_call(d, l, d->d_pos, d->att);
    if (d->profiling) {
        rc |= hpa_event_record(d->prof_ev[1]);
        const float ms = hpa_event_elapsed_ms(d->prof_ev[0], d->prof_ev[1]); /* waits for this launch */
        if (ms < 0) return 1;
        d->prof_ms += ms;
        d->prof_launches++;
    }
    return rc;
}

#ifndef DEC_FIRST_LAUNCH
#define DEC_FIRST_LAUNCH 1 /* A/B builds: 0 = the embed kernel + the one-shot qkv(0) GEMM */
#endif
/* the step's first launch under chain form 6 (hpa_decode_first): the
 * embedding into res, layer 0's q and K/V (LN1 folded), and zb bytes of the
 * counter block (error word + hand-off counters) zeroed */
static int dec_first(GPT2* model, size_t zb) {
    GPT2Decode* d = model->decode;
    const GPT2Config c = model->config;
    const ParameterTensors* w = &model->params;
    const int C = c.channels;
    HpaLayerArgs a;
    memset(&a, 0, sizeof(a));
    a.B = d->B;
    a.C = C;
    a.num_heads = c.num_heads;
    a.pool = &d->pool;
    a.block_table = d->d_bt;
    a.bt_stride = d->bt_stride;
    a.pos = d->d_pos;
    a.res = d->res;
    a.w_qkv = wpack_at(d, d->wpack_off[0]); /* layer 0 */
    a.qkv_c1 = d->d_fold;
    a.qkv_c2 = d->d_fold + 3 * C;
    a.q_out = d->d_q;
    return hpa_decode_first(&a, d->d_tokens, w->wte, w->wpe, d->pl_ctr, zb);
}

/* the bf16 chain's first launch: embedding + qkv(0) + the counter zeroing */
static int dec_first_b16(GPT2* model, size_t zb) {
    GPT2Decode* d = model->decode;
    const ParameterTensors* w = &model->params;
    HpaChainB16Args a;
    memset(&a, 0, sizeof(a));
    a.B = d->B;
    a.pool = &d->pool;
    a.block_table = d->d_bt;
    a.bt_stride = d->bt_stride;
    a.pos = d->d_pos;
    a.res = d->res;
    a.w_qkv = wpack_at(d, d->wpack_off[0]); /* layer 0 */
    a.b_qkv = w->qkvb;
    a.ln1_w = w->ln1w;
    a.ln1_b = w->ln1b;
    a.q_out = d->d_q;
    return hpa_decode_chain_b16_first(&a, d->d_tokens, w->wte, w->wpe, d->pl_ctr, zb);
}

/* every layer of the step as the pipelined halves' one launch (pl_on 5) */
static int dec_pipe(GPT2* model) {
    GPT2Decode* d = model->decode;
    HpaPipeArgs a;
    memset(&a, 0, sizeof(a));
    a.B = d->B;
    a.num_layers = model->config.num_layers;
    a.pool = &d->pool;
    a.block_table = d->d_bt;
    a.bt_stride = d->bt_stride;
    a.pos = d->d_pos;
    a.layers = d->d_pipe_lay;
    a.q = d->d_q;
    a.att = d->att;
    a.res = d->res;
    a.res2 = d->res2;
    a.fch = d->fch;
    a.slab = d->pipe_slab;
    a.stats_out = d->st1; /* LNf statistics for the logits */
    a.stats_mp = d->Mp;
    a.counters = d->pl_ctr + DEC_ERR_INTS;
    a.layer_ctr_ints = d->pl_ctr_ints;
    a.err = d->pl_ctr;
    a.err_sticky = d->d_next + d->B;
    a.g_cus = d->pipe_g;
    return hpa_decode_pipe(&a);
}

/* the whole step on the library stream */
static int dec_launch(GPT2* model) {
    GPT2Decode* d = model->decode;
    const ParameterTensors* w = &model->params;
    const int L = model->config.num_layers;
    const int C = model->config.channels;
    const int pl = d->pl_on && !d->profiling;
    /* persistent layers: the embed kernel also zeroes their hand-off counters */
    const size_t zb = (DEC_ERR_INTS + (size_t)L * d->pl_ctr_ints) * sizeof(int);
    /* chain form 6 (and form 8 at C = 768, which sums as form 6): embed +
     * qkv(0) + the counter zeroing in one launch */
    const int first = pl && DEC_FIRST_LAUNCH && (((d->pl_on == 3 || d->pl_on == 5) &&
                      (d->pl_wform == 6 || (d->pl_wform == 8 && model->config.num_heads == 12))) || d->pl_on == 4);
    int rc = first ? (d->pl_on == 4 ? dec_first_b16(model, zb) : dec_first(model, zb))
           : !pl   ? hpa_embed_frag(d->d_tokens, d->d_pos, w->wte, w->wpe, d->res, d->st1, d->B, C)
                   : hpa_embed_frag_zero(d->d_tokens, d->d_pos, w->wte, w->wpe, d->res, d->st1, d->B, C, d->pl_ctr, zb);
#define DEC_TRACE(i) \
    if (d->trace_x) rc |= hpa_unpack_frag(d->res, d->B, C, d->trace_x + (size_t)(i) * d->B * C, C)
    DEC_TRACE(0);
    if (pl && d->pl_on == 5 && first && !d->trace_x) { /* the pipelined halves: every layer in one launch */
        rc |= dec_pipe(model);
        rc |= dec_gemm(model, 0, G_LOGITS);
        rc |= dec_pick(model, NULL);
        return rc;
    }
    if (pl) { /* qkv(0), then one persistent launch per layer */
        if (!first) rc |= dec_gemm(model, 0, G_QKV);
        for (int l = 0; l < L && !rc; l++) {
            if (d->pl_on >= 2) rc |= dec_attention(model, l); /* chain form: the attention's own launch */
            rc |= dec_layer(model, l);
            DEC_TRACE(l + 1);
        }
        rc |= dec_gemm(model, 0, G_LOGITS);
        rc |= dec_pick(model, NULL); /* a separate argmax launch: the in-launch pick (HpaFusedGemm.pick_next)
                                      * measured no faster, profiles/r4/experiments/in_launch_pick.txt */
        return rc;
    }
    for (int l = 0; l < L && !rc; l++) {
        rc |= dec_gemm(model, l, G_QKV);
        rc |= dec_attention(model, l);
        rc |= dec_gemm(model, l, G_ATTPROJ);
        rc |= dec_gemm(model, l, G_FC);
        rc |= dec_gemm(model, l, G_FCPROJ);
        DEC_TRACE(l + 1);
    }
#undef DEC_TRACE
    rc |= dec_gemm(model, 0, G_LOGITS);
    rc |= dec_pick(model, NULL);
    return rc;
}

/* token choice: greedy argmax (enable = 0, the north star's), or the
 * reference driver's multinomial sampling (softmax_forward + sample_mult,
 * paged_infer.c:259-286, :837-848) with sequence b drawing its coins from
 * xorshift state seed + b (B = 1 reproduces the reference's single stream) */
int gpt2_decode_set_sampling(GPT2* model, int enable, unsigned long long seed) {
    GPT2Decode* d = model->decode;
    if (!d) return 1;
    if (hpa_synchronize()) return 1;
    if (!d->d_rng) {
        d->d_rng = (unsigned long long*)hpa_malloc(d->B * sizeof(unsigned long long));
        if (!d->d_rng) return 1;
    }
    unsigned long long* h = (unsigned long long*)malloc(d->B * sizeof(unsigned long long));
    if (!h) return 1;
    for (int b = 0; b < d->B; b++) h[b] = seed + (unsigned long long)b;
    const int rc = hpa_memcpy(d->d_rng, h, d->B * sizeof(unsigned long long));
    free(h);
    if (rc) return 1;
    d->sample = enable ? 1 : 0;
    if (d->graph) { /* recapture with the other token-choice kernel */
        hpa_graph_destroy(d->graph);
        d->graph = NULL;
        if (dec_rezero(d)) return 1;
    }
    return 0;
}

int gpt2_decode_set_graph(GPT2* model, int enable) {
    GPT2Decode* d = model->decode;
    if (!d) return 1;
    d->use_graph = enable;
    if (!enable && d->graph) {
        hpa_synchronize();
        hpa_graph_destroy(d->graph);
        d->graph = NULL;
    }
    return 0;
}

/* 0 = by shape (hpa_attn_pick_splits), else 1..HPA_ATTN_MAX_SPLITS */
int gpt2_decode_set_attn_splits(GPT2* model, int splits) {
    GPT2Decode* d = model->decode;
    if (!d) return 1;
    if (splits == 0) {
        int ncu = 0;
        hpa_device_info(NULL, 0, &ncu, NULL);
        splits = hpa_attn_pick_splits(dec_pick_B(d), d->pool.num_heads, d->max_ctx, ncu);
    }
    if (hpa_synchronize()) return 1;
    return dec_set_splits(d, splits);
}

int gpt2_decode_attn_splits(GPT2* model) { return model->decode ? model->decode->attn_splits : 0; }

/* waves per attention workgroup the engine picked (hpa_set_attention_waves may override it) */
int gpt2_decode_attn_waves(GPT2* model) { return model->decode ? model->decode->attn_waves : 0; }

static int dec_enqueue(GPT2* model, const int* tokens) {
    GPT2Decode* d = model->decode;
    if (!d) { fprintf(stderr, "[paged_infer] gpt2_decode_init first\n"); return 1; }
    if (tokens) {
        for (int b = 0; b < d->B; b++)
            if (tokens[b] < 0 || tokens[b] >= model->config.vocab_size) {
                fprintf(stderr, "[paged_infer] token out of range\n"); /* :591-596 */
                return 1;
            }
    }
    if (dec_ensure_pages(d)) return 1;
    if (dec_sync_block_table(d)) return 1;
    if (tokens && dec_upload_tokens(d, tokens)) return 1;
    if (d->use_graph && !d->profiling && !d->trace_x) {
        if (!d->graph) {
            if (hpa_graph_begin()) return 1;
            const int rc = dec_launch(model);
            void* g = hpa_graph_end();
            if (rc || !g) return 1;
            d->graph = g;
        }
        if (hpa_graph_launch(d->graph)) return 1;
    } else if (dec_launch(model)) {
        return 1;
    }
    for (int b = 0; b < d->B; b++) d->h_pos[b]++;
    return 0;
}

/* ---- prefill: the new tokens of every sequence in one pass ----
 * All rows go through the fused GEMMs (row r of sequence b at absolute
 * position pos[b] + t; the QKV epilogue appends each row's K/V through its
 * sequence's block table), the causal multi-query attention runs on MFMA
 * (hpa_paged_attention_prefill_ragged), and the last row of every sequence
 * is gathered for the logits and the token choice.  Equivalent to one decode
 * step per token (tested against the oracle's token-by-token decode). */
static int dec_prefill_reserve(GPT2* model, int R) {
    GPT2Decode* d = model->decode;
    if (R <= d->pf_cap) return 0;
    dec_prefill_free(d);
    const size_t C = model->config.channels, ct = C / 16;
    const size_t Rp = (size_t)(R + 15) / 16 * 16;
    d->pf_res = (float*)hpa_malloc(Rp * C * 4);
    d->pf_res2 = (float*)hpa_malloc(Rp * C * 4);
    d->pf_att = (float*)hpa_malloc(Rp * C * 4);
    d->pf_fch = (float*)hpa_malloc(Rp * 4 * C * 4);
    d->pf_st1 = (float*)hpa_malloc(ct * Rp * 2 * 4);
    d->pf_st2 = (float*)hpa_malloc(ct * Rp * 2 * 4);
    d->pf_q = (float*)hpa_malloc(Rp * C * 4);
    d->pf_tok = (int*)hpa_malloc(Rp * sizeof(int));
    d->pf_pos = (int*)hpa_malloc(Rp * sizeof(int));
    d->pf_seq = (int*)hpa_malloc(Rp * sizeof(int));
    d->pf_start = (int*)hpa_malloc(3 * (size_t)d->B * sizeof(int)); /* start[B], row0[B], len[B] */
    d->pf_last = (int*)hpa_malloc(d->B * sizeof(int));
    d->h_pf = (int*)malloc((3 * Rp + 4 * (size_t)d->B) * sizeof(int));
    if (!d->pf_res || !d->pf_res2 || !d->pf_att || !d->pf_fch || !d->pf_st1 || !d->pf_st2 || !d->pf_q ||
        !d->pf_tok || !d->pf_pos || !d->pf_seq || !d->pf_start || !d->pf_last || !d->h_pf) {
        dec_prefill_free(d);
        return 1;
    }
    /* padded rows stay zero */
    if (hpa_memset_async(d->pf_res, 0, Rp * C * 4) || hpa_memset_async(d->pf_res2, 0, Rp * C * 4) ||
        hpa_memset_async(d->pf_att, 0, Rp * C * 4) || hpa_memset_async(d->pf_fch, 0, Rp * 4 * C * 4))
        return 1;
    d->pf_cap = R;
    return 0;
}

static int prefill_gemm(GPT2* model, int l, int which, int R) {
    GPT2Decode* d = model->decode;
    const GPT2Config c = model->config;
    const int C = c.channels, ct = C / 16;
    const ParameterTensors* w = &model->params;
    const size_t lc = (size_t)l * C;
    const size_t e_layer = d->wpack_off[3] + hpa_frag_elems(C, 4 * C);
    HpaFusedGemm g;
    memset(&g, 0, sizeof(g));
    g.M = R;
    g.w_dtype = d->w_bf16 ? HPA_BF16 : HPA_F32;
    /* many rows: reuse every activation fragment over 2 weight tiles and every
     * weight fragment over 4 row blocks (MFMA-bound at this M) */
    g.waves = d->w_bf16 ? 0 : 8; /* bf16 weights: the library's shapes by (M, N, K) */
    g.row_blocks = d->w_bf16 ? 0 : 4;
    g.col_tiles = d->w_bf16 ? 0 : 2;
    g.pool = &d->pool;
    g.layer = l;
    g.block_table = d->d_bt;
    g.bt_stride = d->bt_stride;
    g.pos = d->pf_pos;
    g.row_seq = d->pf_seq;
    switch (which) {
        case G_QKV:
            g.epilogue = HPA_FEPI_QKV; g.x = d->pf_res; g.K = C; g.ln_stats = d->pf_st1;
            g.ln_ntiles = l == 0 ? 1 : ct; g.ln_w = w->ln1w + lc; g.ln_b = w->ln1b + lc;
            g.w = wpack_at(d, e_layer * l + d->wpack_off[0]); g.N = 3 * C; g.bias = w->qkvb + 3 * lc; g.out = d->pf_q;
            if (d->d_fold) { g.ln_fold_c1 = d->d_fold + 14 * lc; g.bias = g.ln_fold_c1 + 3 * C; }
            break;
        case G_ATTPROJ:
            g.epilogue = HPA_FEPI_RESID; g.x = d->pf_att; g.K = C; g.w = wpack_at(d, e_layer * l + d->wpack_off[1]);
            g.N = C; g.bias = w->attprojb + lc; g.out = d->pf_res2; g.res_in = d->pf_res;
            g.stats_out = d->d_fold ? NULL : d->pf_st2;
            break;
        case G_FC:
            g.epilogue = HPA_FEPI_GELU; g.x = d->pf_res2; g.K = C; g.ln_stats = d->pf_st2; g.ln_ntiles = ct;
            g.ln_w = w->ln2w + lc; g.ln_b = w->ln2b + lc; g.w = wpack_at(d, e_layer * l + d->wpack_off[2]);
            g.N = 4 * C; g.bias = w->fcb + 4 * lc; g.out = d->pf_fch;
            if (d->d_fold) { g.ln_fold_c1 = d->d_fold + 14 * lc + 6 * C; g.bias = g.ln_fold_c1 + 4 * C; }
            break;
        default: /* G_FCPROJ */
            g.epilogue = HPA_FEPI_RESID; g.x = d->pf_fch; g.K = 4 * C; g.w = wpack_at(d, e_layer * l + d->wpack_off[3]);
            g.N = C; g.bias = w->fcprojb + lc; g.out = d->pf_res; g.res_in = d->pf_res2;
            g.stats_out = d->d_fold && l + 1 < c.num_layers ? NULL : d->pf_st1;
            break;
    }
    return hpa_gemm_fused(&g);
}

/* the logits of EVERY prefill row (gpt2_forward's window, paged_infer.c:727:
 * the reference writes logits for all T rows): LNf(res) . wte^T over the R
 * packed rows into rows_out [R][V] (device), one LOGITS GEMM on the looped /
 * bf16 kernels (any row count); its argmax partials go to a scratch buffer */
static int prefill_all_logits(GPT2* model, int R, float* rows_out, const int* out_rows) {
    GPT2Decode* d = model->decode;
    const GPT2Config c = model->config;
    const int C = c.channels, V = c.vocab_size;
    const size_t Rp = (size_t)(R + 15) / 16 * 16;
    float* part = (float*)hpa_malloc((size_t)(V + 15) / 16 * Rp * 2 * sizeof(float));
    if (!part) return 1;
    HpaFusedGemm g;
    memset(&g, 0, sizeof(g));
    g.M = R;
    g.w_dtype = d->w_bf16 ? HPA_BF16 : HPA_F32;
    g.epilogue = HPA_FEPI_LOGITS;
    g.x = d->pf_res;
    g.K = C;
    g.ln_stats = d->pf_st1; /* the last fcproj's 16-column statistics (prefill_gemm) */
    g.ln_ntiles = C / 16;
    g.ln_w = model->params.lnfw;
    g.ln_b = model->params.lnfb;
    g.w = wpack_at(d, d->wpack_off[4]);
    g.N = V;
    g.out = rows_out;
    g.row_seq = out_rows; /* LOGITS: GEMM row -> row of rows_out (NULL: the same) */
    g.part_out = part;
    const int rc = hpa_gemm_fused(&g) || hpa_synchronize();
    hpa_free(part);
    return rc;
}

/* One pass over lens[b] >= 0 new tokens of every sequence b (tokens packed
 * in sequence order): all rows through the fused GEMMs, causal multi-query
 * paged attention per sequence, then the last row of every sequence with
 * lens[b] > 0 through the logits and the greedy / sampled pick.  Sequences
 * with lens[b] = 0 are untouched (position, next token, sampler state).
 * all_logits (device [R][V], nullable): every row's logits too. */
static int dec_prefill_rows(GPT2* model, const int* tokens, const int* lens, int* next_tokens, float* all_logits,
                            const int* all_rows) {
    GPT2Decode* d = model->decode;
    if (!d) { fprintf(stderr, "[paged_infer] gpt2_decode_init first\n"); return 1; }
    const GPT2Config c = model->config;
    const int B = d->B, C = c.channels, L = c.num_layers;
    long R = 0;
    int T = 0;
    for (int b = 0; b < B; b++) {
        if (lens[b] < 0) { fprintf(stderr, "[paged_infer] negative length for sequence %d\n", b); return 1; }
        if (d->h_pos[b] + lens[b] > d->max_ctx) {
            fprintf(stderr, "[paged_infer] prefill of %d tokens overflows sequence %d\n", lens[b], b);
            return 1;
        }
        R += lens[b];
        if (lens[b] > T) T = lens[b];
    }
    if (R == 0) return 0;
    if (R > (1L << 24)) { fprintf(stderr, "[paged_infer] prefill too large\n"); return 1; }
    for (long i = 0; i < R; i++)
        if (tokens[i] < 0 || tokens[i] >= c.vocab_size) {
            fprintf(stderr, "[paged_infer] token out of range\n"); /* :591-596 */
            return 1;
        }
    for (int b = 0; b < B; b++)
        if (lens[b] > 0 && dec_grow(d, b, lens[b], lens, NULL)) return 1;
    if (dec_sync_block_table(d)) return 1;
    if (dec_prefill_reserve(model, (int)R)) return 1;
    /* row tables: token, absolute position, sequence; per-sequence start,
     * first row, length, last row (-1: skipped) */
    if (hpa_synchronize()) return 1; /* h_pf staging reuse */
    const int Rp = (int)((R + 15) / 16 * 16);
    int *ht = d->h_pf, *hp = ht + Rp, *hs = hp + Rp, *hst = hs + Rp, *hr0 = hst + B, *hln = hr0 + B, *hl = hln + B;
    int r = 0;
    for (int b = 0; b < B; b++) {
        hst[b] = d->h_pos[b];
        hr0[b] = r;
        hln[b] = lens[b];
        for (int t = 0; t < lens[b]; t++, r++) {
            ht[r] = tokens[r];
            hp[r] = d->h_pos[b] + t;
            hs[r] = b;
        }
        hl[b] = lens[b] > 0 ? r - 1 : -1;
    }
    if (hpa_memcpy(d->pf_tok, ht, R * sizeof(int)) || hpa_memcpy(d->pf_pos, hp, R * sizeof(int)) ||
        hpa_memcpy(d->pf_seq, hs, R * sizeof(int)) || hpa_memcpy(d->pf_start, hst, 3 * (size_t)B * sizeof(int)) ||
        hpa_memcpy(d->pf_last, hl, B * sizeof(int)))
        return 1;
    const int* d_row0 = d->pf_start + B;
    const int* d_len = d->pf_start + 2 * B;
    const ParameterTensors* w = &model->params;
    int rc = hpa_embed_frag(d->pf_tok, d->pf_pos, w->wte, w->wpe, d->pf_res, d->pf_st1, (int)R, C);
    for (int l = 0; l < L && !rc; l++) {
        rc |= prefill_gemm(model, l, G_QKV, (int)R);
        rc |= hpa_paged_attention_prefill_ragged(d->pf_q, &d->pool, l, d->d_bt, d->bt_stride, d->pf_start, d_row0,
                                                 d_len, B, T, d->pf_att);
        rc |= prefill_gemm(model, l, G_ATTPROJ, (int)R);
        rc |= prefill_gemm(model, l, G_FC, (int)R);
        rc |= prefill_gemm(model, l, G_FCPROJ, (int)R);
    }
    if (all_logits && !rc) rc |= prefill_all_logits(model, (int)R, all_logits, all_rows);
    /* last row of every active sequence -> the decode rows, logits, pick; the
     * pick advances pos by one: set pos = start + len - 1 first */
    for (int b = 0; b < B; b++) hst[b] = d->h_pos[b] + (lens[b] > 0 ? lens[b] - 1 : 0);
    rc |= hpa_memcpy(d->d_pos, hst, B * sizeof(int));
    rc |= hpa_gather_rows_frag(d->pf_res, d->pf_st1, Rp, d->pf_last, B, d->res, d->st1, d->Mp, C);
    rc |= dec_gemm(model, 0, G_LOGITS);
    rc |= dec_pick(model, d_len);
    if (rc) return 1;
    for (int b = 0; b < B; b++) d->h_pos[b] += lens[b];
    if (next_tokens) {
        if (hpa_memcpy(d->h_next, d->d_next, B * sizeof(int))) return 1;
        memcpy(next_tokens, d->h_next, B * sizeof(int));
    }
    return hpa_synchronize();
}

int gpt2_decode_prefill(GPT2* model, const int* tokens, int T, int* next_tokens) {
    GPT2Decode* d = model->decode;
    if (!d) { fprintf(stderr, "[paged_infer] gpt2_decode_init first\n"); return 1; }
    if (T <= 0) return 1;
    int* lens = (int*)malloc(d->B * sizeof(int));
    if (!lens) return 1;
    for (int b = 0; b < d->B; b++) lens[b] = T;
    const int rc = dec_prefill_rows(model, tokens, lens, next_tokens, NULL, NULL);
    free(lens);
    return rc;
}

int gpt2_decode_prefill_ragged(GPT2* model, const int* tokens, const int* lens, int* next_tokens) {
    if (!model->decode) { fprintf(stderr, "[paged_infer] gpt2_decode_init first\n"); return 1; }
    if (!lens || !tokens) return 1;
    return dec_prefill_rows(model, tokens, lens, next_tokens, NULL, NULL);
}

int gpt2_decode_release(GPT2* model, int seq) {
    GPT2Decode* d = model->decode;
    if (!d) { fprintf(stderr, "[paged_infer] gpt2_decode_init first\n"); return 1; }
    if (seq < 0 || seq >= d->B) { fprintf(stderr, "[paged_infer] no sequence %d\n", seq); return 1; }
    if (hpa_synchronize()) return 1; /* the pages may still be read by queued work */
    if (d->bm->prompt_block_count[seq]) free_blocks_for_prompt(d->bm, seq);
    d->h_pos[seq] = 0;
    if (hpa_memcpy(d->d_pos + seq, &d->h_pos[seq], sizeof(int))) return 1;
    return dec_sync_block_table(d);
}

int gpt2_decode_step_async(GPT2* model, const int* tokens) { return dec_enqueue(model, tokens); }

int gpt2_decode_step(GPT2* model, const int* tokens, int* next_tokens) {
    if (dec_enqueue(model, tokens)) return 1;
    GPT2Decode* d = model->decode;
    if (next_tokens) {
        if (hpa_memcpy_async(d->h_next, d->d_next, (d->B + 1) * sizeof(int)) || hpa_synchronize()) return 1;
        if (d->h_next[d->B]) return gpt2_decode_status(model) ? 1 : 1;
        memcpy(next_tokens, d->h_next, d->B * sizeof(int));
    }
    return 0;
}

/* one step, eager, that also writes the residual stream entering every
 * layer and the final one (the rows LNf reads) to host_x [L+1][B][C]: the
 * per-layer parity tests hand it to the oracle (oracle_paged_step_ex) so that
 * each layer is checked on the GPU's own input */
int gpt2_decode_step_traced(GPT2* model, const int* tokens, int* next_tokens, float* host_x) {
    GPT2Decode* d = model->decode;
    if (!d || !host_x) return 1;
    const size_t n = (size_t)(model->config.num_layers + 1) * d->B * model->config.channels;
    d->trace_x = (float*)hpa_malloc(n * sizeof(float));
    if (!d->trace_x) return 1;
    int rc = gpt2_decode_step(model, tokens, next_tokens);
    rc |= hpa_memcpy(host_x, d->trace_x, n * sizeof(float));
    hpa_free(d->trace_x);
    d->trace_x = NULL;
    return rc;
}

int gpt2_decode_status(GPT2* model) {
    GPT2Decode* d = model->decode;
    if (!d) return -1;
    if (hpa_memcpy_async(d->h_next, d->d_next, (d->B + 1) * sizeof(int)) || hpa_synchronize()) return -1;
    const int code = d->h_next[d->B];
    if (code) {
        static const char* what[] = {"", "attention", "attproj", "fc", "fcproj"};
        fprintf(stderr, "[paged_infer] persistent layer: in-launch wait for %s timed out (code %d); step invalid\n",
                code >= 1 && code <= 4 ? what[code] : "?", code);
        const int zero = 0;
        if (hpa_memcpy(d->d_next + d->B, &zero, sizeof(int)) || dec_rezero(d)) return -1;
    }
    return code;
}

int gpt2_decode_set_layer_kernel(GPT2* model, int enable) {
    GPT2Decode* d = model->decode;
    if (!d) return 1;
    if (hpa_synchronize()) return 1;
    d->pl_want = enable < 0 ? 0 : enable > 7 ? 7 : enable;
    if (dec_layer_setup(model, d)) return 1;
    if (d->graph) { /* recapture with the other step */
        hpa_graph_destroy(d->graph);
        d->graph = NULL;
        if (dec_rezero(d)) return 1;
    }
    return 0;
}

int gpt2_decode_layer_kernel(GPT2* model) { return model->decode ? model->decode->pl_on : 0; }

int gpt2_decode_set_pipe_split(GPT2* model, int g_cus) {
    GPT2Decode* d = model->decode;
    if (!d || g_cus < 0 || g_cus % 8) return 1;
    if (hpa_synchronize()) return 1;
    d->pipe_g = g_cus;
    if (d->graph) { /* recapture with the other split */
        hpa_graph_destroy(d->graph);
        d->graph = NULL;
        if (dec_rezero(d)) return 1;
    }
    return 0;
}


/* sequences the LRU policy paged out since the last call (their position
 * restarted at 0: the caller must prefill them again); mask (nullable, [B])
 * gets 1 for each.  Returns how many. */
int gpt2_decode_evicted(GPT2* model, int* mask) {
    GPT2Decode* d = model->decode;
    if (!d) return -1;
    int n = 0;
    for (int b = 0; b < d->B; b++) {
        if (mask) mask[b] = d->h_evicted[b];
        n += d->h_evicted[b];
        d->h_evicted[b] = 0;
    }
    return n;
}

int gpt2_decode_reset(GPT2* model) {
    GPT2Decode* d = model->decode;
    if (!d) return 1;
    if (hpa_synchronize()) return 1;
    for (int b = 0; b < d->B; b++) {
        if (d->bm->prompt_block_count[b]) free_blocks_for_prompt(d->bm, b);
        d->h_pos[b] = 0;
    }
    if (hpa_memset_async(d->d_pos, 0, d->B * sizeof(int))) return 1;
    return dec_sync_block_table(d) || hpa_synchronize();
}

int gpt2_decode_fill_random(GPT2* model, int ctx, unsigned long long seed) {
    return gpt2_decode_fill_random_ex(model, ctx, seed, 0);
}

int gpt2_decode_fill_random_ex(GPT2* model, int ctx, unsigned long long seed, int seq_offset) {
    GPT2Decode* d = model->decode;
    if (!d) return 1;
    if (ctx < 0 || ctx >= d->max_ctx) {
        fprintf(stderr, "[paged_infer] fill_random: ctx must be < max_ctx\n");
        return 1;
    }
    if (gpt2_decode_reset(model)) return 1;
    for (int b = 0; b < d->B; b++) {
        const int need = (ctx + d->P - 1) / d->P;
        while (d->bm->prompt_block_count[b] < need)
            if (!request_block(d->bm, b)) return 1;
        d->h_pos[b] = ctx;
    }
    if (dec_sync_block_table(d)) return 1;
    if (hpa_pool_fill_random_ex(&d->pool, d->d_bt, d->bt_stride, d->B, ctx, seed, seq_offset)) return 1;
    if (hpa_memcpy(d->d_pos, d->h_pos, d->B * sizeof(int))) return 1;
    return 0;
}

float* gpt2_decode_logits(GPT2* model) { return model->decode ? model->decode->d_logits : NULL; }
int* gpt2_decode_next(GPT2* model) { return model->decode ? model->decode->d_next : NULL; }
int gpt2_decode_batch(GPT2* model) { return model->decode ? model->decode->B : 0; }

int gpt2_decode_positions(GPT2* model, int* host_pos) {
    GPT2Decode* d = model->decode;
    if (!d) return 1;
    memcpy(host_pos, d->h_pos, d->B * sizeof(int));
    return 0;
}

/* K/V of positions [0, n) of sequence b at layer l, in the reference's
 * token-major layout: k, v = [n][C] host arrays (parity tests hand the same
 * cache to the oracle) */
int gpt2_decode_read_kv(GPT2* model, int l, int b, int n, float* k, float* v) {
    GPT2Decode* d = model->decode;
    if (!d || l < 0 || l >= model->config.num_layers || b < 0 || b >= d->B || n < 0 || n > d->h_pos[b]) return 1;
    const int C = model->config.channels, NH = model->config.num_heads, P = d->P;
    const size_t tile = (size_t)P * 64, eb = d->pool.elem_bytes;
    unsigned char* buf = (unsigned char*)malloc(2 * NH * tile * eb);
    if (!buf || hpa_synchronize()) { free(buf); return 1; }
    int rc = 0;
    for (int p0 = 0; p0 < n && !rc; p0 += P) {
        const int page = d->pv.map[d->bm->prompt_block_list[b][p0 / P]];
        rc = hpa_memcpy(buf, hpa_pool_tile(&d->pool, l, page, 0, 0), 2 * NH * tile * eb);
        for (int t = p0; t < n && t < p0 + P && !rc; t++)
            for (int h = 0; h < NH; h++)
                for (int x = 0; x < 64; x++) {
                    const int s = t - p0;
                    /* K [chunk][slot][4|8], V [slot][64] (hip_paged_attn.h pool layout) */
                    const size_t ki = eb == 4 ? ((size_t)(x >> 2) * P + s) * 4 + (x & 3)
                                              : ((size_t)(x >> 3) * P + s) * 8 + (x & 7);
                    const size_t vi = (size_t)s * 64 + x;
                    const size_t kt = (size_t)h * tile, vt = (size_t)(NH + h) * tile;
                    float kf, vf;
                    if (eb == 4) {
                        kf = ((const float*)buf)[kt + ki];
                        vf = ((const float*)buf)[vt + vi];
                    } else {
                        const unsigned ku = (unsigned)((const unsigned short*)buf)[kt + ki] << 16;
                        const unsigned vu = (unsigned)((const unsigned short*)buf)[vt + vi] << 16;
                        memcpy(&kf, &ku, 4);
                        memcpy(&vf, &vu, 4);
                    }
                    k[(size_t)t * C + h * 64 + x] = kf;
                    v[(size_t)t * C + h * 64 + x] = vf;
                }
    }
    free(buf);
    return rc;
}

/* launch shapes of the fused GEMMs (qkv, attproj, fc, fcproj, logits):
 * set = 0 copies them out; set = 1 applies the nonzero entries */
int gpt2_decode_gemm_config(GPT2* model, int* waves5, int* row_blocks5, int* col_tiles5, int set) {
    GPT2Decode* d = model->decode;
    if (!d) return 1;
    if (!set) {
        if (waves5) memcpy(waves5, d->fwaves, sizeof(d->fwaves));
        if (row_blocks5) memcpy(row_blocks5, d->frb, sizeof(d->frb));
        if (col_tiles5) memcpy(col_tiles5, d->fct, sizeof(d->fct));
        return 0;
    }
    for (int i = 0; i < 5; i++) {
        if (waves5 && waves5[i] != 0 && waves5[i] != 4 && waves5[i] != 8 && waves5[i] != 16) return 1;
        if (row_blocks5 && row_blocks5[i] != 0 && row_blocks5[i] != 1 && row_blocks5[i] != 2 &&
            row_blocks5[i] != 4)
            return 1;
        if (col_tiles5 && col_tiles5[i] != 0 && col_tiles5[i] != 1 && col_tiles5[i] != 2 && col_tiles5[i] != 4)
            return 1;
    }
    for (int i = 0; i < 5; i++) {
        if (waves5 && waves5[i]) d->fwaves[i] = waves5[i];
        if (row_blocks5 && row_blocks5[i]) d->frb[i] = row_blocks5[i];
        if (col_tiles5 && col_tiles5[i]) d->fct[i] = col_tiles5[i];
    }
    if (d->graph) { /* recapture with the new launch shapes */
        hpa_synchronize();
        hpa_graph_destroy(d->graph);
        d->graph = NULL;
    }
    return 0;
}

/* the decode attention kernel alone, `iters` back-to-back launches over the
 * layers (layer = i % L) on the engine's pool, block tables and q, at the
 * positions of the LAST completed step (ctx = pos), bracketed by HIP events on
 * the launch stream: the roofline measurement of bench.py.  Writes the average
 * launch time and the algorithmic bytes per launch (K+V rows read, q in, out). */
int gpt2_decode_time_attention(GPT2* model, int iters, double* ms_per_launch, double* bytes_per_launch) {
    GPT2Decode* d = model->decode;
    if (!d || iters <= 0) return 1;
    const int B = d->B, C = model->config.channels, L = model->config.num_layers;
    for (int b = 0; b < B; b++)
        if (d->h_pos[b] < 1) {
            fprintf(stderr, "[paged_infer] time_attention: run a step first\n");
            return 1;
        }
    int* d_p = (int*)hpa_malloc(B * sizeof(int));
    int* h_p = (int*)malloc(B * sizeof(int));
    float* out = (float*)hpa_malloc(hpa_frag_elems(B, C) * sizeof(float));
    void* e0 = hpa_event_create();
    void* e1 = hpa_event_create();
    int rc = !d_p || !h_p || !out || !e0 || !e1;
    if (!rc) {
        for (int b = 0; b < B; b++) h_p[b] = d->h_pos[b] - 1;
        rc |= hpa_memcpy(d_p, h_p, B * sizeof(int));
        /* warm-up launch, then the timed ones */
        rc |= dec_attn_call(d, 0, d_p, out);
        rc |= hpa_event_record(e0);
        for (int i = 0; i < iters && !rc; i++) rc |= dec_attn_call(d, i % L, d_p, out);
        rc |= hpa_event_record(e1);
        const float ms = rc ? -1.f : hpa_event_elapsed_ms(e0, e1);
        if (ms < 0) rc = 1;
        if (!rc) {
            double kv = 0.0;
            for (int b = 0; b < B; b++) kv += 2.0 * d->h_pos[b] * C * (double)d->pool.elem_bytes;
            if (ms_per_launch) *ms_per_launch = ms / iters;
            if (bytes_per_launch) *bytes_per_launch = kv + 2.0 * B * C * 4.0;
        }
    }
    hpa_event_destroy(e0);
    hpa_event_destroy(e1);
    hpa_free(out);
    hpa_free(d_p);
    free(h_p);
    return rc;
}

/* Infinity-Cache probe (tools/l3_probe.py): per iteration, the first `frac`
 * of layer l's pool slab is read by hpa_l3_prefetch (grid pf_grid), then the
 * attention of layer l runs; HIP events around each part, synchronised per
 * iteration.  frac = 0 times the attention alone in the same form. */
int gpt2_decode_time_attention_pf(GPT2* model, int iters, double frac, int pf_grid, double* ms_attn,
                                  double* ms_pf) {
    GPT2Decode* d = model->decode;
    if (!d || iters <= 0 || frac < 0.0 || frac > 1.0) return 1;
    const int B = d->B, C = model->config.channels, L = model->config.num_layers;
    for (int b = 0; b < B; b++)
        if (d->h_pos[b] < 1) return 1;
    int* d_p = (int*)hpa_malloc(B * sizeof(int));
    int* h_p = (int*)malloc(B * sizeof(int));
    float* out = (float*)hpa_malloc(hpa_frag_elems(B, C) * sizeof(float));
    void* e[3] = {hpa_event_create(), hpa_event_create(), hpa_event_create()};
    int rc = !d_p || !h_p || !out || !e[0] || !e[1] || !e[2];
    double ta = 0.0, tp = 0.0;
    const size_t slab = d->pool.layer_elems * d->pool.elem_bytes;
    const size_t nb = ((size_t)(frac * (double)slab)) & ~(size_t)4095;
    if (!rc) {
        for (int b = 0; b < B; b++) h_p[b] = d->h_pos[b] - 1;
        rc |= hpa_memcpy(d_p, h_p, B * sizeof(int));
        for (int i = -1; i < iters && !rc; i++) { /* i = -1: warm-up */
            const int l = (i + L) % L;
            rc |= hpa_event_record(e[0]);
            if (nb) rc |= hpa_l3_prefetch((const char*)d->pool.base + (size_t)l * slab, nb, pf_grid);
            rc |= hpa_event_record(e[1]);
            rc |= dec_attn_call(d, l, d_p, out);
            rc |= hpa_event_record(e[2]);
            if (rc) break;
            const float a = hpa_event_elapsed_ms(e[1], e[2]), p = hpa_event_elapsed_ms(e[0], e[1]);
            if (a < 0 || p < 0) rc = 1;
            if (i >= 0) {
                ta += a;
                tp += p;
            }
        }
    }
    if (!rc) {
        if (ms_attn) *ms_attn = ta / iters;
        if (ms_pf) *ms_pf = tp / iters;
    }
    for (int k = 0; k < 3; k++) hpa_event_destroy(e[k]);
    hpa_free(out);
    hpa_free(d_p);
    free(h_p);
    return rc;
}

/* weights + wpe rows + KV read (ctx = pos+1) + KV append + logits */
double gpt2_decode_step_bytes(GPT2* model, double* attn_bytes) {
    GPT2Decode* d = model->decode;
    if (!d) return 0.0;
    const GPT2Config c = model->config;
    const double C = c.channels, L = c.num_layers, V = c.vocab_size, w = 4.0;
    const double wkv = (double)d->pool.elem_bytes; /* fp32 or bf16 KV storage */
    const double wm = d->w_bf16 ? 2.0 : 4.0; /* GEMM weight matrices: bf16 or fp32 */
    const double weights = (L * 12 * C * C + V * C) * wm + (L * 13 * C + 2 * C) * w;
    double kv = 0.0;
    for (int b = 0; b < d->B; b++) kv += 2.0 * L * (d->h_pos[b] + 1) * C * wkv;
    const double append = 2.0 * L * d->B * C * wkv;
    const double logits = (double)d->B * V * 4.0;
    if (attn_bytes) *attn_bytes = kv;
    return weights + d->B * C * w + kv + append + logits;
}

/* ------------------------------------------------------------------------ */
/* sequence-sharded decode: one process per GPU, RCCL gather  */
/* ------------------------------------------------------------------------ */
/* The batch the engine's shape picks follow (attention split count and
 * waves, layer-loop form and unit widths, logits form, ring GEMM): total = 0
 * (the default) picks by the engine's own B, so a shard computes exactly what
 * a single-GPU engine of its rows computes (the small-batch forms: what the
 * metric's 2/4/8-GPU points time); total > 0 picks as the unsharded engine of
 * `total` sequences does where total <= 64 (fp32 weights) or 256 (bf16
 * weights: the bf16 chain's range), so each of a shard's rows equals that
 * engine's row bit for bit (row results depend on M only through these
 * picks); above that the unsharded engine has no persistent forms and the
 * engine's own B is used.  Needs no communicator (tests emulate a rank of an
 * N-GPU decode on one GPU with it).  Replaces the global-batch picks that
 * gpt2_decode_shard used to force. */
int gpt2_decode_set_global_batch(GPT2* model, int total) {
    GPT2Decode* d = model ? model->decode : NULL;
    if (!d) { fprintf(stderr, "[paged_infer] gpt2_decode_init first\n"); return 1; }
    if (total < 0 || (total > 0 && total < d->B)) {
        fprintf(stderr, "[paged_infer] gpt2_decode_set_global_batch: total %d < this engine's %d rows\n", total, d->B);
        return 1;
    }
    int ncu = 0;
    hpa_device_info(NULL, 0, &ncu, NULL);
    d->pl_global_B = total;
    if (hpa_synchronize() ||
        dec_set_splits(d, hpa_attn_pick_splits(dec_pick_B(d), model->config.num_heads, d->max_ctx, ncu)) ||
        dec_layer_setup(model, d))
        return 1;
    if (d->graph) {
        hpa_graph_destroy(d->graph);
        d->graph = NULL;
    }
    return dec_rezero(d);
}

int gpt2_decode_global_batch(GPT2* model) { return model && model->decode ? model->decode->pl_global_B : -1; }

/* This rank's engine decodes rows_per_rank[rank] sequences (its slice of the
 * global batch, in rank order); hpa_comm_init must have bound the
 * communicator.  The gather runs on a communication stream of its own.  The
 * shape picks stay the engine's own (its B); gpt2_decode_set_global_batch
 * makes them follow the whole batch instead. */
int gpt2_decode_shard(GPT2* model, const int* rows_per_rank, int root) {
    GPT2Decode* d = model->decode;
    if (!d) { fprintf(stderr, "[paged_infer] gpt2_decode_init first\n"); return 1; }
    const int n = hpa_comm_size(), rank = hpa_comm_rank();
    if (n < 1 || rank < 0 || !rows_per_rank || root < 0 || root >= n) {
        fprintf(stderr, "[paged_infer] gpt2_decode_shard: hpa_comm_init first, rows per rank, root\n");
        return 1;
    }
    if (rows_per_rank[rank] != d->B) {
        fprintf(stderr, "[paged_infer] gpt2_decode_shard: this rank's engine has %d sequences, not %d\n", d->B,
                rows_per_rank[rank]);
        return 1;
    }
    dec_shard_free(d);
    DecShard* s = (DecShard*)calloc(1, sizeof(DecShard));
    if (!s) return 1;
    d->shard = s;
    s->nranks = n;
    s->rank = rank;
    s->root = root;
    s->last = -1;
    s->rows = (int*)malloc(n * sizeof(int));
    s->bytes = (size_t*)malloc(n * sizeof(size_t));
    long total = 0;
    if (!s->rows || !s->bytes) { dec_shard_free(d); return 1; }
    for (int r = 0; r < n; r++) {
        s->rows[r] = rows_per_rank[r];
        total += rows_per_rank[r];
    }
    const size_t V = model->config.vocab_size;
    s->stream = hpa_stream_create();
    int ok = s->stream != NULL;
    for (int k = 0; k < 2 && ok; k++) {
        s->send[k] = (float*)hpa_malloc((size_t)d->B * V * 4);
        s->send_ids[k] = (int*)hpa_malloc((size_t)d->B * 4);
        if (rank == root) {
            s->recv[k] = (float*)hpa_malloc((size_t)total * V * 4);
            s->recv_ids[k] = (int*)hpa_malloc((size_t)total * 4);
        }
        s->ev_done[k] = hpa_event_create_nt();
        ok = s->send[k] && s->send_ids[k] && (rank != root || (s->recv[k] && s->recv_ids[k])) && s->ev_done[k];
    }
    if (ok && hpa_stream_value_ops()) {
        s->d_seq = (unsigned*)hpa_malloc(64);
        ok = s->d_seq && hpa_memset_async(s->d_seq, 0, 64) == 0 && hpa_synchronize() == 0;
    } else {
        for (int k = 0; k < 2 && ok; k++) ok = (s->ev_ready[k] = hpa_event_create_nt()) != NULL;
    }
    if (!ok) { dec_shard_free(d); return 1; }
    return 0;
}

/* the end-of-step gather (the north star's one collective): this rank's
 * logits (what = 0, [B][V] fp32) or greedy ids (what = 1, [B] int32) of the
 * last enqueued step go to the root, rows in rank order.  The copy into send
 * buffer k (k alternates) is enqueued on the compute stream; the
 * communication stream waits for it and runs the RCCL gather, so it overlaps
 * the next step's kernels.  Before buffer k is refilled (two gathers later)
 * the compute stream waits for that buffer's gather.  Asynchronous: the
 * result is read with gpt2_decode_gathered after gpt2_decode_gather_wait. */
int gpt2_decode_gather(GPT2* model, int what) {
    GPT2Decode* d = model->decode;
    DecShard* s = d ? d->shard : NULL;
    if (!s || (what != 0 && what != 1)) { fprintf(stderr, "[paged_infer] gpt2_decode_shard first\n"); return 1; }
    const size_t V = model->config.vocab_size;
    const size_t per = what ? sizeof(int) : V * sizeof(float);
    const int k = s->k;
    void* main_stream = hpa_get_stream();
    int rc = 0;
    if (s->pending[k]) rc |= hpa_stream_wait_event(s->ev_done[k]); /* buffer k's previous gather */
    void* src = what ? (void*)d->d_next : (void*)d->d_logits;
    void* snd = what ? (void*)s->send_ids[k] : (void*)s->send[k];
    rc |= hpa_memcpy_async(snd, src, (size_t)d->B * per);
    /* compute -> comm through a device word, not an event: a stream waiting
     * on an event of the decode stream slows the decode kernels ~25 us per
     * step while the wait is pending; a wait-value 5-9 us
     * (profiles/r6/recv_coresidency.txt) */
    const unsigned seq = ++s->seq;
    rc |= s->d_seq ? hpa_stream_write_value32(s->d_seq, seq) : hpa_event_record(s->ev_ready[k]);
    for (int r = 0; r < s->nranks; r++) s->bytes[r] = (size_t)s->rows[r] * per;
    hpa_set_stream(s->stream);
    rc |= s->d_seq ? hpa_stream_wait_value32(s->d_seq, seq) : hpa_stream_wait_event(s->ev_ready[k]);
    rc |= hpa_comm_gatherv(snd, (size_t)d->B * per, what ? (void*)s->recv_ids[k] : (void*)s->recv[k], s->bytes,
                           s->root, s->stream);
    rc |= hpa_event_record(s->ev_done[k]);
    hpa_set_stream(main_stream);
    s->pending[k] = 1;
    s->last = k;
    s->k ^= 1;
    return rc;
}

/* the single-process form (hpa_comm_init_all): one thread
 * drives the engines of n devices; models[i] runs on device i of the
 * communicator set.  Every engine's gather is posted inside ONE NCCL group
 * (an ungrouped ncclSend to the root would block the thread before the other
 * devices' calls are posted); the current device returns to index 0. */
int gpt2_decode_gather_all(GPT2** models, int n, int what) {
    if (!models || n < 1 || n != hpa_comm_size()) {
        fprintf(stderr, "[paged_infer] gpt2_decode_gather_all: one engine per device of hpa_comm_init_all\n");
        return 1;
    }
    int rc = hpa_comm_group_start();
    for (int i = 0; i < n && !rc; i++) {
        rc |= hpa_comm_use(i);
        rc |= gpt2_decode_gather(models[i], what);
    }
    rc |= hpa_comm_group_end();
    rc |= hpa_comm_use(0);
    return rc;
}

/* host waits for the last gather */
int gpt2_decode_gather_wait(GPT2* model) {
    GPT2Decode* d = model->decode;
    if (!d || !d->shard || d->shard->last < 0) return 1;
    return hpa_event_synchronize(d->shard->ev_done[d->shard->last]);
}

/* root: device pointer to the last gather's rows ([sum rows][V] fp32 logits
 * or [sum rows] int32 ids); NULL elsewhere */
void* gpt2_decode_gathered(GPT2* model, int what) {
    GPT2Decode* d = model->decode;
    if (!d || !d->shard || d->shard->last < 0 || d->shard->rank != d->shard->root) return NULL;
    return what ? (void*)d->shard->recv_ids[d->shard->last] : (void*)d->shard->recv[d->shard->last];
}

/* ------------------------------------------------------------------------ */
/* gpt2_forward (paged_infer.c:575-729) on the decode engine                */
/* ------------------------------------------------------------------------ */
/* inputs (B, T) hold the token window at absolute positions offset..offset+T-1
 * (the reference driver's convention, :1028-1080: the context-filling loop
 * calls it again and again at offset 0 with one more real token each time,
 * then the window slides).  The engine keeps the token at every cached
 * position; the first position whose token differs from the cached one (or
 * is not cached yet) is where recomputation starts, one decode step per
 * position, all L layers at absolute positions.  logits/probs rows r = 0..T-1
 * of every b are those of position offset + r, as the reference's full
 * window forward writes them (:727-728): rows of unchanged positions come
 * from the per-position logits kept since they were computed.  targets are
 * accepted and ignored (mean_loss = -1). */
void gpt2_forward(GPT2* model, int* inputs, int* targets, size_t B, size_t T, size_t max_total,
                  int offset) {
    (void)targets;
    if (model->params_memory == NULL) {
        printf("Error: model was not initialized properly.\n");
        exit(1);
    }
    const size_t V = model->config.vocab_size;
    for (size_t i = 0; i < B * T; i++) /* :591-596 */
        if (inputs[i] < 0 || (size_t)inputs[i] >= V) PI_FATAL("token out of range");
    if (offset < 0) PI_FATAL("negative window offset");
    if (!model->acts_memory) {
        model->batch_size = (int)B;
        model->seq_len = (int)T;
        const size_t n = B * T * V;
        model->acts_memory = (float*)hpa_malloc_managed(2 * n * sizeof(float));
        if (!model->acts_memory) PI_FATAL("activation allocation failed");
        memset(model->acts_memory, 0, 2 * n * sizeof(float));
        model->acts.logits = model->acts_memory;
        model->acts.probs = model->acts_memory + n;
        model->inputs = (int*)malloc(B * T * sizeof(int));
        model->targets = (int*)malloc(B * T * sizeof(int));
        size_t maxctx = max_total > (size_t)model->config.max_seq_len ? (size_t)model->config.max_seq_len
                                                                       : max_total;
        if (maxctx < (size_t)offset + T) maxctx = (size_t)offset + T;
        if (gpt2_decode_init(model, (int)B, model->manager ? 0 : 16, (int)maxctx) != 0)
            PI_FATAL("decode engine init failed");
        GPT2Decode* d = model->decode;
        d->h_hist = (int*)malloc(B * (size_t)d->max_ctx * sizeof(int));
        if (!d->h_hist) PI_FATAL("history allocation failed");
        const double cache = (double)B * d->max_ctx * V * 4.0;
        if (cache <= 4e9) { /* per-position logits for the rows of unchanged positions */
            d->pos_logits = (float*)hpa_malloc((size_t)cache);
            if (!d->pos_logits) PI_FATAL("per-position logits allocation failed");
        }
    } else if ((int)B != model->batch_size || (int)T != model->seq_len) {
        printf("Model: B=%d T=%d, Desired: B=%d T=%d\n", model->batch_size, model->seq_len, (int)B,
               (int)T);
        exit(EXIT_FAILURE);
    }
    memcpy(model->inputs, inputs, B * T * sizeof(int));
    GPT2Decode* d = model->decode;
    if (!d->h_hist) PI_FATAL("gpt2_forward: the engine was not created by gpt2_forward");
    if ((size_t)offset + T > (size_t)d->max_ctx) PI_FATAL("window past max_total / max_seq_len");
    /* sequences share the window, so they advance together: the first
     * position (over all b) whose token is new or changed starts the redo */
    int cached = d->h_pos[0];
    for (size_t b = 1; b < B; b++)
        if (d->h_pos[b] != cached) PI_FATAL("gpt2_forward: sequences at different positions");
    if (cached < offset) PI_FATAL("window starts after uncached positions");
    int start = offset + (int)T;
    for (size_t b = 0; b < B; b++)
        for (int t = 0; t < (int)T; t++) {
            const int p = offset + t;
            if (p >= start) break;
            if (p >= cached || d->h_hist[b * d->max_ctx + p] != inputs[b * T + t]) {
                start = p;
                break;
            }
        }
    if (!d->pos_logits) { /* only row T-1 is written: its position must be the last one decoded */
        if (start < offset + (int)T - 1)
            PI_FATAL("gpt2_forward: changed tokens before the window's last position need the per-position "
                     "logits cache (B * max_total * V too large)");
        if (start == offset + (int)T && cached != offset + (int)T) start = offset + (int)T - 1;
    }
    if (start < cached) { /* rewind: pages are kept, positions >= start are rewritten */
        int* p = (int*)malloc(B * sizeof(int));
        for (size_t b = 0; b < B; b++) p[b] = start;
        if (gpt2_decode_set_positions(model, p)) PI_FATAL("rewind failed");
        free(p);
    }
    const int n_new = offset + (int)T - start;
    if (n_new >= 2 && d->pos_logits) {
        /* the window's changed positions in ONE multi-row prefill pass that
         * returns every row's logits (the reference's T-row matmul_forward,
         * :703-704 / :727), not n_new single-row decode steps */
        int* toks = (int*)malloc(B * (size_t)n_new * sizeof(int));
        int* lens = (int*)malloc(B * sizeof(int));
        int* map = (int*)malloc(B * (size_t)n_new * sizeof(int));
        int* d_map = (int*)hpa_malloc(B * (size_t)n_new * sizeof(int));
        if (!toks || !lens || !map || !d_map) PI_FATAL("prefill window allocation failed");
        for (size_t b = 0; b < B; b++) {
            lens[b] = n_new;
            for (int t = 0; t < n_new; t++) {
                const int tk = inputs[b * T + (start - offset) + t];
                toks[b * n_new + t] = tk;
                map[b * n_new + t] = (int)(b * d->max_ctx) + start + t; /* its row of pos_logits */
                d->h_hist[b * d->max_ctx + start + t] = tk;
            }
        }
        /* every row's logits straight into its position's row of pos_logits
         * (the GEMM's output row map): no [B][n_new][V] staging copy */
        PI_CHECK(hpa_memcpy(d_map, map, B * (size_t)n_new * sizeof(int)));
        if (dec_prefill_rows(model, toks, lens, NULL, d->pos_logits, d_map)) PI_FATAL("window prefill failed");
        if (gpt2_decode_evicted(model, NULL) > 0) PI_FATAL("gpt2_forward: page pool too small, a sequence was evicted");
        hpa_free(d_map);
        free(map);
        free(lens);
        free(toks);
    }
    int* tok = (int*)malloc(B * sizeof(int));
    for (int pos = n_new >= 2 && d->pos_logits ? offset + (int)T : start; pos < offset + (int)T; pos++) {
        for (size_t b = 0; b < B; b++) {
            tok[b] = inputs[b * T + (pos - offset)];
            d->h_hist[b * d->max_ctx + pos] = tok[b];
        }
        if (gpt2_decode_step(model, tok, NULL)) PI_FATAL("decode step failed");
        /* every sequence of the window is live: an LRU eviction inside the
         * loop would restart one at position 0 mid-window */
        if (gpt2_decode_evicted(model, NULL) > 0) PI_FATAL("gpt2_forward: page pool too small, a sequence was evicted");
        if (d->pos_logits)
            for (size_t b = 0; b < B; b++)
                PI_CHECK(hpa_memcpy_async(d->pos_logits + (b * d->max_ctx + pos) * V, d->d_logits + b * V,
                                          V * sizeof(float)));
    }
    free(tok);
    PI_CHECK(hpa_synchronize());
    /* logits rows: every position of the window when kept, else row T-1 */
    for (size_t b = 0; b < B; b++)
        for (int t = d->pos_logits ? 0 : (int)T - 1; t < (int)T; t++) {
            const float* src = d->pos_logits ? d->pos_logits + (b * d->max_ctx + offset + t) * V : d->d_logits + b * V;
            PI_CHECK(hpa_memcpy(model->acts.logits + (b * T + t) * V, src, V * sizeof(float)));
        }
    /* probs of the same rows (softmax_forward, :259-286) */
    const int r0 = d->pos_logits ? 0 : (int)T - 1;
    for (size_t b = 0; b < B; b++)
        PI_CHECK(hpa_ref_softmax(model->acts.probs + (b * T + r0) * V, model->acts.logits + (b * T + r0) * V,
                                 (int)T - r0, (int)V));
    PI_CHECK(hpa_synchronize());
    model->mean_loss = -1.0f;
}

/* paged_infer.c:736-745 (does not free model->manager, like the reference;
 * the engine hands a caller-owned manager its pages back, dec_free) */
void gpt2_free(GPT2* model) {
    gpt2_decode_free(model);
    hpa_free(model->params_memory);
    hpa_free(model->acts_memory);
    free(model->inputs);
    free(model->targets);
    model->params_memory = NULL;
    model->acts_memory = NULL;
    model->inputs = NULL;
    model->targets = NULL;
}

/* heap GPT2 handle for FFI callers that cannot size the struct (ctypes) */
GPT2* gpt2_alloc(void) {
    GPT2* m = (GPT2*)calloc(1, sizeof(GPT2));
    if (m) m->mean_loss = -1.0f;
    return m;
}
void gpt2_release(GPT2* model) {
    if (!model) return;
    gpt2_free(model);
    free(model);
}
void gpt2_set_manager(GPT2* model, BlockManager* manager) { model->manager = manager; }
float* gpt2_acts_logits(GPT2* model) { return model->acts.logits; }
float* gpt2_acts_probs(GPT2* model) { return model->acts.probs; }

/* allocate (but do not fill) the pages of positions [0, ctx) for every
 * sequence, so decode steps up to ctx never touch the allocator */
int gpt2_decode_reserve(GPT2* model, int ctx) {
    GPT2Decode* d = model->decode;
    if (!d || ctx < 0 || ctx > d->max_ctx) return 1;
    for (int b = 0; b < d->B; b++) {
        const int need = (ctx + d->P - 1) / d->P;
        while (d->bm->prompt_block_count[b] < need)
            if (!request_block(d->bm, b)) return 1;
    }
    return dec_sync_block_table(d) || hpa_synchronize();
}

/* move every sequence to position pos[b] (pages are kept; positions >= pos
 * will be overwritten).  Requires pages for pos[b] to exist already. */
int gpt2_decode_set_positions(GPT2* model, const int* pos) {
    GPT2Decode* d = model->decode;
    if (!d) return 1;
    for (int b = 0; b < d->B; b++) {
        if (pos[b] < 0 || pos[b] >= d->max_ctx) return 1;
        if (d->bm->prompt_block_count[b] * d->P < pos[b]) return 1;
    }
    for (int b = 0; b < d->B; b++) d->h_pos[b] = pos[b];
    return hpa_memcpy(d->d_pos, d->h_pos, d->B * sizeof(int));
}

/* attention-kernel timing with HIP events on the launch stream: enable (1)
 * switches the engine to eager launches with events around every layer's
 * attention launch; read returns (total ms, launches). */
int gpt2_decode_profile(GPT2* model, int enable) {
    GPT2Decode* d = model->decode;
    if (!d) return 1;
    if (hpa_synchronize()) return 1;
    d->profiling = enable ? 1 : 0;
    d->prof_ms = 0.0;
    d->prof_launches = 0;
    return 0;
}

double gpt2_decode_profile_read(GPT2* model, long* launches) {
    GPT2Decode* d = model->decode;
    if (!d) return -1.0;
    if (launches) *launches = d->prof_launches;
    return d->prof_ms;
}
