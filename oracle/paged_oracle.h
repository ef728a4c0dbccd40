/*
 * paged_oracle.h -- CPU restatement of mx60s/llm.c-paged's paged-attention
 * decode path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library, and only as the checker / the timed CPU baseline.  The
 * product path (llm.c-paged_amd/) never links or calls it.
 *
 * Every function cites the reference file:line it restates (paths relative
 * to the reference checkout).  Arithmetic order is kept as in the reference
 * (sequential-i fp32 dots, 4-pass softmax with max init -10000.0f, scale =
 * 1.0/sqrtf(hs)) so that, built with -O2 -fno-fast-math, results are
 * bit-identical to the reference functions on the same inputs; this is pinned
 * by tests/test_oracle.py against tests/golden/ (generated from the
 * reference itself by tests/golden/gen_golden.py via oracle/_ref).
 *
 * Deliberate semantic corrections vs. the reference's end-to-end driver
 * (SURVEY.md section 0): all L layers run (reference: `l < 1`,
 * paged_infer.c:659), positions are absolute (reference: window-relative,
 * paged_infer.c:24-47 + :1055-1080), each sequence has its own block table
 * (reference: prompt 0 hard-coded, paged_infer.c:515,713), and the page size
 * is a runtime value (reference: BLOCK_SIZE 32, block_manager.c:6).
 */
#ifndef PAGED_ORACLE_H
#define PAGED_ORACLE_H
#include <stddef.h>
#ifdef __cplusplus
extern "C" {
#endif

/* GPT2Config, paged_infer.c:397-403 */
typedef struct {
    int max_seq_len;
    int vocab_size;
    int num_layers;
    int num_heads;
    int channels;
} OracleConfig;

/* ParameterTensors sizes/offsets in the checkpoint order, paged_infer.c:308-326,461-476 */
int oracle_set_threads(int n);
size_t oracle_num_params(OracleConfig c);
void oracle_param_offsets(OracleConfig c, size_t off[16]);

/* ---- layer functions (paged_infer.c:24-302) ---- */
void oracle_encoder_forward(float* out, const int* inp, const float* wte, const float* wpe,
                            int B, int T, int C);                               /* :24-47 */
void oracle_encoder_forward_pos(float* out, const int* inp, const int* pos, const float* wte,
                                const float* wpe, int N, int C);    /* :24-47, absolute pos */
void oracle_layernorm_forward(float* out, float* mean, float* rstd, const float* inp,
                              const float* weight, const float* bias, int B, int T, int C); /* :49-89 */
void oracle_matmul_forward(float* out, const float* inp, const float* weight, const float* bias,
                           int B, int T, int C, int OC);                        /* :92-114 */
void oracle_matmul_cached(float* out, const float* inp, const float* weight, const float* bias,
                          int B, int T, int C, int OC);                         /* :117-160 */
void oracle_gelu_forward(float* out, const float* inp, int N);                  /* :243-251 */
void oracle_residual_forward(float* out, const float* inp1, const float* inp2, int N); /* :253-257 */
void oracle_softmax_forward(float* probs, const float* logits, int B, int T, int V);   /* :259-286 */
int  oracle_argmax(const float* x, int n);          /* greedy, first max wins (:937-951) */
unsigned int oracle_random_u32(unsigned long long* state);                      /* :826-832 */
float oracle_random_f32(unsigned long long* state);                             /* :833-835 */
int  oracle_sample_mult(const float* probabilities, int n, float coin);         /* :837-848 */

/* contiguous attention, train_scratch.c:218-291 == test_paged_attn.c:10-84 */
void oracle_attention_forward(float* out, float* preatt, float* att, const float* inp,
                              int B, int T, int C, int NH);
/* paged attention, paged_infer.c:163-240, with the page size a runtime value
 * (reference: BLOCK_SIZE 32).  Query row t attends logical positions
 * offset..offset+t through key_blocks[p / block_size] + (p % block_size) * C. */
void oracle_attention_paged(float* out, float* preatt, float* att, const float* inp,
                            float* const* key_blocks, float* const* value_blocks,
                            int B, int T, int C, int NH, int offset, int block_size);

/* one decode query (C floats) over positions 0..ctx-1 of a sequence's pages */
void oracle_attention_decode(float* out, const float* q, float* const* key_blocks,
                             float* const* value_blocks, int ctx, int C, int NH, int block_size);

/* full-recompute GPT-2 forward with all L layers, train_scratch.c:658-798
 * (the model-level oracle; logits only).  logits: (B,T,V). */
void oracle_gpt2_forward(const float* params, OracleConfig cfg, const int* tokens,
                         int B, int T, float* logits);

/* ---- paged incremental decode with corrected semantics ----
 * Per-sequence page lists over a page pool laid out like the reference's
 * pages (token-major [page_size][C] per page and layer, block_manager.c:145-146).
 * Pages are handed out from a seeded permutation so block tables are never
 * contiguous. */
typedef struct OraclePaged OraclePaged;
OraclePaged* oracle_paged_create(const float* params, OracleConfig cfg, int B, int page_size,
                                 int max_ctx, unsigned long long page_seed);
/* one decode step: token[b] at absolute position pos[b] for every b.  Appends
 * K,V (add_to_cache, paged_infer.c:505-573), runs attention over 0..pos[b]
 * (attention_paged arithmetic, :163-240), all L layers, final LN, logits
 * (matmul_forward with wte, :727); next[b] = argmax(logits[b]).  logits may
 * be NULL.  Returns 0, or -1 when a sequence would exceed max_ctx. */
int  oracle_paged_step(OraclePaged* o, const int* tokens, float* logits, int* next);
/* the step with each layer's input taken from forced_x [L+1][B][C] (nullable)
 * and every layer's output written to layer_out [L][B][C] (nullable) */
int  oracle_paged_step_ex(OraclePaged* o, const int* tokens, const float* forced_x, float* layer_out,
                          float* logits, int* next);
/* synthetic K/V fill: set every pos[b] = ctx and fill those slots with U(-1,1)
 * (the bounded CPU-baseline sample; bench.py only). */
void oracle_paged_fill_random(OraclePaged* o, int ctx, unsigned long long seed);
int  oracle_paged_pos(const OraclePaged* o, int b);
/* parity tests: the K/V of positions [0, n) of sequence b at layer l
 * (token-major [n][C]); pos[b] becomes n */
int  oracle_paged_set_kv(OraclePaged* o, int layer, int b, int n, const float* k, const float* v);
/* bf16 KV pool semantics (BASELINE config 5): appended K/V are rounded to
 * bf16 (nearest even) and read back exactly; all arithmetic stays fp32 */
void oracle_paged_set_kv_bf16(OraclePaged* o, int on);
/* bf16 weights mode (the engine's HPA_BF16 weights): GEMM weights and GEMM
 * input rows rounded to bf16 (nearest even), fp32 sums; 0 or -1 (no memory) */
int oracle_paged_set_w_bf16(OraclePaged* o, int on);
float oracle_round_bf16(float f);
void oracle_paged_free(OraclePaged* o);

#ifdef __cplusplus
}
#endif
#endif
