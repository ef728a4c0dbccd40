/*
 * paged_infer.h -- drop-in for the API of mx60s/llm.c-paged paged_infer.c
 * (GPT-2 inference over a paged KV cache), backed by MI355X kernels.
 *
 * Reference-named functions keep the reference signatures
 * (paged_infer.c:24-302, :436-745, :826-951).  Their data may live on the
 * host or in device memory: host buffers are staged through HBM and the
 * result copied back, so a caller written for the reference works unchanged.
 * The layer functions compute on the GPU with the reference's arithmetic
 * order (hpa_ref_* kernels).
 *
 * The decode hot path is additive: gpt2_decode_* run one batched decode
 * step (one token for each of B sequences at absolute positions) entirely
 * on device through hand-written gfx950 kernels, the page pool in HBM and
 * per-sequence block tables from the BlockManager.  gpt2_forward() is
 * implemented on top of it with corrected semantics (all L layers, absolute
 * positions, one page list per sequence).
 */
#ifndef PAGED_INFER_H
#define PAGED_INFER_H
#include <stddef.h>
#include <stdint.h>

#include "block_manager.h"
#ifdef __cplusplus
extern "C" {
#endif

/* paged_infer.c:397-403 */
typedef struct {
    int max_seq_len;
    int vocab_size;
    int num_layers;
    int num_heads;
    int channels;
} GPT2Config;

/* paged_infer.c:308-326; DEVICE pointers into params_memory */
#define NUM_PARAMETER_TENSORS 16
typedef struct {
    float* wte;      /* (V, C) */
    float* wpe;      /* (maxT, C) */
    float* ln1w;     /* (L, C) */
    float* ln1b;     /* (L, C) */
    float* qkvw;     /* (L, 3C, C) */
    float* qkvb;     /* (L, 3C) */
    float* attprojw; /* (L, C, C) */
    float* attprojb; /* (L, C) */
    float* ln2w;     /* (L, C) */
    float* ln2b;     /* (L, C) */
    float* fcw;      /* (L, 4C, C) */
    float* fcb;      /* (L, 4C) */
    float* fcprojw;  /* (L, C, 4C) */
    float* fcprojb;  /* (L, C) */
    float* lnfw;     /* (C) */
    float* lnfb;     /* (C) */
} ParameterTensors;

/* the caller-visible outputs of gpt2_forward (paged_infer.c:350-375 keeps 23
 * activation tensors; decode needs only these, host-readable) */
typedef struct {
    float* logits; /* (B, T, V): row T-1 of every b written by gpt2_forward */
    float* probs;  /* (B, T, V): softmax of those rows */
} ActivationTensors;

typedef struct GPT2Decode GPT2Decode;

/* paged_infer.c:405-434 (training-only fields dropped) */
typedef struct {
    GPT2Config config;
    ParameterTensors params;
    size_t param_sizes[NUM_PARAMETER_TENSORS];
    float* params_memory; /* device */
    size_t num_parameters;
    ActivationTensors acts;
    float* acts_memory;   /* managed memory behind acts */
    int batch_size;
    int seq_len;
    int* inputs;
    int* targets;
    float mean_loss;
    BlockManager* manager; /* kv cache stuff (set by the caller, paged_infer.c:986-987) */
    GPT2Decode* decode;    /* device decode engine (lazily created) */
} GPT2;

/* ---------------- reference API ---------------- */
void encoder_forward(float* out, int* inp, float* wte, float* wpe, int B, int T, int C);
void layernorm_forward(float* out, float* mean, float* rstd, float* inp, float* weight, float* bias,
                       int B, int T, int C);
void matmul_forward(float* out, float* inp, float* weight, float* bias, int B, int T, int C, int OC);
void matmul_cached(float* out, float* inp, float* weight, float* bias, int B, int T, int C, int OC);
void attention_paged(float* out, float* preatt, float* att, float* inp, float** key_blocks,
                     float** value_blocks, int B, int T, int C, int NH, int offset);
void gelu_forward(float* out, float* inp, int N);
void residual_forward(float* out, float* inp1, float* inp2, int N);
void softmax_forward(float* probs, float* logits, int B, int T, int V);
void add_to_cache(BlockManager* manager, float* qkv, int B, int T, int C,
                  int how_many_tokens_to_copy_from_the_end_of_sequence);
void gpt2_build_from_checkpoint(GPT2* model, const char* checkpoint_path);
void gpt2_forward(GPT2* model, int* inputs, int* targets, size_t B, size_t T, size_t max_total,
                  int offset);
void gpt2_free(GPT2* model);
unsigned int random_u32(unsigned long long* state);
float random_f32(unsigned long long* state);
int sample_mult(float* probabilities, int n, float coin);
int* generate_tokens_from_logits(float* probs, int B, int T, int V);
void print_generated_sequence(int* tokens, int B, int T);   /* :930-935 */

/* tokenizer, decode only (paged_infer.c:852-928); file written by
 * train_gpt2.py:350-363 */
typedef struct {
    uint32_t vocab_size;
    char** token_table;
    int init_ok;
} Tokenizer;
void safe_printf(const char* piece);
void tokenizer_init(Tokenizer* tokenizer, const char* filename);
const char* tokenizer_decode(Tokenizer* tokenizer, uint32_t token_id);
void tokenizer_free(Tokenizer* tokenizer);

/* attention_paged with the page size as an argument (the reference fixes
 * BLOCK_SIZE = 32); attention_paged() uses BLOCK_SIZE */
void attention_paged_bs(float* out, float* preatt, float* att, float* inp, float** key_blocks,
                        float** value_blocks, int B, int T, int C, int NH, int offset,
                        int block_size);

/* ---------------- model construction (additive) ---------------- */
/* upload host params (checkpoint order) to the device; 0 on success */
int gpt2_build_from_params(GPT2* model, GPT2Config config, const float* host_params);
/* seeded synthetic GPT-2 weights (the reference xorshift, paged_infer.c:826-835) */
int gpt2_build_synthetic(GPT2* model, GPT2Config config, unsigned long long seed);
size_t gpt2_num_parameters(GPT2Config config);
int gpt2_synthetic_params(GPT2Config config, unsigned long long seed, float* host_params);
int gpt2_write_checkpoint(const char* path, GPT2Config config, const float* host_params);
/* version 1 (fp32) or 2 (bf16 weights, LN fp32 and last: train_gpt2.py:267-293,
 * rounded to nearest even as torch .to(bfloat16)) */
int gpt2_write_checkpoint_ex(const char* path, GPT2Config config, const float* host_params, int version);
/* host-only reader of v1 and v2 checkpoints: config (nullable) from the
 * header; host_params (nullable: header only) receives the parameters in
 * ParameterTensors order as fp32 (bf16 widened exactly).  Nonzero + stderr
 * on a bad file (gpt2_build_from_checkpoint prints and exits instead, as
 * the reference :436-502). */
int gpt2_read_checkpoint(const char* path, GPT2Config* config, float* host_params);

/* heap handle for FFI callers (ctypes / cgo) that cannot size GPT2 */
GPT2* gpt2_alloc(void);
void gpt2_release(GPT2* model); /* gpt2_free + free */
void gpt2_set_manager(GPT2* model, BlockManager* manager);
float* gpt2_acts_logits(GPT2* model);
float* gpt2_acts_probs(GPT2* model);

/* ---------------- decode engine (the MI355X hot path) ---------------- */
/* B sequences, page_size tokens per page, up to max_ctx tokens per sequence.
 * Uses model->manager when it was set by the caller (its block_size becomes
 * the page size), otherwise creates one sized B x ceil(max_ctx/page_size). */
int  gpt2_decode_init(GPT2* model, int B, int page_size, int max_ctx);
/* the same with the KV pool's storage type: HPA_F32 (0, default) or HPA_BF16
 * (1: BASELINE config 5; page size a multiple of 8) */
int  gpt2_decode_init_ex(GPT2* model, int B, int page_size, int max_ctx, int kv_dtype);
/* ... and the weights' storage type: HPA_F32 (0, default) or HPA_BF16 (1:
 * "bf16 decode" -- the layer and logits weights packed bf16 in HBM, GEMM
 * inputs rounded to bf16 after their LayerNorm, fp32 accumulation on
 * v_mfma_f32_16x16x32_bf16; LayerNorm, attention, residuals, GELU, softmax
 * stay fp32) */
int  gpt2_decode_init_w(GPT2* model, int B, int page_size, int max_ctx, int kv_dtype, int w_dtype);
/* one decode step for every sequence: tokens[b] (host) at position pos[b];
 * tokens == NULL feeds back the previous step's greedy ids (device-resident).
 * next_tokens (host, may be NULL) receives argmax(logits[b]). */
int  gpt2_decode_step(GPT2* model, const int* tokens, int* next_tokens);
/* prefill: tokens[b*T + t] (host) at positions pos[b] + t for every sequence,
 * all T tokens in one pass (B*T-row GEMMs, causal multi-query paged
 * attention on MFMA); afterwards logits / next ids are those of each
 * sequence's last token and pos[b] += T, so decode continues with
 * gpt2_decode_step(model, NULL, ...). */
int  gpt2_decode_prefill(GPT2* model, const int* tokens, int T, int* next_tokens);
/* continuous batching: one pass over lens[b] >= 0 new tokens per sequence
 * (tokens packed in sequence order, sum(lens) of them): prompts of newly
 * admitted sequences and single decode tokens of running ones go through
 * the same call.  Sequences with lens[b] = 0 are untouched (position, next
 * id, sampler state).  next_tokens[b] is each sequence's next id. */
int  gpt2_decode_prefill_ragged(GPT2* model, const int* tokens, const int* lens, int* next_tokens);
/* retire sequence seq: its pages go back to the pool (block_manager.c:78-90),
 * its position restarts at 0, so the slot can admit a new prompt */
int  gpt2_decode_release(GPT2* model, int seq);
/* the same, but enqueue only (no host sync; next ids stay on device) */
int  gpt2_decode_step_async(GPT2* model, const int* tokens);
/* one eager step that also copies the residual stream entering every layer
 * and the final one to host_x, row-major [L+1][B][C] (per-layer parity tests) */
int  gpt2_decode_step_traced(GPT2* model, const int* tokens, int* next_tokens, float* host_x);
/* free every sequence's pages and rewind positions to 0 */
int  gpt2_decode_reset(GPT2* model);
/* synthetic K/V for positions [0, ctx) of every sequence (benchmark prefill) */
int  gpt2_decode_fill_random(GPT2* model, int ctx, unsigned long long seed);
/* the same with the K/V of global sequences seq_offset.. (a shard of a larger
 * batch gets exactly its rows of the unsharded fill) */
int  gpt2_decode_fill_random_ex(GPT2* model, int ctx, unsigned long long seed, int seq_offset);
/* allocate the pages of positions [0, ctx) up front (no host work per step) */
int  gpt2_decode_reserve(GPT2* model, int ctx);
/* rewind/advance positions (pages kept) */
int  gpt2_decode_set_positions(GPT2* model, const int* pos);
/* capture the step into a hipGraph and replay it (1) or launch eagerly (0) */
int  gpt2_decode_set_graph(GPT2* model, int enable);
/* context ranges per (sequence, head) of the decode attention
 * (hpa_paged_attention_decode_split): 0 = by shape (hpa_attn_pick_splits:
 * GPT-2 124M 1 at B >= 64 and 16, 2 at 32 and 8), else 1..16 */
int  gpt2_decode_set_attn_splits(GPT2* model, int splits);
int  gpt2_decode_attn_splits(GPT2* model);
/* waves per attention workgroup the engine picked for its batch (hpa_attn_pick_waves) */
int  gpt2_decode_attn_waves(GPT2* model);
/* the layer loop's form: 0 five launches per layer; 2 one persistent launch
 * per layer (hpa_decode_layer: attention -> attproj -> fc -> fcproj -> next
 * qkv); 3 the decode attention's own launch + one persistent launch of the
 * GEMM chain (attproj -> fc -> fcproj -> next qkv) in 4-wave units; 4 the
 * chain in round 3's wide units (C = 768); 5 chain form 6: every phase in
 * 12-wave units of T tiles, one per workgroup, 16-byte epilogues, waits per
 * row block (C = 768); 6 chain form 8: streamed-weight units for MFMA-bound
 * wide layers (C = 768 / 1024 / 1280 / 1600: GPT-2 124M to XL); 1 (default, "auto") the form
 * measured fastest (profiles/r4: 5 at C = 768, 6 at C >= 1024, else 3).
 * The persistent forms need fp32 weights and B <= 64 (else five launches).
 * HPA_LAYER_KERNEL=0..6 in the environment
 * sets the default.  A persistent launch needs every CU for its 12-wave
 * workgroups: a GPU shared with another process's persistent kernels should
 * use 0. */
int  gpt2_decode_set_layer_kernel(GPT2* model, int enable);
/* 7: the pipelined halves (hpa_decode_pipe, hpa_pipe.hip): the step's first
 * launch, ONE persistent launch of every layer with the batch in two halves
 * (the GEMM chain of one half on g_cus CUs beside the attention of the other
 * on the rest), the logits; bit-identical to form 5.  GPT-2 124M shapes, fp32
 * weights and pool, 17..64 rows (else form 5).  Traced steps run form 5. */
/* CUs of the pipelined halves' GEMM role (multiple of 8; 0: the default, 64) */
int  gpt2_decode_set_pipe_split(GPT2* model, int g_cus);
/* the form in use: 0 five launches, 1 full persistent layer, 2 attention
 * launch + persistent chain of 4-wave units, 3 the chain in wide / multi-tile
 * units (forms 4..6 of gpt2_decode_set_layer_kernel), 4 the bf16-weight
 * chain, 5 the pipelined halves (form 7) */
int  gpt2_decode_layer_kernel(GPT2* model);
/* waits for the queued work; 0, or the code of a timed-out in-launch wait of
 * the persistent layer (the step's outputs are then invalid), which it clears */
int  gpt2_decode_status(GPT2* model);
/* attention-kernel timing with HIP events around every layer's attention
 * launch (forces eager launches while enabled) */
int    gpt2_decode_profile(GPT2* model, int enable);
double gpt2_decode_profile_read(GPT2* model, long* launches);
/* device buffers: logits [B][V], next ids [B]; host positions [B]; batch */
float* gpt2_decode_logits(GPT2* model);
int*   gpt2_decode_next(GPT2* model);
int    gpt2_decode_positions(GPT2* model, int* host_pos);
int    gpt2_decode_batch(GPT2* model);
/* sequences the LRU policy paged out since the last call (block_manager.c:
 * 104-113 evicts a whole sequence when the pool is full; it restarts at
 * position 0 and must be prefilled again); mask (nullable, [B]) marks them.
 * Returns how many. */
int    gpt2_decode_evicted(GPT2* model, int* mask);
/* K/V of positions [0, n) of sequence b at layer l, token-major [n][C] host
 * arrays (the reference page layout, block_manager.c:145-146) */
int    gpt2_decode_read_kv(GPT2* model, int layer, int b, int n, float* k, float* v);
/* fused GEMM launch shapes [qkv, attproj, fc, fcproj, logits]: waves per
 * workgroup (4/8/16), 16-row blocks (1/2/4) and 16-column tiles (1/2/4) per
 * workgroup.  set = 0 copies them out; set = 1 applies the nonzero entries
 * (NULL = keep).  Invalid combinations fail at the next step's launch. */
int    gpt2_decode_gemm_config(GPT2* model, int* waves5, int* row_blocks5, int* col_tiles5, int set);
/* attention kernel timed alone: `iters` back-to-back launches on the engine's
 * pool at the last step's positions; average ms and algorithmic bytes per
 * launch (bench.py roofline) */
int    gpt2_decode_time_attention(GPT2* model, int iters, double* ms_per_launch,
                                  double* bytes_per_launch);
/* Infinity-Cache probe: the first `frac` of layer l's pool slab read by
 * hpa_l3_prefetch (pf_grid workgroups), then layer l's attention; average ms
 * of each part (per-iteration events) */
int    gpt2_decode_time_attention_pf(GPT2* model, int iters, double frac, int pf_grid, double* ms_attn,
                                     double* ms_pf);
/* token choice: 0 = greedy argmax (default); 1 = multinomial sampling as the
 * reference driver (softmax_forward + sample_mult with random_f32 coins),
 * sequence b seeded with seed + b; the coins stay on the device */
int    gpt2_decode_set_sampling(GPT2* model, int enable, unsigned long long seed);
/* algorithmic HBM bytes one step reads+writes at the current positions
 * (SURVEY.md 8d formula) and the attention kernel's share of them */
double gpt2_decode_step_bytes(GPT2* model, double* attention_bytes);

/* ---------------- sequence-sharded decode ----------------
 * One process per GPU: every rank runs its own engine (gpt2_decode_init with
 * its B_local sequences, private page pool, replicated weights); nothing is
 * exchanged inside a step.  After hpa_comm_init (hip_paged_attn.h),
 * gpt2_decode_shard tells the engine every rank's row count (rank order) and
 * the root; gpt2_decode_gather then enqueues the end-of-step RCCL gather of
 * the logits (what = 0) or greedy ids (what = 1) on a communication stream
 * (double-buffered: it overlaps the next step).  gpt2_decode_gathered (root)
 * returns the device rows of the last gather after gpt2_decode_gather_wait. */
/* the batch the shape picks follow (attention splits / waves, layer-loop
 * form, logits form): 0 (default) the engine's own B -- a shard computes what
 * a single-GPU engine of its rows computes; total > 0 (<= 64 applies with
 * fp32 weights, <= 256 with bf16 weights -- the bf16 chain's row limit --
 * above that the own B) -- what the unsharded engine of `total` rows computes, bit
 * for bit.  No communicator needed.  Replaces the global-batch picks
 * gpt2_decode_shard forced until round 3. */
int    gpt2_decode_set_global_batch(GPT2* model, int total);
/* the value set by gpt2_decode_set_global_batch (0: own B), -1 without an engine */
int    gpt2_decode_global_batch(GPT2* model);
int    gpt2_decode_shard(GPT2* model, const int* rows_per_rank, int root);
int    gpt2_decode_gather(GPT2* model, int what);
/* the single-process form (hpa_comm_init_all): models[i] on device i, every
 * gather posted inside one NCCL group */
int    gpt2_decode_gather_all(GPT2** models, int n, int what);
int    gpt2_decode_gather_wait(GPT2* model);
void*  gpt2_decode_gathered(GPT2* model, int what);
void   gpt2_decode_free(GPT2* model);

#ifdef __cplusplus
}
#endif
#endif
