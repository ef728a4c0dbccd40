/*
 * hip_paged_attn.h -- C-ABI of the MI355X (gfx950) paged-attention decode
 * library libpaged_hip.so.  Plain pointers and sizes only.
 *
 * Two families of entry points:
 *
 *  hpa_*            MI355X-native building blocks of the decode step
 *                   (device memory, page pool, fused kernels).  Called by
 *                   paged_infer.c's decode driver (gpt2_decode_*), which is
 *                   the replacement for the reference's gpt2_forward
 *                   (paged_infer.c:575-729 of mx60s/llm.c-paged).
 *  reference-named  the drop-in functions of the reference's
 *                   paged_infer.c / block_manager.c API, declared in
 *                   paged_infer.h and block_manager.h.
 *
 * Error convention (reference: stderr + NULL from the allocator,
 * block_manager.c:117,139,149; exit(1) with location for device errors like
 * cudaCheck, train_gpt2.cu:27-34): hpa_* return 0 on success and a nonzero
 * code after printing "[hpa] <file>:<line> <error>" to stderr; with
 * HPA_FATAL=1 in the environment they exit(1) instead.
 *
 * Device pointers passed to hpa_* kernels must live in device-accessible
 * memory (hpa_malloc / hpa_malloc_managed / hipHostMalloc).  All launches go
 * to the library's current stream (hpa_set_stream) and are asynchronous.
 */
#ifndef HIP_PAGED_ATTN_H
#define HIP_PAGED_ATTN_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* ---------------- device, stream, memory, events ---------------- */
int   hpa_init(int device);            /* select device, create the default stream */
int   hpa_device_count(void);
int   hpa_get_device(void);
int   hpa_set_stream(void* hip_stream); /* NULL = library default stream */
void* hpa_get_stream(void);
int   hpa_synchronize(void);            /* stream sync */
int   hpa_device_synchronize(void);
void* hpa_malloc(size_t bytes);          /* hipMalloc; NULL on failure */
void* hpa_malloc_managed(size_t bytes);  /* hipMallocManaged (host-dereferenceable) */
void* hpa_host_alloc(size_t bytes);      /* pinned host memory */
int   hpa_free(void* p);
int   hpa_host_free(void* p);
int   hpa_memcpy(void* dst, const void* src, size_t bytes);       /* hipMemcpyDefault, sync */
int   hpa_memcpy_async(void* dst, const void* src, size_t bytes); /* on the current stream */
int   hpa_memset_async(void* dst, int value, size_t bytes);
/* read [p, p + bytes) on the current stream and drop it, so a later kernel
 * finds those lines in the 256 MiB Infinity Cache (grid: workgroups of 256) */
int   hpa_l3_prefetch(const void* p, size_t bytes, int grid);
int   hpa_is_device_accessible(const void* p); /* 1 if a kernel may dereference p */
void* hpa_event_create(void);
int   hpa_event_record(void* ev);
float hpa_event_elapsed_ms(void* start, void* stop); /* syncs on stop */
int   hpa_event_destroy(void* ev);
void* hpa_event_create_nt(void);          /* no timing: fork/join ordering only */
int   hpa_event_synchronize(void* ev);     /* host waits until the work before ev is done */
/* extra streams for concurrent work (e.g. a communication stream);
 * hpa_stream_wait_event: the CURRENT stream waits for `ev` (recorded on any
 * stream).  Inside a capture, fork/join through events pulls the other
 * stream into the same graph as parallel branches. */
void* hpa_stream_create(void);
int   hpa_stream_destroy(void* stream);
int   hpa_stream_wait_event(void* ev);
/* a dependency through a device word (round 6): write_value -- the current
 * stream sets *flag = value once its earlier work is done; wait_value -- the
 * current stream waits until *flag >= value.  The decode gather's
 * compute -> comm hand-off uses it: a pending event wait on another stream
 * slows the decode stream's kernels ~25 us per step, a pending wait-value
 * 5-9 us (profiles/r6/recv_coresidency.txt). */
int   hpa_stream_value_ops(void);  /* 1 if the device supports them (else use events) */
int   hpa_stream_write_value32(unsigned* flag, unsigned value);
int   hpa_stream_wait_value32(unsigned* flag, unsigned value);
const char* hpa_last_error(void);
/* build flags of this library: bit 0 = an A/B build (-DHPA_AB: the layer
 * forms measured slower -- the full persistent layer, the wide-unit chains --
 * and the measurement env knobs HPA_LAYER_SPLITS, HPA_GEMM_RING,
 * HPA_LOGITS_FORM, HPA_BF16_ARES; the product library has none of them) */
int hpa_build_flags(void);
/* hipGraph capture of everything enqueued on the current stream between
 * begin and end (the decode step: 5 launches per layer); replay with
 * hpa_graph_launch.  Kernel arguments are frozen at capture, so per-step
 * state (tokens, positions, block tables) must live in device memory. */
int   hpa_graph_begin(void);
void* hpa_graph_end(void);               /* instantiated executable graph, NULL on failure */
int   hpa_graph_launch(void* graph_exec);
int   hpa_graph_destroy(void* graph_exec);
/* waves per (sequence, head) workgroup of every decode attention launch of
 * the process: 1, 2, 4, 8 (an override for timing tools); 0 (default): the
 * caller's choice (the engine's hpa_attn_pick_waves, else 4) */
int   hpa_set_attention_waves(int nw);
int   hpa_device_info(char* name, int name_len, int* num_cus, size_t* total_mem);

/* ---------------- paged KV pool (fast layout) ----------------
 * One allocation per device: pool[layer][page][kv][head][tile], tile =
 * page_size x head_size elements.  K tiles are stored as
 * [head_size/4][page_size][4] (so one wave64 instruction reads 4-byte x 4
 * columns of 64 consecutive tokens = 128..512 contiguous bytes per page, the
 * lane-per-token QK^T layout); V tiles are token-major [page_size][head_size]
 * (one 256-byte row per token-head, the lane-per-dimension PV layout).
 * bf16 pools (HPA_BF16, BASELINE config 5; storage only, all arithmetic
 * fp32): K tiles [head_size/8][page_size][8] (one 16-byte chunk per
 * lane-per-token load), V tiles [page_size][head_size] (128-byte rows);
 * values are rounded to nearest-even when appended.  Page size multiple of 8.
 * A page id names the same slot in every layer's pool (vLLM-style shared
 * block table), so the block table is [seq][logical page] int32. */
typedef struct HpaKVPool {
    void*  base;          /* device pointer */
    int    num_layers, num_heads, head_size, page_size, num_pages;
    int    dtype;         /* HPA_F32 or HPA_BF16 */
    size_t elem_bytes;
    size_t page_elems;    /* elements of one page of one layer (K and V, all heads) */
    size_t layer_elems;   /* num_pages * page_elems */
    size_t bytes;
    int    managed;
} HpaKVPool;
enum { HPA_F32 = 0, HPA_BF16 = 1 };
int  hpa_pool_create(HpaKVPool* pool, int num_layers, int num_heads, int head_size, int page_size,
                     int num_pages, int dtype, int managed);
void hpa_pool_destroy(HpaKVPool* pool);
/* device address of the K (kv=0) or V (kv=1) tile of (layer, page, head) */
void* hpa_pool_tile(const HpaKVPool* pool, int layer, int page, int kv, int head);
/* host-side layout helpers (tests / compat copies) */
size_t hpa_pool_k_index(const HpaKVPool* pool, int layer, int page, int head, int slot, int d);
size_t hpa_pool_v_index(const HpaKVPool* pool, int layer, int page, int head, int slot, int d);

/* ---------------- decode-step kernels (fp32) ----------------
 * B = sequences in the batch, C = channels, NH heads of head_size 64.
 * pos[b] = absolute position of the token decoded this step (== tokens
 * already cached for b); the token's K/V go to slot pos[b] and attention
 * covers positions 0..pos[b]. */

/* paged decode attention (attention_paged paged_infer.c:163-240 for one
 * query row per sequence at absolute position pos[b]): block-table gather of
 * K/V pages -> q.k^T -> online softmax -> PV.  q, out: [B][C]. */
int hpa_paged_attention_decode(const float* q, const HpaKVPool* pool, int layer,
                               const int* block_table, int bt_stride, const int* pos, float* out,
                               int B);

/* split-context (flash-decoding) form: each (sequence, head)'s context is cut
 * into `splits` (1..HPA_ATTN_MAX_SPLITS) ranges of 64-token tiles, one
 * workgroup each; the last range to finish merges the ranges' (max, sum,
 * acc) in range order (so the result does not depend on timing) and writes
 * out[b] -- row-major [B][C] or, out_frag != 0, the frag layout.  ws:
 * hpa_attn_ws_bytes(B, NH, splits) bytes of device memory whose counter part
 * is zero before the first launch (hpa_memset_async the whole buffer once;
 * every launch leaves it zero).  splits = 1 is the single-pass kernel above
 * (ws may be NULL).  Within fp32 rounding of the single pass (another
 * summation grouping), bit-identical across launches for a given splits. */
#define HPA_ATTN_MAX_SPLITS 16
size_t hpa_attn_ws_bytes(int B, int num_heads, int splits);
/* the engine's choice by shape only (num_cus <= 0: 256): ranges while B*NH*S
 * stays within one workgroup per CU, 2 between one and two per CU, else 1 */
int hpa_attn_pick_splits(int B, int num_heads, int max_ctx, int num_cus);
/* the same with the waves per workgroup (0: 4; 1, 2, 4 or 8) -- the engine
 * passes hpa_attn_pick_waves of its (global) batch */
int hpa_paged_attention_decode_split_w(const float* q, const HpaKVPool* pool, int layer, const int* block_table,
                                       int bt_stride, const int* pos, float* out, int B, int splits, void* ws,
                                       int out_frag, int waves);
/* 8 when the B*num_heads*splits workgroups fit one per CU, else 4 */
int hpa_attn_pick_waves(int B, int num_heads, int splits, int num_cus);
int hpa_paged_attention_decode_split(const float* q, const HpaKVPool* pool, int layer, const int* block_table,
                                     int bt_stride, const int* pos, float* out, int B, int splits, void* ws,
                                     int out_frag);
/* synthetic K/V fill of positions [0, ctx) for every sequence with U(-1,1)
 * from a counter-based hash (attention microbench / bench synthetic prefill) */
int hpa_pool_fill_random(const HpaKVPool* pool, const int* block_table, int bt_stride, int B,
                         int ctx, uint64_t seed);
/* the same for sequences seq_offset .. seq_offset+B-1 of a larger batch (a
 * shard fills exactly the rows the unsharded batch would get) */
int hpa_pool_fill_random_ex(const HpaKVPool* pool, const int* block_table, int bt_stride, int B,
                            int ctx, uint64_t seed, int seq_offset);

/* ---------------- fused decode-layer GEMMs (the engine's path) ----------------
 * "frag" layout: a [rows][K] fp32 matrix with rows padded to a multiple of 16
 * stored so that the v_mfma_f32_16x16x4_f32 operand fragment of (16-row
 * block, 16-deep k-step) is 1 KiB contiguous: element (m,k) at
 * ((m/16 * K/16 + k/16) * 64 + m%16 + 16*((k%16)/4)) * 4 + k%4.  Weights are
 * packed once at load; activations that feed a GEMM are written in it. */
size_t hpa_frag_elems(int rows, int K);           /* padded element count */
int hpa_pack_frag(const float* src, int rows, int K, int ld, float* dst); /* device -> device */
int hpa_unpack_frag(const float* src, int rows, int K, float* dst, int ld);
/* bf16 frag layout ([rows][K], rows padded to 16, K % 32 == 0): the
 * v_mfma_f32_16x16x32_bf16 operand fragment of (16-row block, 32-deep k-step s)
 * is 1 KiB contiguous; lane l = (m % 16) + 16*g holds k = 32s + 4g + {0..3} then
 * k = 32s + 16 + 4g + {0..3} (the two float4 the same lane reads from the fp32
 * frag layout at k16-steps 2s, 2s+1).  Element (m, k) at
 * ((m/16 * K/32 + k/32) * 64 + m%16 + 16*((k%16)/4)) * 8 + k%4 + 4*((k%32)/16).
 * Values are fp32 rounded to nearest even (hpa_pack_frag_bf16, device -> device). */
size_t hpa_frag_bf16_elems(int rows, int K);      /* padded element count (2 bytes each) */
int hpa_pack_frag_bf16(const float* src, int rows, int K, int ld, void* dst);

/* per-row LayerNorm statistics travel between kernels as partial sums
 * (sum x, sum x^2) over 16-column tiles: stats[tile][Mp][2]; a consumer sums
 * the `ntiles` partials of a row in order: mean = S1/C, var = S2/C - mean^2,
 * rstd = 1/sqrtf(var + 1e-5) (layernorm_forward, paged_infer.c:49-89, in its
 * one-pass form) and applies (x - mean) * rstd * w + b to its A fragments. */
enum { HPA_FEPI_QKV = 0, HPA_FEPI_RESID = 1, HPA_FEPI_GELU = 2, HPA_FEPI_LOGITS = 3 };
typedef struct {
    /* A = x (frag layout, M rows, K cols), optionally LayerNorm'ed on the fly */
    const float* x;
    int M, K;
    const float* ln_stats; /* NULL: no LN */
    int ln_ntiles;
    const float* ln_w;
    const float* ln_b;
    /* B = W^T, W (frag layout, N rows of K) */
    const float* w;
    int N;
    const float* bias;    /* [N] or NULL */
    int epilogue;         /* HPA_FEPI_* */
    /* QKV: out = q [M][C] row-major; K/V rows appended to pool pages at pos[m] */
    /* RESID: out = res_in + acc + bias (frag layout [M][N]); stats_out[N/16][Mp][2]
       (NULL: no statistics -- the consumer folds its LN and sums its own) */
    /* GELU: out = gelu(acc + bias) (frag layout [M][N]) */
    /* LOGITS: out = acc [M][N] row-major (ld = N); part_out[N/16 tiles][Mp][2] = (max, argmax) */
    float* out;
    const float* res_in;
    float* stats_out;
    float* part_out;
    const HpaKVPool* pool;
    int layer;
    const int* block_table;
    int bt_stride;
    const int* pos;
    int waves;            /* waves per workgroup sharing the K range: 4, 8 or 16; 0 = by shape.
                             Variant 4 on the resident logits kernel: 16 = its 16-wave
                             K-split form, 12 = its ring form, else by M (the two sum a
                             row's K in different orders: give sharded callers the
                             global batch's form) */
    int row_blocks;       /* 16-row blocks per workgroup: 1, 2 or 4; 0 = by shape */
    int variant;          /* 0 = by shape; 1 = looped (two trips in flight);
                             2 = one-shot (every operand load issued up front; one
                             row block; (waves, K/16) in {(4,48),(8,48),(16,48),(8,192),(16,192),(10,100)});
                             3 = loader / MFMA-wave ring (hpa_gemm_ring.hip): <= 64 padded rows,
                             LN folded (ln_fold_c1) or absent, QKV / GELU / RESID; one
                             12-wave workgroup per 32 columns and K part; waves = K parts
                             (0/1 = none; 2..4 need sk_slab / sk_count sized by
                             hpa_gemm_ring_workspace: the last part of a column pair sums
                             the parts in part order); row_blocks / col_tiles ignored;
                             4 = LOGITS only: activation-resident persistent kernel
                             (K = 768, rows <= 64; 16 waves); else stream-K (6) when
                             sk_slab / sk_count are given and rows <= 64; else as 1;
                             5 = bf16 weights only: A-resident kernel (col_tiles = rounds,
                             K <= 3200);
                             6 = stream-K (hpa_gemm_sk.hip; M <= 64, fp32 weights): one
                             8-wave workgroup per CU walks an equal contiguous share of
                             the (32-column super-tile, k16) steps, all M rows at once;
                             tiles split between workgroups are summed in workgroup
                             order by the last to arrive (sk_slab / sk_count).  LN
                             folded (ln_fold_c1) or applied on load (K <= 2048) */
    int col_tiles;        /* 16-column tiles per workgroup: 1; 2 (waves 4/8, row_blocks
                             2/4); 4 (waves 4, row_blocks 4); 0 = by shape.  A hint:
                             where M's row blocks or the waves cannot carry it, 1 */
    const int* row_seq;   /* QKV: block-table row of each GEMM row (NULL = the row
                             itself; prefill rows b*T+t -> b); LOGITS (looped and
                             bf16 kernels): the output row of each GEMM row
                             (gpt2_forward's per-position logits, written in place) */
    const float* ln_fold_c1; /* non-NULL: the LayerNorm is folded into w (packed by
                             hpa_ln_fold_pack: w = W*ln_w per column k, bias = c2):
                             A is x as it stands, and the epilogue applies
                             out[n] = rstd*(acc[n] - mean*c1[n]) + bias[n] with the
                             row statistics (one-pass) summed from the A fragments
                             the workgroup already holds (K = the LN width).  No LN
                             prologue and no statistics loads; ln_stats, ln_w and
                             ln_b are not read. */
    float* sk_slab;       /* variant 6: hpa_gemm_sk_workspace floats */
    int* sk_count;        /* variant 6: per-super-tile counters, zero before the first launch
                             (every launch leaves them zero) */
    int w_dtype;          /* HPA_F32 (0): w is fp32 frag layout.  HPA_BF16: w points at bf16
                             weights in the bf16 frag layout (hpa_pack_frag_bf16), K % 32 == 0;
                             A is rounded to bf16 (RNE) after the LayerNorm, products are
                             summed in fp32 on v_mfma_f32_16x16x32_bf16 (variant 0, 1
                             or 5; ln_fold_c1 must be NULL); waves 4/8. */
    /* LOGITS on the activation-resident kernel (variant 4, fp32) only: non-NULL
     * pick_next makes the launch's last workgroup to finish (an arrival ticket on
     * pick_count: one int, zero before the first launch, left zero) reduce the
     * argmax partials as hpa_argmax_final(part_out, ..., pick_next, pick_tokens,
     * pick_pos, NULL) would: next[m] = the lowest column of row m's maximum;
     * pick_tokens (nullable) gets it too, pick_pos (nullable) += 1.  Saves the
     * argmax launch. */
    int* pick_next;
    int* pick_tokens;
    int* pick_pos;
    int* pick_count;
} HpaFusedGemm;
/* LayerNorm folding for hpa_gemm_fused (layernorm_forward :49-89 followed by
 * matmul_forward :92-114, restated): for W [N][K] row-major (device), writes
 * dst_frag = frag-packed W[n][k]*ln_w[k], c1[n] = sum_k of those products and
 * c2[n] = sum_k ln_b[k]*W[n][k] + bias[n] (bias may be NULL); sums in double,
 * rounded once.  Then sum_k LN(x)_k W[n][k] + bias[n] =
 * rstd*(sum_k x_k W'[n][k] - mean*c1[n]) + c2[n]. */
int hpa_ln_fold_pack(const float* W, int N, int K, const float* ln_w, const float* ln_b, const float* bias,
                     float* dst_frag, float* c1, float* c2);
int hpa_gemm_fused(const HpaFusedGemm* g);
/* variant 3 K-split workspace for an (N) GEMM in `parts` K parts: slab
 * floats and counters (zero before the first launch; every launch leaves them
 * zero); nonzero on bad arguments */
int hpa_gemm_ring_workspace(int N, int parts, size_t* slab_floats, size_t* counters);
/* variant 6 workspace: slab floats and counters for an (N) GEMM on this
 * device's CU count (enough for any K and M <= 64) */
int hpa_gemm_sk_workspace(int N, size_t* slab_floats, size_t* counters);
/* argmax partials per row a LOGITS launch of g writes into part_out (the
 * `ntiles` of hpa_argmax_final): N/16 tiles, or one per workgroup of the
 * activation-resident kernel (variant 4) on the current stream; -1 if g is
 * not a valid LOGITS descriptor */
int hpa_logits_partials(const HpaFusedGemm* g);
/* the kernel a variant-4 fp32 LOGITS GEMM of this shape runs (LN applied):
 * 4 = activation-resident, 6 = stream-K (when given its workspace), 1 =
 * looped; -1 on a bad shape.  The engine allocates the stream-K workspace
 * exactly when this says 6. */
int hpa_logits_kernel(int M, int N, int K);
/* the launch shape hpa_gemm_fused picks when waves / row_blocks / col_tiles
 * are 0: out3 = {waves, row_blocks, col_tiles} */
void hpa_fused_pick(int M, int N, int K, int* out3);
/* the launch shape of a bf16-weight GEMM (w_dtype = HPA_BF16) when waves /
 * row_blocks / col_tiles are 0 */
void hpa_fused_pick_bf16(int M, int N, int K, int* out3);
/* bf16 weights, A-resident kernel (variant 5: the workgroup's rows of A
 * LayerNorm'ed and rounded into LDS once, waves walking waves*rounds column
 * tiles over the whole K; col_tiles = rounds for this variant):
 * out3 = {waves, row_blocks, rounds}; returns 1 where variant 0 uses it */
int hpa_fused_pick_bf16_ares(int M, int N, int K, int* out3);
int hpa_fused_pick_waves(int M, int N, int K);
/* ---------------- persistent decode layer (hpa_layer.hip) ----------------
 * The decode step's layer loop (reference gpt2_forward, paged_infer.c:659-722)
 * as ONE launch per layer l instead of five:
 *   attention(l) -> attproj(l) -> fc(l) -> fcproj(l) -> qkv(l+1)
 * or, chain_only, the decode attention as its own launch before and one
 * launch of attproj(l) -> fc(l) -> fcproj(l) -> qkv(l+1) (the engine's
 * default form: measured faster at every batch, profiles/r3/pl_ab.txt).
 * One 12-wave workgroup per CU (grid = CU count, residency checked with the
 * occupancy API), split into three 4-wave slots; every phase deals its units
 * (a 16x16 output tile over a K range, or an attention unit) one per slot.
 * Each slot loads its next phase's weight fragments into registers BEFORE
 * that phase's wait, so the weight stream overlaps the hand-off.  Hand-offs
 * inside the launch: write-through (sc1) stores, drained, one agent-scope
 * arrival per workgroup on a counter sharded 8 ways, polled with sc1 loads
 * (MI355X_MICROARCH.md "Valid forms", row 1).  fcproj is split over K into 4
 * parts and the last part of a tile to draw its ticket adds the parts in part
 * order.  qkv and fc follow the one-shot kernel's summation order (4 waves x
 * K/4, folded in wave order): their rows are bit-identical to the launch path.
 * fp32 frag-packed weights with the LayerNorms folded (hpa_ln_fold_pack);
 * C = 128 or 768 (num_heads 2 or 12), B <= 64, B*num_heads*splits <= 3 x CUs.
 * Every spin is bounded (200 ms): a timeout stores a nonzero code in *err and
 * ends the launch (the outputs are then garbage). */
typedef struct {
    int B, C, num_heads, splits;  /* splits: context ranges of the attention */
    int last;                     /* 1: no qkv(l+1) phase (last layer) */
    int chain_only;               /* 1: no attention phase -- the caller launched the decode
                                     attention (frag output into att) before: the launch is
                                     attproj -> fc -> fcproj -> qkv(l+1); 2..5: the same with wide
                                     units (C = 768), waves per unit of (attproj, fc / fcproj,
                                     qkv): 2 (12, 12, 12) B <= 16; 3 (12, 6, 6) B <= 32;
                                     4 (12, 4, 6) B <= 48; 5 (12, 4, 4) B <= 64; 6: every phase
                                     in units of all 12 waves of a workgroup holding T 16-column
                                     tiles (T by batch, one unit per workgroup, the 12-wave
                                     summation order at every B <= 64), 16-byte epilogues,
                                     waits per row block (C = 768); 8: the chain for
                                     MFMA-bound wide layers (C = 768, 1024, 1280 or 1600: GPT-2 124M to XL): units of
                                     12 waves x up to 7 tiles, weights streamed per tile */
    const HpaKVPool* pool;
    int layer;
    const int* block_table;
    int bt_stride;
    const int* pos;
    const float* q;               /* q of layer l [B][C] row-major (read) */
    float* att;                   /* attention output, frag [Mp][C] */
    float* res;                   /* residual in (frag [Mp][C]); fcproj writes the next */
    float* res2;                  /* res + attproj, frag [Mp][C] */
    float* fch;                   /* gelu(fc), frag [Mp][4C] */
    const float* w_ap;            /* frag-packed attprojw [C][C] */
    const float* b_ap;
    const float* w_fc;            /* LN2-folded fcw [4C][C] */
    const float* fc_c1;
    const float* fc_c2;
    const float* w_fp;            /* frag-packed fcprojw [C][4C] */
    const float* b_fp;
    const float* w_qkv;           /* layer l+1, LN1-folded qkvw [3C][C] (unused when last) */
    const float* qkv_c1;
    const float* qkv_c2;
    float* q_out;                 /* q of layer l+1 [B][C]; its K/V go into layer l+1's pages */
    float* stats_out;             /* last layer: LNf statistics [C/16][Mp][2] of res; else NULL */
    float* rec;                   /* attention split records (hpa_decode_layer_sizes) */
    float* slab;                  /* K-part partial sums */
    int* counters;                /* this layer's counter block, zero before the launch */
    int* err;                     /* this step's: 0, or the code of the first timed-out wait; zeroed
                                     with the counters before every step (the launch's waits bail
                                     out at once when it is set) */
    int* err_sticky;              /* nullable: the first code also lands here, never zeroed by a
                                     step (gpt2_decode_status reads and clears it) */
    int stats_mp;                 /* row stride of stats_out; 0: this launch's Mp */
} HpaLayerArgs;
/* 1 if the persistent layer applies (shape, CU count, residency), else 0 */
int hpa_decode_layer_eligible(int B, int C, int num_heads, int splits);
/* 1 if chain form `form` (HpaLayerArgs.chain_only 6, 7: C = 768; 8: C = 768,
 * 1024, 1280 or 1600) applies to B rows on this device's CU count, else 0 */
int hpa_decode_chain_eligible(int B, int C, int num_heads, int form);
/* splits the persistent layer uses by default for this batch */
int hpa_decode_layer_pick_splits(int B, int num_heads, int max_ctx);
/* sizes: out[0] = rec floats, out[1] = slab floats, out[2] = counter ints per layer */
int hpa_decode_layer_sizes(int B, int C, int num_heads, int splits, size_t* out3);
int hpa_decode_layer(const HpaLayerArgs* a);
/* the decode step's first launch at GPT-2 124M shapes (C = 768, 12 heads,
 * B <= 64, LN1 folded into w_qkv / qkv_c1 / qkv_c2 of layer 0): the embedding
 * wte[tokens[b]] + wpe[pos[b]] (encoder_forward, paged_infer.c:41-47) into
 * res (frag), layer 0's q into q_out and its K/V into layer 0's pages (chain
 * form 6's qkv phase), and zero_bytes of `zero` (the step's counter block,
 * 16-byte granules) zeroed -- one launch for the embed kernel and the qkv
 * GEMM.  Reads a->B, pool, block_table, bt_stride, pos, res, w_qkv, qkv_c1,
 * qkv_c2, q_out; the layer fields are ignored. */
int hpa_decode_first(const HpaLayerArgs* a, const int* tokens, const float* wte, const float* wpe, void* zero,
                     size_t zero_bytes);
/* ---------------- pipelined halves (hpa_pipe.hip) ----------------
 * The whole layer loop of a decode step (gpt2_forward, paged_infer.c:659-722,
 * every layer l = 0..L-1: attention(l) -> attproj(l) -> fc(l) -> fcproj(l) ->
 * qkv(l+1)) as ONE persistent launch, after the step's first launch
 * (hpa_decode_first: embedding, qkv(0), the counter block zeroed) and before
 * the logits.  The batch is cut into two halves of row blocks; the CUs take
 * fixed roles: `g_cus` CUs run the GEMM chain of one half while the others
 * stream the paged attention of the other half (software pipeline, slot s:
 * attention(s/2, s%2) beside chain((s-1)/2, (s-1)%2)).  The attention is
 * paged_attn_decode_f32's (4 waves per (sequence, head), one context range)
 * and the chain units are chain form 6's (12 waves over K), so a step equals
 * the chain-form step bit for bit.  GPT-2 124M shapes: C = 768, 12 heads,
 * fp32 weights (LN-folded frag packs) and an fp32 pool, 17..64 rows with both
 * halves non-empty.  Bounded spins, error words as hpa_decode_layer. */
typedef struct {
    const float *w_ap, *b_ap;                 /* layer l: attprojw (frag), attprojb */
    const float *w_fc, *fc_c1, *fc_c2;        /* LN2-folded fcw (frag), c1, c2 */
    const float *w_fp, *b_fp;                 /* fcprojw (frag), fcprojb */
    const float *w_qkv, *qkv_c1, *qkv_c2;     /* layer l+1's LN1-folded qkvw (NULL at the last layer) */
} HpaPipeLayer;
typedef struct {
    int B, num_layers;
    const HpaKVPool* pool;        /* fp32 pages; layer l+1's K/V appended by qkv(l+1) */
    const int* block_table;
    int bt_stride;
    const int* pos;
    const HpaPipeLayer* layers;   /* DEVICE array [num_layers] */
    float* q;                     /* q [B][C] row-major: layer 0's from the first launch, rewritten per layer */
    float* att;                   /* frag [Mp][C] */
    float* res;                   /* residual (frag [Mp][C]): the embedding in, the last layer's out */
    float* res2;                  /* frag [Mp][C] */
    float* fch;                   /* frag [Mp][4C] */
    float* slab;                  /* fcproj K-part partials: hpa_decode_pipe_sizes out[0] floats */
    float* stats_out;             /* LNf statistics of the last layer's res [C/16][stats_mp][2] */
    int stats_mp;
    int* counters;                /* [num_layers][layer_ctr_ints], zero before the launch */
    size_t layer_ctr_ints;        /* >= hpa_decode_pipe_sizes out[1] */
    int* err;                     /* as HpaLayerArgs.err / err_sticky */
    int* err_sticky;
    int g_cus;                    /* CUs of the GEMM role (multiple of 8; 0: 64) */
} HpaPipeArgs;
/* 1 if the pipelined-halves launch applies to B rows (C, heads, pool dtype, CU count) */
int hpa_decode_pipe_eligible(int B, int C, int num_heads, int kv_dtype);
/* out2 = {slab floats, counter ints per layer} */
int hpa_decode_pipe_sizes(int B, size_t* out2);
int hpa_decode_pipe(const HpaPipeArgs* a);
/* diagnostic builds (-DHPA_PIPE_TRACE) only: the per-(layer, half, workgroup)
 * event stamps of the last launch, [2 * layers][256][12] u64 (10-ns ticks);
 * host NULL clears them; returns 1 in the product library */
int hpa_decode_pipe_trace(unsigned long long* host, int layers);
/* ---------------- bf16-weight decode chain (hpa_chain_b16.hip) ----------------
 * The layer's GEMMs on bf16 weights (BASELINE config 5) as ONE persistent
 * launch after the layer's decode-attention launch:
 *   attproj(l) -> fc(l) -> fcproj(l) -> qkv(l+1)
 * (gpt2_forward, paged_infer.c:659-722), in place of four bf16 GEMM launches.
 * C = 768, 12 heads, B = 1..256; one 8-wave workgroup per CU; LayerNorms on
 * the operand path with the row statistics from the consumer's own operand
 * fragments; weights in the bf16 frag layout (hpa_pack_frag_bf16); operands
 * rounded to bf16, fp32 accumulation.  Same hand-off protocol, bounded spins
 * and error words as hpa_decode_layer. */
typedef struct {
    int B, layer, last;           /* last: no qkv(l+1) phase; stats_out then written */
    const HpaKVPool* pool;        /* fp32 or bf16 pages; K/V of layer l+1 appended */
    const int* block_table;
    int bt_stride;
    const int* pos;
    const float* att;             /* attention output of layer l, frag [Mp][C] */
    float* res;                   /* residual in (frag [Mp][C]); fcproj writes the next */
    float* res2;                  /* res + attproj, frag [Mp][C] */
    float* fch;                   /* gelu(fc), bf16 frag layout [Mp][4C] (half the buffer) */
    const void* w_ap;             /* bf16 frag packs: attprojw [C][C], fcw [4C][C], */
    const void* w_fc;             /* fcprojw [C][4C], qkvw of layer l+1 [3C][C] */
    const void* w_fp;
    const void* w_qkv;
    const float *b_ap, *ln2_w, *ln2_b, *b_fc, *b_fp, *ln1_w, *ln1_b, *b_qkv; /* ln1 / b_qkv: layer l+1 */
    float* q_out;                 /* q of layer l+1 [B][C] row-major */
    float* stats_out;             /* last layer: LNf statistics [C/16][stats_mp][2] of res; else NULL */
    int stats_mp;                 /* 0: ceil(B/16)*16 */
    float* slab;                  /* fcproj K-part partials (hpa_decode_chain_b16_sizes out[0] floats) */
    int* counters;                /* this layer's counter block (out[1] ints), zero before the launch */
    int* err;                     /* as HpaLayerArgs.err / err_sticky */
    int* err_sticky;
} HpaChainB16Args;
int hpa_decode_chain_b16_eligible(int B, int C, int num_heads);
/* out2 = {slab floats, counter ints per layer} */
int hpa_decode_chain_b16_sizes(int B, size_t* out2);
int hpa_decode_chain_b16(const HpaChainB16Args* a);
/* the step's first launch on this path: the embedding wte[tokens[b]] +
 * wpe[pos[b]] (encoder_forward, paged_infer.c:41-47) into res, layer 0's q
 * and K/V (the chain's qkv phase; w_qkv / b_qkv / ln1_* of layer 0), and
 * zero_bytes of `zero` (the step's counter block) zeroed -- one launch for
 * the embed kernel and the qkv(0) GEMM.  Reads B, pool, block_table,
 * bt_stride, pos, res, w_qkv, b_qkv, ln1_w, ln1_b, q_out. */
int hpa_decode_chain_b16_first(const HpaChainB16Args* a, const int* tokens, const float* wte, const float* wpe,
                               void* zero, size_t zero_bytes);
/* diagnostic builds (-DHPA_LAYER_TRACE) only, else returns 1: the bf16
 * chain's per-(layer, workgroup) event stamps, as hpa_decode_layer_trace */
int hpa_decode_chain_b16_trace(unsigned long long* host, int layers);
/* diagnostic builds (-DHPA_LAYER_TRACE) only, else returns 1: per-(layer,
 * workgroup) event stamps [layers][256][16] of the last launches (10 ns
 * ticks); host = NULL clears them */
int hpa_decode_layer_trace(unsigned long long* host, int layers);
/* diagnostic builds only, else returns 1: chain form 8's fc phase of layer 5,
 * per wave ([256][12][16] u64 s_memtime: A loads issued, each half-tile's
 * MFMAs issued, loop done); host = NULL clears them */
int hpa_decode_cx_wave_trace(unsigned long long* host);
/* diagnostic builds (-DHPA_RG_TRACE) only, else returns 1: the ring logits
 * kernel's per-workgroup stamps of the last launch: [2][256][24] u64, s_memrealtime
 * (10 ns ticks) then s_memtime (shader clock) */
int hpa_logits_trace(unsigned long long* host);
/* residual = wte[tok] + wpe[pos] in frag layout [Mp][C], stats (1 tile) */
int hpa_embed_frag(const int* tokens, const int* pos, const float* wte, const float* wpe,
                   float* res_frag, float* stats, int B, int C);
/* the same, also zeroing zero[0 .. zero_bytes) (16-byte granules): the
 * decode step's hand-off counters without a memset node of their own */
int hpa_embed_frag_zero(const int* tokens, const int* pos, const float* wte, const float* wpe,
                        float* res_frag, float* stats, int B, int C, void* zero, size_t zero_bytes);
/* greedy id from the logits GEMM's per-tile (max, argmax) partials:
 * lowest index wins ties; next[b], tokens[b] = next[b], pos[b] += 1.
 * active (nullable, [B]): rows with active[b] <= 0 are left untouched */
int hpa_argmax_final(const float* part, int ntiles, int Mp, int B, int* next, int* tokens, int* pos,
                     const int* active);
/* multinomial draw per row from softmax(logits) with the reference's
 * generator and arithmetic order (softmax_forward :259-286, sample_mult
 * :837-848, random_f32 :826-835), one xorshift state per row advanced on the
 * device; next[b], tokens[b] = next[b], pos[b] += 1 (tokens/pos may be NULL);
 * active as hpa_argmax_final (an inactive row's state does not advance) */
int hpa_sample_final(const float* logits, int B, int V, unsigned long long* state, int* next, int* tokens,
                     int* pos, const int* active);
/* the same draw from the single-lane sequential kernel (the ordered fp32
 * additions as one dependent chain); kept as the measured baseline and as a
 * cross-check of hpa_sample_final's integer-scan formulation */
int hpa_sample_final_serial(const float* logits, int B, int V, unsigned long long* state, int* next, int* tokens,
                            int* pos, const int* active);
/* paged decode attention writing its output in frag layout ([B][C]) */
int hpa_paged_attention_decode_frag(const float* q, const HpaKVPool* pool, int layer,
                                    const int* block_table, int bt_stride, const int* pos,
                                    float* out_frag, int B);

/* ---------------- prefill (multi-query) ----------------
 * attention_paged (paged_infer.c:163-240) for T query rows per sequence at
 * absolute positions start[b] + t, causal over the sequence's pages: q
 * [B*T][C] row-major (row = b*T + t), out frag layout [ceil16(B*T)][C].
 * S = QK^T and O += PV on v_mfma_f32_16x16x4_f32 (dense here), online
 * softmax from the reference's -10000 floor.  The K/V of every query
 * position must already be in the pages (the prefill QKV GEMM appends them). */
int hpa_paged_attention_prefill(const float* q, const HpaKVPool* pool, int layer, const int* block_table,
                                int bt_stride, const int* start, int B, int T, float* out_frag);
/* ragged form (continuous batching): sequence b has len[b] >= 0 query rows
 * starting at row row0[b] of q / out (device arrays, given together);
 * T = max(len).  row0 = len = NULL is the uniform form above. */
int hpa_paged_attention_prefill_ragged(const float* q, const HpaKVPool* pool, int layer, const int* block_table,
                                       int bt_stride, const int* start, const int* row0, const int* len, int B,
                                       int T, float* out_frag);
/* rows[i] of a frag-layout [src_Mp][C] matrix and of its LN statistics
 * ([C/16][src_Mp][2]) -> row i of dst / dst_stats (n rows; prefill -> logits);
 * rows[i] < 0 leaves row i of dst as it is */
int hpa_gather_rows_frag(const float* src, const float* src_stats, int src_Mp, const int* rows, int n,
                         float* dst, float* dst_stats, int dst_Mp, int C);

/* ---------------- multi-GPU: RCCL over xGMI (hpa_comm.hip) ----------------
 * One process per GPU.  Rank 0 makes the id
 * (hpa_comm_unique_id), the launcher hands it to every rank (any out-of-band
 * channel: a file -- bench.py --, sockets, MPI), and each rank binds its
 * current device with hpa_comm_init.  The decode engine's end-of-step gather
 * (gpt2_decode_gather) runs on it. */
size_t hpa_comm_id_bytes(void);                     /* sizeof(ncclUniqueId) = 128 */
int    hpa_comm_unique_id(void* id, size_t id_bytes);
int    hpa_comm_init(int nranks, int rank, const void* id);
int    hpa_comm_destroy(void);
int    hpa_comm_size(void);                         /* 0 before hpa_comm_init */
int    hpa_comm_rank(void);                         /* -1 before hpa_comm_init */
/* root receives every rank's bytes in rank order (ncclSend/ncclRecv group;
 * uneven sizes allowed) on `stream` (NULL = the library stream), async */
int    hpa_comm_gatherv(const void* send, size_t send_bytes, void* recv, const size_t* bytes_per_rank, int root,
                        void* stream);
/* the gather's layout, host arithmetic only (what hpa_comm_gatherv posts):
 * recv_off[r] = byte offset of rank r's rows in root's buffer (rank order);
 * returns the number of ncclRecv the root posts (ranks != root with bytes),
 * or 1 / 0 on a non-root rank (it sends iff its bytes are nonzero); -1 on bad
 * arguments.  *own_off = root's own rows' offset (its local copy). */
int    hpa_comm_gather_layout(int nranks, int rank, int root, const size_t* bytes_per_rank, size_t* recv_off,
                              size_t* own_off);
/* the gather's schedule, host arithmetic only: the point-to-point operations
 * THIS rank posts for one hpa_comm_gatherv, in posting order.  hpa_comm_gatherv
 * executes exactly this list (ncclSend / ncclRecv inside one NCCL group, then
 * the root's local copy), so a host transport can run the same schedule (the
 * world-size-2..4 gloo tests, tests/test_multi_rank.py).  SEND: send_bytes of
 * the send buffer to `peer` (offset 0); RECV: `bytes` from `peer` at `offset`
 * of recv; COPY (root): its own rows into recv at `offset`.  Zero-byte
 * operations are never listed.  Returns the operation count (<= nranks), -1 on
 * bad arguments or when max_ops is too small (ops may be NULL to count). */
enum { HPA_COMM_SEND = 0, HPA_COMM_RECV = 1, HPA_COMM_COPY = 2 };
typedef struct {
    int op;        /* HPA_COMM_* */
    int peer;      /* the other rank (COPY: this rank) */
    size_t offset; /* byte offset in recv (SEND: 0, in send) */
    size_t bytes;
} HpaCommOp;
int    hpa_comm_gather_plan(int nranks, int rank, int root, const size_t* bytes_per_rank, HpaCommOp* ops,
                            int max_ops);
/* timing helpers over the communicator (RCCL all-reduce on the library
 * stream, then a host wait): a barrier, and the maximum of one host double
 * over the ranks (bench.py's max-over-ranks step time) */
int    hpa_comm_barrier(void);
int    hpa_comm_allreduce_max(double* value);
/* single-process form (one process driving ndev GPUs,
 * ncclCommInitAll): communicators for devices devs[0..ndev-1], rank i =
 * devs[i]; hpa_comm_use(i) makes comm i (and device devs[i]) current for the
 * calls above.  Exclusive with hpa_comm_init. */
int    hpa_comm_init_all(int ndev, const int* devs);
int    hpa_comm_use(int index);
/* ncclGroupStart / ncclGroupEnd around the collectives posted between them
 * (the single-process form: every device's gather from one thread) */
int    hpa_comm_group_start(void);
int    hpa_comm_group_end(void);

/* ---------------- reference-layout kernels (drop-in compat) ----------------
 * Pages in the reference layout: token-major [block_size][C] per page
 * (block_manager.c:145-146).  key_blocks/value_blocks: DEVICE arrays of
 * DEVICE page pointers.  Reference arithmetic order (no FMA contraction), so
 * results match the reference bit-for-bit up to expf/tanhf ulps. */
int hpa_ref_attention_paged(float* out, float* preatt, float* att, const float* inp,
                            float* const* key_blocks, float* const* value_blocks, int B, int T,
                            int C, int NH, int offset, int block_size);
/* cached == 0: matmul_forward (:92-114); cached == 1: matmul_cached
 * (:117-160): rows t < T-1 compute only the first C outputs (Q) */
int hpa_ref_matmul(float* out, const float* inp, const float* weight, const float* bias, int B,
                   int T, int C, int OC, int cached);
int hpa_ref_layernorm(float* out, float* mean, float* rstd, const float* inp, const float* weight,
                      const float* bias, int N, int C);
int hpa_ref_encoder(float* out, const int* inp, const float* wte, const float* wpe, int B, int T,
                    int C, int pos_offset);
int hpa_ref_gelu(float* out, const float* inp, int N);
int hpa_ref_residual(float* out, const float* a, const float* b, int N);
int hpa_ref_softmax(float* probs, const float* logits, int N, int V);

#ifdef __cplusplus
}
#endif
#endif
