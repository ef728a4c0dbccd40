/*
 * block_manager.h -- drop-in for mx60s/llm.c-paged block_manager.c
 * (the paged KV page allocator, reference block_manager.c:1-201).
 *
 * Source compatibility: the reference's callers (block_manager_test.c,
 * paged_infer.c) `#include "block_manager.c"` and touch the structs'
 * fields directly; every field they use keeps its name and type, and
 * `manager->blocks[i]`, `manager->prompt_block_list[p][i]`,
 * `manager->prompt_block_count[p]` index exactly as before.  The capacity
 * macros MAX_PROMPTS / MAX_BLOCKS / BLOCK_SIZE (block_manager.c:4-6) remain
 * the defaults of create_block_manager(); create_block_manager_ex() takes
 * them at run time (a GPT-2 124M batch of 64 x 1024 tokens at page 16 needs
 * 4096 pages; GPT-2 XL or bf16 configs up to 65536).  The manager, its page
 * descriptors and its page lists are ONE malloc block, so the reference
 * idiom `free(manager)` still releases everything the manager owns.
 *
 * Page payloads come from a backend: host malloc (the reference behaviour,
 * the default when built without HIP), HIP managed memory (default inside
 * libpaged_hip.so, so host code can still dereference keys/values), or a
 * view into a device page pool (the decode engine: keys/values then point at
 * layer 0's K/V tiles of that page in HBM and nothing is allocated per page).
 *
 * Behavioural notes vs the reference:
 *  - lru_epoch and every page's filled/lru_counter start at 0 (the reference
 *    leaves them uninitialised, block_manager.c:38-52);
 *  - allocation is first-fit by page index exactly like the linear scan of
 *    block_manager.c:121-128, found through a free-page bitmap;
 *  - eviction is the reference's: the page with the smallest lru_counter
 *    strictly below lru_epoch loses its whole prompt (:92-113);
 *  - a prompt's page list that is full makes request_block return NULL with
 *    a message (the reference would overflow its fixed row);
 *  - the debug printf chatter of get_current_block / free_blocks_for_prompt /
 *    page_out_lru_block is off unless bm_set_verbose(1).
 */
#ifndef BLOCK_MANAGER_H
#define BLOCK_MANAGER_H
#include <stddef.h>
#ifdef __cplusplus
extern "C" {
#endif

#ifndef MAX_PROMPTS
#define MAX_PROMPTS 100
#endif
#ifndef MAX_BLOCKS
#define MAX_BLOCKS 100
#endif
#ifndef BLOCK_SIZE
#define BLOCK_SIZE 32
#endif

/* block_manager.c:9-15 */
typedef struct {
    float* keys;
    float* values;
    int filled;
    int prompt_id;
    int lru_counter;
} KVBlock;

/* where page payloads live; alloc returns the payload for (page, kv) */
typedef struct {
    void* (*alloc)(void* ctx, int page, int kv, size_t bytes);
    void (*release)(void* ctx, int page, int kv, void* payload);
    void* ctx;
} BMPageBackend;

/* block_manager.c:17-23, plus run-time capacity */
typedef struct {
    int C;
    KVBlock* blocks;             /* [max_blocks] */
    int** prompt_block_list;     /* [max_prompts] rows of [max_blocks_per_prompt] */
    int* prompt_block_count;     /* [max_prompts] */
    int lru_epoch;
    /* ---- extensions ---- */
    int max_prompts;
    int max_blocks;
    int block_size;              /* tokens per page */
    int max_blocks_per_prompt;
    int* block_table;            /* contiguous storage behind prompt_block_list */
    unsigned long long* free_bits; /* bit set = page free */
    int free_words;
    int free_hint;               /* lowest word that may hold a free page */
    int free_count;
    BMPageBackend backend;
    int dirty_lo, dirty_hi;      /* prompt rows changed since bm_clear_dirty */
    int last_evicted_prompt;     /* prompt paged out by the last request_block, or -1 */
} BlockManager;

/* ---- reference API (signatures as block_manager.c) ---- */
void print_state(BlockManager* manager, int prompt);
BlockManager* create_block_manager(int channels);
int get_next_block_id(BlockManager* manager, int prompt, int block_id);
KVBlock* get_current_block(BlockManager* manager, int prompt_id);
void free_blocks_for_prompt(BlockManager* manager, int prompt_id);
int find_least_recently_used_block(BlockManager* manager);
void page_out_lru_block(BlockManager* manager);
KVBlock* request_block(BlockManager* manager, int prompt_id);
float*** collect_kv_blocks(BlockManager* manager, int prompt_id, int* num_blocks);

/* ---- additive API ---- */
BlockManager* create_block_manager_ex(int channels, int max_prompts, int max_blocks, int block_size,
                                      int max_blocks_per_prompt);
void destroy_block_manager(BlockManager* manager); /* frees live pages, then the manager */
void bm_set_backend(BlockManager* manager, const BMPageBackend* backend); /* NULL = default */
void bm_use_host_pages(BlockManager* manager); /* malloc'd pages, as the reference */
void bm_set_verbose(int on);
int  bm_block_index(const BlockManager* manager, const KVBlock* block);
int  bm_free_pages(const BlockManager* manager);
void bm_clear_dirty(BlockManager* manager);
/* the backend compiled in as default: 0 host malloc, 1 HIP managed memory */
int  bm_default_backend_kind(void);

#ifdef __cplusplus
}
#endif
#endif
