/*
 * block_manager.c -- drop-in page allocator for the paged KV cache.
 * Same API and allocation policy as the reference block_manager.c of
 * mx60s/llm.c-paged (first-fit page, per-prompt ordered page lists, LRU
 * whole-prompt eviction); run-time capacity, bitmap first-fit, pluggable
 * page storage.  See include/block_manager.h for the differences.
 *
 * This file can be #included textually (as the reference's tests and
 * paged_infer.c do with the reference file) or compiled into
 * libpaged_hip.so (with -DBM_WITH_HIP, where pages default to HIP managed
 * memory so host code may still read and write keys/values).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "block_manager.h"

#ifdef BM_WITH_HIP
#include "hip_paged_attn.h"
#endif

static int g_bm_verbose = 0;
void bm_set_verbose(int on) { g_bm_verbose = on; }

/* ---------------- page payload backends ---------------- */
static void* bm_host_alloc(void* ctx, int page, int kv, size_t bytes) {
    (void)ctx; (void)page; (void)kv;
    return malloc(bytes);
}
static void bm_host_release(void* ctx, int page, int kv, void* p) {
    (void)ctx; (void)page; (void)kv;
    free(p);
}
#ifdef BM_WITH_HIP
static void* bm_managed_alloc(void* ctx, int page, int kv, size_t bytes) {
    (void)ctx; (void)page; (void)kv;
    return hpa_malloc_managed(bytes);
}
static void bm_managed_release(void* ctx, int page, int kv, void* p) {
    (void)ctx; (void)page; (void)kv;
    hpa_free(p);
}
#endif

int bm_default_backend_kind(void) {
#ifdef BM_WITH_HIP
    return 1;
#else
    return 0;
#endif
}

static BMPageBackend bm_default_backend(void) {
    BMPageBackend b;
#ifdef BM_WITH_HIP
    b.alloc = bm_managed_alloc;
    b.release = bm_managed_release;
#else
    b.alloc = bm_host_alloc;
    b.release = bm_host_release;
#endif
    b.ctx = NULL;
    return b;
}

void bm_set_backend(BlockManager* m, const BMPageBackend* backend) {
    m->backend = backend ? *backend : bm_default_backend();
}

/* explicit host-malloc pages (the reference behaviour), e.g. CPU-only tests */
void bm_use_host_pages(BlockManager* m) {
    m->backend.alloc = bm_host_alloc;
    m->backend.release = bm_host_release;
    m->backend.ctx = NULL;
}

/* ---------------- free-page bitmap ---------------- */
static void bm_mark_free(BlockManager* m, int i) {
    m->free_bits[i >> 6] |= 1ull << (i & 63);
    if ((i >> 6) < m->free_hint) m->free_hint = i >> 6;
    m->free_count++;
}
static void bm_mark_used(BlockManager* m, int i) {
    m->free_bits[i >> 6] &= ~(1ull << (i & 63));
    m->free_count--;
}
/* lowest free page index == the reference's linear first-fit scan (:121-128) */
static int bm_first_free(BlockManager* m) {
    for (int w = m->free_hint; w < m->free_words; w++) {
        if (m->free_bits[w]) {
            m->free_hint = w;
            return (w << 6) + __builtin_ctzll(m->free_bits[w]);
        }
    }
    m->free_hint = m->free_words;
    return -1;
}

static size_t bm_align16(size_t x) { return (x + 15) & ~(size_t)15; }

BlockManager* create_block_manager_ex(int channels, int max_prompts, int max_blocks, int block_size,
                                      int max_blocks_per_prompt) {
    if (channels <= 0 || max_prompts <= 0 || max_blocks <= 0 || block_size <= 0 ||
        max_blocks_per_prompt <= 0) {
        fprintf(stderr, "create_block_manager: invalid capacity.\n");
        return NULL;
    }
    int words = (max_blocks + 63) / 64;
    size_t o_blocks = bm_align16(sizeof(BlockManager));
    size_t o_rows = o_blocks + bm_align16(sizeof(KVBlock) * (size_t)max_blocks);
    size_t o_count = o_rows + bm_align16(sizeof(int*) * (size_t)max_prompts);
    size_t o_table = o_count + bm_align16(sizeof(int) * (size_t)max_prompts);
    size_t o_bits = o_table + bm_align16(sizeof(int) * (size_t)max_prompts * max_blocks_per_prompt);
    size_t total = o_bits + sizeof(unsigned long long) * (size_t)words;
    char* mem = (char*)calloc(1, total); /* block_manager.c:39 (one block: free(manager) works) */
    if (!mem) {
        fprintf(stderr, "create_block_manager: out of memory.\n");
        return NULL;
    }
    BlockManager* m = (BlockManager*)mem;
    m->C = channels;
    m->blocks = (KVBlock*)(mem + o_blocks);
    m->prompt_block_list = (int**)(mem + o_rows);
    m->prompt_block_count = (int*)(mem + o_count);
    m->block_table = (int*)(mem + o_table);
    m->free_bits = (unsigned long long*)(mem + o_bits);
    m->max_prompts = max_prompts;
    m->max_blocks = max_blocks;
    m->block_size = block_size;
    m->max_blocks_per_prompt = max_blocks_per_prompt;
    m->free_words = words;
    m->lru_epoch = 0;
    m->last_evicted_prompt = -1;
    for (int p = 0; p < max_prompts; p++) {
        m->prompt_block_list[p] = m->block_table + (size_t)p * max_blocks_per_prompt;
        m->prompt_block_count[p] = 0; /* :42-44 */
        for (int i = 0; i < max_blocks_per_prompt; i++) m->prompt_block_list[p][i] = -1;
    }
    for (int i = 0; i < max_blocks; i++) { /* :46-50 */
        m->blocks[i].keys = NULL;
        m->blocks[i].values = NULL;
        m->blocks[i].prompt_id = -1;
        m->blocks[i].filled = 0;
        m->blocks[i].lru_counter = 0;
    }
    m->free_count = 0;
    for (int i = 0; i < max_blocks; i++) bm_mark_free(m, i);
    m->free_hint = 0;
    m->backend = bm_default_backend();
    m->dirty_lo = max_prompts;
    m->dirty_hi = -1;
    return m;
}

/* block_manager.c:38-52 */
BlockManager* create_block_manager(int channels) {
    return create_block_manager_ex(channels, MAX_PROMPTS, MAX_BLOCKS, BLOCK_SIZE, MAX_BLOCKS);
}

void destroy_block_manager(BlockManager* m) {
    if (!m) return;
    for (int p = 0; p < m->max_prompts; p++)
        if (m->prompt_block_count[p]) free_blocks_for_prompt(m, p);
    free(m);
}

/* block_manager.c:25-36 */
void print_state(BlockManager* manager, int prompt) {
    printf("Block manager llru %d\n", manager->lru_epoch);
    int n = manager->prompt_block_count[prompt];
    printf("Prompt %d block count: %d\n", prompt, n);
    for (int i = 0; i < n; i++) {
        int id = manager->prompt_block_list[prompt][i];
        printf("Block %d: filled %d, llru %d\n", id, manager->blocks[id].filled,
               manager->blocks[id].lru_counter);
    }
}

/* block_manager.c:54-63: the id after block_id in the prompt's list, else -1 */
int get_next_block_id(BlockManager* manager, int prompt, int block_id) {
    if (prompt < 0 || prompt >= manager->max_prompts) return -1;
    int n = manager->max_blocks_per_prompt;
    const int* list = manager->prompt_block_list[prompt];
    for (int i = 0; i < n; i++)
        if (list[i] == block_id && i + 1 < n) return list[i + 1];
    return -1;
}

/* block_manager.c:65-76 */
KVBlock* get_current_block(BlockManager* manager, int prompt_id) {
    if (prompt_id < 0 || prompt_id >= manager->max_prompts) return NULL;
    int n = manager->prompt_block_count[prompt_id];
    if (g_bm_verbose) printf("Current num_blocks in prompt is %d\n", n);
    if (n == 0) return NULL;
    int idx = manager->prompt_block_list[prompt_id][n - 1];
    if (g_bm_verbose) printf("Current block idx is %d\n", idx);
    return &manager->blocks[idx];
}

static void bm_mark_dirty(BlockManager* m, int p) {
    if (p < m->dirty_lo) m->dirty_lo = p;
    if (p > m->dirty_hi) m->dirty_hi = p;
}

void bm_clear_dirty(BlockManager* m) {
    m->dirty_lo = m->max_prompts;
    m->dirty_hi = -1;
}

/* block_manager.c:78-90 */
void free_blocks_for_prompt(BlockManager* manager, int prompt_id) {
    if (prompt_id < 0 || prompt_id >= manager->max_prompts) return;
    if (g_bm_verbose) printf("Freeing all blocks for prompt\n");
    for (int i = 0; i < manager->prompt_block_count[prompt_id]; i++) {
        int bi = manager->prompt_block_list[prompt_id][i];
        KVBlock* b = &manager->blocks[bi];
        if (b->keys) manager->backend.release(manager->backend.ctx, bi, 0, b->keys);
        if (b->values) manager->backend.release(manager->backend.ctx, bi, 1, b->values);
        b->keys = NULL;
        b->values = NULL;
        b->filled = 0;
        b->prompt_id = -1;
        manager->prompt_block_list[prompt_id][i] = -1;
        bm_mark_free(manager, bi);
    }
    manager->prompt_block_count[prompt_id] = 0;
    bm_mark_dirty(manager, prompt_id);
}

/* block_manager.c:92-102: smallest lru_counter strictly below lru_epoch */
int find_least_recently_used_block(BlockManager* manager) {
    int lru_index = -1;
    int min_lru = manager->lru_epoch;
    for (int i = 0; i < manager->max_blocks; i++) {
        if (manager->blocks[i].prompt_id != -1 && manager->blocks[i].lru_counter < min_lru) {
            min_lru = manager->blocks[i].lru_counter;
            lru_index = i;
        }
    }
    return lru_index;
}

/* block_manager.c:104-113: evict the whole prompt owning the LRU page */
void page_out_lru_block(BlockManager* manager) {
    if (g_bm_verbose) printf("Paging out lru block\n");
    int lru = find_least_recently_used_block(manager);
    if (lru != -1) {
        int p = manager->blocks[lru].prompt_id;
        manager->last_evicted_prompt = p;
        free_blocks_for_prompt(manager, p);
    }
}

/* block_manager.c:115-162 */
KVBlock* request_block(BlockManager* manager, int prompt_id) {
    manager->last_evicted_prompt = -1;
    if (prompt_id < 0 || prompt_id >= manager->max_prompts) {
        fprintf(stderr, "Invalid prompt ID.\n");
        return NULL;
    }
    if (manager->prompt_block_count[prompt_id] >= manager->max_blocks_per_prompt) {
        fprintf(stderr, "Prompt page list is full.\n");
        return NULL;
    }
    int bi = bm_first_free(manager);
    if (bi == -1) {
        page_out_lru_block(manager);
        bi = bm_first_free(manager);
        if (bi == -1) {
            fprintf(stderr, "No blocks available.\n");
            return NULL;
        }
    }
    /* the reference mallocs BLOCK_SIZE*C floats each for keys and values (:145-146) */
    size_t bytes = (size_t)manager->block_size * manager->C * sizeof(float);
    KVBlock* b = &manager->blocks[bi];
    b->keys = (float*)manager->backend.alloc(manager->backend.ctx, bi, 0, bytes);
    b->values = (float*)manager->backend.alloc(manager->backend.ctx, bi, 1, bytes);
    if (b->keys == NULL || b->values == NULL) {
        fprintf(stderr, "Failed to allocate memory for block keys/values.\n");
        if (b->keys) manager->backend.release(manager->backend.ctx, bi, 0, b->keys);
        if (b->values) manager->backend.release(manager->backend.ctx, bi, 1, b->values);
        b->keys = b->values = NULL;
        return NULL;
    }
    bm_mark_used(manager, bi);
    b->prompt_id = prompt_id;
    b->filled = 0;
    b->lru_counter = ++manager->lru_epoch;
    int n = manager->prompt_block_count[prompt_id];
    manager->prompt_block_list[prompt_id][n] = bi;
    manager->prompt_block_count[prompt_id] = n + 1;
    bm_mark_dirty(manager, prompt_id);
    return b;
}

/* block_manager.c:165-201: caller frees kv[0], kv[1], kv */
float*** collect_kv_blocks(BlockManager* manager, int prompt_id, int* num_blocks) {
    if (prompt_id < 0 || prompt_id >= manager->max_prompts) {
        fprintf(stderr, "Invalid prompt ID.\n");
        return NULL;
    }
    *num_blocks = manager->prompt_block_count[prompt_id];
    if (*num_blocks == 0) return NULL;
    float*** kv = (float***)malloc(2 * sizeof(float**));
    if (!kv) {
        fprintf(stderr, "Memory allocation failed for kv_pointers.\n");
        return NULL;
    }
    kv[0] = (float**)malloc(*num_blocks * sizeof(float*));
    kv[1] = (float**)malloc(*num_blocks * sizeof(float*));
    if (!kv[0] || !kv[1]) {
        fprintf(stderr, "Memory allocation failed for key/value pointers.\n");
        free(kv[0]);
        free(kv[1]);
        free(kv);
        return NULL;
    }
    for (int i = 0; i < *num_blocks; i++) {
        int bi = manager->prompt_block_list[prompt_id][i];
        kv[0][i] = manager->blocks[bi].keys;
        kv[1][i] = manager->blocks[bi].values;
    }
    return kv;
}

int bm_block_index(const BlockManager* manager, const KVBlock* block) {
    if (!block) return -1;
    return (int)(block - manager->blocks);
}

int bm_free_pages(const BlockManager* manager) { return manager->free_count; }
