/*
 * ref_paged_driver.c -- builds the REFERENCE paged_infer.c (which textually
 * includes the reference block_manager.c) into oracle/_ref/libref_paged.so so
 * tests/golden/gen_golden.py can run the reference's own functions.
 * TEST INFRASTRUCTURE ONLY; needs /root/reference (this container only).
 * The reference source is compiled where it lies (-DREF_PAGED_INFER=path);
 * nothing from it is copied into this repository.
 */
#define main ref_paged_infer_main
#include REF_PAGED_INFER
#undef main

/* Field accessors so ctypes never has to mirror the fixed-size reference
 * structs (block_manager.c:9-23). */
int ref_bm_block_size(void) { return BLOCK_SIZE; }
int ref_bm_max_blocks(void) { return MAX_BLOCKS; }
int ref_bm_max_prompts(void) { return MAX_PROMPTS; }
/* create_block_manager (block_manager.c:38-52) leaves lru_epoch and every
 * page's filled/lru_counter uninitialised; a trace needs them defined, so the
 * generator zeroes them right after creation (the drop-in does the same). */
BlockManager* ref_bm_create(int C) {
    BlockManager* m = create_block_manager(C);
    m->lru_epoch = 0;
    for (int i = 0; i < MAX_BLOCKS; i++) { m->blocks[i].filled = 0; m->blocks[i].lru_counter = 0; }
    return m;
}
int ref_bm_block_index(BlockManager* m, KVBlock* b) { return b ? (int)(b - m->blocks) : -1; }
int ref_bm_block_prompt(BlockManager* m, int i) { return m->blocks[i].prompt_id; }
int ref_bm_block_filled(BlockManager* m, int i) { return m->blocks[i].filled; }
void ref_bm_set_filled(BlockManager* m, int i, int f) { m->blocks[i].filled = f; }
int ref_bm_block_lru(BlockManager* m, int i) { return m->blocks[i].lru_counter; }
int ref_bm_prompt_count(BlockManager* m, int p) { return m->prompt_block_count[p]; }
int ref_bm_prompt_list(BlockManager* m, int p, int i) { return m->prompt_block_list[p][i]; }
int ref_bm_lru_epoch(BlockManager* m) { return m->lru_epoch; }
void ref_bm_touch(BlockManager* m, int i) { m->blocks[i].lru_counter = ++m->lru_epoch; } /* paged_infer.c:524 */
