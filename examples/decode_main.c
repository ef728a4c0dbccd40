/*
 * decode_main.c -- a batched greedy decode driver written against the
 * drop-in C API, the way the reference's own driver (paged_infer.c:953-1101)
 * uses it: build the model, hand it a BlockManager, run decode steps.
 *
 *   gcc -O2 examples/decode_main.c -Iinclude -Lllm.c-paged_amd -lpaged_hip \
 *       -Wl,-rpath,$PWD/llm.c-paged_amd -o decode_main
 *   ./decode_main [checkpoint.bin] [B] [steps]
 *
 * Without a checkpoint it builds seeded synthetic GPT-2 124M weights (the
 * reference's xorshift, seed 1337).
 */
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include "block_manager.h"
#include "paged_infer.h"

static double now_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

int main(int argc, char** argv) {
    const char* ckpt = argc > 1 && argv[1][0] ? argv[1] : NULL;
    int B = argc > 2 ? atoi(argv[2]) : 8;
    int steps = argc > 3 ? atoi(argv[3]) : 32;
    const int page_size = 16, max_ctx = 1024;

    GPT2 model;
    if (ckpt) {
        gpt2_build_from_checkpoint(&model, ckpt); /* paged_infer.c:436-502; exits on error */
    } else {
        GPT2Config c = {1024, 50257, 12, 12, 768};
        if (gpt2_build_synthetic(&model, c, 1337ULL)) return 1;
    }
    /* the caller owns the manager and hands it to the model (paged_infer.c:986-987) */
    BlockManager* bm = create_block_manager_ex(model.config.channels, B, B * (max_ctx / page_size),
                                               page_size, max_ctx / page_size);
    if (!bm) return 1;
    model.manager = bm;
    if (gpt2_decode_init(&model, B, page_size, max_ctx)) return 1;

    int* tok = (int*)malloc(B * sizeof(int));
    int* next = (int*)malloc(B * sizeof(int));
    unsigned long long rng = 42;
    for (int b = 0; b < B; b++) tok[b] = (int)(random_u32(&rng) % model.config.vocab_size);
    if (gpt2_decode_step(&model, tok, next)) return 1; /* first token of every sequence */
    double t0 = now_s();
    for (int s = 1; s < steps; s++)
        if (gpt2_decode_step(&model, NULL, next)) return 1; /* greedy ids fed back on device */
    double dt = now_s() - t0;
    printf("decoded %d steps x %d sequences: %.1f tokens/s; seq 0 last id %d\n", steps - 1, B,
           (steps - 1) * B / dt, next[0]);
    free(tok);
    free(next);
    gpt2_free(&model);               /* does not free the manager (reference ownership) */
    destroy_block_manager(bm);
    return 0;
}
