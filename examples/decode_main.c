/*
 * decode_main.c -- the reference driver (paged_infer.c:953-1101) on the
 * MI355X decode path, written against the drop-in C API only:
 *
 *   build the model (checkpoint, :436-502; or seeded synthetic GPT-2 124M)
 *   -> hand it a caller-owned BlockManager (:986-987)
 *   -> read the prompt tokens (the reference's DataLoader reads int32
 *      tokens, :753-818; synthetic ids when no file is given)
 *   -> prefill every prompt in one pass (gpt2_decode_prefill: B*T-row GEMMs,
 *      causal multi-query paged attention on MFMA)
 *   -> decode: sample_mult with random_f32 coins from xorshift state 1337
 *      (:1060-1062; on the device, sequence b seeded 1337 + b) or greedy
 *   -> print every token through the tokenizer (:875-928; ids when there is
 *      no tokenizer file), time the generation (:1019-1020, :1085-1087).
 *
 *   gcc -O2 examples/decode_main.c -Iinclude -Lllm.c-paged_amd -lpaged_hip \
 *       -Wl,-rpath,$PWD/llm.c-paged_amd -o decode_main
 *   ./decode_main [-c checkpoint.bin] [-k tokenizer.bin] [-t tokens.bin]
 *                 [-b B] [-p prompt_len] [-n new_tokens] [-g] [-o ids.bin] [-q]
 *     -g greedy (default: sampling as the reference), -o writes the B x
 *     (prompt + new) token ids as int32, -q prints only the summary line.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "block_manager.h"
#include "paged_infer.h"

static double now_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

static void print_token(Tokenizer* tk, int id) {
    if (tk->init_ok) safe_printf(tokenizer_decode(tk, (unsigned)id));
    else printf("%d ", id);
}

int main(int argc, char** argv) {
    const char *ckpt = NULL, *tok_path = NULL, *tokens_path = NULL, *ids_out = NULL;
    int B = 4, prompt_len = 32, new_tokens = 32, greedy = 0, quiet = 0;
    for (int i = 1; i < argc; i++) {
        const char* a = argv[i];
        const char* v = i + 1 < argc ? argv[i + 1] : NULL;
        if (!strcmp(a, "-g")) { greedy = 1; continue; }
        if (!strcmp(a, "-q")) { quiet = 1; continue; }
        if (!v) { fprintf(stderr, "missing value for %s\n", a); return 2; }
        if (!strcmp(a, "-c")) ckpt = v;
        else if (!strcmp(a, "-k")) tok_path = v;
        else if (!strcmp(a, "-t")) tokens_path = v;
        else if (!strcmp(a, "-o")) ids_out = v;
        else if (!strcmp(a, "-b")) B = atoi(v);
        else if (!strcmp(a, "-p")) prompt_len = atoi(v);
        else if (!strcmp(a, "-n")) new_tokens = atoi(v);
        else { fprintf(stderr, "unknown option %s\n", a); return 2; }
        i++;
    }
    GPT2 model;
    if (ckpt) {
        gpt2_build_from_checkpoint(&model, ckpt); /* exits on error, as the reference */
    } else {
        GPT2Config c = {1024, 50257, 12, 12, 768};
        if (gpt2_build_synthetic(&model, c, 1337ULL)) return 1;
    }
    const int V = model.config.vocab_size, total = prompt_len + new_tokens;
    if (B <= 0 || prompt_len <= 0 || new_tokens < 0 || total > model.config.max_seq_len) {
        fprintf(stderr, "need B > 0, prompt > 0 and prompt + new <= %d\n", model.config.max_seq_len);
        return 2;
    }
    const int page_size = 16, max_pages = (total + page_size - 1) / page_size;
    /* the caller owns the manager and hands it to the model (paged_infer.c:986-987) */
    BlockManager* bm = create_block_manager_ex(model.config.channels, B, B * max_pages, page_size, max_pages);
    if (!bm) return 1;
    model.manager = bm;
    if (gpt2_decode_init(&model, B, page_size, total)) return 1;
    if (!greedy && gpt2_decode_set_sampling(&model, 1, 1337ULL)) return 1; /* rng_state = 1337 (:975) */
    gpt2_decode_set_graph(&model, 1);

    int* gen = (int*)malloc((size_t)B * total * sizeof(int));
    int* prompt = (int*)malloc((size_t)B * prompt_len * sizeof(int));
    int* next = (int*)malloc(B * sizeof(int));
    if (!gen || !prompt || !next) return 1;
    if (tokens_path) { /* int32 tokens, e.g. a prepro_tinyshakespeare.py .bin */
        FILE* f = fopen(tokens_path, "rb");
        if (!f || fread(prompt, sizeof(int), (size_t)B * prompt_len, f) != (size_t)B * prompt_len) {
            fprintf(stderr, "cannot read %d x %d tokens from %s\n", B, prompt_len, tokens_path);
            return 1;
        }
        fclose(f);
    } else {
        unsigned long long rng = 42;
        for (int i = 0; i < B * prompt_len; i++) prompt[i] = (int)(random_u32(&rng) % (unsigned)V);
    }
    for (int i = 0; i < B * prompt_len; i++)
        if (prompt[i] < 0 || prompt[i] >= V) { fprintf(stderr, "prompt token out of range\n"); return 1; }
    Tokenizer tk;
    tk.init_ok = 0;
    if (tok_path) tokenizer_init(&tk, tok_path);

    if (!quiet) {
        printf("==============Prompt (sequence 0):==================\n");
        for (int t = 0; t < prompt_len; t++) print_token(&tk, prompt[t]);
        printf("\n========================================\n");
    }
    double t0 = now_s();
    /* the whole prompt of every sequence in one pass; next[b] = the first new token */
    if (gpt2_decode_prefill(&model, prompt, prompt_len, next)) return 1;
    double t1 = now_s();
    for (int b = 0; b < B; b++) {
        memcpy(gen + (size_t)b * total, prompt + (size_t)b * prompt_len, prompt_len * sizeof(int));
        if (new_tokens > 0) gen[(size_t)b * total + prompt_len] = next[b];
    }
    if (!quiet) printf("\ngenerating:\n---\n");
    for (int t = 1; t < new_tokens; t++) {
        if (!quiet) print_token(&tk, next[0]);
        /* the previous ids stay on the device and feed this step */
        if (gpt2_decode_step(&model, NULL, next)) return 1;
        for (int b = 0; b < B; b++) gen[(size_t)b * total + prompt_len + t] = next[b];
    }
    if (!quiet && new_tokens > 0) print_token(&tk, next[0]);
    double t2 = now_s();
    if (!quiet) printf("\n---\nFinished!\n");
    printf("prefill %d x %d tokens in %.3f ms; generated %d tokens x %d sequences (%s) in %.3f ms: "
           "%.1f tokens/s\n", B, prompt_len, 1e3 * (t1 - t0), new_tokens, B, greedy ? "greedy" : "sampled",
           1e3 * (t2 - t0), new_tokens > 1 ? (double)(new_tokens - 1) * B / (t2 - t1) : 0.0);
    if (ids_out) {
        FILE* f = fopen(ids_out, "wb");
        if (!f || fwrite(gen, sizeof(int), (size_t)B * total, f) != (size_t)B * total) return 1;
        fclose(f);
    }
    tokenizer_free(&tk);
    free(gen);
    free(prompt);
    free(next);
    gpt2_free(&model);         /* does not free the manager (reference ownership) */
    destroy_block_manager(bm);
    return 0;
}
