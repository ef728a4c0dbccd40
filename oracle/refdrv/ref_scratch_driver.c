/*
 * ref_scratch_driver.c -- builds the REFERENCE train_scratch.c (the full-L
 * fp32 forward, train_scratch.c:658-798) into
 * oracle/_ref/libref_scratch.so for golden generation.  TEST INFRASTRUCTURE
 * ONLY; compiled where the source lies, never copied.
 */
#define TESTING
#include REF_TRAIN_SCRATCH

/* load a v1 checkpoint with the reference loader, run the reference forward,
 * copy out (B,T,V) logits */
int ref_full_forward(const char* ckpt, const int* tokens, int B, int T, float* logits_out) {
    GPT2 model;
    gpt2_build_from_checkpoint(&model, (char*)ckpt);
    gpt2_forward(&model, (int*)tokens, NULL, B, T);
    memcpy(logits_out, model.acts.logits, (size_t)B * T * model.config.vocab_size * sizeof(float));
    gpt2_free(&model);
    return 0;
}
