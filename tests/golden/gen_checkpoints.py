"""Fixture generator for the on-disk formats.  Runs in
the build container only (it imports the reference from /root/reference);
the GPU box and the tests read only the files it writes:

  ckpt_v1.bin   write_model(model, ..., "float32")   (train_gpt2.py:295-320, 242-265)
  ckpt_v2.bin   write_model(model, ..., "bfloat16")  (train_gpt2.py:295-320, 267-293)
  tokenizer.bin write_tokenizer(enc, ...)            (train_gpt2.py:350-363)
  ckpt_expected.npz
      psum    per-tensor sums of the parameters in ParameterTensors order
              (paged_infer.c:308-326), fp64: pins the loaders' tensor order
      tokens  a token sequence (T,)
      logits  the reference model's forward logits at every position (T, V)
              (GPT.forward, train_gpt2.py:122-146: last-position logits of
              each prefix)
      pieces  the tokenizer's byte strings, concatenated, and their offsets

Usage: python tests/golden/gen_checkpoints.py   (writes next to this file)
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, "/root/reference")
import train_gpt2 as ref  # noqa: E402

CFG = dict(block_size=32, vocab_size=128, n_layer=1, n_head=2, n_embd=128)


class ByteEnc:
    """a tiny byte-level vocabulary standing in for tiktoken (absent offline):
    id i < 96 -> one printable/space byte, the rest multi-byte pieces and
    control bytes (exercising safe_printf's filter)"""

    def __init__(self, n):
        self.max_token_value = n - 1
        self.n = n

    def decode_bytes(self, ids):
        i = ids[0]
        if i < 95:
            return bytes([32 + i])          # ' ' .. '~'
        if i < 100:
            return bytes([i - 95 + 1])      # control bytes 1..5
        return ("tok%d" % i).encode()       # multi-byte pieces


def main():
    torch.manual_seed(1234)
    model = ref.GPT(ref.GPTConfig(**CFG))
    model.eval()
    v1 = os.path.join(HERE, "ckpt_v1.bin")
    v2 = os.path.join(HERE, "ckpt_v2.bin")
    ref.write_model(model, v1, "float32")
    ref.write_model(model, v2, "bfloat16")
    enc = ByteEnc(CFG["vocab_size"])
    ref.write_tokenizer(enc, os.path.join(HERE, "tokenizer.bin"))

    P = {n: p.detach().float().numpy() for n, p in model.named_parameters()}
    L = CFG["n_layer"]

    def per_layer(fmt):
        return np.concatenate([P[fmt % i].reshape(-1) for i in range(L)])

    order = [P["transformer.wte.weight"].reshape(-1), P["transformer.wpe.weight"].reshape(-1),
             per_layer("transformer.h.%d.ln_1.weight"), per_layer("transformer.h.%d.ln_1.bias"),
             per_layer("transformer.h.%d.attn.c_attn.weight"), per_layer("transformer.h.%d.attn.c_attn.bias"),
             per_layer("transformer.h.%d.attn.c_proj.weight"), per_layer("transformer.h.%d.attn.c_proj.bias"),
             per_layer("transformer.h.%d.ln_2.weight"), per_layer("transformer.h.%d.ln_2.bias"),
             per_layer("transformer.h.%d.mlp.c_fc.weight"), per_layer("transformer.h.%d.mlp.c_fc.bias"),
             per_layer("transformer.h.%d.mlp.c_proj.weight"), per_layer("transformer.h.%d.mlp.c_proj.bias"),
             P["transformer.ln_f.weight"].reshape(-1), P["transformer.ln_f.bias"].reshape(-1)]
    params = np.concatenate(order).astype(np.float32)
    psum = np.array([o.astype(np.float64).sum() for o in order])

    T = 24
    tokens = torch.randint(0, CFG["vocab_size"], (1, T), generator=torch.Generator().manual_seed(7))
    with torch.no_grad():
        logits = np.stack([model(tokens[:, :t + 1])[0][0, -1].float().numpy() for t in range(T)])
    pieces = [enc.decode_bytes([i]) for i in range(CFG["vocab_size"])]
    offs = np.cumsum([0] + [len(p) for p in pieces]).astype(np.int32)
    np.savez_compressed(os.path.join(HERE, "ckpt_expected.npz"), psum=psum,
                        tokens=tokens[0].numpy().astype(np.int32), logits=logits.astype(np.float32),
                        pieces=np.frombuffer(b"".join(pieces), np.uint8), offsets=offs,
                        config=np.array([CFG["block_size"], CFG["vocab_size"], CFG["n_layer"], CFG["n_head"],
                                         CFG["n_embd"]], np.int32))
    print("wrote", v1, v2, "tokenizer.bin, ckpt_expected.npz;", params.size, "parameters")


if __name__ == "__main__":
    main()
