"""ctypes bindings for the CPU oracle (oracle/liboracle*.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, always as the checker / the timed CPU baseline,
never as the product path.  The oracle restates the reference algorithm
(see paged_oracle.h for the file:line map).
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_F = ctypes.POINTER(ctypes.c_float)
_I = ctypes.POINTER(ctypes.c_int)
_PF = ctypes.POINTER(_F)


class OracleConfig(ctypes.Structure):
    _fields_ = [("max_seq_len", ctypes.c_int), ("vocab_size", ctypes.c_int),
                ("num_layers", ctypes.c_int), ("num_heads", ctypes.c_int),
                ("channels", ctypes.c_int)]


def build(fast=False):
    """(Re)build the oracle libraries with make; returns the library path."""
    name = "liboracle_fast.so" if fast else "liboracle.so"
    subprocess.run(["make", "-s", "-C", HERE, name], check=True)
    return os.path.join(HERE, name)


_libs = {}


def lib(fast=False):
    key = bool(fast)
    if key in _libs:
        return _libs[key]
    path = os.path.join(HERE, "liboracle_fast.so" if fast else "liboracle.so")
    src = os.path.join(HERE, "paged_oracle.c")
    if not os.path.exists(path) or os.path.getmtime(path) < os.path.getmtime(src):
        build(fast)
    L = ctypes.CDLL(path)
    L.oracle_num_params.restype = ctypes.c_size_t
    L.oracle_set_threads.argtypes = [ctypes.c_int]
    L.oracle_set_threads.restype = ctypes.c_int
    L.oracle_num_params.argtypes = [OracleConfig]
    L.oracle_param_offsets.argtypes = [OracleConfig, ctypes.POINTER(ctypes.c_size_t)]
    L.oracle_attention_paged.argtypes = [_F, _F, _F, _F, _PF, _PF] + [ctypes.c_int] * 6
    L.oracle_attention_decode.argtypes = [_F, _F, _PF, _PF] + [ctypes.c_int] * 4
    L.oracle_attention_forward.argtypes = [_F, _F, _F, _F] + [ctypes.c_int] * 4
    L.oracle_matmul_forward.argtypes = [_F, _F, _F, _F] + [ctypes.c_int] * 4
    L.oracle_matmul_cached.argtypes = [_F, _F, _F, _F] + [ctypes.c_int] * 4
    L.oracle_layernorm_forward.argtypes = [_F, _F, _F, _F, _F, _F] + [ctypes.c_int] * 3
    L.oracle_gelu_forward.argtypes = [_F, _F, ctypes.c_int]
    L.oracle_gpt2_forward.argtypes = [_F, OracleConfig, _I, ctypes.c_int, ctypes.c_int, _F]
    L.oracle_paged_create.restype = ctypes.c_void_p
    L.oracle_paged_create.argtypes = [_F, OracleConfig, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_ulonglong]
    L.oracle_paged_set_kv.restype = ctypes.c_int
    L.oracle_paged_set_kv.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, _F, _F]
    L.oracle_paged_step.restype = ctypes.c_int
    L.oracle_paged_step.argtypes = [ctypes.c_void_p, _I, _F, _I]
    L.oracle_paged_step_ex.restype = ctypes.c_int
    L.oracle_paged_step_ex.argtypes = [ctypes.c_void_p, _I, _F, _F, _F, _I]
    L.oracle_paged_fill_random.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_ulonglong]
    L.oracle_paged_pos.argtypes = [ctypes.c_void_p, ctypes.c_int]
    L.oracle_paged_pos.restype = ctypes.c_int
    L.oracle_paged_free.argtypes = [ctypes.c_void_p]
    L.oracle_paged_set_kv_bf16.argtypes = [ctypes.c_void_p, ctypes.c_int]
    L.oracle_paged_set_w_bf16.argtypes = [ctypes.c_void_p, ctypes.c_int]
    L.oracle_round_bf16.argtypes = [ctypes.c_float]
    L.oracle_round_bf16.restype = ctypes.c_float
    L.oracle_softmax_forward.argtypes = [_F, _F, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    L.oracle_random_f32.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
    L.oracle_random_f32.restype = ctypes.c_float
    L.oracle_sample_mult.argtypes = [_F, ctypes.c_int, ctypes.c_float]
    L.oracle_sample_mult.restype = ctypes.c_int
    L.oracle_argmax.argtypes = [_F, ctypes.c_int]
    L.oracle_argmax.restype = ctypes.c_int
    _libs[key] = L
    return L


def fp(a):
    assert a.dtype == np.float32 and a.flags.c_contiguous
    return a.ctypes.data_as(_F)


def ip(a):
    assert a.dtype == np.int32 and a.flags.c_contiguous
    return a.ctypes.data_as(_I)


def cfg(maxT, V, L, NH, C):
    return OracleConfig(maxT, V, L, NH, C)


def num_params(c, fast=False):
    return lib(fast).oracle_num_params(c)


def attention_paged(inp, kpool, vpool, page_order, B, T, C, NH, offset, block_size):
    """oracle_attention_paged on a pool whose logical page i lives at
    kpool[page_order[i]] (kpool: (npages, block_size, C))."""
    L = lib()
    out = np.zeros((B, T, C), np.float32)
    preatt = np.zeros((B, NH, T, T), np.float32)
    att = np.zeros((B, NH, T, T), np.float32)
    n = len(page_order)
    kb = (_F * n)(*[kpool[p].ctypes.data_as(_F) for p in page_order])
    vb = (_F * n)(*[vpool[p].ctypes.data_as(_F) for p in page_order])
    L.oracle_attention_paged(fp(out), fp(preatt), fp(att), fp(inp), kb, vb, B, T, C, NH, offset,
                             block_size)
    return out, preatt, att


def attention_decode(q, kpages, vpages, ctx, NH):
    """oracle_attention_decode: q (C,), kpages/vpages lists of (block_size, C)
    float32 arrays in logical order; returns out (C,)."""
    L = lib()
    C = q.shape[0]
    bs = kpages[0].shape[0]
    out = np.zeros(C, np.float32)
    n = len(kpages)
    kb = (_F * n)(*[fp(p) for p in kpages])
    vb = (_F * n)(*[fp(p) for p in vpages])
    L.oracle_attention_decode(fp(out), fp(np.ascontiguousarray(q, np.float32)), kb, vb, ctx, C, NH, bs)
    return out


def gpt2_forward(params, c, tokens, fast=False):
    B, T = tokens.shape
    logits = np.zeros((B, T, c.vocab_size), np.float32)
    lib(fast).oracle_gpt2_forward(fp(params), c, ip(np.ascontiguousarray(tokens, np.int32)), B, T,
                                  fp(logits))
    return logits


class PagedDecoder:
    """oracle_paged_* : incremental paged decode, absolute positions, all layers."""

    def __init__(self, params, c, B, page_size, max_ctx, page_seed=7, fast=False, kv_bf16=False,
                 w_bf16=False):
        self.L = lib(fast)
        self.params = params  # keep alive
        self.c = c
        self.B = B
        self.h = self.L.oracle_paged_create(fp(params), c, B, page_size, max_ctx, page_seed)
        if not self.h:
            raise MemoryError("oracle_paged_create failed")
        if kv_bf16:
            self.L.oracle_paged_set_kv_bf16(self.h, 1)
        if w_bf16 and self.L.oracle_paged_set_w_bf16(self.h, 1) != 0:
            raise MemoryError("oracle_paged_set_w_bf16")

    def step(self, tokens, want_logits=True):
        tokens = np.ascontiguousarray(tokens, np.int32)
        nxt = np.zeros(self.B, np.int32)
        logits = np.zeros((self.B, self.c.vocab_size), np.float32) if want_logits else None
        rc = self.L.oracle_paged_step(self.h, ip(tokens), fp(logits) if want_logits else None,
                                      ip(nxt))
        if rc != 0:
            raise RuntimeError("oracle_paged_step failed (context full)")
        return nxt, logits

    def step_forced(self, tokens, forced_x):
        """one step with layer l's input taken from forced_x[l] ((L+1, B, C):
        the GPU engine's residual stream, gpt2_decode_step_traced; forced_x[L]
        feeds LNf); returns next ids, logits and every layer's output (L, B, C)"""
        tokens = np.ascontiguousarray(tokens, np.int32)
        Lc, C = self.c.num_layers, self.c.channels
        fx = None
        if forced_x is not None:  # None: the decoder's own stream (layer outputs still returned)
            fx = np.ascontiguousarray(forced_x, np.float32)
            assert fx.shape == (Lc + 1, self.B, C)
        nxt = np.zeros(self.B, np.int32)
        logits = np.zeros((self.B, self.c.vocab_size), np.float32)
        out = np.zeros((Lc, self.B, C), np.float32)
        if self.L.oracle_paged_step_ex(self.h, ip(tokens), fp(fx) if fx is not None else None, fp(out), fp(logits),
                                       ip(nxt)) != 0:
            raise RuntimeError("oracle_paged_step_ex failed (context full)")
        return nxt, logits, out

    def set_kv(self, layer, b, k, v):
        """positions [0, len(k)) of sequence b at `layer` take these K/V rows
        (token-major (n, C)); pos[b] becomes n"""
        k = np.ascontiguousarray(k, np.float32)
        v = np.ascontiguousarray(v, np.float32)
        if self.L.oracle_paged_set_kv(self.h, int(layer), int(b), k.shape[0], fp(k), fp(v)) != 0:
            raise RuntimeError("oracle_paged_set_kv failed")

    def fill_random(self, ctx, seed=1):
        self.L.oracle_paged_fill_random(self.h, ctx, seed)

    def pos(self, b):
        return self.L.oracle_paged_pos(self.h, b)

    def close(self):
        if self.h:
            self.L.oracle_paged_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Sampler:
    """the reference driver's token choice (softmax_forward :259-286 +
    sample_mult :837-848 with random_f32 coins :826-835), one xorshift stream
    per sequence seeded seed + b (as gpt2_decode_set_sampling)"""

    def __init__(self, B, seed=1337):
        self.states = [ctypes.c_ulonglong(seed + b) for b in range(B)]

    def sample(self, logits):
        L = lib()
        B, V = logits.shape
        logits = np.ascontiguousarray(logits, np.float32)
        probs = np.empty_like(logits)
        L.oracle_softmax_forward(fp(probs), fp(logits), B, 1, V)
        out = np.empty(B, np.int32)
        for b in range(B):
            coin = L.oracle_random_f32(ctypes.byref(self.states[b]))
            out[b] = L.oracle_sample_mult(fp(probs[b]), V, coin)
        return out
