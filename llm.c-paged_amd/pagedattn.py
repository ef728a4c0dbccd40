"""Python host mirror of libpaged_hip.so (ctypes over the C-ABI).

This is a thin binding, not a compute path: every call lands in the C
library (include/hip_paged_attn.h, paged_infer.h, block_manager.h), which
runs the MI355X kernels.  There is no fallback: if the library is missing or
no HIP device is visible, the calls raise.

Names mirror the reference API (paged_infer.c / block_manager.c of
mx60s/llm.c-paged): Model wraps GPT2 + gpt2_decode_* (the decode hot path),
BlockManager wraps create_block_manager / request_block / ... .
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("HPA_LIB") or os.path.join(HERE, "libpaged_hip.so")  # HPA_LIB: tool A/B builds
INCLUDE_DIR = os.path.join(os.path.dirname(HERE), "include")

_F = ctypes.POINTER(ctypes.c_float)
_I = ctypes.POINTER(ctypes.c_int)
_V = ctypes.c_void_p


class GPT2Config(ctypes.Structure):
    """paged_infer.c:397-403"""
    _fields_ = [("max_seq_len", ctypes.c_int), ("vocab_size", ctypes.c_int),
                ("num_layers", ctypes.c_int), ("num_heads", ctypes.c_int),
                ("channels", ctypes.c_int)]

    def as_dict(self):
        return dict(maxT=self.max_seq_len, V=self.vocab_size, L=self.num_layers,
                    NH=self.num_heads, C=self.channels)


class KVBlock(ctypes.Structure):
    """block_manager.c:9-15"""
    _fields_ = [("keys", _F), ("values", _F), ("filled", ctypes.c_int),
                ("prompt_id", ctypes.c_int), ("lru_counter", ctypes.c_int)]


class HpaKVPool(ctypes.Structure):
    _fields_ = [("base", _V), ("num_layers", ctypes.c_int), ("num_heads", ctypes.c_int),
                ("head_size", ctypes.c_int), ("page_size", ctypes.c_int),
                ("num_pages", ctypes.c_int), ("dtype", ctypes.c_int),
                ("elem_bytes", ctypes.c_size_t), ("page_elems", ctypes.c_size_t),
                ("layer_elems", ctypes.c_size_t), ("bytes", ctypes.c_size_t),
                ("managed", ctypes.c_int)]


class HpaFusedGemm(ctypes.Structure):
    _fields_ = [("x", _V), ("M", ctypes.c_int), ("K", ctypes.c_int), ("ln_stats", _V),
                ("ln_ntiles", ctypes.c_int), ("ln_w", _V), ("ln_b", _V), ("w", _V),
                ("N", ctypes.c_int), ("bias", _V), ("epilogue", ctypes.c_int), ("out", _V),
                ("res_in", _V), ("stats_out", _V), ("part_out", _V),
                ("pool", ctypes.POINTER(HpaKVPool)), ("layer", ctypes.c_int), ("block_table", _V),
                ("bt_stride", ctypes.c_int), ("pos", _V), ("waves", ctypes.c_int),
                ("row_blocks", ctypes.c_int), ("variant", ctypes.c_int), ("col_tiles", ctypes.c_int),
                ("row_seq", _V), ("ln_fold_c1", _V), ("sk_slab", _V), ("sk_count", _V),
                ("w_dtype", ctypes.c_int), ("pick_next", _V), ("pick_tokens", _V), ("pick_pos", _V),
                ("pick_count", _V)]


HPA_FEPI_QKV, HPA_FEPI_RESID, HPA_FEPI_GELU, HPA_FEPI_LOGITS = 0, 1, 2, 3
HPA_COMM_SEND, HPA_COMM_RECV, HPA_COMM_COPY = 0, 1, 2


class HpaCommOp(ctypes.Structure):
    """include/hip_paged_attn.h HpaCommOp: one operation of the gather schedule"""
    _fields_ = [("op", ctypes.c_int), ("peer", ctypes.c_int), ("offset", ctypes.c_size_t),
                ("bytes", ctypes.c_size_t)]


def frag_index(m, k, K):
    """numpy mirror of hpa_internal.h frag_index (vectorised over m, k)"""
    m = np.asarray(m)
    k = np.asarray(k)
    return ((((m >> 4) * (K >> 4) + (k >> 4)) * 64 + ((m & 15) + 16 * ((k >> 2) & 3))) << 2) + (k & 3)


def to_frag(a, pad=16):
    """host [rows][K] -> frag-layout flat array (rows padded to `pad`)"""
    rows, K = a.shape
    rp = (rows + pad - 1) // pad * pad
    out = np.zeros(rp * K, np.float32)
    m, k = np.meshgrid(np.arange(rows), np.arange(K), indexing="ij")
    out[frag_index(m, k, K)] = a
    return out


def from_frag(f, rows, K):
    m, k = np.meshgrid(np.arange(rows), np.arange(K), indexing="ij")
    return f[frag_index(m, k, K)]


GPT2_124M = dict(maxT=1024, V=50257, L=12, NH=12, C=768)
GPT2_XL = dict(maxT=1024, V=50257, L=48, NH=25, C=1600)

def config(d):
    return GPT2Config(d["maxT"], d["V"], d["L"], d["NH"], d["C"])


def gather_plan(nranks, rank, root, nbytes):
    """hpa_comm_gather_plan: the (op, peer, offset, bytes) operations this rank
    posts for one end-of-step gather -- the list hpa_comm_gatherv executes over
    RCCL (host arithmetic, no GPU needed)"""
    L = lib()
    b = (ctypes.c_size_t * nranks)(*nbytes)
    ops = (HpaCommOp * nranks)()
    n = L.hpa_comm_gather_plan(nranks, rank, root, b, ops, nranks)
    if n < 0:
        raise ValueError("hpa_comm_gather_plan: bad arguments")
    return [(o.op, o.peer, o.offset, o.bytes) for o in ops[:n]]


def build(force=False):
    """Compile libpaged_hip.so in-tree (hipcc --offload-arch=gfx950)."""
    cmd = ["make", "-s", "-C", HERE, "-j8"]
    if force:
        cmd.insert(2, "-B")
    subprocess.run(cmd, check=True)
    return LIB_PATH


_lib = None


def _sig(L, name, res, args):
    f = getattr(L, name)
    f.restype = res
    f.argtypes = args


def lib():
    """Load libpaged_hip.so (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} missing: run __graft_entry__.build() (no CPU fallback)")
    L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    i, v, f, sz = ctypes.c_int, _V, ctypes.c_float, ctypes.c_size_t
    P = ctypes.POINTER(HpaKVPool)
    # runtime
    _sig(L, "hpa_init", i, [i])
    _sig(L, "hpa_device_count", i, [])
    _sig(L, "hpa_get_device", i, [])
    _sig(L, "hpa_set_stream", i, [v])
    _sig(L, "hpa_get_stream", v, [])
    _sig(L, "hpa_synchronize", i, [])
    _sig(L, "hpa_device_synchronize", i, [])
    _sig(L, "hpa_malloc", v, [sz])
    _sig(L, "hpa_malloc_managed", v, [sz])
    _sig(L, "hpa_host_alloc", v, [sz])
    _sig(L, "hpa_free", i, [v])
    _sig(L, "hpa_memcpy", i, [v, v, sz])
    _sig(L, "hpa_memcpy_async", i, [v, v, sz])
    _sig(L, "hpa_memset_async", i, [v, i, sz])
    _sig(L, "hpa_is_device_accessible", i, [v])
    _sig(L, "hpa_event_create", v, [])
    _sig(L, "hpa_event_record", i, [v])
    _sig(L, "hpa_event_elapsed_ms", f, [v, v])
    _sig(L, "hpa_event_destroy", i, [v])
    _sig(L, "hpa_event_create_nt", v, [])
    _sig(L, "hpa_stream_create", v, [])
    _sig(L, "hpa_stream_destroy", i, [v])
    _sig(L, "hpa_stream_wait_event", i, [v])
    _sig(L, "hpa_event_synchronize", i, [v])
    _sig(L, "hpa_last_error", ctypes.c_char_p, [])
    _sig(L, "hpa_build_flags", i, [])
    _sig(L, "hpa_device_info", i, [ctypes.c_char_p, i, _I, ctypes.POINTER(sz)])
    _sig(L, "hpa_set_attention_waves", i, [i])
    _sig(L, "hpa_attn_pick_waves", i, [i, i, i, i])
    # pool + kernels
    _sig(L, "hpa_pool_create", i, [P, i, i, i, i, i, i, i])
    _sig(L, "hpa_pool_destroy", None, [P])
    _sig(L, "hpa_pool_tile", v, [P, i, i, i, i])
    _sig(L, "hpa_pool_k_index", sz, [P, i, i, i, i, i])
    _sig(L, "hpa_pool_v_index", sz, [P, i, i, i, i, i])
    _sig(L, "hpa_pool_fill_random", i, [P, v, i, i, i, ctypes.c_uint64])
    _sig(L, "hpa_paged_attention_decode", i, [v, P, i, v, i, v, v, i])
    _sig(L, "hpa_attn_ws_bytes", sz, [i, i, i])
    _sig(L, "hpa_attn_pick_splits", i, [i, i, i, i])
    _sig(L, "hpa_paged_attention_decode_split", i, [v, P, i, v, i, v, v, i, i, v, i])
    _sig(L, "hpa_comm_id_bytes", sz, [])
    _sig(L, "hpa_comm_unique_id", i, [v, sz])
    _sig(L, "hpa_comm_init", i, [i, i, v])
    _sig(L, "hpa_comm_destroy", i, [])
    _sig(L, "hpa_comm_size", i, [])
    _sig(L, "hpa_comm_rank", i, [])
    _sig(L, "hpa_comm_gatherv", i, [v, sz, v, ctypes.POINTER(sz), i, v])
    _sig(L, "hpa_comm_gather_layout", i, [i, i, i, ctypes.POINTER(sz), ctypes.POINTER(sz), ctypes.POINTER(sz)])
    _sig(L, "hpa_comm_gather_plan", i, [i, i, i, ctypes.POINTER(sz), ctypes.POINTER(HpaCommOp), i])
    _sig(L, "hpa_comm_barrier", i, [])
    _sig(L, "hpa_comm_allreduce_max", i, [ctypes.POINTER(ctypes.c_double)])
    _sig(L, "hpa_comm_init_all", i, [i, ctypes.POINTER(i)])
    _sig(L, "hpa_comm_use", i, [i])
    _sig(L, "hpa_ref_attention_paged", i, [v, v, v, v, v, v, i, i, i, i, i, i])
    _sig(L, "hpa_ref_matmul", i, [v, v, v, v, i, i, i, i, i])
    # block manager (block_manager.c API)
    _sig(L, "create_block_manager", v, [i])
    _sig(L, "create_block_manager_ex", v, [i, i, i, i, i])
    _sig(L, "destroy_block_manager", None, [v])
    _sig(L, "request_block", ctypes.POINTER(KVBlock), [v, i])
    _sig(L, "get_current_block", ctypes.POINTER(KVBlock), [v, i])
    _sig(L, "free_blocks_for_prompt", None, [v, i])
    _sig(L, "find_least_recently_used_block", i, [v])
    _sig(L, "page_out_lru_block", None, [v])
    _sig(L, "get_next_block_id", i, [v, i, i])
    _sig(L, "collect_kv_blocks", v, [v, i, _I])
    _sig(L, "bm_block_index", i, [v, v])
    _sig(L, "bm_free_pages", i, [v])
    _sig(L, "bm_use_host_pages", None, [v])
    _sig(L, "bm_default_backend_kind", i, [])
    # model + decode engine
    _sig(L, "gpt2_alloc", v, [])
    _sig(L, "gpt2_release", None, [v])
    _sig(L, "gpt2_set_manager", None, [v, v])
    _sig(L, "gpt2_acts_logits", _F, [v])
    _sig(L, "gpt2_acts_probs", _F, [v])
    _sig(L, "gpt2_num_parameters", sz, [GPT2Config])
    _sig(L, "gpt2_synthetic_params", i, [GPT2Config, ctypes.c_ulonglong, _F])
    _sig(L, "gpt2_write_checkpoint", i, [ctypes.c_char_p, GPT2Config, _F])
    _sig(L, "gpt2_write_checkpoint_ex", i, [ctypes.c_char_p, GPT2Config, _F, i])
    _sig(L, "gpt2_read_checkpoint", i, [ctypes.c_char_p, ctypes.POINTER(GPT2Config), _F])
    _sig(L, "tokenizer_init", None, [v, ctypes.c_char_p])
    _sig(L, "tokenizer_decode", ctypes.c_char_p, [v, ctypes.c_uint32])
    _sig(L, "tokenizer_free", None, [v])
    _sig(L, "safe_printf", None, [ctypes.c_char_p])
    _sig(L, "gpt2_build_from_params", i, [v, GPT2Config, _F])
    _sig(L, "gpt2_build_synthetic", i, [v, GPT2Config, ctypes.c_ulonglong])
    _sig(L, "gpt2_build_from_checkpoint", None, [v, ctypes.c_char_p])
    _sig(L, "gpt2_forward", None, [v, _I, _I, sz, sz, sz, i])
    _sig(L, "gpt2_decode_init", i, [v, i, i, i])
    _sig(L, "gpt2_decode_init_ex", i, [v, i, i, i, i])
    _sig(L, "gpt2_decode_init_w", i, [v, i, i, i, i, i])
    _sig(L, "hpa_pack_frag_bf16", i, [v, i, i, i, v])
    _sig(L, "hpa_frag_bf16_elems", ctypes.c_size_t, [i, i])
    _sig(L, "gpt2_decode_prefill", i, [v, _I, i, _I])
    _sig(L, "gpt2_decode_prefill_ragged", i, [v, _I, _I, _I])
    _sig(L, "gpt2_decode_release", i, [v, i])
    _sig(L, "gpt2_decode_set_sampling", i, [v, i, ctypes.c_ulonglong])
    _sig(L, "hpa_paged_attention_prefill", i, [_F, v, i, _I, i, _I, i, i, _F])
    _sig(L, "hpa_paged_attention_prefill_ragged", i, [_F, v, i, _I, i, _I, _I, _I, i, i, _F])
    _sig(L, "hpa_gather_rows_frag", i, [_F, _F, i, _I, i, _F, _F, i, i])
    _sig(L, "gpt2_decode_step", i, [v, _I, _I])
    _sig(L, "gpt2_decode_step_async", i, [v, _I])
    _sig(L, "gpt2_decode_step_traced", i, [v, _I, _I, _F])
    _sig(L, "gpt2_decode_reset", i, [v])
    _sig(L, "gpt2_decode_fill_random", i, [v, i, ctypes.c_ulonglong])
    _sig(L, "gpt2_decode_set_graph", i, [v, i])
    _sig(L, "gpt2_decode_reserve", i, [v, i])
    _sig(L, "gpt2_decode_free", None, [v])
    _sig(L, "gpt2_decode_set_attn_splits", i, [v, i])
    _sig(L, "gpt2_decode_attn_splits", i, [v])
    _sig(L, "gpt2_decode_attn_waves", i, [v])
    _sig(L, "gpt2_decode_set_global_batch", i, [v, i])
    _sig(L, "gpt2_decode_global_batch", i, [v])
    _sig(L, "gpt2_decode_set_layer_kernel", i, [v, i])
    _sig(L, "gpt2_decode_fill_random_ex", i, [v, i, ctypes.c_uint64, i])
    _sig(L, "hpa_pool_fill_random_ex", i, [P, v, i, i, i, ctypes.c_uint64, i])
    _sig(L, "hpa_logits_kernel", i, [i, i, i])
    _sig(L, "gpt2_decode_layer_kernel", i, [v])
    _sig(L, "gpt2_decode_set_pipe_split", i, [v, i])
    _sig(L, "hpa_decode_pipe_eligible", i, [i, i, i, i])
    _sig(L, "gpt2_decode_status", i, [v])
    _sig(L, "hpa_decode_layer_eligible", i, [i, i, i, i])
    _sig(L, "hpa_decode_layer_pick_splits", i, [i, i, i])
    _sig(L, "hpa_decode_layer_trace", i, [v, i])
    _sig(L, "hpa_decode_chain_b16_trace", i, [v, i])
    _sig(L, "hpa_decode_cx_wave_trace", i, [v])
    _sig(L, "hpa_logits_trace", i, [v])
    _sig(L, "gpt2_decode_evicted", i, [v, _I])
    _sig(L, "gpt2_decode_read_kv", i, [v, i, i, i, _F, _F])
    _sig(L, "gpt2_decode_batch", i, [v])
    _sig(L, "gpt2_decode_shard", i, [v, _I, i])
    _sig(L, "gpt2_decode_gather", i, [v, i])
    _sig(L, "gpt2_decode_gather_all", i, [ctypes.POINTER(v), i, i])
    _sig(L, "hpa_comm_group_start", i, [])
    _sig(L, "hpa_comm_group_end", i, [])
    _sig(L, "gpt2_decode_gather_wait", i, [v])
    _sig(L, "gpt2_decode_gathered", v, [v, i])
    _sig(L, "gpt2_decode_profile", i, [v, i])
    _sig(L, "gpt2_decode_profile_read", ctypes.c_double, [v, ctypes.POINTER(ctypes.c_long)])
    _sig(L, "hpa_frag_elems", sz, [i, i])
    _sig(L, "hpa_pack_frag", i, [v, i, i, i, v])
    _sig(L, "hpa_ln_fold_pack", i, [v, i, i, v, v, v, v, v, v])
    _sig(L, "hpa_unpack_frag", i, [v, i, i, v, i])
    _sig(L, "hpa_gemm_fused", i, [ctypes.POINTER(HpaFusedGemm)])
    _sig(L, "hpa_gemm_sk_workspace", i, [i, ctypes.POINTER(sz), ctypes.POINTER(sz)])
    _sig(L, "hpa_logits_partials", i, [ctypes.POINTER(HpaFusedGemm)])
    _sig(L, "hpa_fused_pick_waves", i, [i, i, i])
    _sig(L, "hpa_fused_pick", None, [i, i, i, _I])
    _sig(L, "hpa_fused_pick_bf16", None, [i, i, i, _I])
    _sig(L, "hpa_fused_pick_bf16_ares", i, [i, i, i, _I])
    _sig(L, "hpa_embed_frag", i, [v, v, v, v, v, v, i, i])
    _sig(L, "hpa_embed_frag_zero", i, [v, v, v, v, v, v, i, i, v, ctypes.c_size_t])
    _sig(L, "hpa_argmax_final", i, [v, i, i, i, v, v, v, v])
    _sig(L, "hpa_sample_final", i, [v, i, i, v, v, v, v, v])
    _sig(L, "hpa_sample_final_serial", i, [v, i, i, v, v, v, v, v])
    _sig(L, "hpa_paged_attention_decode_frag", i, [v, P, i, v, i, v, v, i])
    _sig(L, "gpt2_decode_set_positions", i, [v, _I])
    _sig(L, "gpt2_decode_logits", v, [v])
    _sig(L, "gpt2_decode_next", v, [v])
    _sig(L, "gpt2_decode_positions", i, [v, _I])
    _sig(L, "gpt2_decode_gemm_config", i, [v, _I, _I, _I, i])
    _sig(L, "gpt2_decode_time_attention", i, [v, i, ctypes.POINTER(ctypes.c_double),
                                              ctypes.POINTER(ctypes.c_double)])
    _sig(L, "gpt2_decode_time_attention_pf", i, [v, i, ctypes.c_double, i, ctypes.POINTER(ctypes.c_double),
                                                 ctypes.POINTER(ctypes.c_double)])
    _sig(L, "hpa_l3_prefetch", i, [v, sz, i])
    _sig(L, "hpa_gemm_ring_workspace", i, [i, i, ctypes.POINTER(sz), ctypes.POINTER(sz)])
    _sig(L, "gpt2_decode_step_bytes", ctypes.c_double, [v, ctypes.POINTER(ctypes.c_double)])
    _sig(L, "random_u32", ctypes.c_uint, [ctypes.POINTER(ctypes.c_ulonglong)])
    _sig(L, "random_f32", f, [ctypes.POINTER(ctypes.c_ulonglong)])
    _lib = L
    return L


def check(rc, what=""):
    if rc != 0:
        err = lib().hpa_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed: {err}")


def init(device=0):
    L = lib()
    if L.hpa_device_count() <= 0:
        raise RuntimeError("no HIP device visible: the MI355X path has no CPU fallback")
    check(L.hpa_init(device), "hpa_init")


def device_info():
    L = lib()
    name = ctypes.create_string_buffer(256)
    cus = ctypes.c_int()
    mem = ctypes.c_size_t()
    check(L.hpa_device_info(name, 256, ctypes.byref(cus), ctypes.byref(mem)), "device_info")
    return name.value.decode(), cus.value, mem.value


# ---------------------------------------------------------------- device buffers
class DeviceBuffer:
    """hpa_malloc'd memory with numpy-typed upload/download helpers."""

    def __init__(self, nbytes, managed=False):
        L = lib()
        self.nbytes = int(nbytes)
        self.ptr = L.hpa_malloc_managed(self.nbytes) if managed else L.hpa_malloc(self.nbytes)
        if not self.ptr:
            raise MemoryError(f"device allocation of {nbytes} bytes failed")

    @classmethod
    def from_array(cls, a, managed=False):
        a = np.ascontiguousarray(a)
        b = cls(a.nbytes, managed)
        b.upload(a)
        return b

    def upload(self, a, offset=0):
        a = np.ascontiguousarray(a)
        assert offset + a.nbytes <= self.nbytes
        check(lib().hpa_memcpy(self.ptr + offset, a.ctypes.data, a.nbytes), "upload")

    def download(self, shape, dtype=np.float32, offset=0):
        out = np.empty(shape, dtype)
        assert offset + out.nbytes <= self.nbytes
        check(lib().hpa_memcpy(out.ctypes.data, self.ptr + offset, out.nbytes), "download")
        return out

    def free(self):
        if self.ptr:
            lib().hpa_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def to_bf16_bits(a):
    """fp32 -> bf16 bit patterns, round to nearest even (hpa::f32_to_bf16)"""
    u = np.ascontiguousarray(a, np.float32).view(np.uint32).astype(np.uint64)
    u = (u + 0x7FFF + ((u >> 16) & 1)) >> 16
    return u.astype(np.uint16)


def from_bf16_bits(b):
    return (np.asarray(b, np.uint16).astype(np.uint32) << 16).view(np.float32)


def round_bf16(a):
    """the fp32 value a bf16 KV pool stores for `a`"""
    return from_bf16_bits(to_bf16_bits(a))


HPA_F32, HPA_BF16 = 0, 1


class Pool:
    """HpaKVPool: the HBM page pool in the fast layout (fp32 or bf16)."""

    def __init__(self, num_layers, num_heads, page_size, num_pages, head_size=64, managed=False, dtype=HPA_F32):
        self.s = HpaKVPool()
        check(lib().hpa_pool_create(ctypes.byref(self.s), num_layers, num_heads, head_size, page_size,
                                    num_pages, int(dtype), int(managed)), "pool_create")

    @property
    def ref(self):
        return ctypes.byref(self.s)

    def _k_chunk(self):
        return 8 if self.s.dtype == HPA_BF16 else 4

    def write_tokens(self, layer, pages, k, v):
        """host helper: k, v (ntok, C) -> logical positions 0..ntok-1 of the
        sequence whose page list is `pages` (uploads whole pages; bf16 pools
        store the round-to-nearest-even values)."""
        s = self.s
        P, NH, HS, ch = s.page_size, s.num_heads, s.head_size, self._k_chunk()
        bf = s.dtype == HPA_BF16
        ntok = k.shape[0]
        for lp, page in enumerate(pages):
            t0 = lp * P
            if t0 >= ntok:
                break
            n = min(P, ntok - t0)
            kt = np.zeros((NH, HS // ch, P, ch), np.float32)
            vt = np.zeros((NH, P, HS), np.float32)
            kt[:, :, :n, :] = k[t0:t0 + n].reshape(n, NH, HS // ch, ch).transpose(1, 2, 0, 3)
            vt[:, :n, :] = v[t0:t0 + n].reshape(n, NH, HS).transpose(1, 0, 2)
            if bf:
                kt, vt = to_bf16_bits(kt), to_bf16_bits(vt)
            page_k = lib().hpa_pool_tile(self.ref, layer, int(page), 0, 0)
            page_v = lib().hpa_pool_tile(self.ref, layer, int(page), 1, 0)
            check(lib().hpa_memcpy(page_k, kt.ctypes.data, kt.nbytes), "pool write K")
            check(lib().hpa_memcpy(page_v, vt.ctypes.data, vt.nbytes), "pool write V")

    def read_tokens(self, layer, pages, ntok):
        s = self.s
        P, NH, HS, ch = s.page_size, s.num_heads, s.head_size, self._k_chunk()
        bf = s.dtype == HPA_BF16
        et = np.uint16 if bf else np.float32
        k = np.zeros((ntok, NH * HS), np.float32)
        v = np.zeros((ntok, NH * HS), np.float32)
        for lp, page in enumerate(pages):
            t0 = lp * P
            if t0 >= ntok:
                break
            n = min(P, ntok - t0)
            kt = np.empty((NH, HS // ch, P, ch), et)
            vt = np.empty((NH, P, HS), et)
            check(lib().hpa_memcpy(kt.ctypes.data, lib().hpa_pool_tile(self.ref, layer, int(page), 0, 0),
                                   kt.nbytes), "pool read K")
            check(lib().hpa_memcpy(vt.ctypes.data, lib().hpa_pool_tile(self.ref, layer, int(page), 1, 0),
                                   vt.nbytes), "pool read V")
            if bf:
                kt, vt = from_bf16_bits(kt), from_bf16_bits(vt)
            k[t0:t0 + n] = kt[:, :, :n, :].transpose(2, 0, 1, 3).reshape(n, NH * HS)
            v[t0:t0 + n] = vt[:, :n, :].transpose(1, 0, 2).reshape(n, NH * HS)
        return k, v

    def destroy(self):
        if self.s.base:
            lib().hpa_pool_destroy(self.ref)

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass


# ---------------------------------------------------------------- on-disk formats
def read_checkpoint(path):
    """gpt2_read_checkpoint (host only): (GPT2Config, fp32 params in
    ParameterTensors order) from a v1 or v2 checkpoint"""
    c = GPT2Config()
    check(lib().gpt2_read_checkpoint(str(path).encode(), ctypes.byref(c), None), "read_checkpoint header")
    p = np.empty(lib().gpt2_num_parameters(c), np.float32)
    check(lib().gpt2_read_checkpoint(str(path).encode(), ctypes.byref(c), p.ctypes.data_as(_F)), "read_checkpoint")
    return c, p


def write_checkpoint(path, c, params, version=1):
    p = np.ascontiguousarray(params, np.float32)
    check(lib().gpt2_write_checkpoint_ex(str(path).encode(), c, p.ctypes.data_as(_F), int(version)),
          "write_checkpoint")


class Tokenizer(ctypes.Structure):
    """paged_infer.c:852-856"""
    _fields_ = [("vocab_size", ctypes.c_uint32), ("token_table", ctypes.POINTER(ctypes.c_char_p)),
                ("init_ok", ctypes.c_int)]

    def __init__(self, path):
        super().__init__()
        lib().tokenizer_init(ctypes.byref(self), str(path).encode())

    def decode(self, token_id):
        """the token's bytes, or None (not initialised / out of range)"""
        return lib().tokenizer_decode(ctypes.byref(self), int(token_id))

    def free(self):
        lib().tokenizer_free(ctypes.byref(self))


# ---------------------------------------------------------------- block manager
class BlockManager:
    """block_manager.c API (create_block_manager, request_block, ...)."""

    def __init__(self, channels, max_prompts=None, max_blocks=None, block_size=None,
                 max_blocks_per_prompt=None, host_pages=False):
        L = lib()
        if max_prompts is None:
            self.h = L.create_block_manager(channels)
        else:
            self.h = L.create_block_manager_ex(channels, max_prompts, max_blocks, block_size,
                                               max_blocks_per_prompt or max_blocks)
        if not self.h:
            raise MemoryError("create_block_manager failed")
        if host_pages:
            L.bm_use_host_pages(self.h)

    def request_block(self, prompt):
        blk = lib().request_block(self.h, prompt)
        return lib().bm_block_index(self.h, blk) if blk else -1

    def block(self, index):
        base = ctypes.cast(self.h, ctypes.POINTER(ctypes.c_void_p))
        blocks = ctypes.cast(base[1], ctypes.POINTER(KVBlock))  # BlockManager.blocks
        return blocks[index]

    def close(self):
        if self.h:
            lib().destroy_block_manager(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ---------------------------------------------------------------- model / decode engine
class Model:
    """GPT2 + the decode engine (gpt2_decode_*), i.e. the hot path."""

    def __init__(self, cfg, params=None, seed=1337, checkpoint=None):
        L = lib()
        if checkpoint is not None:  # config from the file's header
            cfg = GPT2Config()
            check(L.gpt2_read_checkpoint(str(checkpoint).encode(), ctypes.byref(cfg), None), "checkpoint header")
        self.cfg = cfg if isinstance(cfg, GPT2Config) else config(cfg)
        self.h = L.gpt2_alloc()
        if checkpoint is not None:
            L.gpt2_build_from_checkpoint(self.h, str(checkpoint).encode())
        elif params is not None:
            p = np.ascontiguousarray(params, np.float32)
            assert p.size == L.gpt2_num_parameters(self.cfg)
            check(L.gpt2_build_from_params(self.h, self.cfg, p.ctypes.data_as(_F)), "build_from_params")
        else:
            check(L.gpt2_build_synthetic(self.h, self.cfg, seed), "build_synthetic")
        self.B = 0

    def set_manager(self, bm):
        """model.manager = bm (paged_infer.c:986-987): the engine's pages come
        from this manager's capacity, with its LRU policy"""
        self._bm = bm
        lib().gpt2_set_manager(self.h, bm.h)

    def decode_init(self, B, page_size=16, max_ctx=None, kv_dtype=HPA_F32, w_dtype=HPA_F32):
        max_ctx = max_ctx or self.cfg.max_seq_len
        check(lib().gpt2_decode_init_w(self.h, B, page_size, max_ctx, int(kv_dtype), int(w_dtype)),
              "gpt2_decode_init")
        self.B = B

    def set_graph(self, on):
        check(lib().gpt2_decode_set_graph(self.h, int(on)), "set_graph")

    def step(self, tokens=None, want_next=True):
        nxt = np.zeros(self.B, np.int32) if want_next else None
        tp = None
        if tokens is not None:
            tokens = np.ascontiguousarray(tokens, np.int32)
            assert tokens.shape == (self.B,)
            tp = tokens.ctypes.data_as(_I)
        check(lib().gpt2_decode_step(self.h, tp, nxt.ctypes.data_as(_I) if want_next else None),
              "gpt2_decode_step")
        return nxt

    def step_traced(self, tokens=None):
        """one eager step; returns (next ids, the residual stream entering every
        layer and the final one, (L+1, B, C))"""
        nxt = np.zeros(self.B, np.int32)
        xs = np.zeros((self.cfg.num_layers + 1, self.B, self.cfg.channels), np.float32)
        tp = None
        if tokens is not None:
            tokens = np.ascontiguousarray(tokens, np.int32)
            tp = tokens.ctypes.data_as(_I)
        check(lib().gpt2_decode_step_traced(self.h, tp, nxt.ctypes.data_as(_I), xs.ctypes.data_as(_F)),
              "gpt2_decode_step_traced")
        return nxt, xs

    def step_async(self, tokens=None):
        tp = None
        if tokens is not None:
            tokens = np.ascontiguousarray(tokens, np.int32)
            tp = tokens.ctypes.data_as(_I)
        check(lib().gpt2_decode_step_async(self.h, tp), "gpt2_decode_step_async")

    def logits(self):
        ptr = lib().gpt2_decode_logits(self.h)
        out = np.empty((self.B, self.cfg.vocab_size), np.float32)
        check(lib().hpa_memcpy(out.ctypes.data, ptr, out.nbytes), "logits download")
        return out

    def logits_ptr(self):
        return lib().gpt2_decode_logits(self.h)

    def next_ptr(self):
        return lib().gpt2_decode_next(self.h)

    def positions(self):
        out = np.zeros(self.B, np.int32)
        check(lib().gpt2_decode_positions(self.h, out.ctypes.data_as(_I)), "positions")
        return out

    def set_attn_splits(self, splits):
        """context ranges per (sequence, head) of the decode attention (0 = by shape)"""
        check(lib().gpt2_decode_set_attn_splits(self.h, int(splits)), "set_attn_splits")
        return lib().gpt2_decode_attn_splits(self.h)

    def attn_splits(self):
        return lib().gpt2_decode_attn_splits(self.h)

    def attn_waves(self):
        return lib().gpt2_decode_attn_waves(self.h)

    def set_global_batch(self, total):
        """shape picks of the unsharded engine of `total` rows (<= 64; 0 = this
        engine's own B): a shard's rows then equal that engine's bit for bit"""
        check(lib().gpt2_decode_set_global_batch(self.h, int(total)), "set_global_batch")

    def set_layer_kernel(self, on):
        """layer loop: 0 five launches, 2 full persistent layer, 3 attention
        launch + persistent chain, 4 the chain with wide units (B <= 16,
        C = 768), 1 the form measured fastest for the batch (bf16 weights:
        any nonzero value is the bf16 chain, B <= 256);
        returns whether a persistent form is now in use"""
        check(lib().gpt2_decode_set_layer_kernel(self.h, int(on)), "set_layer_kernel")
        return bool(lib().gpt2_decode_layer_kernel(self.h))

    def layer_kernel(self):
        return bool(lib().gpt2_decode_layer_kernel(self.h))

    def set_pipe_split(self, g_cus):
        """CUs of the pipelined halves' GEMM role (form 7; multiple of 8, 0 = 64)"""
        check(lib().gpt2_decode_set_pipe_split(self.h, int(g_cus)), "set_pipe_split")

    def layer_form(self):
        """0 five launches per layer, 1 full persistent layer, 2 attention launch + persistent chain,
        3 the chain with wide units, 4 the bf16-weight chain (hpa_chain_b16.hip), 5 the pipelined
        halves (hpa_pipe.hip)"""
        return int(lib().gpt2_decode_layer_kernel(self.h))

    def status(self):
        """waits for queued work; raises if a persistent-layer wait timed out"""
        code = lib().gpt2_decode_status(self.h)
        if code:
            raise RuntimeError(f"decode step failed (status {code})")

    def evicted(self):
        """sequences the LRU policy paged out since the last call (bool mask)"""
        m = np.zeros(self.B, np.int32)
        n = lib().gpt2_decode_evicted(self.h, m.ctypes.data_as(_I))
        if n < 0:
            raise RuntimeError("evicted: no engine")
        return m.astype(bool)

    def read_kv(self, layer, b, n):
        """K, V of positions [0, n) of sequence b, token-major (n, C) fp32"""
        C = self.cfg.channels
        k = np.zeros((n, C), np.float32)
        v = np.zeros((n, C), np.float32)
        check(lib().gpt2_decode_read_kv(self.h, int(layer), int(b), int(n), k.ctypes.data_as(_F),
                                        v.ctypes.data_as(_F)), "read_kv")
        return k, v

    def shard(self, rows_per_rank, root=0):
        """sequence-sharded decode: this rank's row count among rows_per_rank
        (after hpa_comm_init); gather() then runs the RCCL end-of-step gather"""
        r = np.ascontiguousarray(rows_per_rank, np.int32)
        check(lib().gpt2_decode_shard(self.h, r.ctypes.data_as(_I), int(root)), "shard")

    def gather(self, what=0):
        check(lib().gpt2_decode_gather(self.h, int(what)), "gather")

    def gathered(self, total_rows, what=0):
        """root: host copy of the last gather (waits for it)"""
        check(lib().gpt2_decode_gather_wait(self.h), "gather_wait")
        ptr = lib().gpt2_decode_gathered(self.h, int(what))
        if not ptr:
            return None
        out = np.empty((total_rows, self.cfg.vocab_size) if what == 0 else (total_rows,),
                       np.float32 if what == 0 else np.int32)
        check(lib().hpa_memcpy(out.ctypes.data, ptr, out.nbytes), "gathered download")
        return out

    def time_attention(self, iters=48):
        """(avg ms, algorithmic bytes) per launch of the decode attention
        kernel, back-to-back launches at the last step's positions"""
        ms, by = ctypes.c_double(), ctypes.c_double()
        check(lib().gpt2_decode_time_attention(self.h, int(iters), ctypes.byref(ms), ctypes.byref(by)),
              "time_attention")
        return ms.value, by.value

    def time_attention_pf(self, frac, iters=24, grid=1024):
        """(attention ms, prefetch ms) per iteration: the first `frac` of the
        layer's pool slab read into the Infinity Cache, then its attention"""
        a, p = ctypes.c_double(), ctypes.c_double()
        check(lib().gpt2_decode_time_attention_pf(self.h, int(iters), float(frac), int(grid), ctypes.byref(a),
                                                  ctypes.byref(p)), "time_attention_pf")
        return a.value, p.value

    def prefill(self, tokens):
        """tokens (B, T): all T tokens of every sequence in one pass; returns
        the greedy next ids (B,)"""
        tokens = np.ascontiguousarray(tokens, np.int32)
        assert tokens.ndim == 2 and tokens.shape[0] == self.B
        nxt = np.zeros(self.B, np.int32)
        check(lib().gpt2_decode_prefill(self.h, tokens.ctypes.data_as(_I), tokens.shape[1],
                                        nxt.ctypes.data_as(_I)), "prefill")
        return nxt

    def prefill_ragged(self, seqs):
        """seqs: B token lists (empty = sequence untouched); one pass over
        all of them (continuous batching); returns the next ids (B,)"""
        assert len(seqs) == self.B
        lens = np.array([len(t) for t in seqs], np.int32)
        flat = np.ascontiguousarray(np.concatenate([np.asarray(t, np.int32).reshape(-1) for t in seqs])
                                    if lens.sum() else np.zeros(1, np.int32), np.int32)
        nxt = np.zeros(self.B, np.int32)
        check(lib().gpt2_decode_prefill_ragged(self.h, flat.ctypes.data_as(_I), lens.ctypes.data_as(_I),
                                               nxt.ctypes.data_as(_I)), "prefill_ragged")
        return nxt

    def release(self, seq):
        """retire sequence seq: pages back to the pool, position 0"""
        check(lib().gpt2_decode_release(self.h, int(seq)), "release")

    def set_sampling(self, enable=True, seed=1337):
        check(lib().gpt2_decode_set_sampling(self.h, int(bool(enable)), int(seed)), "set_sampling")

    def gemm_config(self, waves=None, row_blocks=None, col_tiles=None):
        """fused GEMM launch shapes [qkv, attproj, fc, fcproj, logits]:
        (waves, 16-row blocks, 16-column tiles) per workgroup; applies the
        nonzero entries of the given lists first"""
        arrs = [np.ascontiguousarray(a if a is not None else [0] * 5, np.int32)
                for a in (waves, row_blocks, col_tiles)]
        if any(a is not None for a in (waves, row_blocks, col_tiles)):
            check(lib().gpt2_decode_gemm_config(self.h, *[a.ctypes.data_as(_I) for a in arrs], 1),
                  "gemm_config")
        out = [np.zeros(5, np.int32) for _ in range(3)]
        check(lib().gpt2_decode_gemm_config(self.h, *[a.ctypes.data_as(_I) for a in out], 0), "gemm_config")
        return tuple(out)

    def step_bytes(self):
        att = ctypes.c_double()
        tot = lib().gpt2_decode_step_bytes(self.h, ctypes.byref(att))
        return tot, att.value

    def reset(self):
        check(lib().gpt2_decode_reset(self.h), "reset")

    def reserve(self, ctx):
        check(lib().gpt2_decode_reserve(self.h, ctx), "reserve")

    def set_positions(self, pos):
        pos = np.ascontiguousarray(pos, np.int32)
        check(lib().gpt2_decode_set_positions(self.h, pos.ctypes.data_as(_I)), "set_positions")

    def fill_random(self, ctx, seed=1, seq_offset=0):
        """synthetic K/V of positions [0, ctx); seq_offset: this engine's rows
        are sequences seq_offset.. of a larger (sharded) batch"""
        check(lib().gpt2_decode_fill_random_ex(self.h, ctx, seed, seq_offset), "fill_random")

    def close(self):
        if self.h:
            lib().hpa_synchronize()
            lib().gpt2_release(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def synthetic_params(cfg, seed=1337):
    L = lib()
    c = cfg if isinstance(cfg, GPT2Config) else config(cfg)
    n = L.gpt2_num_parameters(c)
    p = np.empty(n, np.float32)
    check(L.gpt2_synthetic_params(c, seed, p.ctypes.data_as(_F)), "synthetic_params")
    return p


class Timer:
    """HIP events on the library's stream (where the kernels run)."""

    def __init__(self):
        self.a = lib().hpa_event_create()
        self.b = lib().hpa_event_create()

    def start(self):
        check(lib().hpa_event_record(self.a), "event_record")

    def stop(self):
        check(lib().hpa_event_record(self.b), "event_record")
        return lib().hpa_event_elapsed_ms(self.a, self.b)

    def __del__(self):
        try:
            lib().hpa_event_destroy(self.a)
            lib().hpa_event_destroy(self.b)
        except Exception:
            pass
