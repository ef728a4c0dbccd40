"""Sequence sharding of the paged decode across ranks.

Decode sequences are independent, so a step has no exchange inside it: each
rank owns a contiguous range of sequences, its own page pool and block
tables, and a full replica of the weights.  The one collective is at the end
of the step, the north star's logits gather to rank 0 over RCCL/xGMI
(`ncclGather` of [B_local x V] fp32); the cheaper variant gathers only the
greedy ids.  The same code drives `gloo` on CPU tensors in the multi-process
tests and `nccl` (RCCL) on device tensors in bench.py.
"""


def shard_range(B, world, rank):
    """contiguous sequence range [lo, hi) of `rank` out of B sequences"""
    if B < world:
        raise ValueError(f"batch {B} smaller than world size {world}")
    base, rem = divmod(B, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def batch_layout(batch, world, rank, scaling):
    """(global B, lo, hi) for this rank.  weak: `batch` sequences per rank
    (BASELINE config 4: 64 per GPU, B = 64 * n); strong: `batch` sequences in
    total split across ranks"""
    if scaling == "weak":
        return batch * world, rank * batch, (rank + 1) * batch
    if scaling == "strong":
        lo, hi = shard_range(batch, world, rank)
        return batch, lo, hi
    raise ValueError(scaling)


class StepGather:
    """End-of-step gather to rank 0 of every rank's logits ("logits") or
    greedy ids ("ids"); "none" skips the collective.  Ranks may hold
    different numbers of sequences (strong scaling with B % world != 0): the
    gather is over padded [max_local, ...] buffers and rank 0 trims them.
    `src` tensors live on `device` ("cuda" for RCCL, "cpu" for gloo)."""

    def __init__(self, dist, world, rank, counts, V, mode, device):
        import torch
        self.dist, self.world, self.rank, self.mode = dist, world, rank, mode
        self.counts = list(counts)
        self.max_local = max(self.counts)
        self.V = V
        width = V if mode == "logits" else 1
        dtype = torch.float32 if mode == "logits" else torch.int32
        self.send = torch.zeros(self.max_local, width, dtype=dtype, device=device)
        self.recv = None
        if rank == 0 and mode != "none":
            self.recv = [torch.zeros_like(self.send) for _ in range(world)]

    def buffer(self):
        """the [max_local, width] send buffer the step's output is copied into"""
        return self.send

    def gather(self):
        if self.mode == "none" or self.world == 1:
            return
        self.dist.gather(self.send, gather_list=self.recv, dst=0)

    def result(self):
        """rank 0: the gathered [B, V] logits or [B] ids in global sequence order"""
        import torch
        if self.rank != 0 or self.mode == "none":
            return None
        parts = [self.send[:self.counts[0]]] if self.world == 1 else \
            [r[:n] for r, n in zip(self.recv, self.counts)]
        out = torch.cat(parts, 0)
        return out if self.mode == "logits" else out[:, 0]
