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
    `src` tensors live on `device` ("cuda" for RCCL, "cpu" for gloo).

    nbuf = 2 double-buffers the step output so the gather of step k can run
    asynchronously (async_op) while step k+1 computes: gather(i, async_op=True)
    returns once the collective is queued; before buffer i is refilled,
    wait(i) orders the refill after that collective (on RCCL: the caller's
    current stream waits for it; the host does not block)."""

    def __init__(self, dist, world, rank, counts, V, mode, device, nbuf=1):
        import torch
        self.dist, self.world, self.rank, self.mode = dist, world, rank, mode
        self.counts = list(counts)
        self.max_local = max(self.counts)
        self.V = V
        width = V if mode == "logits" else 1
        dtype = torch.float32 if mode == "logits" else torch.int32
        self.send = [torch.zeros(self.max_local, width, dtype=dtype, device=device) for _ in range(nbuf)]
        self.recv = [None] * nbuf
        if rank == 0 and mode != "none":
            self.recv = [[torch.zeros_like(self.send[0]) for _ in range(world)] for _ in range(nbuf)]
        self.work = [None] * nbuf

    def buffer(self, i=0):
        """the [max_local, width] send buffer i the step's output is copied into"""
        return self.send[i]

    def wait(self, i=0):
        """order the next use of buffer i after its outstanding gather"""
        if self.work[i] is not None:
            self.work[i].wait()
            self.work[i] = None

    def gather(self, i=0, async_op=False):
        if self.mode == "none" or self.world == 1:
            return
        self.wait(i)
        w = self.dist.gather(self.send[i], gather_list=self.recv[i], dst=0, async_op=async_op)
        if async_op:
            self.work[i] = w

    def result(self, i=0):
        """rank 0: the gathered [B, V] logits or [B] ids in global sequence
        order (after wait(i) for an asynchronous gather)"""
        import torch
        if self.rank != 0 or self.mode == "none":
            return None
        parts = [self.send[i][:self.counts[0]]] if self.world == 1 else \
            [r[:n] for r, n in zip(self.recv[i], self.counts)]
        out = torch.cat(parts, 0)
        return out if self.mode == "logits" else out[:, 0]
