"""Sequence sharding of the paged decode across ranks: the
batch layout bench.py and the tests use.

Decode sequences are independent, so a step has no exchange inside it: each
rank owns a contiguous range of sequences, its own page pool and block
tables, and a full replica of the weights.  The one collective is the
north star's end-of-step gather of the logits (or greedy ids) to the root,
which lives in the C library (gpt2_decode_gather -> hpa_comm_gatherv over
RCCL; its schedule is hpa_comm_gather_plan, run over gloo by
tests/test_multi_rank.py).
"""


def shard_range(B, world, rank):
    """contiguous sequence range [lo, hi) of `rank` out of B sequences"""
    if B < world:
        raise ValueError(f"batch {B} smaller than world size {world}")
    base, rem = divmod(B, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def batch_layout(batch, world, rank, scaling):
    """(global B, lo, hi) for this rank.  strong (the metric's 2/4/8-GPU
    points): `batch` sequences in total split across ranks; weak (BASELINE
    config 4: 64 per GPU, B = 64 * n): `batch` sequences per rank"""
    if scaling == "weak":
        return batch * world, rank * batch, (rank + 1) * batch
    if scaling == "strong":
        lo, hi = shard_range(batch, world, rank)
        return batch, lo, hi
    raise ValueError(scaling)
