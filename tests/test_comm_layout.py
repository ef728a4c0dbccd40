"""Host arithmetic of the end-of-step gather (hpa_comm_gather_layout, the
offsets hpa_comm_gatherv posts its ncclRecv at): runs on the CPU through the
C ABI, no GPU and no communicator needed.  Covers uneven rows, a non-zero
root and ranks with zero rows (the multi-rank RCCL branch cannot
run with two ranks on the test box's single GPU)."""
import ctypes

import numpy as np
import pytest

sz = ctypes.c_size_t


@pytest.fixture(scope="module")
def L():
    import pagedattn
    return pagedattn.lib()


def layout(L, nranks, rank, root, nbytes):
    b = (sz * nranks)(*nbytes)
    off = (sz * nranks)()
    own = sz(12345)
    n = L.hpa_comm_gather_layout(nranks, rank, root, b, off, ctypes.byref(own))
    return n, list(off), own.value


@pytest.mark.parametrize("rows,root", [([3, 3], 0), ([4, 3, 0, 5], 0), ([2, 0, 7, 1, 0, 9, 3, 3], 5),
                                       ([0, 0, 4], 2), ([8] * 8, 7), ([1], 0)])
def test_offsets_are_rank_order_prefix_sums(L, rows, root):
    V = 50257 * 4
    nbytes = [r * V for r in rows]
    expect_off = list(np.concatenate([[0], np.cumsum(nbytes)[:-1]]).astype(int))
    for rank in range(len(rows)):
        n, off, own = layout(L, len(rows), rank, root, nbytes)
        assert off == expect_off
        if rank == root:
            assert own == expect_off[root]
            assert n == sum(1 for r, b in enumerate(nbytes) if r != root and b)  # ncclRecv posted
        else:
            assert n == (1 if nbytes[rank] else 0)  # sends iff it has rows


def test_zero_row_ranks_never_post(L):
    n, off, own = layout(L, 4, 0, 0, [0, 0, 0, 0])
    assert n == 0 and off == [0, 0, 0, 0] and own == 0


def test_bad_arguments(L):
    b = (sz * 2)(1, 1)
    assert L.hpa_comm_gather_layout(2, 2, 0, b, None, None) == -1
    assert L.hpa_comm_gather_layout(2, 0, 2, b, None, None) == -1
    assert L.hpa_comm_gather_layout(0, 0, 0, b, None, None) == -1
    assert L.hpa_comm_gather_layout(2, 0, 0, None, None, None) == -1
    assert L.hpa_comm_gather_layout(2, 1, 0, b, None, None) == 1  # NULL outputs allowed
