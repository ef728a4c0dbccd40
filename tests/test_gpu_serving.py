"""Continuous batching: ragged prefill that mixes new
prompts with single decode tokens, admission into released slots, and the
reference's LRU whole-sequence eviction under pool pressure
(block_manager.c:104-162), all against one oracle decoder per request.

Bars as the decode tests: logits within 2e-4 of the oracle, greedy ids
bit-exact where the oracle's top-2 margin exceeds 1e-3.
"""
import numpy as np
import pytest

import oracle_ctypes as oc
import synth

pytestmark = pytest.mark.gpu
SMALL = dict(maxT=256, V=1000, L=2, NH=2, C=128)
LOGIT_TOL = 2e-4
TIE_MARGIN = 1e-3


class Request:
    """one sequence in the oracle: a B = 1 paged decoder fed token by token"""

    def __init__(self, params, c, P, seed):
        self.o = oc.PagedDecoder(params, c, 1, P, SMALL["maxT"], page_seed=seed)

    def feed(self, toks):
        for t in toks:
            nxt, lg = self.o.step(np.array([t], np.int32))
        return int(nxt[0]), lg[0]

    def pos(self):
        return self.o.pos(0)

    def close(self):
        self.o.close()


class Server:
    """the engine's slots next to one oracle Request per live slot"""

    def __init__(self, hip, B, P, seed, bm=None):
        self.params = synth.params(SMALL, seed=seed)
        self.c = oc.cfg(SMALL["maxT"], SMALL["V"], SMALL["L"], SMALL["NH"], SMALL["C"])
        self.model = hip.Model(SMALL, params=self.params)
        if bm is not None:
            self.model.set_manager(bm)
        self.model.decode_init(B, P, SMALL["maxT"])
        self.B, self.P = B, P
        self.rng = np.random.default_rng(seed)
        self.reqs = [None] * B
        self.cur = [0] * B  # the oracle's next id per slot (fed back, so ties cannot diverge)
        self.worst = 0.0
        self.n_req = 0

    def admit(self, b, n):
        """a new prompt of n tokens in slot b (releasing what was there)"""
        if self.reqs[b] is not None:
            self.reqs[b].close()
            self.model.release(b)
        self.n_req += 1
        self.reqs[b] = Request(self.params, self.c, self.P, seed=100 + self.n_req)
        return [int(t) for t in self.rng.integers(0, SMALL["V"], n)]

    def _check(self, b, g_next, o_next, o_logits, logits):
        self.worst = max(self.worst, float(np.abs(logits[b] - o_logits).max()))
        s = np.sort(o_logits)
        if s[-1] - s[-2] > TIE_MARGIN:
            assert g_next[b] == o_next, (b, g_next[b], o_next)
        self.cur[b] = o_next

    def run(self, batch):
        """batch: slot -> tokens; one ragged call for all of them"""
        g_next = self.model.prefill_ragged([batch.get(b, []) for b in range(self.B)])
        logits = self.model.logits()
        for b, toks in batch.items():
            o_next, o_logits = self.reqs[b].feed(toks)
            self._check(b, g_next, o_next, o_logits, logits)
        self.check_positions()

    def decode(self):
        """one plain decode step of every slot (all must be live)"""
        toks = np.array(self.cur, np.int32)
        g_next = self.model.step(toks)
        logits = self.model.logits()
        for b in range(self.B):
            o_next, o_logits = self.reqs[b].feed([int(toks[b])])
            self._check(b, g_next, o_next, o_logits, logits)
        self.check_positions()

    def check_positions(self):
        pos = self.model.positions()
        for b, r in enumerate(self.reqs):
            if r is not None:
                assert pos[b] == r.pos(), (b, pos[b], r.pos())

    def close(self):
        for r in self.reqs:
            if r is not None:
                r.close()
        self.model.close()


def test_ragged_prefill_matches_oracle(hip):
    """ragged lengths incl. 0 (untouched) and lengths across page and 64-row
    query-block boundaries, then decode continues"""
    s = Server(hip, B=4, P=16, seed=1)
    s.run({0: s.admit(0, 37), 2: s.admit(2, 5), 3: s.admit(3, 70)})
    before = s.model.positions()[1]
    s.run({1: s.admit(1, 64)})
    assert before == 0
    for _ in range(3):
        s.decode()
    assert s.worst <= LOGIT_TOL, s.worst
    s.close()


def test_continuous_batching_matches_oracle(hip):
    """admissions while other slots decode, a release and re-admission into
    the same slot (its pages reused), then plain decode steps"""
    s = Server(hip, B=3, P=16, seed=2)
    s.run({0: s.admit(0, 20), 1: s.admit(1, 7)})
    for _ in range(3):
        s.run({0: [s.cur[0]], 1: [s.cur[1]]})
    s.run({0: [s.cur[0]], 1: [s.cur[1]], 2: s.admit(2, 30)})
    s.run({0: [s.cur[0]], 1: s.admit(1, 12), 2: [s.cur[2]]})  # slot 1 retired and re-admitted
    for _ in range(4):
        s.run({b: [s.cur[b]] for b in range(3)})
    for _ in range(3):
        s.decode()
    assert s.worst <= LOGIT_TOL, s.worst
    s.close()


def test_inactive_rows_untouched(hip):
    """a sequence with 0 tokens in a ragged call keeps its position, its next
    id and its logits row"""
    s = Server(hip, B=2, P=8, seed=3)
    s.run({0: s.admit(0, 9), 1: s.admit(1, 4)})
    nxt0 = s.model.step(None)  # device-fed step, then a ragged call touching only slot 1
    lg0 = s.model.logits()[0].copy()
    pos0 = s.model.positions()[0]
    g = s.model.prefill_ragged([[], [3, 4, 5]])
    assert g[0] == nxt0[0]
    assert s.model.positions()[0] == pos0
    assert np.array_equal(s.model.logits()[0], lg0)
    s.close()


def test_lru_eviction_restarts_sequence(hip):
    """a pool of 5 pages for 2 sequences: growing sequence 1 evicts the
    least recently allocated sequence (0) whole, which restarts at
    position 0 with the token it was fed"""
    bm = hip.BlockManager(SMALL["C"], max_prompts=2, max_blocks=5, block_size=16, max_blocks_per_prompt=16)
    s = Server(hip, B=2, P=16, seed=4, bm=bm)
    s.run({0: s.admit(0, 40), 1: s.admit(1, 31)})  # 3 + 2 pages: pool full
    s.decode()  # sequence 1 writes position 31 (its 2nd page): no eviction yet
    # next step: sequence 1 needs a 3rd page -> sequence 0 (LRU) is evicted
    s.reqs[0].close()
    s.reqs[0] = Request(s.params, s.c, 16, seed=999)
    s.decode()
    assert s.model.positions()[0] == 1 and s.reqs[0].pos() == 1
    assert s.worst <= LOGIT_TOL, s.worst
    s.close()
    bm.close()


def test_ragged_prefill_rejects_bad_lengths(hip):
    s = Server(hip, B=2, P=16, seed=5)
    with pytest.raises(RuntimeError):
        s.model.prefill_ragged([[1] * (SMALL["maxT"] + 1), []])
    with pytest.raises(RuntimeError):
        s.model.prefill_ragged([[SMALL["V"]], [1]])  # token out of range
    s.close()
