"""Host logic of the physical-chunk placement (bayesdll_amd.placement) — no GPU:
chunk geometry and the candidate assignments the full-size timing chooses from
(DESIGN.md §4 "Placement")."""
import random

import pytest

from bayesdll_amd import placement as P


@pytest.mark.parametrize("n", [1 << 24, 44549160, 306535400, 305548325, (1 << 28) + 1])
def test_chunk_geometry_covers_the_vector_in_2mib_chunks_of_at_most_1gib(n):
    per, cb = P.chunk_geometry(n)
    assert cb % P.ALIGN == 0 and cb <= P.CHUNK_TARGET + P.ALIGN
    assert per * cb >= 4 * n > (per - 1) * cb
    assert per == -(-4 * n // P.CHUNK_TARGET)


def test_vit_l_32_is_two_chunks_of_586_mib():
    per, cb = P.chunk_geometry(306535400)
    assert (per, cb >> 20) == (2, 586)


@pytest.mark.parametrize("names", [["theta", "grad", "mom"],
                                   ["theta", "grad", "mom", "prior"],
                                   ["theta", "grad", "mom", "prior", "adam_m", "adam_v", "sgd_buf"]])
@pytest.mark.parametrize("per", [1, 2, 3])
def test_candidates_are_disjoint_role_assignments(names, per):
    nchunks = len(names) * per + 2 * per
    rng = random.Random(per * 31 + len(names))
    times = {(i, j): rng.random() for i in range(nchunks) for j in range(nchunks) if i != j}
    cands = P.candidate_assignments(times, nchunks, names, per)
    # allocation order first
    assert cands[0] == {nm: list(range(q * per, (q + 1) * per)) for q, nm in enumerate(names)}
    assert 2 <= len(cands) <= P.COMPOSITES + 1
    seen = []
    for c in cands:
        assert list(c) == names
        ids = [k for nm in names for k in c[nm]]
        assert all(len(c[nm]) == per for nm in names)
        assert len(ids) == len(set(ids)) and all(0 <= k < nchunks for k in ids)
        assert c not in seen
        seen.append(c)
    # the first greedy candidate holds the fastest pair as theta / mom chunk 0
    best = min(times, key=times.get)
    assert (cands[1]["theta"][0], cands[1]["mom"][0]) == best


def test_greedy_completion_takes_the_fastest_disjoint_pairs():
    names = ["theta", "grad", "mom"]
    # chunk pairs (0, 1) and (2, 3) fastest; anything touching 0..3 otherwise slow
    times = {(i, j): 1.0 for i in range(8) for j in range(8) if i != j}
    times[(0, 1)] = 0.1
    times[(2, 3)] = 0.2
    times[(4, 5)] = 0.3
    c = P.candidate_assignments(times, 8, names, 2)[1]
    assert c["theta"] == [0, 2] and c["mom"] == [1, 3] and c["grad"] == [4, 5]
    # seeded by the second-fastest pair: it leads, the fastest disjoint one follows
    c2 = P.candidate_assignments(times, 8, names, 2)[2]
    assert c2["theta"] == [2, 0] and c2["mom"] == [3, 1]


def test_no_pair_times_gives_allocation_order_only():
    names = ["theta", "grad", "mom"]
    assert P.candidate_assignments({}, 6, names, 2) == [
        {"theta": [0, 1], "grad": [2, 3], "mom": [4, 5]}]


def test_draw_buffer_keeps_small_vectors_and_honours_placement_off(monkeypatch):
    """flat.draw_buffer times candidates only for vectors of >= PLACEMENT_MIN_ELEMS
    with placement on; otherwise it returns the draw's own buffer untouched and
    never launches."""
    import torch

    from bayesdll_amd import flat as F

    def launch(_):
        raise AssertionError("no launch expected")

    small = torch.empty(F.PLACEMENT_MIN_ELEMS - 1)
    assert F.draw_buffer(small, launch) == (small, None)
    monkeypatch.setenv("BDL_PLACEMENT", "0")
    big = torch.empty(F.PLACEMENT_MIN_ELEMS)
    out, ms = F.draw_buffer(big, launch)
    assert out is big and ms is None


def test_one_candidates_rank_chunks_by_position_then_allocation_order():
    """placement.one_candidates (the posterior draw's output, placement.place_one):
    position by position the w-th fastest chunk not yet used, then the
    allocation order; each list once, per distinct chunks in range."""
    ms = [0.30, 0.10, 0.40, 0.12, 0.11, 0.50]
    c = P.one_candidates([ms, ms], 2)                    # both positions alike
    assert c[0] == [1, 4]                                # the two fastest chunks
    assert c[1] == [4, 3] and c[2] == [3, 0]             # next windows of the ranking
    assert c[-1] == [0, 1]                               # allocation order last
    assert len(c) == P.ONE_COMPOSITES + 1
    for ids in c:
        assert len(ids) == 2 and len(set(ids)) == 2 and all(0 <= i < len(ms) for i in ids)
    # the chunk fastest at position 1 differs from position 0's
    p0 = [0.30, 0.10, 0.40, 0.50]
    p1 = [0.30, 0.50, 0.40, 0.10]
    assert P.one_candidates([p0, p1], 2)[0] == [1, 3]
    # one chunk per vector, fewer chunks than windows
    assert P.one_candidates([[0.2, 0.1]], 1) == [[1], [0]]
    assert P._one_estimate([p0, p1], 2) == pytest.approx(0.2)


def test_moment_pair_halves_of_one_allocation(monkeypatch):
    """flat.moment_pair: for vectors of >= PLACEMENT_MIN_ELEMS, m1 / m2 are the
    two halves of one allocation (disjoint, m2 on a 256-B boundary, both
    contiguous, n elements each); smaller vectors and BDL_PLACEMENT=0 get two
    plain allocations."""
    import torch

    from bayesdll_amd import flat as F
    monkeypatch.delenv("BDL_PLACEMENT", raising=False)
    for n in (F.PLACEMENT_MIN_ELEMS, F.PLACEMENT_MIN_ELEMS + 3, 306535400):
        m1, m2 = F.moment_pair(n, "cpu")
        assert m1.numel() == n and m2.numel() == n
        assert m1.is_contiguous() and m2.is_contiguous()
        assert m1.untyped_storage().data_ptr() == m2.untyped_storage().data_ptr()
        assert m1.data_ptr() + 4 * n <= m2.data_ptr()
        assert (m2.data_ptr() - m1.data_ptr()) % 256 == 0
        assert m2.data_ptr() + 4 * n <= m1.untyped_storage().data_ptr() + m1.untyped_storage().nbytes()
    small = F.moment_pair(1000, "cpu")
    assert small[0].untyped_storage().data_ptr() != small[1].untyped_storage().data_ptr()
    monkeypatch.setenv("BDL_PLACEMENT", "0")
    a, b = F.moment_pair(F.PLACEMENT_MIN_ELEMS, "cpu")
    assert a.untyped_storage().data_ptr() != b.untyped_storage().data_ptr()


def test_ref_split_needs_two_groups_and_enough_of_each():
    """placement._ref_split (the "ref" search): chunks slow against chunk 0 share
    its group, the rest are the fast group; no split without a spread or
    without per - 1 slow and per fast chunks."""
    t = {1: 1.05, 2: 0.96, 3: 1.06, 4: 0.95, 5: 0.97, 6: 1.04, 7: 0.955}
    slow, fast = P._ref_split(t, 2)
    assert slow == [3, 1, 6] and fast == [4, 7, 2, 5]
    assert P._ref_split({1: 1.0, 2: 0.995, 3: 1.001}, 2) is None      # one group
    assert P._ref_split({1: 0.95, 2: 0.96, 3: 1.05}, 3) is None       # one slow < per - 1
    assert P._ref_split({1: 1.05, 2: 1.06, 3: 0.95}, 2) is None       # one fast < per
    assert P._ref_split({}, 1) is None


@pytest.mark.parametrize("names", [["theta", "mom"], ["theta", "mom", "prior"],
                                   ["theta", "mom", "prior", "adam_m", "adam_v", "sgd_buf"]])
@pytest.mark.parametrize("per", [1, 2, 3])
def test_ref_candidates_pair_chunk0s_group_with_the_fast_group(names, per):
    nchunks = len(names) * per + 2 * per
    rng = random.Random(7 * per + len(names))
    # chunks 0..per (chunk 0's group) slow against 0, the rest fast, with noise
    t0 = {j: (1.05 if j <= per else 0.96) + 0.005 * rng.random() for j in range(1, nchunks)}
    cands = P.ref_candidates(t0, nchunks, names, per)
    assert cands[0] == {nm: list(range(q * per, (q + 1) * per)) for q, nm in enumerate(names)}
    assert 2 <= len(cands) <= P.COMPOSITES + 1
    group0 = set(range(per + 1))
    for c in cands:
        ids = [k for nm in names for k in c[nm]]
        assert all(len(c[nm]) == per for nm in names)
        assert len(ids) == len(set(ids)) and all(0 <= k < nchunks for k in ids)
    for c in cands[1:]:
        th, mo = set(c["theta"]), set(c["mom"])
        # one of theta / mom is chunk 0's group, the other entirely the fast group
        assert (th <= group0 and not mo & group0) or (mo <= group0 and not th & group0)
    # the first: theta = chunk 0 and its group, mom = the fastest chunks
    fastest = sorted((j for j in t0 if j > per), key=t0.get)[:per]
    assert cands[1]["theta"][0] == 0 and cands[1]["mom"] == fastest
    # no split: allocation order only
    assert P.ref_candidates({j: 1.0 for j in range(1, nchunks)}, nchunks, names, per) == cands[:1]


def test_one_found_needs_a_spread_and_per_fast_chunks():
    """placement._one_found (place_one's escalation stop rule)."""
    assert P._one_found([0.30, 0.31, 0.295, 0.311], 2)          # 5 % spread, 2 fast
    assert not P._one_found([0.30, 0.301, 0.302, 0.3005], 1)    # one group
    assert not P._one_found([0.29, 0.31, 0.312, 0.311], 2)      # only one fast chunk
    assert P._one_found([0.29, 0.31], 1)


def test_ref_found_wants_the_best_level_not_the_middle_one():
    """placement._ref_found (the escalation's stop rule): a second group at least
    FAST_REF faster than chunk 0's own group stops it; a middle level (~4.5 %)
    or a single group does not."""
    slow = {j: 0.51 + 0.001 * (j % 3) for j in range(1, 8)}
    assert not P._ref_found(slow, 2)                                    # one group
    mid = {**slow, 8: 0.488, 9: 0.489}                            # ~4.3 % faster
    assert not P._ref_found(mid, 2)
    best = {**slow, 8: 0.476, 9: 0.477}                           # ~6.8 % faster
    assert P._ref_found(best, 2)
    assert not P._ref_found({**slow, 8: 0.476}, 2)               # one fast chunk < per
    # chunk 0 alone in its group (per = 1): compared with the slowest time
    assert P._ref_found({1: 0.47, 2: 0.51}, 1)


class _FakeLaunch:
    def __init__(self, roles):
        self.roles = roles

    def __call__(self):
        pass


@pytest.fixture
def fake_chunks(monkeypatch):
    """placement's chunk allocator and mappings replaced by host fakes: each
    chunk / composite is a CPU tensor; returns {data_ptr: chunk ids}."""
    import torch
    monkeypatch.setattr(P, "CHUNK_TARGET", 2 << 20)     # 2-MiB chunks
    chunks_of = {}

    class FakeMapping:
        def __init__(self, dev_index, handles, chunk_bytes, nelem, adopt=None):
            self.owner = self.role = None
            self.handles, self.nelem = list(handles), nelem
            self.va, self.total = 1, len(handles) * chunk_bytes

        def tensor(self):
            t = torch.zeros(self.nelem)
            chunks_of[t.data_ptr()] = self.handles
            return t

    class FakeChunks:
        def __init__(self, dev_index, chunk_bytes):
            self.chunk_bytes, self.handles, self.views = chunk_bytes, [], []

        def add(self, k):
            for _ in range(k):
                h = len(self.handles)
                self.handles.append(h)
                self.views.append(FakeMapping(0, [h], self.chunk_bytes,
                                              self.chunk_bytes // 4).tensor())

        def release(self):
            self.views, self.handles = [], []

    monkeypatch.setattr(P, "Mapping", FakeMapping)
    monkeypatch.setattr(P, "_Chunks", FakeChunks)
    return chunks_of


def test_place_escalates_until_another_group_shows(fake_chunks):
    """placement.place end to end on the host with fake chunks and a timing
    model in which chunks 0-19 form one physical group and 20-39 another
    (theta / mom in different groups: 0.96, same group: 1.05).  The first pool
    (8 chunks, all pairs) is one group; the escalation adds 4 chunks a round,
    each timed against chunk 0, until chunks 20-23 show; the kept set pairs
    the two groups."""
    def time_launch(f):
        th, mo = fake_chunks[f.roles["theta"].data_ptr()], fake_chunks[f.roles["mom"].data_ptr()]
        return sum(0.96 if a // 20 != b // 20 else 1.05 for a, b in zip(th, mo)) / len(th)

    n = 1 << 20                                          # 4 MB: two 2-MiB chunks per vector
    vecs, info = P.place(n, "cuda:0", ["theta", "mom"], lambda roles, m: _FakeLaunch(roles),
                         time_launch, budget_bytes=1 << 34, with_torch=False)
    assert info["chunks_per_vector"] == 2 and info["pairs"] == "all"
    assert info["chunks_allocated"] == 24 and info["escalation_rounds"] == 4
    assert info["pairs_timed"] == 8 * 7 + 16             # first pool all pairs, then vs chunk 0
    assert len(info["ref_ms"]) == 23
    assert info["chosen_ms"] == pytest.approx(0.96) and info["kept"] == "search"
    assert info["retimed_ms"] is None                    # RETIME off by default
    th, mo = info["theta_chunks"], info["mom_chunks"]
    groups = ({c // 20 for c in th}, {c // 20 for c in mo})
    assert groups in (({0}, {1}), ({1}, {0})), (th, mo)
    assert set(vecs) == {"theta", "mom"} and all(v.numel() == n for v in vecs.values())


def test_place_retimes_the_finalists(fake_chunks, monkeypatch):
    """BDL_PLACEMENT_RETIME=3: the three fastest candidates are timed twice
    more and the best MEAN wins — the composite that was lucky once (0.90,
    then 0.99) loses to one that is fast every time (0.95)."""
    monkeypatch.setattr(P, "RETIME", 3)
    order, calls = [], {}
    seq = {0: [0.90, 0.99, 0.99], 1: [0.95, 0.95, 0.95]}  # by first appearance

    def time_launch(f):
        th, mo = fake_chunks[f.roles["theta"].data_ptr()], fake_chunks[f.roles["mom"].data_ptr()]
        if len(th) == 1:                                 # chunk pairs: two groups of 4
            return 0.5 if th[0] // 4 != mo[0] // 4 else 0.55
        key = (tuple(th), tuple(mo))
        if key not in calls:
            order.append(key)
            calls[key] = 0
        calls[key] += 1
        return seq.get(order.index(key), [1.0] * 3)[calls[key] - 1]

    n = 1 << 20
    _, info = P.place(n, "cuda:0", ["theta", "mom"], lambda roles, m: _FakeLaunch(roles),
                      time_launch, budget_bytes=1 << 34, with_torch=False)
    assert info["composites_ms"][:2] == [0.9, 0.95]
    assert info["retimed_ms"][:2] == [pytest.approx(0.96), pytest.approx(0.95)]  # first-round order
    assert info["chosen_ms"] == pytest.approx(0.95)
    assert [list(order[1][0]), list(order[1][1])] == [info["theta_chunks"], info["mom_chunks"]]


def test_place_one_escalates_until_a_faster_group_shows(fake_chunks):
    """placement.place_one on the host with fake chunks: chunks 0-17 write at
    0.31 ms, 18+ at 0.29 (the group opposite the draw's reads).  The first
    pool (ONE_POOL = 16 chunks) is all slow; one round of 4 reaches chunks
    18-19; the composite is built from them."""
    def time_launch(f):
        ch = fake_chunks[f.roles["out"].data_ptr()]
        return sum(0.29 if c >= 18 else 0.31 for c in ch) / len(ch)

    n = 1 << 20
    buf, info = P.place_one(n, "cuda:0", lambda b, off: _FakeLaunch({"out": b}), time_launch,
                            budget_bytes=1 << 34)
    assert buf is not None and buf.numel() == n
    assert info["chunks_allocated"] == 20 == len(info["chunk_ms"])
    assert info["chosen_ms"] == pytest.approx(0.29) and all(c >= 18 for c in info["chunks"])


def test_place_one_escalates_until_the_plain_allocation_is_beaten(fake_chunks):
    """Two groups inside the first pool (0.31 / 0.30 ms per chunk) but neither
    promising against a plain allocation at 0.585 ms full size: the pool grows
    until chunks at 0.28 appear (from chunk 24)."""
    def time_launch(f):
        ch = fake_chunks[f.roles["out"].data_ptr()]
        return sum(0.28 if c >= 24 else (0.30 if c % 2 else 0.31) for c in ch) / len(ch)

    buf, info = P.place_one(1 << 20, "cuda:0", lambda b, off: _FakeLaunch({"out": b}), time_launch,
                            budget_bytes=1 << 34, beat_ms=0.585)
    assert info["chunks_allocated"] == 28
    assert info["chosen_ms"] == pytest.approx(0.28) and buf is not None


def test_with_grad_takes_the_best_free_chunks():
    """placement.with_grad: the gradient gets the best-ranked chunks theta / mom
    leave free; the other roles are re-filled in allocation order."""
    a = {"theta": [0, 1], "grad": [2, 3], "mom": [4, 5], "prior": [6, 7]}
    out = P.with_grad(a, [4, 9, 1, 8, 2], ["theta", "grad", "mom", "prior"], 2, 10)
    assert out == {"theta": [0, 1], "grad": [9, 8], "mom": [4, 5], "prior": [2, 3]}


def test_place_times_the_gradient_after_the_pair(fake_chunks):
    """A placed gradient ("grad" among the roles) is left out of the pair
    timings and then timed on every other chunk against the fastest pair; the
    candidates put it on the fastest chunks."""
    seen_grad = []

    def time_launch(f):
        th, mo = fake_chunks[f.roles["theta"].data_ptr()], fake_chunks[f.roles["mom"].data_ptr()]
        g = f.roles.get("grad")
        gc = fake_chunks[g.data_ptr()] if g is not None else None
        seen_grad.append(gc is not None)
        t = sum(0.96 if a // 4 != b // 4 else 1.05 for a, b in zip(th, mo)) / len(th)
        if gc is not None:                                # chunks 6, 7 the best gradient home
            t -= 0.01 * sum(c in (6, 7) for c in gc) / len(gc)
        return t

    n = 1 << 20
    vecs, info = P.place(n, "cuda:0", ["theta", "grad", "mom"], lambda roles, m: _FakeLaunch(roles),
                         time_launch, budget_bytes=1 << 34, with_torch=False)
    p0 = 2 * 2 + 2 * 2                                    # the pair-timed share of the first pool
    assert not any(seen_grad[:p0 * (p0 - 1)])             # pair timings: no placed gradient
    assert info["pairs_timed"] == p0 * (p0 - 1) + info["chunks_allocated"] - (3 * 2 + 2 * 2)
    assert info["grad_timed"] == info["chunks_allocated"] - 2
    assert sorted(info["grad_chunks"]) == [6, 7]
    assert set(vecs) == {"theta", "grad", "mom"}


def test_fast_pairs_found_needs_per_disjoint_fast_pairs():
    """placement._fast_pairs_found: with one chunk of the other group in the
    pool every fast pair shares it — not enough for a two-chunk composite."""
    def times_for(groups):
        k = len(groups)
        return {(i, j): (0.48 if groups[i] != groups[j] else 0.52)
                for i in range(k) for j in range(k) if i != j}
    one_b = times_for([0, 0, 0, 0, 0, 0, 0, 1])
    assert P._fast_pairs_found(one_b, 1)
    assert not P._fast_pairs_found(one_b, 2)
    two_b = times_for([0, 0, 0, 0, 0, 0, 1, 1])
    assert P._fast_pairs_found(two_b, 2)
    assert not P._fast_pairs_found(times_for([0] * 8), 1)
    assert not P._fast_pairs_found({}, 1)


def test_place_escalates_when_the_pool_has_one_chunk_of_the_other_group(fake_chunks):
    """First pool: chunks 0-6 one group, chunk 7 the other — fast pairs exist
    but all share chunk 7; the search escalates instead of keeping a fast /
    slow composite."""
    def grp(c):
        return 1 if c == 7 or c >= 12 else 0

    def time_launch(f):
        th, mo = fake_chunks[f.roles["theta"].data_ptr()], fake_chunks[f.roles["mom"].data_ptr()]
        return sum(0.48 if grp(a) != grp(b) else 0.52 for a, b in zip(th, mo)) / len(th)

    _, info = P.place(1 << 20, "cuda:0", ["theta", "mom"], lambda roles, m: _FakeLaunch(roles),
                      time_launch, budget_bytes=1 << 34, with_torch=False)
    assert info["escalation_rounds"] >= 1
    assert info["chosen_ms"] == pytest.approx(0.48)


def test_ref_found_does_not_count_a_straggler_as_the_second_fast_chunk():
    """The box that showed it: one truly fast chunk (0.4819) and a slow-group
    straggler just under the midpoint (0.5023) must not stop the escalation at
    per = 2."""
    t = {1: 0.5188, 2: 0.5203, 3: 0.5131, 4: 0.5174, 5: 0.5188, 6: 0.508, 7: 0.5023,
         8: 0.5112, 9: 0.5044, 10: 0.5031, 11: 0.5072, 12: 0.5101, 13: 0.5178, 14: 0.5241,
         15: 0.5122, 16: 0.5156, 17: 0.4819}
    assert not P._ref_found(t, 2)
    assert P._ref_found({**t, 18: 0.4835}, 2)
