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


def test_moment_pair_halves_of_one_allocation(monkeypatch):
    """flat.moment_pair: for vectors of >= PLACEMENT_MIN_ELEMS, m1 / m2 are the
    two halves of one allocation (disjoint, m2 on a 256-B boundary, both
    contiguous, n elements each) whatever BDL_PLACEMENT says (a layout, not a
    search); smaller vectors get two plain allocations."""
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
    assert a.untyped_storage().data_ptr() == b.untyped_storage().data_ptr()


def test_placement_is_opt_in(monkeypatch):
    """torch's allocator unless BDL_PLACEMENT asks for the chunk search."""
    from bayesdll_amd import placement as P
    monkeypatch.delenv("BDL_PLACEMENT", raising=False)
    assert P.mode() == "0"
    monkeypatch.setenv("BDL_PLACEMENT", "search")
    assert P.mode() == "search"


def test_split_groups_needs_two_groups_and_enough_of_each():
    """placement.split_groups: chunks slow against chunk 0 share its group, the
    rest are the fast group; no split without a spread or without per - 1
    slow and per fast chunks."""
    t = {1: 1.05, 2: 0.96, 3: 1.06, 4: 0.95, 5: 0.97, 6: 1.04, 7: 0.955}
    slow, fast = P.split_groups(t, 2)
    assert slow == [3, 1, 6] and fast == [4, 7, 2, 5]
    assert P.split_groups({1: 1.0, 2: 0.995, 3: 1.001}, 2) is None      # one group
    assert P.split_groups({1: 0.95, 2: 0.96, 3: 1.05}, 3) is None       # one slow < per - 1
    assert P.split_groups({1: 1.05, 2: 1.06, 3: 0.95}, 2) is None       # one fast < per
    assert P.split_groups({}, 1) is None


@pytest.mark.parametrize("names", [["theta", "mom"], ["theta", "mom", "prior"],
                                   ["theta", "mom", "prior", "adam_m", "adam_v", "sgd_buf"]])
@pytest.mark.parametrize("per", [1, 2, 3])
def test_assignments_pair_chunk0s_group_with_the_fast_group(names, per):
    nchunks = len(names) * per + 2 * per
    rng = random.Random(7 * per + len(names))
    # chunks 0..per (chunk 0's group) slow against 0, the rest fast, with noise
    t0 = {j: (1.05 if j <= per else 0.96) + 0.005 * rng.random() for j in range(1, nchunks)}
    cands = P.assignments(t0, nchunks, names, per)
    assert cands[0] == {nm: list(range(q * per, (q + 1) * per)) for q, nm in enumerate(names)}
    assert 2 <= len(cands) <= P.COMPOSITES + 1
    group0 = set(range(per + 1))
    for c in cands:
        ids = [k for nm in names for k in c[nm]]
        assert list(c) == names and all(len(c[nm]) == per for nm in names)
        assert len(ids) == len(set(ids)) and all(0 <= k < nchunks for k in ids)
    for c in cands[1:]:
        th, mo = set(c["theta"]), set(c["mom"])
        # one of theta / mom is chunk 0's group, the other entirely the fast group
        assert (th <= group0 and not mo & group0) or (mo <= group0 and not th & group0)
    # the first: theta = chunk 0 and its group, mom = the fastest chunks
    fastest = sorted((j for j in t0 if j > per), key=t0.get)[:per]
    assert cands[1]["theta"][0] == 0 and cands[1]["mom"] == fastest
    # no split: allocation order only
    assert P.assignments({j: 1.0 for j in range(1, nchunks)}, nchunks, names, per) == cands[:1]


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


def _grouped(fake_chunks, first_fast):
    """Timing model: chunks below `first_fast` form one physical group, the rest
    another; theta / mom in different groups 0.96 ms, same group 1.05."""
    def time_launch(f):
        th, mo = fake_chunks[f.roles["theta"].data_ptr()], fake_chunks[f.roles["mom"].data_ptr()]
        return sum(0.96 if (a >= first_fast) != (b >= first_fast) else 1.05
                   for a, b in zip(th, mo)) / len(th)
    return time_launch


def test_place_grows_the_pool_until_another_group_shows(fake_chunks):
    """placement.place on the host with fake chunks: chunks 0-9 one group,
    10+ another.  The first pool (roles x per + 2 x per = 8 chunks) is one
    group; the pool grows 4 chunks at a time (each new chunk timed against
    chunk 0) until 10, 11 show; the kept set pairs the two groups."""
    n = 1 << 20                                          # 4 MB: two 2-MiB chunks per vector
    vecs, info = P.place(n, "cuda:0", ["theta", "mom"], lambda roles, m: _FakeLaunch(roles),
                         _grouped(fake_chunks, 10), budget_bytes=1 << 34, with_torch=False)
    assert info["chunks_per_vector"] == 2
    assert info["chunks_allocated"] == 12 and info["pairs_timed"] == 11 == len(info["ref_ms"])
    assert info["groups"]["fast"] == [10, 11]
    assert info["chosen_ms"] == pytest.approx(0.96) and info["kept"] == "search"
    th, mo = info["theta_chunks"], info["mom_chunks"]
    assert {c >= 10 for c in th} != {c >= 10 for c in mo} and len({c >= 10 for c in th}) == 1
    assert set(vecs) == {"theta", "mom"} and all(v.numel() == n for v in vecs.values())
    assert info["transient_gb"] == pytest.approx(12 * 2 / 1024, abs=0.01)


def test_place_stops_at_max_chunks(fake_chunks):
    """One physical group throughout: the pool stops at MAX_CHUNKS and the
    allocation order is kept."""
    _, info = P.place(1 << 20, "cuda:0", ["theta", "mom"], lambda roles, m: _FakeLaunch(roles),
                      _grouped(fake_chunks, 1000), budget_bytes=1 << 34, with_torch=False)
    assert info["chunks_allocated"] == P.MAX_CHUNKS and info["groups"] is None
    assert info["kept"] == "default" and info["composites_ms"] == [pytest.approx(1.05)]


def test_place_stops_at_its_time_budget(fake_chunks, monkeypatch):
    """Past SEARCH_SECONDS no more chunks are added and at most the allocation
    order and one group pairing are timed at full size."""
    monkeypatch.setattr(P, "SEARCH_SECONDS", 0.0)
    _, info = P.place(1 << 20, "cuda:0", ["theta", "mom"], lambda roles, m: _FakeLaunch(roles),
                      _grouped(fake_chunks, 6), budget_bytes=1 << 34, with_torch=False)
    assert info["chunks_allocated"] == 8 and len(info["composites_ms"]) <= 2
    assert info["chosen_ms"] == pytest.approx(0.96)


def test_place_refuses_a_budget_below_the_roles():
    with pytest.raises(RuntimeError, match="exceed the budget"):
        P.place(1 << 20, "cuda:0", ["theta", "mom"], None, None, budget_bytes=3 * (2 << 20))
