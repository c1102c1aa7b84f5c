"""Gradient arena (include/bdl_arena.h, bayesdll_amd/arena.py): the backward
pass of a Runner step allocates from one device reservation, so the
per-tensor gradients the fused update reads (methods/csghmc.py:741-778 reads
each p.grad) are sub-ranges of ONE allocation.  The arena changes where the
gradients sit, never a value: chains with and without it are bit-identical
(eager, eager overlap, graph mode).  Opt-in (BDL_GRAD_ARENA=1): measured
not to close the per-tensor gradient gap."""
import ctypes as C

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")


def _run(monkeypatch, arena, graph=False, overlap=False, epochs=2):
    import bayesdll_amd._base as B
    import bayesdll_amd.csghmc as csghmc
    from fakenet import MLP, init_vector, synthetic_mnist
    monkeypatch.setenv("BDL_GRAD_ARENA", "1" if arena else "0")
    monkeypatch.setattr(B, "OVERLAP_BUCKET_ELEMS", 1 << 18)
    n = 2797010
    init = torch.tensor(init_vector(91, n, 0.03))
    data = synthetic_mnist(93, 232, 64, device=DEV)  # 64, 64, 64, 40
    crit = torch.nn.CrossEntropyLoss()
    torch.manual_seed(0)
    net = MLP()
    with torch.no_grad():
        torch.nn.utils.vector_to_parameters(init, net.parameters())
    net = net.to(DEV)
    model = csghmc.Model(30000.0, prior_sig=1.0, momentum_decay=0.18)
    model.noise_mode, model.seed = "philox", 3
    model.graph, model.overlap = graph, overlap
    m1 = m2 = None
    losses, seen = [], []
    step = 0
    for ep in range(epochs):
        for k, (x, y) in enumerate(data):
            coll = None
            if ep >= 1 and k >= 1:
                st = model.flat
                if m1 is None:
                    m1 = torch.empty(st.n, device=DEV)
                    m2 = torch.empty(st.n, device=DEV)
                    coll = (1, m1, m2, 1.0)
                else:
                    coll = (2, m1, m2, float(step))
            lr = 1e-2 * (1.0 + 0.1 * step)
            loss, _ = model(x, y, net, None, crit, [lr, 2 * lr], 1.0, 0.5,
                            should_sample=k % 2 == 1, collect=coll)
            losses.append(float(loss))
            seen.append([None if p.grad is None else p.grad for p in model.flat.params])
            step += 1
    torch.cuda.synchronize()
    model._test_net, model._test_batch = net, data[0]
    return model, m1, m2, losses, seen


def test_backward_gradients_come_from_the_arena(monkeypatch):
    from bayesdll_amd import arena as A
    model, _, _, _, seen = _run(monkeypatch, arena=True, epochs=1)
    st = model.flat
    assert st.grad_mode == "tensor" and st.arena is not None
    # the autograd engine's device thread allocated them inside the routing
    for grads in seen[-2:]:
        for g in grads:
            assert g is not None and A.contains(st.device, g), "gradient outside the arena"
    # steady state: the same batch shape gets the same gradient blocks back
    del seen
    x, y = model._test_batch
    ptrs, s0 = [], None
    for i in range(4):
        model(x, y, model._test_net, None, torch.nn.CrossEntropyLoss(),
              [1e-3, 1e-3], 1.0, 0.5, should_sample=False)
        ptrs.append([p.grad.data_ptr() for p in st.params])
        if i == 1:
            torch.cuda.synchronize()
            s0 = A.stats(st.device)
    torch.cuda.synchronize()
    s1 = A.stats(st.device)
    assert ptrs[2] == ptrs[3]
    assert s1["carvings"] == s0["carvings"], (s0, s1)  # served from the pool's cache
    assert s1["live"] >= 1 and s1["reserved"] >= 4 * st.n


@pytest.mark.parametrize("mode", ["eager", "overlap", "graph"])
def test_arena_chain_equals_default_pool_chain(monkeypatch, mode):
    kw = dict(graph=mode == "graph", overlap=mode == "overlap")
    ma, m1a, m2a, la, _ = _run(monkeypatch, arena=True, **kw)
    md, m1d, m2d, ld, _ = _run(monkeypatch, arena=False, **kw)
    assert ma.flat.arena is not None and md.flat.arena is None
    assert la == ld
    assert torch.equal(ma.flat.theta, md.flat.theta)
    assert torch.equal(ma.flat.mom, md.flat.mom)
    assert torch.equal(m1a, m1d) and torch.equal(m2a, m2d)
    ma.release_graphs()
    md.release_graphs()


def test_arena_regions_grow_reset_and_release():
    """The bump allocator through the C-ABI: carve, grow into a new region
    when the current one is full, reset the current region when it empties,
    release a retired one when its last carving is freed."""
    from bayesdll_amd import _lib as L
    from bayesdll_amd import arena as A
    h = L.lib()
    dev = torch.device("cuda", torch.cuda.current_device())
    idx = dev.index
    mib = 1 << 20
    L.check(h.bdl_arena_reserve(idx, 5 * mib), "reserve")  # rounded to 6 MiB
    s0 = A.stats(dev)
    assert s0["size"] == 6 * mib
    a = h.bdl_arena_alloc(2 * mib, idx, None)   # top-down
    b = h.bdl_arena_alloc(3 * mib, idx, None)   # carved as 4 MiB: the region is full
    assert a == s0["base"] + 4 * mib and b == s0["base"]
    assert h.bdl_arena_contains(idx, C.c_void_p(b), 3 * mib) == 1
    c = h.bdl_arena_alloc(mib, idx, None)        # does not fit: a new region
    s1 = A.stats(dev)
    assert s1["grown"] == s0["grown"] + 1 and s1["size"] == 6 * mib
    assert c == s1["base"] + 4 * mib   # max(2 x 2 MiB, 6 MiB) region, its top 2 MiB
    h.bdl_arena_free(C.c_void_p(c), mib, idx, None)   # current region empties: reset
    assert h.bdl_arena_alloc(mib, idx, None) == c
    h.bdl_arena_free(C.c_void_p(c), mib, idx, None)
    h.bdl_arena_free(C.c_void_p(a), 2 * mib, idx, None)
    assert h.bdl_arena_contains(idx, C.c_void_p(a), 1) == 1  # b still lives in it
    h.bdl_arena_free(C.c_void_p(b), 3 * mib, idx, None)      # retired and empty: released
    assert h.bdl_arena_contains(idx, C.c_void_p(a), 1) == 0
    s2 = A.stats(dev)
    assert s2["regions"] == s0["regions"]
