"""Graph mode with the update captured (BDL_GRAPH=1 + BDL_OVERLAP=1): the
cSGHMC bucket launches are captured with forward and backward on a side
stream, and each step rewrites their kernel nodes' arguments
(bdl_graph_redirect) before the replay.  The chain must equal the eager,
sequential one bit for bit over every step kind (explore, sample, the cycle's
first collect and the Welford collect, each its own graph), a learning rate
that changes every step, and a ragged last batch (another input shape)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")


def _run(graph, overlap, monkeypatch, between=None):
    import bayesdll_amd._base as B
    import bayesdll_amd.csghmc as csghmc
    from fakenet import MLP, init_vector, synthetic_mnist
    monkeypatch.setattr(B, "OVERLAP_BUCKET_ELEMS", 1 << 18)  # several buckets on an MLP
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
    losses = []
    step = 0
    for ep in range(3):
        for k, (x, y) in enumerate(data):
            coll = None
            if ep >= 1 and k >= 1:
                st = model.flat
                if m1 is None:
                    m1 = torch.empty(st.n, device=DEV)
                    m2 = torch.empty(st.n, device=DEV)
                    coll = (1, m1, m2, 1.0)          # COLLECT_WELFORD_INIT
                else:
                    coll = (2, m1, m2, float(step))  # COLLECT_WELFORD
            lr = 1e-2 * (1.0 + 0.1 * step)
            if between is not None:
                between(step)
            loss, _ = model(x, y, net, None, crit, [lr, 2 * lr], 1.0, 0.5,
                            should_sample=k % 2 == 1, collect=coll)
            losses.append(float(loss))
            step += 1
    torch.cuda.synchronize()
    return model, m1, m2, losses


def test_graph_overlap_equals_eager_chain(monkeypatch):
    mg, m1g, m2g, lg = _run(True, True, monkeypatch)
    me, m1e, m2e, le = _run(False, False, monkeypatch)
    keys = [k for k in mg._graphs if "overlap" in k]
    assert not mg.overlap_graph_failed, mg.overlap_graph_error
    # explore, sample, first collect, collect; full and ragged batches
    assert len(keys) >= 5, keys
    assert all(len(mg._graphs[k]["nodes"]) >= 4 for k in keys)
    assert lg == le
    assert torch.equal(mg.flat.theta, me.flat.theta)
    assert torch.equal(mg.flat.mom, me.flat.mom)
    assert torch.equal(m1g, m1e) and torch.equal(m2g, m2e)
    mg.release_graphs()


def _same(a, b):
    ma, m1a, m2a, la = a
    mb, m1b, m2b, lb = b
    assert la == lb
    assert torch.equal(ma.flat.theta, mb.flat.theta)
    assert torch.equal(ma.flat.mom, mb.flat.mom)
    assert torch.equal(m1a, m1b) and torch.equal(m2a, m2b)


def test_failed_node_check_falls_back_once(monkeypatch):
    """A capture whose node check fails is dropped and the sampler stays on
    the eager overlap from then on: ONE capture attempt, not one per step."""
    import bayesdll_amd._base as B
    monkeypatch.setattr(B.FusedModelBase, "_check_overlap_nodes",
                        staticmethod(lambda *a: "forced mismatch"))
    got = _run(True, True, monkeypatch)
    mg = got[0]
    assert mg.overlap_graph_failed and mg.overlap_graph_error == "forced mismatch"
    assert mg.overlap_captures == 1
    assert not any("overlap" in k for k in mg._graphs)
    monkeypatch.undo()
    _same(got, _run(False, False, monkeypatch))
    mg.release_graphs()


def test_geometry_change_between_steps_keeps_the_graph(monkeypatch):
    """Another launch geometry installed between steps (e.g. by another
    sampler's state): every redirect re-installs the geometry its nodes were
    captured with, so no rewrite fails and the chain stays bit-identical."""
    from bayesdll_amd import kernels as K
    geoms = [(1, 4, 1), (2, 2, 1), (3, 1, 1)]
    got = _run(True, True, monkeypatch, between=lambda s: K.set_launch_config(*geoms[s % 3]))
    mg = got[0]
    assert not mg.overlap_graph_failed, mg.overlap_graph_error
    assert mg.overlap_captures == sum(1 for k in mg._graphs if "overlap" in k)
    _same(got, _run(False, False, monkeypatch))
    mg.release_graphs()


def test_graph_cap_reached_steps_run_eager_overlap(monkeypatch):
    """Past MAX_OVERLAP_GRAPHS the remaining step kinds run the eager overlap,
    bit-identical, without capturing more."""
    import bayesdll_amd._base as B
    monkeypatch.setattr(B, "MAX_OVERLAP_GRAPHS", 2)
    got = _run(True, True, monkeypatch)
    mg = got[0]
    assert sum(1 for k in mg._graphs if "overlap" in k) <= 2
    assert mg.overlap_captures <= 2 and not mg.overlap_graph_failed
    _same(got, _run(False, False, monkeypatch))
    mg.release_graphs()
