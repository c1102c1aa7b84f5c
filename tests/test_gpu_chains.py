"""Multi-chain ensemble through the product Runners (config 5's logic at mlp
size): two processes, one chain each, sharing the box's one GPU over gloo (the
same bayesdll_amd.chains calls RCCL makes at one GPU per rank).

Checks, for cSGHMC and SGLD:
  * each rank's chain is exactly the chain a single process computes with the
    same chain id (Philox key = (seed, chain, step)): no cross-chain coupling
    during sampling, bit for bit;
  * the chains differ (chain id separates the noise streams);
  * Runner.evaluate's predictive is the cross-chain posterior-predictive
    average log((1/K) sum_k softmax(s_k)) of the chains' own predictive scores, and
    every rank holds the same one; per-chain logits_all stay per chain.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
pytestmark = pytest.mark.gpu
WORLD = 2


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _run_ranks(method, tmp_path, extra=(), singles=False):
    """WORLD ranks of one ensemble, or (singles=True) WORLD single-chain
    processes with chain ids 0..WORLD-1 and no torch.distributed — fresh
    processes either way, so both sides start from the same library state."""
    port = _free_port()
    procs, outs = [], []
    base = {k: v for k, v in os.environ.items()
            if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    for r in range(WORLD):
        tag = "single" if singles else "rank"
        out = str(tmp_path / f"{method}_{tag}{r}.npz")
        env = base if singles else dict(base, RANK=str(r), LOCAL_RANK="0", WORLD_SIZE=str(WORLD),
                                        MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        args = ["--chain", str(r)] if singles else list(extra)
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "chain_worker.py"),
                                       "--method", method, "--out", out, *args], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
        outs.append(out)
    logs = []
    try:
        for p in procs:
            logs.append(p.communicate(timeout=180)[0].decode(errors="replace"))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    for p, log in zip(procs, logs):
        assert p.returncode == 0, log[-3000:]
    return [dict(np.load(o)) for o in outs]


@pytest.mark.parametrize("method", ["csghmc", "sgld"])
def test_two_chain_ensemble_matches_single_chains(method, tmp_path):
    ranks = _run_ranks(method, tmp_path)
    singles = _run_ranks(method, tmp_path, singles=True)
    for r in range(WORLD):
        assert int(ranks[r]["chain"]) == r
        # each chain writes its checkpoints / logits under <log_dir>/chain<rank>
        assert str(ranks[r]["log_dir"]).endswith(f"chain{r}")
        assert not str(singles[r]["log_dir"]).endswith(f"chain{r}")
        # the chain a rank samples is the single-process chain with its id, bit for bit
        np.testing.assert_array_equal(ranks[r]["theta"], singles[r]["theta"])
        np.testing.assert_array_equal(ranks[r]["logits_all"], singles[r]["logits_all"])
        np.testing.assert_array_equal(ranks[r]["targets"], singles[0]["targets"])
    assert not np.array_equal(singles[0]["theta"], singles[1]["theta"])
    # ensemble predictive = log-mean-exp over the chains' own (normalised) predictives
    lp = np.stack([s["logits"].astype(np.float64) for s in singles])
    lp = lp - np.log(np.exp(lp).sum(axis=2, keepdims=True))  # log_softmax per chain
    want = np.log(np.mean(np.exp(lp), axis=0))
    for r in range(WORLD):
        np.testing.assert_allclose(ranks[r]["logits"], want, rtol=0, atol=2e-6)
    np.testing.assert_array_equal(ranks[0]["logits"], ranks[1]["logits"])
    assert ranks[0]["loss"] == ranks[1]["loss"] and ranks[0]["err"] == ranks[1]["err"]


def test_sharded_likelihood_pass_and_gmm_weights_over_chains(tmp_path):
    """SURVEY §8(f) row 3 through the product Runner: two ranks run the same
    cSGHMC chain (replicas); the cycle-end full_batch_likelihoods sharded
    over them (each scores half the training batches, one all-reduce of the
    loss sums) equals the single-process pass (rtol 1e-6); ranks whose
    moments differ are refused; evaluate() with GMM weights over chains gives
    the single chain's predictive when the chains are identical."""
    ranks = _run_ranks("csghmc", tmp_path, extra=("--replica",))
    single = _run_ranks("csghmc", tmp_path, singles=True)[0]
    for r in range(WORLD):
        np.testing.assert_array_equal(ranks[r]["theta"], single["theta"])
        np.testing.assert_array_equal(ranks[r]["lik_local"], single["lik_local"])
        assert len(ranks[r]["lik_shard"]) == 3  # nst draws
        np.testing.assert_allclose(ranks[r]["lik_shard"], single["lik_local"], rtol=1e-6)
        assert bool(ranks[r]["mismatch_refused"])
        # identical chains: the jointly weighted ensemble is the chain's own mixture
        np.testing.assert_allclose(ranks[r]["logits_gmm_over_chains"],
                                   torch.log_softmax(torch.from_numpy(single["logits"]), 1).numpy(),
                                   rtol=1e-5, atol=1e-5)
