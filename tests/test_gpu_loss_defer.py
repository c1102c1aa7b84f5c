"""The Runners' device-side epoch loss (no per-step loss.item()) equals the
reference's per-step float64 sum bit for bit (BDL_SYNC_LOSS=1 restores it)."""
import logging
from types import SimpleNamespace

import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu


class MLP(nn.Module):
    readout_name = "fc2"

    def __init__(self):
        super().__init__()
        self.fc1 = nn.Linear(20, 16)
        self.fc2 = nn.Linear(16, 4)

    def forward(self, x):
        return self.fc2(torch.relu(self.fc1(x)))


@pytest.mark.parametrize("method", ["csghmc", "sgld", "csgld"])
def test_deferred_epoch_loss_equals_per_step_sum(method, monkeypatch, tmp_path):
    import importlib

    from bayesdll_amd.run import DEFAULT_HPARAMS, SyntheticLoader, parse_hparams
    dev = torch.device("cuda", 0)
    loader = SyntheticLoader(640, (20,), 4, 64, dev, 3)
    out = {}
    for sync in ("1", "0"):
        monkeypatch.setenv("BDL_SYNC_LOSS", sync)
        torch.manual_seed(0)
        hp, _ = parse_hparams(DEFAULT_HPARAMS[method])
        args = SimpleNamespace(
            lr=1e-2, lr_head=1e-2, epochs=4, num_cycles=2, proportion_exploration=0.5, ND=640,
            device=dev, seed=0, hparams=hp, pretrained=None, log_dir=str(tmp_path),
            num_classes=4, ece_num_bins=15, momentum=0.5, clip_grad=None, test_eval_freq=100)
        R = importlib.import_module(f"bayesdll_amd.{method}").Runner(
            MLP().to(dev), None, args, logging.getLogger("t"))
        res = [R.train_one_epoch(loader) if method != "sgld" else
               R.train_one_epoch(loader, False, 0) for _ in range(2)]
        out[sync] = [(float(r[0]), float(r[1])) for r in res]
        assert not R.model.defer_loss  # reset after the epoch: direct calls get floats
        assert all(type(r[0]) is float for r in res)
    assert out["1"] == out["0"]
