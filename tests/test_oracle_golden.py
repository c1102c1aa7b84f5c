"""The oracle (CPU restatement) must reproduce the reference BIT-EXACTLY.

Golden fixtures were produced by running the reference's own Runner/Model code
(tests/golden/gen_golden.py); here the oracle replays the same prescribed
gradients and captured noise and must land on identical bits.
"""
import numpy as np
import pytest

from golden_util import FIXTURES, grad_fn, load, noise_fn
from oracle import sgmcmc_oracle as O


@pytest.mark.parametrize("name", FIXTURES)
def test_oracle_matches_reference_bitexact(name):
    fx = load(name)
    out = O.simulate(fx["config"], fx["segments"], fx["readout"], fx["theta_init"],
                     fx["prior_mean"], grad_fn(fx), noise_fn(fx))
    np.testing.assert_array_equal(out["lrs"], fx["lrs"])
    np.testing.assert_array_equal(out["theta"], fx["theta"])
    np.testing.assert_array_equal(out["mom"], fx["mom"])
    for key in ("adam_m", "adam_v", "sgd_buf"):
        if key in fx and key in out:
            np.testing.assert_array_equal(out[key], fx[key], err_msg=key)
    if fx["config"]["method"].startswith("adam_"):
        assert "adam_m" in out and "adam_v" in out
    if fx["config"]["method"] in ("csghmc", "csghmc_fs"):
        np.testing.assert_array_equal(out["should_sample"], fx["should_sample"])
    if "cycles" in fx:
        np.testing.assert_array_equal(out["cycles"], fx["cycles"])
        np.testing.assert_array_equal(out["cycle_mom1"], fx["cycle_mom1"])
        np.testing.assert_array_equal(out["cycle_mom2"], fx["cycle_mom2"])
        np.testing.assert_array_equal(out["samples_per_cycle"], fx["samples_per_cycle"])
        assert out["samples_collected"] == int(fx["samples_collected"])
        assert out["current_cycle"] == int(fx["current_cycle"])
    else:
        np.testing.assert_array_equal(out["post_mom1"], fx["post_mom1"])
        np.testing.assert_array_equal(out["post_mom2"], fx["post_mom2"])
        assert out["post_cnt"] == int(fx["post_cnt"])


def test_schedule_tables_match_reference():
    import json
    import os
    from golden_util import GOLDEN
    d = np.load(os.path.join(GOLDEN, "schedule.npz"), allow_pickle=False)
    for (E, B, M, beta) in json.loads(str(d["configs"])):
        key = f"E{E}_B{B}_M{M}_beta{beta}"
        s = O.CyclicalSchedule(0.1, M, E, beta)
        lr, ss, last, cyc = [], [], [], []
        for ep in range(E):
            for b in range(B):
                lr.append(s.calculate_lr(ep, b, B))
                ss.append(s.should_sample(ep, b, B))
                last.append(s.last_in_cycle(ep, b, B))
                cyc.append(s.get_cycle_number(ep, b, B))
        np.testing.assert_array_equal(np.array(lr), d[key + "_lr"])
        np.testing.assert_array_equal(np.array(ss), d[key + "_sample"])
        np.testing.assert_array_equal(np.array(last), d[key + "_last"])
        np.testing.assert_array_equal(np.array(cyc), d[key + "_cycle"])
