"""Product cyclical schedule (host scalar feed) vs the reference's tables."""
import json
import os

import numpy as np

from bayesdll_amd.cyclical import CyclicalSGMCMC
from golden_util import GOLDEN


def test_product_schedule_matches_reference_tables():
    d = np.load(os.path.join(GOLDEN, "schedule.npz"), allow_pickle=False)
    for (E, B, M, beta) in json.loads(str(d["configs"])):
        key = f"E{E}_B{B}_M{M}_beta{beta}"
        s = CyclicalSGMCMC(0.1, M, E, beta)
        got = [(s.calculate_lr(e, b, B), s.should_sample(e, b, B), s.last_in_cycle(e, b, B),
                s.get_cycle_number(e, b, B)) for e in range(E) for b in range(B)]
        np.testing.assert_array_equal([g[0] for g in got], d[key + "_lr"])
        np.testing.assert_array_equal([g[1] for g in got], d[key + "_sample"])
        np.testing.assert_array_equal([g[2] for g in got], d[key + "_last"])
        np.testing.assert_array_equal([g[3] for g in got], d[key + "_cycle"])


def test_quirk_q3_last_in_cycle_never_fires_when_k_mod_m_nonzero():
    s = CyclicalSGMCMC(0.1, 3, 7, 0.5)  # K = 70, M = 3
    B = 10
    assert not any(s.last_in_cycle(e, b, B) for e in range(7) for b in range(B))
    restarts = [e * B + b + 1 for e in range(7) for b in range(B)
                if e * B + b > 0 and s.calculate_lr(e, b, B) == 0.1]
    assert restarts == [24, 47, 70]
