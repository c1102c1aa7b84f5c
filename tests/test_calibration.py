"""bayesdll_amd.calibration vs the reference's calibration.py, pinned by
tests/golden/calibration.npz (gen_golden.py GOLDEN_ONLY=calib: the
reference's own analyze / find_optimal_temperature on seeded logits)."""
import os

import numpy as np

from golden_util import GOLDEN


def test_calibration_matches_reference(tmp_path):
    from bayesdll_amd import calibration as C
    d = np.load(os.path.join(GOLDEN, "calibration.npz"), allow_pickle=False)
    for name in ("c10", "c37"):
        logits, labels = d[f"{name}_logits"], d[f"{name}_labels"]
        for t in (1.0, 1.7):
            got = C.analyze(labels, logits, 15, plot_save_path=str(tmp_path / "r.png"),
                            temperature=t)
            np.testing.assert_allclose(got, d[f"{name}_analyze_T{t}"], rtol=1e-12, atol=0)
        topt, ok = C.find_optimal_temperature(d[f"{name}_vlabels"], d[f"{name}_vlogits"],
                                              plot_save_path=str(tmp_path / "t.png"))
        assert ok == bool(d[f"{name}_topt_ok"])
        np.testing.assert_allclose(topt, d[f"{name}_topt"], rtol=1e-9)
    assert (tmp_path / "r.png").exists() and (tmp_path / "t.png").exists()


def test_log_calibration_lines(tmp_path):
    import logging
    from types import SimpleNamespace
    from bayesdll_amd.calibration import log_calibration
    d = np.load(os.path.join(GOLDEN, "calibration.npz"), allow_pickle=False)
    args = SimpleNamespace(ece_num_bins=15, log_dir=str(tmp_path))
    msgs = []

    class H(logging.Handler):
        def emit(self, rec):
            msgs.append(rec.getMessage())
    log = logging.getLogger("calib-test")
    log.setLevel(logging.INFO)
    log.addHandler(H())
    out = log_calibration(args, log, d["c10_labels"], d["c10_logits"], d["c10_vlabels"],
                          d["c10_vlogits"])
    assert msgs[0].startswith("[Calibration - Default T=1] ECE = ")
    assert msgs[1].startswith("[Calibration - Temp-scaled Topt=3.3391]")
    assert {"reliability_T1.png", "reliability_Topt.png", "temp_scale_optim_curve.png"} <= \
        set(os.listdir(tmp_path))
    np.testing.assert_allclose(out["T1"], d["c10_analyze_T1.0"], rtol=1e-12)
