"""Calibration metrics the reference Runners log after each new best
evaluation (calibration.py: calc_bins :24-67, analyze :215-259,
find_optimal_temperature :123-212): confidence-binned ECE / MCE over all
(example, class) probabilities, NLL, and a scalar temperature fitted on the
validation logits.  Host-side numpy/scipy on the predictions the fused sampler
produced; the reliability plots are written when matplotlib is importable.
"""
from __future__ import annotations

import numpy as np
import scipy.optimize
import scipy.special


def _softmax_flat(logits, temperature):
    return scipy.special.softmax(logits / temperature, axis=1).ravel()


def calc_bins(labels, logits, num_bins, temperature=1):
    """Bin every p(y=j|x_i) by confidence (right edges linspace(0, 1+1e-8)[1:],
    np.digitize), per bin: mean accuracy of the one-hot targets, mean
    confidence, size (calibration.py:24-67)."""
    labels = np.asarray(labels)
    k = logits.shape[1]
    onehot = np.eye(k)[labels].ravel()
    probs = _softmax_flat(logits, temperature)
    edges = np.linspace(0, 1 + 1e-8, num_bins + 1)[1:]
    member = np.digitize(probs, edges)
    accs, confs, sizes = np.zeros(num_bins), np.zeros(num_bins), np.zeros(num_bins)
    for b in range(num_bins):
        sel = member == b
        sizes[b] = sel.sum()
        if sizes[b] > 0:
            accs[b] = onehot[sel].sum() / sizes[b]
            confs[b] = probs[sel].sum() / sizes[b]
    return edges, member, accs, confs, sizes


def nll(labels, logits, temperature=1):
    """Mean negative log-likelihood of the temperature-scaled logits."""
    z = logits / temperature
    return float(np.mean(scipy.special.logsumexp(z, axis=1) - z[np.arange(len(labels)), labels]))


def _plot(edges, accs, path, title, ece, mce, nll_):
    try:
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.patches as mpatches
        import matplotlib.pyplot as plt
    except ImportError:
        return
    centers = (np.insert(edges, 0, 0)[:-1] + edges) / 2
    w = centers[1] - centers[0]
    fig = plt.figure(figsize=(8, 8))
    ax = fig.gca()
    ax.set_xlim(0, 1 + 1e-8)
    ax.set_ylim(0, 1)
    ax.set_xlabel("Confidence")
    ax.set_ylabel("Accuracy")
    ax.set_axisbelow(True)
    ax.grid(color="gray", linestyle="dashed")
    p1 = ax.bar(centers, centers, width=w, alpha=0.3, edgecolor="black", color="r", hatch="\\")
    p2 = ax.bar(centers, accs, width=w, alpha=0.3, edgecolor="black", color="b")
    p3 = ax.plot([0, 1], [0, 1], "--", color="gray", linewidth=2)
    ax.set_aspect("equal", adjustable="box")
    first = ax.legend([p1, p2, p3[0]], ["Ideal", "Model", "Y=X"], loc="upper left")
    ax.legend(handles=[mpatches.Patch(color="green", label=f"ECE = {ece * 100:.2f}%"),
                       mpatches.Patch(color="red", label=f"MCE = {mce * 100:.2f}%"),
                       mpatches.Patch(color="blue", label=f"NLL = {nll_:.4f}")],
              loc="lower right")
    ax.add_artist(first)
    if title is not None:
        ax.set_title(title)
    fig.savefig(path, bbox_inches="tight")
    plt.close(fig)


def analyze(labels, logits, num_bins, plot_save_path=None, temperature=1):
    """(ECE, MCE, NLL) at `temperature` (calibration.py:215-259): ECE = sum over
    bins of |acc - conf| weighted by bin size, MCE = max |acc - conf|."""
    edges, _, accs, confs, sizes = calc_bins(labels, logits, num_bins, temperature)
    gap = np.abs(accs - confs)
    ece = float((gap * (sizes / sizes.sum())).sum())
    mce = float(gap.max())
    n = nll(labels, logits, temperature)
    if plot_save_path is not None:
        _plot(edges, accs, plot_save_path, f"Temperature = {temperature}", ece, mce, n)
    return ece, mce, n


def find_optimal_temperature(labels, logits, plot_save_path=None, max_iter=10000):
    """Temperature minimising the validation NLL, scipy.optimize.minimize from
    T = 1 with its default method (calibration.py:123-212, the numpy branch).
    Returns (Topt as a 1-element array, success)."""
    labels = np.asarray(labels)
    trace_t, trace_l = [], []

    def f(t):
        return nll(labels, logits, t)

    def cb(x):
        trace_t.append(np.array(x))
        trace_l.append(f(x))

    res = scipy.optimize.minimize(f, np.ones(1), options={"maxiter": max_iter}, callback=cb)
    if plot_save_path is not None:
        try:
            import matplotlib
            matplotlib.use("Agg")
            import matplotlib.pyplot as plt
            fig, (a1, a2) = plt.subplots(1, 2)
            a1.plot(range(len(trace_t)), [float(np.ravel(t)[0]) for t in trace_t])
            a1.set_title("Temperature T")
            a1.set_xlabel("Iterations")
            a2.plot(range(len(trace_l)), trace_l)
            a2.set_title("NLL on validation set")
            a2.set_xlabel("Iterations")
            fig.savefig(plot_save_path)
            plt.close(fig)
        except ImportError:
            pass
    return res.x, bool(res.success)


def log_calibration(args, logger, targets_test, logits_test, targets_val=None, logits_val=None):
    """The reference Runners' block after a new best evaluation
    (methods/csghmc.py:170-196, methods/sgld.py:160-186): ECE / MCE / NLL at
    T = 1, then, with a validation set, at the temperature fitted on it; the
    same log lines and plot file names."""
    import os
    ece, mce, n = analyze(targets_test, logits_test, num_bins=args.ece_num_bins,
                          plot_save_path=os.path.join(args.log_dir, "reliability_T1.png"),
                          temperature=1)
    logger.info(f"[Calibration - Default T=1] ECE = {ece:.4f}, MCE = {mce:.4f}, NLL = {n:.4f}")
    out = {"T1": (ece, mce, n)}
    if logits_val is not None:
        topt, ok = find_optimal_temperature(
            targets_val, logits_val,
            plot_save_path=os.path.join(args.log_dir, "temp_scale_optim_curve.png"))
        if ok:
            ece, mce, n = analyze(targets_test, logits_test, num_bins=args.ece_num_bins,
                                  plot_save_path=os.path.join(args.log_dir, "reliability_Topt.png"),
                                  temperature=topt)
            logger.info(f"[Calibration - Temp-scaled Topt={topt[0]:.4f}] ECE = {ece:.4f}, "
                        f"MCE = {mce:.4f}, NLL = {n:.4f}")
            out["Topt"] = (float(topt[0]), ece, mce, n)
        else:
            logger.info("!! Temperature scaling optimization failed !!")
    return out
