"""bayesdll — the reference's import surface over the MI355X-native samplers.

The reference installs a package `bayesdll` (setup.py:3-11, package_dir
src/bayesdll) that callers import as `from bayesdll.sgld import Runner`
(src/bayesdll/sgld.py), and its demos import the SG-MCMC Runners as
`from methods.<name> import Runner` (demo_mnist.py:190-230,
demo_vision.py:188-239).  Every SG-MCMC module of that surface answers here
under `bayesdll.<name>` and IS the corresponding `bayesdll_amd.<name>` module
(same object: attributes, monkeypatching and isinstance checks carry over):

    bayesdll.sgld         methods/sgld.py, src/bayesdll/sgld.py
    bayesdll.csghmc       methods/csghmc.py
    bayesdll.sghmc        methods/sghmc.py
    bayesdll.csgld        methods/csgld.py
    bayesdll.csghmc_fs    methods/csghmc_fs.py
    bayesdll.adam_sghmc   methods/adam_sghmc.py
    bayesdll.adam_csghmc  methods/adam_csghmc.py
    bayesdll.cyclical     methods/cyclical.py
    bayesdll.calibration  src/bayesdll/calibration.py (calibration.py)

The non-SG-MCMC modules of src/bayesdll (vanilla, vi, mc_dropout, la) are out
of scope and are not provided.
"""
__all__ = ["sgld", "csghmc", "sghmc", "csgld", "csghmc_fs", "adam_sghmc", "adam_csghmc",
           "cyclical", "calibration"]

# the reference's `methods.<name>` modules that are SG-MCMC samplers (and the
# schedule they import, methods/csghmc.py:12)
METHODS = ("sgld", "csgld", "csghmc", "sghmc", "adam_sghmc", "adam_csghmc", "csghmc_fs",
           "cyclical")


def alias_methods():
    """Make the reference's own import lines (`from methods.csghmc import
    Runner`, demo_mnist.py:190-230, demo_vision.py:188-239,
    pretrain_resnet101.py:24-31) resolve to these samplers, so its scripts run
    unchanged: registers `methods` and `methods.<name>` in sys.modules.
    Returns the `methods` module."""
    import importlib
    import sys
    import types
    pkg = sys.modules.get("methods")
    if pkg is None or not getattr(pkg, "__bayesdll_alias__", False):
        pkg = types.ModuleType("methods", "BayesDLL's methods/ package, served by bayesdll_amd")
        pkg.__path__ = []
        pkg.__bayesdll_alias__ = True
        sys.modules["methods"] = pkg
    for name in METHODS:
        mod = importlib.import_module(f"bayesdll_amd.{name}")
        sys.modules[f"methods.{name}"] = mod
        setattr(pkg, name, mod)
    return pkg
