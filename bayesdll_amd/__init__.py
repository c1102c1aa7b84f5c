"""bayesdll_amd — MI355X-native fused SG-MCMC samplers with BayesDLL's Runner API.

Drop-in modules (same Runner/Model interfaces as the reference's methods/*.py):
    bayesdll_amd.csghmc   cyclical SGHMC  (methods/csghmc.py)
    bayesdll_amd.sghmc    SGHMC           (methods/sghmc.py)
    bayesdll_amd.csgld    cyclical SGLD   (methods/csgld.py)
    bayesdll_amd.sgld     SGLD            (methods/sgld.py, src/bayesdll/sgld.py)
    bayesdll_amd.adam_sghmc   Adam-preconditioned SGHMC          (methods/adam_sghmc.py)
    bayesdll_amd.adam_csghmc  cyclical Adam-preconditioned SGHMC (methods/adam_csghmc.py)
    bayesdll_amd.csghmc_fs    cSGHMC with cold restarts + full-sample BMA (methods/csghmc_fs.py)
    bayesdll_amd.cyclical CyclicalSGMCMC  (methods/cyclical.py)
    bayesdll_amd.calibration  ECE / MCE / NLL / temperature (calibration.py)
    bayesdll_amd.chains   one chain per GPU; the cross-chain predictive (RCCL)
    bayesdll_amd.stacked  K cSGHMC / SGHMC / SGLD / cSGLD chains per device in one launch (not in the reference)
    bayesdll_amd.run      command-line driver with the demos' flags (demo_mnist.py)

The per-step update runs in hand-written HIP kernels for gfx950
(bayesdll_amd/csrc/, one translation unit per kernel family) behind the C-ABI in include/bdl_sgmcmc.h,
loaded with ctypes.  There is no CPU path: without a HIP device or without the
built library, the samplers raise.
"""
from . import cyclical  # noqa: F401

__version__ = "0.1.0"


def library_path():
    from ._lib import LIB_PATH
    return LIB_PATH
