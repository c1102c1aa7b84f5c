"""The reference-side binding a maintainer would add to BayesDLL's
methods/csghmc.py to run its per-tensor cSGHMC update (methods/csghmc.py:747-778)
through the fused MI355X kernel — ctypes over include/bdl_sgmcmc.h, ABI
version 8.  INTEGRATION.md §3 shows this file verbatim; tests/test_abi.py
checks its struct against the C header and the shipped library, and
tests/test_gpu_reference_binding.py runs it against the product's own binding
(bit for bit).

Usage inside the reference's Model.forward, after loss.backward():

    lib = load("/path/to/bayesdll_amd/libbdl_sgmcmc.so")          # once
    runs, nruns = run_table(lib, net, readout_name)                   # once
    csghmc_step(lib, theta, grad, mom, runs, nruns, lrs, momentum_decay,
                prior_sig, N, nd, should_sample, seed, chain, step)

theta / grad / mom are flat fp32 HIP tensors in parameters_to_vector order
(the parameters and their .grad as views into theta / grad).
"""
import ctypes as C

import numpy as np

ABI_VERSION = 8
BDL_CSGHMC = 0
BDL_NOISE_NONE, BDL_NOISE_PHILOX = 0, 2
BDL_ATTR_HEAD, BDL_ATTR_PRIOR = 0x1, 0x2
BDL_FLAG_RECIP_DIV = 0x2


class Segment(C.Structure):      # bdl_segment
    _fields_ = [("offset", C.c_int64), ("numel", C.c_int64), ("attr", C.c_uint32),
                ("pad", C.c_uint32)]


class Run(C.Structure):          # bdl_run
    _fields_ = [("end", C.c_int64), ("attr", C.c_uint32), ("pad", C.c_uint32)]


class StepArgs(C.Structure):     # bdl_step_args, ABI v8
    _fields_ = [(f, C.c_void_p) for f in
                ("theta", "grad", "mom", "prior_mean", "noise", "mom1", "mom2", "runs")] + [
        ("nruns", C.c_int32), ("method", C.c_int32), ("noise_mode", C.c_int32),
        ("collect", C.c_int32), ("flags", C.c_int32), ("pad0", C.c_int32), ("n", C.c_int64),
        ("lr", C.c_float * 2), ("noise_scale", C.c_float * 2), ("one_minus_alpha", C.c_float),
        ("prior_sig", C.c_float), ("sigma2", C.c_float), ("n_data", C.c_float), ("mu", C.c_float),
        ("collect_a", C.c_float), ("collect_b", C.c_float),
        ("inv_sigma2", C.c_float), ("inv_n_data", C.c_float),      # 0 -> 1/fl32(s)
        ("inv_collect_a", C.c_float), ("inv_collect_b", C.c_float), ("pad1", C.c_float),
        ("seed", C.c_uint64), ("chain", C.c_uint64), ("step", C.c_uint64),
        ("grad_base", C.c_void_p),       # null: read `grad` (flat); else per-run bases
        ("nonfinite", C.c_void_p),       # optional int32 device flag: set on NaN/Inf writes
        ("philox_offset", C.c_uint64),   # Philox group offset of a sub-range launch (else 0)
        ("chain_groups", C.c_uint64)]    # stacked chains (0: the vectors hold one chain)


def load(path):
    """Open the library, declare the two entry points used here, and refuse a
    library built for another ABI version (its struct would differ)."""
    lib = C.CDLL(path)
    lib.bdl_version.restype = C.c_int
    lib.bdl_version.argtypes = []
    lib.bdl_last_error.restype = C.c_char_p
    lib.bdl_last_error.argtypes = []
    lib.bdl_build_runs.restype = C.c_int
    lib.bdl_build_runs.argtypes = [C.POINTER(Segment), C.c_int32, C.c_int64, C.POINTER(Run),
                                   C.c_int32]
    lib.bdl_sgmcmc_step.restype = C.c_int
    lib.bdl_sgmcmc_step.argtypes = [C.POINTER(StepArgs), C.c_void_p]
    if lib.bdl_version() != ABI_VERSION:
        raise RuntimeError(f"libbdl_sgmcmc ABI {lib.bdl_version()} != {ABI_VERSION}")
    return lib


def run_table(lib, named_numels, readout_name):
    """The host-side run table of methods/csghmc.py:750-753 (lr group by
    `readout_name in pname`; csghmc applies the prior everywhere, quirk Q1):
    returns (host array of Run, count) — copy it to the device once."""
    segs = (Segment * len(named_numels))()
    off = 0
    for i, (name, k) in enumerate(named_numels):
        head = BDL_ATTR_HEAD if readout_name in name else 0
        segs[i].offset, segs[i].numel, segs[i].attr = off, k, BDL_ATTR_PRIOR | head
        off += k
    cap = 2 * len(named_numels) + 2
    runs = (Run * cap)()
    nr = lib.bdl_build_runs(segs, len(named_numels), off, runs, cap)
    if nr < 0:
        raise RuntimeError(lib.bdl_last_error().decode())
    return runs, nr


def csghmc_step(lib, theta, grad, mom, runs_dev, nruns, lrs, momentum_decay, prior_sig, N, nd,
                should_sample, seed, chain, step, stream=None):
    """methods/csghmc.py:747-778 for every parameter at once.  Scalars are
    formed in float64 exactly as the reference's Python does; ctypes rounds
    them to fp32 as torch does at the op.  `stream`: a hipStream_t (int),
    default torch's current stream."""
    import torch
    a = StepArgs(theta=theta.data_ptr(), grad=grad.data_ptr(), mom=mom.data_ptr(),
                 runs=runs_dev.data_ptr(), nruns=nruns, method=BDL_CSGHMC,
                 noise_mode=BDL_NOISE_PHILOX if should_sample else BDL_NOISE_NONE,
                 flags=BDL_FLAG_RECIP_DIV, n=theta.numel(),
                 one_minus_alpha=1 - momentum_decay, prior_sig=prior_sig,
                 seed=seed, chain=chain, step=step)
    a.lr[:] = [lrs[0], lrs[1]]
    a.noise_scale[:] = [nd * np.sqrt(2 * momentum_decay * lr) / N for lr in lrs]
    if stream is None:
        stream = torch.cuda.current_stream().cuda_stream
    rc = lib.bdl_sgmcmc_step(C.byref(a), C.c_void_p(stream))
    if rc != 0:
        raise RuntimeError(lib.bdl_last_error().decode())
