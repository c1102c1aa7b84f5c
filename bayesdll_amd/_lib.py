"""ctypes binding of the C-ABI in include/bdl_sgmcmc.h (libbdl_sgmcmc.so).

The shared library is built in-tree (`make -C bayesdll_amd/csrc`, or
`__graft_entry__.build()`).  There is no fallback: if the library is missing
or a call fails, a RuntimeError is raised.  The product path never computes
the update anywhere else.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import torch  # noqa: F401  — load torch's HIP runtime first so the .so binds to it

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("BDL_SGMCMC_LIB", os.path.join(HERE, "libbdl_sgmcmc.so"))

# enums / bits — must match include/bdl_sgmcmc.h
BDL_OK = 0
CSGHMC, SGHMC, SGLD, SGHMC_GRAD, SGLD_GRAD, ADAM_SGHMC, ADAM_SGHMC_GRAD = range(7)
NOISE_NONE, NOISE_BUFFER, NOISE_PHILOX = 0, 1, 2
COLLECT_NONE, COLLECT_WELFORD_INIT, COLLECT_WELFORD, COLLECT_MEAN_INIT, COLLECT_MEAN = range(5)
MIX_BARE, MIX_PIPELINED, MIX_PACED = 0, 1, 2  # include/bdl_measure.h bdl_mix_schedule
ATTR_HEAD, ATTR_PRIOR, ATTR_SKIP, ATTR_GUNALIGNED = 0x1, 0x2, 0x4, 0x8
FLAG_FIRST_STEP, FLAG_RECIP_DIV, FLAG_MOMENTUM, FLAG_GRAD_READY = 0x1, 0x2, 0x4, 0x8
VAR_GIVEN, VAR_RAW_MOMENTS, VAR_WELFORD = 0, 1, 2
ABI_VERSION = 8

_fp = C.c_void_p


class Segment(C.Structure):
    _fields_ = [("offset", C.c_int64), ("numel", C.c_int64), ("attr", C.c_uint32),
                ("pad", C.c_uint32)]


class Run(C.Structure):
    _fields_ = [("end", C.c_int64), ("attr", C.c_uint32), ("pad", C.c_uint32)]


class StepArgs(C.Structure):
    _fields_ = [
        ("theta", _fp), ("grad", _fp), ("mom", _fp), ("prior_mean", _fp), ("noise", _fp),
        ("mom1", _fp), ("mom2", _fp), ("runs", _fp),
        ("nruns", C.c_int32), ("method", C.c_int32), ("noise_mode", C.c_int32),
        ("collect", C.c_int32), ("flags", C.c_int32), ("pad0", C.c_int32),
        ("n", C.c_int64),
        ("lr", C.c_float * 2), ("noise_scale", C.c_float * 2),
        ("one_minus_alpha", C.c_float), ("prior_sig", C.c_float), ("sigma2", C.c_float),
        ("n_data", C.c_float), ("mu", C.c_float), ("collect_a", C.c_float),
        ("collect_b", C.c_float), ("inv_sigma2", C.c_float), ("inv_n_data", C.c_float),
        ("inv_collect_a", C.c_float), ("inv_collect_b", C.c_float), ("pad1", C.c_float),
        ("seed", C.c_uint64), ("chain", C.c_uint64), ("step", C.c_uint64),
        ("grad_base", _fp), ("nonfinite", _fp), ("philox_offset", C.c_uint64),
        ("chain_groups", C.c_uint64),
    ]


class AdamArgs(C.Structure):
    _fields_ = [("adam_m", _fp), ("adam_v", _fp), ("sgd_buf", _fp),
                ("beta1", C.c_float), ("one_minus_beta1", C.c_float), ("beta2", C.c_float),
                ("one_minus_beta2", C.c_float), ("bias_corr1", C.c_float),
                ("bias_corr2", C.c_float), ("eps", C.c_float), ("two_alpha", C.c_float),
                ("nd", C.c_float), ("temperature", C.c_float), ("inv_bias_corr1", C.c_float),
                ("inv_bias_corr2", C.c_float), ("inv_temperature", C.c_float),
                ("pad2", C.c_float), ("grad_is_mom", C.c_int32)]


class MomentsArgs(C.Structure):
    _fields_ = [("theta", _fp), ("mom1", _fp), ("mom2", _fp), ("n", C.c_int64),
                ("collect", C.c_int32), ("flags", C.c_int32), ("collect_a", C.c_float),
                ("collect_b", C.c_float), ("inv_collect_a", C.c_float),
                ("inv_collect_b", C.c_float)]


class SampleArgs(C.Structure):
    _fields_ = [("out", _fp), ("mom1", _fp), ("mom2", _fp), ("noise", _fp), ("n", C.c_int64),
                ("var_mode", C.c_int32), ("noise_mode", C.c_int32), ("ratio", C.c_float),
                ("var_floor", C.c_float), ("inv_ratio", C.c_float), ("blocks_per_cu", C.c_int32),
                ("seed", C.c_uint64), ("chain", C.c_uint64),
                ("step", C.c_uint64), ("chain_groups", C.c_uint64), ("unroll", C.c_int32),
                ("pad", C.c_int32)]


EXPORTS = {
    "bdl_version": (C.c_int, []),
    "bdl_last_error": (C.c_char_p, []),
    "bdl_build_runs": (C.c_int, [C.POINTER(Segment), C.c_int32, C.c_int64, C.POINTER(Run),
                                 C.c_int32]),
    "bdl_sgmcmc_step": (C.c_int, [C.POINTER(StepArgs), C.c_void_p]),
    "bdl_moments_update": (C.c_int, [C.POINTER(MomentsArgs), C.c_void_p]),
    "bdl_adam_step": (C.c_int, [C.POINTER(StepArgs), C.POINTER(AdamArgs), C.c_void_p]),
    "bdl_clip_workspace_bytes": (C.c_int64, [C.c_int64]),
    "bdl_sgld_step_clipped": (C.c_int, [C.POINTER(StepArgs), C.c_float, C.c_void_p, C.c_void_p]),
    "bdl_posterior_sample": (C.c_int, [C.POINTER(SampleArgs), C.c_void_p]),
    "bdl_philox_normal": (C.c_int, [C.c_void_p, C.c_int64, C.c_uint64, C.c_uint64, C.c_uint64,
                                    C.c_void_p]),
    "bdl_set_launch_config": (C.c_int, [C.c_int32, C.c_int32, C.c_int32]),
    "bdl_graph_find_step_node": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64,
                                            C.POINTER(C.c_void_p)]),
    "bdl_graph_node_step_args": (C.c_int, [C.c_void_p, C.POINTER(C.c_int64), C.c_int32]),
    "bdl_graph_redirect": (C.c_int, [C.c_void_p, C.c_void_p]),
    # include/bdl_measure.h
    "bdl_stream_mix": (C.c_int, [C.POINTER(C.c_void_p), C.c_int32, C.POINTER(C.c_void_p),
                                 C.c_int32, C.c_int64, C.c_int32, C.c_int32, C.c_void_p]),
    "bdl_sgmcmc_step_bare": (C.c_int, [C.POINTER(StepArgs), C.c_void_p]),
    "bdl_stream_mix_schedule": (C.c_int, [C.POINTER(C.c_void_p), C.c_int32,
                                          C.POINTER(C.c_void_p), C.c_int32, C.c_int64,
                                          C.c_int32, C.c_int32, C.c_int32, C.c_void_p]),
    # include/bdl_arena.h
    "bdl_arena_reserve": (C.c_int, [C.c_int32, C.c_int64]),
    "bdl_arena_alloc": (C.c_void_p, [C.c_size_t, C.c_int, C.c_void_p]),
    "bdl_arena_free": (None, [C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]),
    "bdl_arena_stats": (C.c_int, [C.c_int32, C.POINTER(C.c_int64), C.c_int32]),
    "bdl_arena_contains": (C.c_int, [C.c_int32, C.c_void_p, C.c_int64]),
}

_lib = None
_lock = threading.Lock()


def lib():
    """Load libbdl_sgmcmc.so once; raise if it is missing (no CPU fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(
                    f"bayesdll_amd: HIP library not found at {LIB_PATH}; build it with "
                    "`make -C bayesdll_amd/csrc` (or __graft_entry__.build()). There is no CPU "
                    "fallback for the fused SG-MCMC step.")
            h = C.CDLL(LIB_PATH)
            for name, (res, argt) in EXPORTS.items():
                fn = getattr(h, name)
                fn.restype = res
                fn.argtypes = argt
            if h.bdl_version() != ABI_VERSION:
                raise RuntimeError(f"bayesdll_amd: ABI version mismatch ({h.bdl_version()} != "
                                   f"{ABI_VERSION}); rebuild the library")
            _lib = h
    return _lib


def check(rc: int, what: str):
    if rc != BDL_OK:
        msg = lib().bdl_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed (status {rc}): {msg}")
    return rc


def ptr(t):
    """Device pointer of a tensor (or None)."""
    return None if t is None else C.c_void_p(t.data_ptr())


def current_stream_handle(device=None):
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def require_hip(t: torch.Tensor, what: str):
    if not t.is_cuda:
        raise RuntimeError(f"bayesdll_amd: {what} must live on a HIP device (got {t.device}); "
                           "the fused SG-MCMC step has no CPU path")
    if t.dtype != torch.float32:
        raise RuntimeError(f"bayesdll_amd: {what} must be float32 (got {t.dtype})")
