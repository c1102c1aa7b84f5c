"""C-ABI checks that need no GPU: the library loads, exports every symbol the
header declares, the ctypes mirrors match the C struct layouts (compiled with
gcc from include/bdl_sgmcmc.h), and the host-only run builder behaves."""
import ctypes as C
import os
import re
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "bdl_sgmcmc.h")


def declared_functions():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^(?:int|int64_t|const char\*)\s+(bdl_\w+)\(", txt, re.M)))


def test_header_declares_expected_api():
    assert declared_functions() == sorted([
        "bdl_version", "bdl_last_error", "bdl_build_runs", "bdl_sgmcmc_step",
        "bdl_moments_update", "bdl_posterior_sample", "bdl_philox_normal",
        "bdl_set_launch_config", "bdl_clip_workspace_bytes", "bdl_sgld_step_clipped", "bdl_adam_step"])


def test_library_loads_and_exports_every_declared_symbol():
    from bayesdll_amd import _lib as L
    h = L.lib()
    for name in declared_functions():
        assert hasattr(h, name), name
    assert set(declared_functions()) == set(L.EXPORTS)
    assert h.bdl_version() == L.ABI_VERSION


def _c_layout():
    src = r"""
#include <stdio.h>
#include <stddef.h>
#include "bdl_sgmcmc.h"
#define P(T, f) printf(#T "." #f " %zu\n", offsetof(T, f));
int main(void) {
  printf("bdl_segment %zu\nbdl_run %zu\nbdl_step_args %zu\nbdl_moments_args %zu\nbdl_sample_args %zu\n",
         sizeof(bdl_segment), sizeof(bdl_run), sizeof(bdl_step_args), sizeof(bdl_moments_args),
         sizeof(bdl_sample_args));
  printf("bdl_adam_args %zu\n", sizeof(bdl_adam_args));
  P(bdl_adam_args, sgd_buf) P(bdl_adam_args, beta1) P(bdl_adam_args, bias_corr2)
  P(bdl_adam_args, temperature) P(bdl_adam_args, grad_is_mom)
  P(bdl_step_args, runs) P(bdl_step_args, nruns) P(bdl_step_args, n) P(bdl_step_args, lr)
  P(bdl_step_args, noise_scale) P(bdl_step_args, mu) P(bdl_step_args, collect_b)
  P(bdl_step_args, seed) P(bdl_step_args, step) P(bdl_moments_args, collect_a)
  P(bdl_sample_args, ratio) P(bdl_sample_args, step) P(bdl_run, attr) P(bdl_segment, attr)
  return 0;
}
"""
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "probe.c")
        exe = os.path.join(d, "probe")
        open(c, "w").write(src)
        subprocess.check_call(["gcc", "-std=c99", "-I", os.path.dirname(HEADER), c, "-o", exe])
        out = subprocess.check_output([exe]).decode()
    return dict(line.rsplit(" ", 1) for line in out.strip().splitlines())


def test_ctypes_layout_matches_c_header():
    from bayesdll_amd import _lib as L
    lay = {k: int(v) for k, v in _c_layout().items()}
    assert lay["bdl_segment"] == C.sizeof(L.Segment)
    assert lay["bdl_run"] == C.sizeof(L.Run)
    assert lay["bdl_step_args"] == C.sizeof(L.StepArgs)
    assert lay["bdl_moments_args"] == C.sizeof(L.MomentsArgs)
    assert lay["bdl_sample_args"] == C.sizeof(L.SampleArgs)
    assert lay["bdl_adam_args"] == C.sizeof(L.AdamArgs)
    for key, v in lay.items():
        if "." not in key:
            continue
        struct, field = key.split(".")
        cls = {"bdl_step_args": L.StepArgs, "bdl_moments_args": L.MomentsArgs,
               "bdl_adam_args": L.AdamArgs,
               "bdl_sample_args": L.SampleArgs, "bdl_run": L.Run, "bdl_segment": L.Segment}[struct]
        assert getattr(cls, field).offset == v, key


def test_build_runs_merges_equal_attributes():
    from bayesdll_amd import _lib as L
    from bayesdll_amd.flat import build_runs, segment_attrs
    names = ["a.weight", "a.bias", "b.weight", "b.bias", "classifier.weight", "classifier.bias"]
    numels = [10, 3, 7, 1, 5, 2]
    offsets = [0, 10, 13, 20, 21, 26]
    # informative: only the head boundary matters
    attrs = segment_attrs(names, "classifier", "informative", [True] * 6)
    runs = build_runs(offsets, numels, attrs, 28)
    assert runs.tolist() == [[21, L.ATTR_PRIOR], [28, L.ATTR_PRIOR | L.ATTR_HEAD]]
    # uninformative bias: bias segments lose the prior bit
    attrs = segment_attrs(names, "classifier", "uninformative", [True] * 6)
    runs = build_runs(offsets, numels, attrs, 28)
    assert runs.tolist() == [[10, 2], [13, 0], [20, 2], [21, 0], [26, 3], [28, 1]]
    # frozen parameter -> skip run; trailing gap -> skip
    attrs = segment_attrs(names, "classifier", "informative", [True, False] + [True] * 4)
    runs = build_runs(offsets, numels, attrs, 30)
    assert runs.tolist() == [[10, 2], [13, 6], [21, 2], [28, 3], [30, 4]]


def test_build_runs_rejects_bad_tables():
    from bayesdll_amd.flat import build_runs
    with pytest.raises(RuntimeError, match="overlap"):
        build_runs([0, 5], [10, 3], [0, 0], 20)
    with pytest.raises(RuntimeError, match="exceed"):
        build_runs([0], [30], [0], 20)


def test_empty_vector_is_one_skip_run():
    from bayesdll_amd import _lib as L
    from bayesdll_amd.flat import build_runs
    assert build_runs([], [], [], 0).tolist() == [[0, L.ATTR_SKIP]]


def test_product_refuses_cpu_tensors():
    """No CPU fallback: a net on the CPU is rejected before any kernel call."""
    from fakenet import FakeNet
    from bayesdll_amd.flat import FlatState
    with pytest.raises(RuntimeError, match="HIP device"):
        FlatState(FakeNet())


def test_step_rejects_null_and_misaligned_pointers_without_launching():
    from bayesdll_amd import _lib as L
    a = L.StepArgs()
    a.n = 16
    a.method = L.CSGHMC
    rc = L.lib().bdl_sgmcmc_step(a, None)
    assert rc == -1 and b"required" in L.lib().bdl_last_error()
    a.theta, a.grad, a.mom, a.runs, a.nruns = 0x1004, 0x2000, 0x3000, 0x4000, 1
    rc = L.lib().bdl_sgmcmc_step(a, None)
    assert rc == -2 and b"aligned" in L.lib().bdl_last_error()
    a.theta, a.method = 0x1000, 9
    assert L.lib().bdl_sgmcmc_step(a, None) == -3


def test_entry_points_validate_before_touching_the_device():
    """Argument errors come back as negative bdl_status codes with a message,
    before any HIP call (so this runs without a GPU)."""
    from bayesdll_amd import _lib as L
    h = L.lib()
    a = L.StepArgs()
    assert h.bdl_sgmcmc_step(None, None) == -1                     # BDL_ERR_NULL
    assert b"null args" in h.bdl_last_error()
    a.n, a.method = 8, 9
    assert h.bdl_sgmcmc_step(a, None) == -3                         # unknown method
    a.method, a.noise_mode = L.CSGHMC, 7
    assert h.bdl_sgmcmc_step(a, None) == -3                         # unknown noise mode
    a.noise_mode = L.NOISE_NONE
    assert h.bdl_sgmcmc_step(a, None) == -1                         # theta/grad/runs missing
    a.theta, a.grad, a.mom, a.runs, a.nruns = 0x1000, 0x2000, 0x3000, 0x4000, 5000
    assert h.bdl_sgmcmc_step(a, None) == -5                         # > 4096 runs
    a.nruns = 1
    a.grad = 0x2004
    assert h.bdl_sgmcmc_step(a, None) == -2                         # misaligned vector
    a.grad = 0x2000
    # per-tensor gradient bases instead of the flat grad vector
    a.grad, a.grad_base = None, None
    assert h.bdl_sgmcmc_step(a, None) == -1                         # neither grad nor grad_base
    assert b"grad_base" in h.bdl_last_error()
    a.grad_base = 0x5004
    assert h.bdl_sgmcmc_step(a, None) == -2                         # base table not 8-B aligned
    a.grad_base, a.nruns = 0x5000, 2731
    assert h.bdl_sgmcmc_step(a, None) == -5                         # runs + bases > 64 KiB LDS
    a.grad, a.grad_base, a.nruns = 0x2000, None, 1
    a.method = L.SGLD
    assert h.bdl_sgmcmc_step(a, None) == -1                         # sgld needs prior_mean
    a.n = 0
    assert h.bdl_sgmcmc_step(a, None) == 0                          # empty: no-op
    # clipped step: only SGLD, max_norm > 0, no GRAD_READY
    a.n, a.prior_mean = 8, 0x5000
    a.method = L.CSGHMC
    assert h.bdl_sgld_step_clipped(a, 1.0, C.c_void_p(0x6000), None) == -3
    a.method = L.SGLD
    assert h.bdl_sgld_step_clipped(a, 0.0, C.c_void_p(0x6000), None) == -3
    assert h.bdl_sgld_step_clipped(a, 1.0, None, None) == -1
    a.flags = L.FLAG_GRAD_READY
    assert h.bdl_sgld_step_clipped(a, 1.0, C.c_void_p(0x6000), None) == -3
    a.flags = 0
    assert h.bdl_clip_workspace_bytes(10 ** 9) >= 8
    # Adam: method, Adam buffers, SGD buffer with MOMENTUM
    ad = L.AdamArgs()
    assert h.bdl_adam_step(a, ad, None) == -3                       # method is SGLD
    a.method = L.ADAM_SGHMC
    assert h.bdl_adam_step(a, ad, None) == -1                       # adam_m / adam_v missing
    ad.adam_m, ad.adam_v = 0x7000, 0x8000
    a.flags = L.FLAG_MOMENTUM
    assert h.bdl_adam_step(a, ad, None) == -1                       # sgd_buf missing
    a.flags, a.collect = 0, L.COLLECT_WELFORD
    a.mom1 = 0x9000
    assert h.bdl_adam_step(a, ad, None) == -3                       # Welford not an Adam collect
    assert b"bdl_adam_step" in h.bdl_last_error()


def test_plain_c_host_links_and_calls_the_abi(tmp_path):
    """A C host (no Python, no torch) compiles against include/bdl_sgmcmc.h,
    links libbdl_sgmcmc.so and uses the host-only entry points — the same
    boundary a cgo / JNI / N-API binding would use."""
    from bayesdll_amd import _lib as L
    src = r"""
#include <stdio.h>
#include "bdl_sgmcmc.h"
int main(void) {
  bdl_segment segs[3] = {{0, 10, BDL_ATTR_PRIOR, 0}, {10, 3, 0, 0},
                         {13, 5, BDL_ATTR_PRIOR | BDL_ATTR_HEAD, 0}};
  bdl_run runs[8];
  int nr = bdl_build_runs(segs, 3, 20, runs, 8);
  printf("version %d runs %d", bdl_version(), nr);
  for (int i = 0; i < nr; ++i) printf(" %lld:%u", (long long)runs[i].end, runs[i].attr);
  int rc = bdl_sgmcmc_step(0, 0);
  printf(" rc %d msg %s\n", rc, bdl_last_error());
  return 0;
}
"""
    c = tmp_path / "host.c"
    exe = tmp_path / "host"
    c.write_text(src)
    libdir = os.path.dirname(L.LIB_PATH)
    subprocess.check_call(["gcc", "-std=c99", "-I", os.path.dirname(HEADER), str(c), "-o", str(exe),
                           "-L", libdir, "-lbdl_sgmcmc", f"-Wl,-rpath,{libdir}",
                           "-Wl,-rpath,/opt/rocm/lib"])
    out = subprocess.check_output([str(exe)]).decode()
    assert out.startswith(f"version {L.ABI_VERSION} runs 4")
    assert " 10:2 13:0 18:3 20:4 " in out
    assert "rc -1 msg bdl_sgmcmc_step: null args" in out


def test_missing_library_fails_loudly():
    """No CPU fallback: without the built library the product raises."""
    code = ("import bayesdll_amd._lib as L\n"
            "try:\n    L.lib()\nexcept RuntimeError as e:\n    print('raised', e)\n")
    env = dict(os.environ, BDL_SGMCMC_LIB="/nonexistent/libbdl_sgmcmc.so")
    out = subprocess.run(["python", "-c", code], env=env, capture_output=True, text=True,
                         cwd=os.path.dirname(HEADER) + "/..", timeout=300)
    assert "raised" in out.stdout and "libbdl_sgmcmc" in out.stdout, out.stdout + out.stderr


def test_reference_written_checkpoints_load_weights_only():
    """The reference-written checkpoint fixtures (tests/golden/ckpt_ref_*.pt)
    load through the product's loader (torch.load weights_only=True plus the
    numpy types csghmc's cycle_likelihoods hold): nothing is unpickled as code.
    Keys are the reference's (methods/csghmc.py:530-549, methods/sgld.py:367-385)."""
    import os
    import torch
    from bayesdll_amd._runner import load_checkpoint
    golden = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    ck = load_checkpoint(os.path.join(golden, "ckpt_ref_csghmc.pt"), "cpu")
    assert set(ck) == {"last_theta", "cycle_theta_mom1", "cycle_theta_mom2", "cycle_likelihoods",
                       "cycle_states", "epoch", "current_cycle", "samples_per_cycle"}
    assert sorted(ck["cycle_theta_mom1"]) == [1, 2] and ck["current_cycle"] == 2
    assert ck["last_theta"].shape == ck["cycle_theta_mom1"][1].shape
    ck = load_checkpoint(os.path.join(golden, "ckpt_ref_sgld.pt"), "cpu")
    assert set(ck) == {"last_theta", "post_theta_mom1", "post_theta_mom2", "post_theta_cnt",
                       "prior_sig", "optimizer", "epoch"}
    n = sum(v.numel() for v in ck["last_theta"].values())
    assert ck["post_theta_mom1"].numel() == n and isinstance(ck["post_theta_mom1"], torch.Tensor)
