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
HEADERS = [HEADER, os.path.join(ROOT, "include", "bdl_measure.h"),
           os.path.join(ROOT, "include", "bdl_arena.h")]


def declared_functions(headers=HEADERS):
    txt = "".join(open(h).read() for h in headers)
    return sorted(set(re.findall(r"^(?:int|int64_t|const char\*|void\*?)\s+(bdl_\w+)\(", txt, re.M)))


def test_header_declares_expected_api():
    assert declared_functions([HEADERS[1]]) == ["bdl_sgmcmc_step_bare", "bdl_stream_mix",
                                                "bdl_stream_mix_schedule"]
    assert declared_functions([HEADERS[2]]) == sorted([
        "bdl_arena_reserve", "bdl_arena_alloc", "bdl_arena_free", "bdl_arena_stats",
        "bdl_arena_contains"])
    assert declared_functions([HEADER]) == sorted([
        "bdl_version", "bdl_last_error", "bdl_build_runs", "bdl_sgmcmc_step",
        "bdl_moments_update", "bdl_posterior_sample", "bdl_philox_normal",
        "bdl_set_launch_config", "bdl_clip_workspace_bytes", "bdl_sgld_step_clipped", "bdl_adam_step",
        "bdl_graph_find_step_node", "bdl_graph_node_step_args", "bdl_graph_redirect"])


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
  P(bdl_step_args, grad_base) P(bdl_step_args, nonfinite) P(bdl_step_args, philox_offset)
  P(bdl_step_args, chain_groups) P(bdl_step_args, inv_collect_b) P(bdl_sample_args, chain_groups)
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
    # stacked chains: every float4 group index (+ philox_offset) below 2^32
    a.chain_groups, a.n = 1 << 32, 8
    assert h.bdl_sgmcmc_step(a, None) == -3                         # chain_groups >= 2^32
    a.chain_groups, a.n, a.philox_offset = 2, 8, (1 << 32) - 1
    assert h.bdl_sgmcmc_step(a, None) == -3                         # offset + n/4 >= 2^32
    assert b"stacked chains" in h.bdl_last_error()
    sa = L.SampleArgs()
    sa.n, sa.out, sa.mom1, sa.noise_mode, sa.chain_groups = 8, 0x1000, 0x2000, L.NOISE_PHILOX, 1 << 32
    assert h.bdl_posterior_sample(sa, None) == -3
    a.chain_groups, a.philox_offset = 0, 0
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


def test_other_entry_points_refuse_while_a_graph_redirect_is_active():
    """Only bdl_sgmcmc_step rewrites a captured node: while a redirect is set,
    every other launching entry point launches nothing and says why (a
    pointer check before any HIP call; the fake handles are never used)."""
    from bayesdll_amd import _lib as L
    h = L.lib()
    assert h.bdl_graph_redirect(C.c_void_p(0x10), C.c_void_p(0x20)) == 0
    try:
        a, ad = L.StepArgs(), L.AdamArgs()
        a.method, a.n = L.ADAM_SGHMC, 8
        calls = {
            "bdl_adam_step": lambda: h.bdl_adam_step(a, ad, None),
            "bdl_sgld_step_clipped": lambda: h.bdl_sgld_step_clipped(a, 1.0, C.c_void_p(0x6000),
                                                                     None),
            "bdl_moments_update": lambda: h.bdl_moments_update(L.MomentsArgs(), None),
            "bdl_posterior_sample": lambda: h.bdl_posterior_sample(L.SampleArgs(), None),
            "bdl_philox_normal": lambda: h.bdl_philox_normal(C.c_void_p(0x1000), 8, 0, 0, 0, None),
            "bdl_stream_mix": lambda: h.bdl_stream_mix((C.c_void_p * 1)(0x1000), 1,
                                                       (C.c_void_p * 1)(0x2000), 1, 8, 1, 1, None),
            "bdl_sgmcmc_step_bare": lambda: h.bdl_sgmcmc_step_bare(a, None),
            "bdl_stream_mix_schedule": lambda: h.bdl_stream_mix_schedule(
                (C.c_void_p * 1)(0x1000), 1, (C.c_void_p * 1)(0x2000), 1, 8, 1, 1, 2, None),
        }
        for name, call in calls.items():
            assert call() == -3, name
            assert b"graph redirect is active" in h.bdl_last_error(), name
    finally:
        h.bdl_graph_redirect(None, None)
    assert h.bdl_moments_update(None, None) == -1  # back to ordinary validation


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


ASAN_HOST = r"""
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "bdl_sgmcmc.h"
static unsigned long long s = 88172645463325252ULL;
static unsigned long long rnd(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
#define EXPECT(c) do { if (!(c)) { printf("FAIL line %d\n", __LINE__); return 1; } } while (0)
int main(void) {
  long ok = 0, rejected = 0;
  for (int it = 0; it < 4000; ++it) {           /* bdl_build_runs on random tables */
    int nseg = (int)(rnd() % 40);
    bdl_segment* segs = (bdl_segment*)malloc(sizeof(bdl_segment) * (nseg ? nseg : 1));
    long long pos = 0;
    for (int i = 0; i < nseg; ++i) {
      long long gap = (rnd() % 4 == 0) ? (long long)(rnd() % 5) : 0;
      if (rnd() % 97 == 0) gap = -(long long)(1 + rnd() % 3);   /* overlap */
      long long k = (long long)(rnd() % 50);
      segs[i].offset = pos + gap; segs[i].numel = k;
      segs[i].attr = (unsigned)(rnd() % 16); segs[i].pad = 0;
      pos = segs[i].offset + k;
    }
    long long n = pos + (long long)(rnd() % 5);
    if (rnd() % 50 == 0) n = pos - 1;                             /* segment past n */
    int cap = (rnd() % 3 == 0) ? (int)(rnd() % (2 * nseg + 3)) : 2 * nseg + 2;
    if (cap < 1) cap = 1;
    bdl_run* runs = (bdl_run*)malloc(sizeof(bdl_run) * cap);
    int nr = bdl_build_runs(segs, nseg, n, runs, cap);
    if (nr > 0) {
      EXPECT(nr <= cap);
      for (int r = 1; r < nr; ++r) EXPECT(runs[r].end > runs[r - 1].end && runs[r].attr != runs[r - 1].attr);
      EXPECT(runs[nr - 1].end == n);
      int r = 0;
      for (long long e = 0; e < n; ++e) {                          /* every element's attributes */
        unsigned want = BDL_ATTR_SKIP;
        for (int i = 0; i < nseg; ++i)
          if (e >= segs[i].offset && e < segs[i].offset + segs[i].numel) want = segs[i].attr & 0xF;
        while (runs[r].end <= e) ++r;
        EXPECT(runs[r].attr == want);
      }
      ++ok;
    } else {
      EXPECT(nr < 0 && strlen(bdl_last_error()) > 0);
      ++rejected;
    }
    free(segs);
    free(runs);
  }
  /* argument validation of every entry point (returns before any device call) */
  bdl_step_args a; memset(&a, 0, sizeof a);
  a.n = 16; a.method = BDL_CSGHMC;
  EXPECT(bdl_sgmcmc_step(NULL, NULL) == BDL_ERR_NULL);
  EXPECT(bdl_sgmcmc_step(&a, NULL) == BDL_ERR_NULL);
  a.theta = (float*)0x1000; a.runs = (const bdl_run*)0x4000; a.nruns = 1; a.mom = (float*)0x3000;
  EXPECT(bdl_sgmcmc_step(&a, NULL) == BDL_ERR_NULL);            /* no grad, no grad_base */
  a.grad_base = (const int64_t*)0x5004;
  EXPECT(bdl_sgmcmc_step(&a, NULL) == BDL_ERR_ALIGN);
  a.grad_base = (const int64_t*)0x5000; a.nruns = 2731;
  EXPECT(bdl_sgmcmc_step(&a, NULL) == BDL_ERR_RUNS);
  a.grad_base = NULL; a.grad = (float*)0x2000; a.nruns = 4097;
  EXPECT(bdl_sgmcmc_step(&a, NULL) == BDL_ERR_RUNS);
  a.nruns = 1; a.theta = (float*)0x1004;
  EXPECT(bdl_sgmcmc_step(&a, NULL) == BDL_ERR_ALIGN);
  a.theta = (float*)0x1000; a.method = 99;
  EXPECT(bdl_sgmcmc_step(&a, NULL) == BDL_ERR_ARG);
  a.method = BDL_SGLD;
  EXPECT(bdl_sgmcmc_step(&a, NULL) == BDL_ERR_NULL);            /* prior_mean */
  a.method = BDL_SGLD_GRAD; a.prior_mean = (const float*)0x6000; a.collect = BDL_COLLECT_MEAN;
  a.mom1 = (float*)0x7000;
  EXPECT(bdl_sgmcmc_step(&a, NULL) == BDL_ERR_ARG);             /* grad-only cannot collect */
  EXPECT(bdl_sgld_step_clipped(&a, 1.0f, (void*)0x8000, NULL) == BDL_ERR_ARG);
  a.method = BDL_SGLD; a.collect = 0;
  EXPECT(bdl_sgld_step_clipped(&a, 0.0f, (void*)0x8000, NULL) == BDL_ERR_ARG);
  EXPECT(bdl_sgld_step_clipped(&a, 1.0f, (void*)0x8004, NULL) == BDL_ERR_ALIGN);
  bdl_adam_args ad; memset(&ad, 0, sizeof ad);
  a.method = BDL_ADAM_SGHMC;
  EXPECT(bdl_adam_step(&a, &ad, NULL) == BDL_ERR_NULL);         /* adam_m / adam_v */
  EXPECT(bdl_adam_step(&a, NULL, NULL) == BDL_ERR_NULL);
  bdl_moments_args m; memset(&m, 0, sizeof m); m.n = 8; m.collect = 9;
  EXPECT(bdl_moments_update(&m, NULL) == BDL_ERR_ARG);
  m.collect = BDL_COLLECT_MEAN;
  EXPECT(bdl_moments_update(&m, NULL) == BDL_ERR_NULL);
  bdl_sample_args sa; memset(&sa, 0, sizeof sa); sa.n = 8; sa.var_mode = 7;
  EXPECT(bdl_posterior_sample(&sa, NULL) == BDL_ERR_ARG);
  EXPECT(bdl_philox_normal(NULL, 8, 0, 0, 0, NULL) == BDL_ERR_NULL);
  EXPECT(bdl_philox_normal((float*)0x1004, 8, 0, 0, 0, NULL) == BDL_ERR_ALIGN);
  printf("OK %ld %ld\n", ok, rejected);
  return 0;
}
"""


def test_host_abi_under_address_sanitizer(tmp_path):
    """SURVEY §5 'race detection / sanitizers': the C-ABI's host code (run
    building, every entry point's validation and error paths) built with
    host-side AddressSanitizer (`make asan`; device code unchanged, GPU
    sanitizers are not available) and driven by a C host over 4000 random
    segment tables (gaps, overlaps, segments past n, undersized outputs) —
    no ASan report, every accepted table exactly right, every rejected one
    with a message.  No device calls."""
    import shutil
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    csrc = os.path.join(root, "bayesdll_amd", "csrc")
    lib = os.path.join(root, "bayesdll_amd", "libbdl_sgmcmc_asan.so")
    subprocess.check_call(["make", "-C", csrc, "-j8", "asan"], stdout=subprocess.DEVNULL)
    clang = "/opt/rocm/lib/llvm/bin/clang"
    if not os.path.exists(clang):
        clang = shutil.which("clang")
    c = tmp_path / "fuzz.c"
    exe = tmp_path / "fuzz"
    c.write_text(ASAN_HOST)
    shutil.copy(lib, tmp_path / "libbdl_sgmcmc_asan.so")
    subprocess.check_call([clang, "-std=c99", "-g", "-fsanitize=address", "-fno-omit-frame-pointer",
                           "-I", os.path.dirname(HEADER), str(c), "-o", str(exe),
                           "-L", str(tmp_path), "-lbdl_sgmcmc_asan", f"-Wl,-rpath,{tmp_path}",
                           "-Wl,-rpath,/opt/rocm/lib"])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:verify_asan_link_order=0:abort_on_error=0")
    p = subprocess.run([str(exe)], env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0 and p.stdout.startswith("OK"), (p.stdout + p.stderr)[-3000:]
    assert "AddressSanitizer" not in p.stderr
    ok, rejected = map(int, p.stdout.split()[1:3])
    assert ok > 1000 and rejected > 10


def test_algorithmic_bytes_per_element_match_design_table():
    """kernels.alg_bytes_per_elem (used by the per-epoch GB/s log) reproduces
    DESIGN §4's table / bench.BYTES_PER_ELEM from a launch's own arguments."""
    from bayesdll_amd import _lib as L
    from bayesdll_amd.kernels import alg_bytes_per_elem

    def args(method, collect=0, flags=0, prior=True, m2=True, noise=L.NOISE_PHILOX):
        a = L.StepArgs()
        a.method, a.collect, a.flags, a.noise_mode = method, collect, flags, noise
        a.prior_mean = 0x1000 if prior else None
        a.mom2 = 0x2000 if m2 else None
        return a
    assert alg_bytes_per_elem(args(L.CSGHMC, prior=False, noise=L.NOISE_NONE)) == 20
    assert alg_bytes_per_elem(args(L.CSGHMC, L.COLLECT_WELFORD_INIT, prior=False)) == 28
    assert alg_bytes_per_elem(args(L.CSGHMC, L.COLLECT_WELFORD, prior=False)) == 36
    assert alg_bytes_per_elem(args(L.CSGHMC, prior=False, noise=L.NOISE_BUFFER)) == 24
    mom = L.FLAG_MOMENTUM
    assert alg_bytes_per_elem(args(L.SGLD, flags=mom)) == 24
    assert alg_bytes_per_elem(args(L.SGLD, flags=mom | L.FLAG_FIRST_STEP)) == 20
    assert alg_bytes_per_elem(args(L.SGLD, L.COLLECT_MEAN, flags=mom)) == 40
    assert alg_bytes_per_elem(args(L.SGHMC)) == 24
    ad = L.AdamArgs()
    ad.sgd_buf = 0x3000
    assert alg_bytes_per_elem(args(L.ADAM_SGHMC, flags=mom), ad) == 48
    assert alg_bytes_per_elem(args(L.ADAM_SGHMC, flags=mom | L.FLAG_FIRST_STEP), ad) == 44
    assert alg_bytes_per_elem(args(L.ADAM_SGHMC, L.COLLECT_MEAN, flags=mom), ad) == 64


def test_tools_and_examples_compile():
    """The measurement scripts under tools/ stay importable-syntax clean."""
    import glob
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    files = glob.glob(os.path.join(root, "tools", "*.py"))
    assert len(files) >= 8
    for f in files:
        with open(f) as fh:
            compile(fh.read(), f, "exec")


def _reference_binding():
    import importlib.util
    path = os.path.join(ROOT, "examples", "reference_binding.py")
    spec = importlib.util.spec_from_file_location("reference_binding", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod, path


def test_integration_snippet_is_the_tested_reference_binding():
    """INTEGRATION.md §3 shows examples/reference_binding.py verbatim, so the
    documented binding is the one these tests check."""
    _, path = _reference_binding()
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    assert open(path).read() in doc
    from bayesdll_amd import _lib as L
    assert f"ABI version {L.ABI_VERSION}" in doc
    for old in range(1, L.ABI_VERSION):  # no stale version number in the doc or the binding
        for text in (doc, open(path).read()):
            assert f"ABI version {old}" not in text and f"ABI v{old}," not in text
            assert not re.search(rf"ABI\s+version {old}\b", text), old


def test_reference_binding_struct_matches_header_and_library():
    """The maintainer's ctypes StepArgs has the v6 header's size and every
    field at the header's offset (so the library never reads past it), and
    load() accepts the shipped library and refuses another ABI version."""
    from bayesdll_amd import _lib as L
    rb, _ = _reference_binding()
    lay = {k: int(v) for k, v in _c_layout().items()}
    assert C.sizeof(rb.StepArgs) == lay["bdl_step_args"] == C.sizeof(L.StepArgs)
    assert C.sizeof(rb.Run) == lay["bdl_run"] and C.sizeof(rb.Segment) == lay["bdl_segment"]
    assert [f for f, _ in rb.StepArgs._fields_] == [f for f, _ in L.StepArgs._fields_]
    for f, _ in L.StepArgs._fields_:
        assert getattr(rb.StepArgs, f).offset == getattr(L.StepArgs, f).offset, f
    for key, v in lay.items():
        if key.startswith("bdl_step_args."):
            assert getattr(rb.StepArgs, key.split(".")[1]).offset == v, key
    lib = rb.load(L.LIB_PATH)
    assert lib.bdl_version() == rb.ABI_VERSION == L.ABI_VERSION
    runs, nr = rb.run_table(lib, [("enc.weight", 10), ("enc.bias", 3), ("head.weight", 5)], "head")
    assert [(runs[i].end, runs[i].attr) for i in range(nr)] == [(13, 2), (18, 3)]
    rb.ABI_VERSION = L.ABI_VERSION - 1
    with pytest.raises(RuntimeError, match="ABI"):
        rb.load(L.LIB_PATH)
