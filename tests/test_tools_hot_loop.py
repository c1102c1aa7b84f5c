"""tools/hot_loop_spills.py (the spill-location evidence of DESIGN §4): on a
small hand-written amdgcn listing it finds the sweep loop through its back
edge and counts only the spill code inside it."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

ASM = """\t.text
_Z6kernelv:                             ; @_Z6kernelv
\ts_load_dwordx2 s[0:1], s[4:5], 0x0
\tv_writelane_b32 v9, s6, 0
\tv_readlane_b32 s6, v9, 0
.LBB0_1:                                ; =>This Inner Loop Header: Depth=1
\tglobal_load_dwordx4 v[0:3], v[4:5], off nt
\tv_readlane_b32 s7, v9, 1
\ts_cmp_lt_u32 s2, s3
\ts_cbranch_scc0 .LBB0_3
; %bb.2:
\tv_writelane_b32 v9, s8, 2
\tglobal_store_dwordx4 v[4:5], v[0:3], off nt
\ts_branch .LBB0_1
.LBB0_3:
\tv_readlane_b32 s9, v9, 2
\ts_endpgm
.Lfunc_end0:
"""


def test_counts_spills_inside_and_outside_the_sweep_loop():
    import hot_loop_spills as H
    rows = H.analyse(ASM)
    assert len(rows) == 1
    r = rows[0]
    assert (r["readlane"], r["writelane"], r["scratch"]) == (3, 2, 0)
    assert r["in_sweeps"] == {"readlane": 1, "writelane": 1, "scratch": 0}
    assert r["main"]["load16"] == 1 and r["main"]["blocks"] == 2
