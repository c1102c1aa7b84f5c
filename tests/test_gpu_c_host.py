"""The C-ABI from a plain C host on the GPU: examples/c_abi_step.c (gcc, HIP
runtime C API for device memory, no Python / torch in the process) runs five
cSGHMC steps through bdl_sgmcmc_step and checks theta and v bit for bit
against the same update computed op by op on the CPU.  Built by
__graft_entry__.build()."""
import os
import subprocess

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def test_plain_c_host_runs_the_step_bitexact():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    exe = os.path.join(ROOT, "examples", "c_abi_step")
    assert os.path.exists(exe), "build it with __graft_entry__.build()"
    p = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    assert p.stdout.startswith("OK 4194317 5")
