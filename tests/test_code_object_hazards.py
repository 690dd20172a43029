"""CPU: static hazard checks on the gfx950 code objects inside the built libsiren_mri_amd.so.

* LDS reads (tools/check_lds_hazard.py): the kernels issue their fragment reads as inline asm with
  counted lgkmcnt waits; no instruction on any control-flow path may read a read's destination
  registers before a wait covers it (round 3: a register copy at a branch did, and one wave's block
  of the forward came out wrong in a few launches out of 100).
* Stores (tools/check_store_hazard.py): the forward's store data registers stay untouched until the
  store has completed.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "siren_mri_amd", "libsiren_mri_amd.so")
sys.path.insert(0, os.path.join(ROOT, "tools"))


@pytest.fixture(scope="module")
def disassembly(tmp_path_factory):
    if not os.path.exists(LIB):
        pytest.skip("libsiren_mri_amd.so not built")
    if not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-objdump"):
        pytest.skip("llvm-objdump not available")
    import extract_code_objects as eco
    paths = eco.extract(LIB, str(tmp_path_factory.mktemp("co")))
    assert len(paths) >= 2  # the runtime TU and the forward's TU
    return paths


def _check(tool, dis, filt):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", tool), dis, filt],
                       capture_output=True, text=True)
    return r.returncode, r.stdout


def test_no_lds_read_consumed_before_its_wait(disassembly):
    total = 0
    for dis in disassembly:
        rc, out = _check("check_lds_hazard.py", dis, "_kernel")
        assert rc == 0, out
        total += int(out.strip().split("\n")[-1].split()[0])
    assert total > 150  # every kernel of both translation units was looked at


def test_forward_store_data_held_until_complete(disassembly):
    n = 0
    for dis in disassembly:
        rc, out = _check("check_store_hazard.py", dis, "fused_fwd_reg_kernel")
        assert rc == 0, out
        n += int(out.strip().split("\n")[-1].split()[0])
    assert n == 20  # 5 input forms x 2 output classes x 2 epilogue forms
