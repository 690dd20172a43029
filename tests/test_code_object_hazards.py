"""CPU: static hazard checks on the gfx950 code objects inside the built libsiren_mri_amd.so.

* LDS reads (tools/check_lds_hazard.py): the kernels issue their fragment reads as inline asm with
  counted lgkmcnt waits; no instruction on any control-flow path may read a read's destination
  registers before a wait covers it (round 3: a register copy at a branch did, and one wave's block
  of the forward came out wrong in a few launches out of 100).
* Stores (tools/check_store_hazard.py --window=2): no store of more than 8 bytes, in any kernel of
  either code object, has a data VGPR rewritten with fewer than 2 wait states after its issue —
  the hazard tools/probe_store_hazard.hip measured on gfx950 (1 wait state
  corrupts lanes 12-15 of each 16-lane group, 0 lanes 8-15; 2 or more, none).
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


def test_no_store_data_rewritten_inside_the_measured_window(disassembly):
    kernels = stores = 0
    for dis in disassembly:
        r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "check_store_hazard.py"), dis, "_kernel",
                            "--window=2"], capture_output=True, text=True)
        assert r.returncode == 0, r.stdout
        last = r.stdout.strip().split("\n")[-1].split()
        kernels += int(last[0])
        stores += int(last[2])
    assert kernels > 150 and stores > 2000  # every kernel of both translation units was looked at


def test_forward_stores_carry_their_wait_states(disassembly):
    """The register-resident forward's phase-code and y stores are asm stores followed by s_nop 1
    (siren_common.h store_b128_ws2 / store_b32_ws2): checked on the disassembly of all 26 forms."""
    import re
    forms = 0
    for dis in disassembly:
        text = open(dis).read()
        for m in re.finditer(r"<(_ZN5siren20fused_fwd_reg_kernel\S+)>:\n(.*?)(?:\n\n|\Z)", text, re.S):
            forms += 1
            lines = [ln.split("//")[0].strip() for ln in m.group(2).split("\n")]
            for i, ln in enumerate(lines):
                if ln.startswith("buffer_store"):
                    assert lines[i + 1].startswith("s_nop 1"), (m.group(1), ln, lines[i + 1])
    assert forms == 32  # 6 input forms (1..4, wide, wide with the Fourier input) x 2 output classes x 2 epilogue forms + 8 fused-loss forms
