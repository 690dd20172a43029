"""The C-ABI library loads (no GPU needed), exports every symbol include/siren_mri_amd.h declares,
and validates descriptors / sizes workspaces without touching a device."""
import ctypes
import os
import re

import pytest

from siren_mri_amd import _native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "siren_mri_amd.h")


def header_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(siren_[a-z0-9_]+)\s*\(", text)))


def test_library_builds_and_exports_every_declared_symbol():
    lib = _native.load_library()
    declared = header_functions()
    assert declared, "no functions parsed from the header"
    assert sorted(_native.EXPORTED_SYMBOLS) == declared
    for name in declared:
        assert hasattr(lib, name), f"missing export {name}"
    assert b"gfx950" in lib.siren_version()


def test_library_is_gfx950_code_object():
    data = open(_native.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def _desc(dims, prec=_native.PREC_BF16, **kw):
    return _native.describe_only(dims, prec=prec, **kw)


def test_check_accepts_reference_configs():
    lib = _native.load_library()
    for dims, kw in [([2, 256, 256, 256, 256, 1], dict(rows_per_batch=512 * 512)),
                     ([2, 256, 256, 1], dict(rows_per_batch=64 * 64)),
                     ([16, 256, 256, 256, 256, 2], dict(batch=32, rows_per_batch=16384, weights_batched=True)),
                     # config 4 (2*60 Fourier features) and config 5 (2*228, hidden 512; fp32 too)
                     ([120, 256, 256, 256, 256, 2], dict(batch=32, rows_per_batch=16384, weights_batched=True)),
                     ([456] + [512] * 5 + [2], dict(batch=32, rows_per_batch=16384, weights_batched=True))]:
        for prec in (_native.PREC_F32, _native.PREC_BF16):
            d = _desc(dims, prec=prec, **kw)
            assert lib.siren_mlp_check(ctypes.byref(d)) == 0, _native.last_error()
            assert lib.siren_mlp_saved_bytes(ctypes.byref(d)) > 0
            assert lib.siren_mlp_workspace_bytes(ctypes.byref(d)) > 0


@pytest.mark.parametrize("dims,msg", [
    ([2, 100, 1], "hidden width"),          # not a multiple of 32
    ([600, 256, 1], "in_features"),         # wider than one MFMA K panel
    ([2, 256, 9], "out_features"),          # too wide an output layer
    ([2, 1], "num_layers"),                 # a single linear layer is not an FCBlock
])
def test_check_rejects_unsupported(dims, msg):
    lib = _native.load_library()
    d = _desc(dims)
    assert lib.siren_mlp_check(ctypes.byref(d)) != 0
    assert msg in _native.last_error()


def test_saved_bytes_formula_bf16():
    """saved = prepared bf16 weights (W, W^T and the fused forward's fragment-order copy of each
    MFMA layer, plus the register-resident forward's 4 KiB output-layer fragments and its 4-byte
    weight bound per hidden row) + one 16-bit phase tensor per sine layer except the first
    (recomputed from x by the backward) — 2 bytes per activation element."""
    lib = _native.load_library()
    rows = 512 * 512
    d = _desc([2, 256, 256, 256, 256, 1], rows_per_batch=rows)
    got = lib.siren_mlp_saved_bytes(ctypes.byref(d))
    weights = 3 * 3 * 256 * 256 * 2 + 4096 + 3 * 256 * 4
    phases = 3 * rows * 256 * 2
    assert got == weights + phases


def test_saved_bytes_ragged_rows_recompute_p0():
    """Row counts whose x is not a whole number of 16-byte pieces (rows x C odd multiples of 2)
    also rebuild P_0 from x in the backward: no layer-0 phase tensor is kept."""
    lib = _native.load_library()
    for rows, batch, batched in ((16385, 1, False), (16415, 5, True)):
        d = _desc([2, 256, 256, 256, 256, 1], rows_per_batch=rows, batch=batch, weights_batched=batched)
        got = lib.siren_mlp_saved_bytes(ctypes.byref(d))
        weights = batch * (3 * 3 * 256 * 256 * 2 + 4096 + 3 * 256 * 4)
        assert got == weights + 3 * batch * rows * 256 * 2, (rows, batch)


def test_config_options():
    lib = _native.load_library()
    assert lib.siren_config_get(b"fused_forward") in (0, 1)
    assert lib.siren_config_get(b"nope") == -1
    assert lib.siren_config_get(b"freg_magic") == 0
    assert lib.siren_config_set(b"nope", 1) != 0
    assert "unknown option" in _native.last_error()


def test_empty_input_rejected():
    lib = _native.load_library()
    d = _desc([2, 64, 1], rows_per_batch=0)
    assert lib.siren_mlp_check(ctypes.byref(d)) != 0
    assert "empty" in _native.last_error()


def test_adam_rejects_bad_descriptors():
    lib = _native.load_library()
    d = _native.SirenAdamDesc()
    d.num_tensors = 49
    assert lib.siren_adam_step(ctypes.byref(d), None) != 0
    d.num_tensors = 1  # null pointers
    assert lib.siren_adam_step(ctypes.byref(d), None) != 0
    d.num_tensors = 0
    assert lib.siren_adam_step(ctypes.byref(d), None) == 0


def _loss_desc(**kw):
    ld = _native.SirenLossDesc()
    ld.target = ld.dy = ld.loss = ld.loss_workspace = 256
    ld.loss_workspace_bytes = int(_native.load_library().siren_sse_workspace_bytes())
    for k, v in kw.items():
        setattr(ld, k, v)
    return ld


def test_fused_loss_check_paths():
    """siren_mlp_loss_check: the bf16 register forward's shapes and (round 5) the per-layer path —
    fp32 mode, the reference's arithmetic — take the fused image loss; a sine output layer or an
    incomplete descriptor does not."""
    lib = _native.load_library()
    ok = [([2, 256, 256, 256, 256, 1], _native.PREC_BF16, {}),
          ([2, 256, 256, 256, 256, 1], _native.PREC_F32, {}),
          ([16, 256, 256, 256, 256, 2], _native.PREC_F32, dict(batch=32, weights_batched=True)),
          ([2, 128, 128, 3], _native.PREC_BF16, {})]
    for dims, prec, kw in ok:
        d = _desc(dims, prec=prec, rows_per_batch=16384, **kw)
        assert lib.siren_mlp_loss_check(ctypes.byref(d), ctypes.byref(_loss_desc())) == 0, (dims, _native.last_error())
    d = _desc([2, 256, 256, 1], prec=_native.PREC_F32, rows_per_batch=4096, outermost_linear=False)
    assert lib.siren_mlp_loss_check(ctypes.byref(d), ctypes.byref(_loss_desc())) != 0
    assert "outermost_linear" in _native.last_error()
    d = _desc([2, 256, 256, 1], prec=_native.PREC_F32, rows_per_batch=4096)
    bad = _loss_desc(k0=256)  # k0 without mask / y_dc
    assert lib.siren_mlp_loss_check(ctypes.byref(d), ctypes.byref(bad)) != 0
    assert "together" in _native.last_error()
