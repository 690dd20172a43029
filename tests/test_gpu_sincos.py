"""GPU: the fp32 mode's sin / cos (siren_common.h sin_f32 / cos_f32: Cody-Waite reduction by pi/2
and minimax polynomials) against float64, through the C ABI's siren_sincos_f32.

These functions replace torch.sin in Sine.forward (modules.py:35-38) and its derivative cos in the
fp32 kernels (forward epilogues, backward cos weighting, tangent streams). SIREN phases w0 (W x + b)
reach a few hundred radians at w0 = 30 (first layer: |x| <= 1, |W| <= 1/in, |b| <= 1/sqrt(in)
scaled by 30; hidden layers: |sum| grows with the fit), so the range checked is |x| <= 2000 rad,
dense around the reduction's quadrant boundaries, plus arguments past the Cody-Waite range (those
take OCML's functions through a call). Tolerance: 2.5e-7 absolute (about 2 ulp of 1.0), what
float32 libm itself reaches.
"""
import ctypes
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
TOL = 2.5e-7


def run(x: np.ndarray, impl: int):
    from siren_mri_amd import _native
    xd = torch.from_numpy(x.astype(np.float32)).to(DEV)
    s = torch.empty_like(xd)
    c = torch.empty_like(xd)
    rc = _native.lib().siren_sincos_f32(xd.data_ptr(), s.data_ptr(), c.data_ptr(), xd.numel(), impl,
                                        _native.stream_handle(DEV))
    _native.check(rc, "siren_sincos_f32")
    torch.cuda.synchronize()
    return s.cpu().numpy().astype(np.float64), c.cpu().numpy().astype(np.float64)


def arguments():
    rng = np.random.default_rng(0)
    parts = [
        rng.uniform(-2000.0, 2000.0, 1 << 20),
        rng.uniform(-4.0, 4.0, 1 << 18),
        # around k pi/2 for k up to 1300 (the reduction's quadrant switches)
        (np.arange(-1300, 1301)[:, None] * (math.pi / 2) + np.linspace(-1e-3, 1e-3, 65)[None, :]).ravel(),
        np.array([0.0, -0.0, 1e-30, -1e-30, 1e-7, math.pi, -math.pi, 99999.0, -99999.0]),
    ]
    return np.concatenate(parts).astype(np.float32)


@pytest.mark.parametrize("impl", [0, 1], ids=["cody_waite", "ocml"])
def test_sincos_f32_against_float64(impl):
    x = arguments()
    s, c = run(x, impl)
    xd = x.astype(np.float64)
    es = np.abs(s - np.sin(xd)).max()
    ec = np.abs(c - np.cos(xd)).max()
    print(f"\n[sincos impl {impl}] max |err| sin {es:.3e} cos {ec:.3e} over {x.size} args")
    assert es <= TOL and ec <= TOL, (es, ec)


def test_sincos_f32_far_arguments_take_the_library_path():
    x = np.array([1.0e5, -1.0e5, 3.3e6, -7.7e7, 1.0e20], dtype=np.float32)
    s0, c0 = run(x, 0)
    s1, c1 = run(x, 1)
    assert np.array_equal(s0, s1) and np.array_equal(c0, c1)


def test_sincos_f32_nonfinite():
    x = np.array([np.inf, -np.inf, np.nan], dtype=np.float32)
    s, c = run(x, 0)
    assert np.all(np.isnan(s)) and np.all(np.isnan(c))
