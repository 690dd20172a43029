"""GPU: the k-space epilogue of the hypernetwork SIREN (siren_kspace.hip)
against the reference's recorded values and the fp64 oracle.

  DataConsistencyInKspace (data_consistency.py:32-48): native op, bit-equal to the reference's
      output recorded in features.npz; its backward (1 - m) g exact.
  image_mse (loss_functions.py:66-101): native op on the [B, N, C] layout against losses.npz
      (image_mse_hf, image_mse_plain: the reference's values at 128^2, B = 2).
  DC + image_mse fused: loss and dL/dpred against the oracle's autograd in fp64 (noiseless and
      noisy DC), and fewer kernel launches per forward + backward than the unfused chain.
"""
import os

import numpy as np
import pytest
import torch

from oracle import siren_oracle as orc

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_dc_matches_reference_bitwise():
    from siren_mri_amd.data_consistency import DataConsistencyInKspace
    d = np.load(os.path.join(G, "features.npz"), allow_pickle=False)
    out = DataConsistencyInKspace()(torch.from_numpy(d["pred"]).to(DEV), torch.from_numpy(d["k0"]).to(DEV),
                                    torch.from_numpy(d["mask"]).to(DEV))
    assert hasattr(out, "_siren_dc")  # the native op ran
    assert np.array_equal(out.cpu().numpy(), d["dc"])


@pytest.mark.parametrize("noise", [None, 0.3])
def test_dc_backward(noise):
    from siren_mri_amd.data_consistency import DataConsistencyInKspace
    g = torch.Generator().manual_seed(1)
    pred = torch.randn(3, 64, 2, generator=g)
    k0 = torch.randn(3, 2, 8, 8, generator=g)
    mask = (torch.rand(3, 2, 8, 8, generator=g) < 0.4).float()
    up = torch.randn(3, 64, 2, generator=g)
    p = pred.to(DEV).requires_grad_(True)
    out = DataConsistencyInKspace(noise)(p, k0.to(DEV), mask.to(DEV))
    (out * up.to(DEV)).sum().backward()
    pr = pred.double().requires_grad_(True)
    ref = orc.data_consistency(pr, k0.double(), mask.double()) if noise is None else None
    if ref is None:
        k = k0.double().permute(0, 2, 3, 1).reshape(3, -1, 2)
        m = mask.double().permute(0, 2, 3, 1).reshape(3, -1, 2)
        ref = (1 - m) * pr + m * (pr + noise * k) / (1 + noise)
    (ref * up.double()).sum().backward()
    assert orc.norm_rel(out.detach().cpu(), ref.detach()) < 1e-7
    assert orc.norm_rel(p.grad.cpu(), pr.grad) < 1e-7


def test_image_mse_native_matches_reference_values():
    from siren_mri_amd import loss_functions
    d = np.load(os.path.join(G, "losses.npz"), allow_pickle=False)
    out = {"model_out": torch.from_numpy(d["pred"]).to(DEV)}
    gt = {"img": torch.from_numpy(d["tgt"]).to(DEV)}
    hf = loss_functions.image_mse(None, out, gt, high_freq=True)["img_loss"]
    plain = loss_functions.image_mse(None, out, gt, high_freq=False)["img_loss"]
    assert float(hf) == pytest.approx(float(d["image_mse_hf"]), rel=2e-6)
    assert float(plain) == pytest.approx(float(d["image_mse_plain"]), rel=2e-6)


@pytest.mark.parametrize("noise", [None, 0.25])
@pytest.mark.parametrize("high_freq", [True, False])
def test_fused_dc_image_mse_against_oracle(noise, high_freq):
    from siren_mri_amd import loss_functions
    from siren_mri_amd.data_consistency import DataConsistencyInKspace
    B, side = 3, 128
    g = torch.Generator().manual_seed(7)
    pred = torch.randn(B, side * side, 2, generator=g)
    k0 = torch.randn(B, 2, side, side, generator=g)
    mask = (torch.rand(B, 2, side, side, generator=g) < 0.33).float()
    tgt = torch.randn(B, side * side, 2, generator=g)
    p = pred.to(DEV).requires_grad_(True)
    y = DataConsistencyInKspace(noise)(p, k0.to(DEV), mask.to(DEV))
    loss = loss_functions.image_mse(None, {"model_out": y}, {"img": tgt.to(DEV)}, high_freq=high_freq)["img_loss"]
    (3.0 * loss).backward()
    pr = pred.double().requires_grad_(True)
    k = k0.double().permute(0, 2, 3, 1).reshape(B, -1, 2)
    m = mask.double().permute(0, 2, 3, 1).reshape(B, -1, 2)
    yr = (1 - m) * pr + (m * k if noise is None else m * (pr + noise * k) / (1 + noise))
    ref = orc.image_mse(None, {"model_out": yr}, {"img": tgt.double()}, high_freq=high_freq)["img_loss"]
    (3.0 * ref).backward()
    assert float(loss) == pytest.approx(float(ref), rel=1e-5)
    assert orc.norm_rel(p.grad.cpu(), pr.grad) < 1e-6


def _launches(fn):
    from torch.profiler import ProfilerActivity, profile
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        fn()
        torch.cuda.synchronize()
    return sum(1 for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA)


def test_fusion_removes_launches():
    """DC + image_mse forward and backward: the fused op launches fewer kernels than the chain."""
    from siren_mri_amd import loss_functions
    from siren_mri_amd.data_consistency import DataConsistencyInKspace
    B, side = 4, 128
    g = torch.Generator().manual_seed(3)
    pred = torch.randn(B, side * side, 2, generator=g).to(DEV)
    k0 = torch.randn(B, 2, side, side, generator=g).to(DEV)
    mask = (torch.rand(B, 2, side, side, generator=g) < 0.33).float().to(DEV)
    tgt = torch.randn(B, side * side, 2, generator=g).to(DEV)
    dc = DataConsistencyInKspace()

    def step():
        p = pred.clone().requires_grad_(True)
        loss = loss_functions.image_mse(None, {"model_out": dc(p, k0, mask)}, {"img": tgt})["img_loss"]
        loss.backward()
        return p.grad

    g_fused = step()
    n_fused = _launches(step)
    loss_functions.set_kspace_fusion(False)
    try:
        g_chain = step()
        n_chain = _launches(step)
    finally:
        loss_functions.set_kspace_fusion(True)
    print(f"\n[k-space epilogue] kernel launches fused {n_fused}, unfused {n_chain}")
    assert torch.allclose(g_fused, g_chain, rtol=1e-6, atol=1e-9)
    assert n_fused < n_chain
