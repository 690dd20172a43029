"""GPU: the native SSE kernels of image_mse (the k-space op of siren_kspace.hip on the [B, N, C]
layout; weighted_sse's siren_loss.hip kernels) against the autograd chain of
loss_functions.py:66-101, with and without the 128x128 high-frequency mask (utils.py:25-40)."""
import pytest
import torch

from oracle import siren_oracle as orc

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.mark.parametrize("high_freq", [True, False])
@pytest.mark.parametrize("batch,channels", [(1, 1), (3, 2)])
def test_image_mse_native_matches_autograd(high_freq, batch, channels):
    from siren_mri_amd import loss_functions
    from siren_mri_amd.dataio import lin2img
    g = torch.Generator().manual_seed(5)
    pred = torch.randn(batch, 128 * 128, channels, generator=g).to(DEV).requires_grad_(True)
    tgt = torch.randn(batch, 128 * 128, channels, generator=g).to(DEV)
    loss = loss_functions.image_mse(None, {"model_out": pred}, {"img": tgt}, high_freq=high_freq)["img_loss"]
    assert loss.grad_fn is not None and "KspaceSSE" in type(loss.grad_fn).__name__, \
        "the native k-space SSE path did not run"
    loss.backward()
    # autograd reference of the same expression (the reference's arithmetic), in fp64
    p64 = pred.detach().double().requires_grad_(True)
    diff = lin2img(p64) - lin2img(tgt.double())
    if high_freq:
        diff = loss_functions._high_freq_mask(DEV).double() * diff
    ref = (diff.abs() ** 2).sum() * (1.0 / (128 * 128))
    ref.backward()
    assert abs(float(loss) - float(ref)) <= 1e-5 * abs(float(ref))
    assert orc.norm_rel(pred.grad.double().cpu(), p64.grad.cpu()) < 1e-6


def test_weighted_sse_native_matches_autograd():
    """weighted_sse (a shard's share of image_mse in a coordinate-sharded fit): siren_loss.hip."""
    from siren_mri_amd import loss_functions
    g = torch.Generator().manual_seed(6)
    pred = torch.randn(1, 5000, 1, generator=g).to(DEV).requires_grad_(True)
    tgt = torch.randn(1, 5000, 1, generator=g).to(DEV)
    loss = loss_functions.weighted_sse(pred, tgt)
    assert "WeightedSSE" in type(loss.grad_fn).__name__
    loss.backward()
    p64 = pred.detach().double().requires_grad_(True)
    ref = ((p64 - tgt.double()) ** 2).sum() / (128 * 128)
    ref.backward()
    assert abs(float(loss) - float(ref)) <= 1e-5 * abs(float(ref))
    assert orc.norm_rel(pred.grad.double().cpu(), p64.grad.cpu()) < 1e-6


def test_high_freq_mask_is_float32():
    from siren_mri_amd import loss_functions
    m = loss_functions._high_freq_mask(torch.device("cpu"))
    assert m.dtype == torch.float32 and m.shape == (128, 128)
