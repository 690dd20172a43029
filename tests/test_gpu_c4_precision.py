"""GPU: config 4 at equal steps in the precision it is benched in (bf16 encoder + bf16 SIREN) against
the reference's arithmetic (fp32 encoder on MIOpen + fp32 SIREN), VERDICT r5 missing 1 / weak 1.

The reference trains configs 4/5 in fp32 (encoder modules.py:340-380,433-450, hypernetwork
meta_modules.py:175-225, loop train_mri_neural_process.py:182-185 through training.py:19-146).
Both models start from ONE seed (identical parameters, checked), see the same 32 training slices
of 128^2 k-space every step (bench.py's c4 step: FF transform, DC, image_hypernetwork_loss,
clip_grad_norm_(1.0), Adam(5.57e-5)) and are evaluated on 8 held-out slices (another data seed):

* steps 50 and 100 (the fit's slow phase): the validation slices' PSNR — the reference's own metric
  for this script (utils.write_image_summary_small -> write_psnr on model_out,
  utils.py:216-239,593-616) — and the image-domain PSNR of |ifft2(k-space)| agree within 0.1 dB
  (north_star's PSNR criterion); training and validation loss within 3 %.
* step 200: the fit is in a steep descent (3e-3 -> 1e-3 within ~50 steps) where a few steps' lead
  or lag moves the instantaneous loss by tens of percent, and the reference arithmetic does not
  reproduce itself there: MIOpen's fp32 convolution gradients are not run-to-run deterministic, and
  three fp32 runs of this test gave val loss 2.73e-4 / 3.41e-4 / 2.67e-4, write_psnr 45.575 /
  45.477 / 45.569 dB, image PSNR 27.298 / 27.163 / 27.297 dB (spread 28 %, 0.10 dB, 0.14 dB). The
  bound there is that spread with margin: PSNRs within 0.2 dB, losses within a factor 1.5.
  The three bf16 runs against them: write_psnr +0.021 / +0.072 / -0.057 dB, image PSNR +0.079 /
  +0.121 / -0.091 dB, val loss 2.57e-4 / 2.88e-4 / 3.20e-4 (profiles/r6_c4_precision.txt,
  r6_c4_precision_run2.txt, r6_c4_precision_run3.txt).
Measured at steps 50 / 100: train loss 3.2125e-3 / 3.2124e-3, 2.9943e-3 / 2.9951e-3; val PSNR
44.914 / 44.914, 44.947 / 44.947 dB; image PSNR 26.280 / 26.280, 26.270 / 26.269 dB (bf16 / fp32).
"""
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
CHECK = (50, 100, 200)


def _image_psnr(pred_k, gt_k, res):
    """PSNR of the magnitude images |ifft2(ifftshift(k))| (k-space [B, N, 2] real/imag), each
    normalised by the ground truth's maximum."""
    def mag(k):
        k = k.detach().double().reshape(k.shape[0], res, res, 2)
        c = torch.complex(k[..., 0], k[..., 1])
        return torch.fft.ifft2(torch.fft.ifftshift(c, dim=(-2, -1))).abs()
    p, t = mag(pred_k), mag(gt_k)
    s = t.amax(dim=(-2, -1), keepdim=True)
    mse = ((p / s - t / s) ** 2).mean(dim=(-2, -1))
    return float((10 * torch.log10(1.0 / mse)).mean())


def _run(precision, encoder_precision, monkeypatch, val):
    import bench
    from siren_mri_amd import dataio, utils
    monkeypatch.setattr(sys, "argv", ["bench.py", "--no-psnr", "--no-cpu-baseline", "--no-other-configs",
                                      "--config", "c4"])
    args = bench.parse()
    wl = bench.build_c4(args, DEV, 0, 1, precision, encoder_precision=encoder_precision)
    model, ff, loss_fn = wl.extra["model"], wl.extra["ff"], wl.extra["loss_fn"]
    vinp, vgt = val
    res = bench.C4["res"]
    init = [p.detach().clone() for p in model.parameters()]
    losses, rec = [], {}
    for s in range(max(CHECK) + 1):
        if s in CHECK:
            with torch.no_grad():
                model.eval()
                out = model(ff.model_input(model, dict(vinp)))
                model.train()
                vloss = float(loss_fn(out, vgt)["img_loss"].mean())
                y = out["model_out"]
                ref_psnr = float(np.mean(utils.batch_psnr(dataio.lin2img(y, (res, res)),
                                                          dataio.lin2img(vgt["img"], (res, res)))))
                rec[s] = dict(val_loss=vloss, psnr=ref_psnr, image_psnr=_image_psnr(y, vgt["img"], res))
        losses.append(wl.step().detach())
        if s % 25 == 0 or s < 3:  # progress (a silent GPU command is taken to be hung)
            print(f"  [{precision}/{encoder_precision}] step {s}", flush=True)
    torch.cuda.synchronize()
    return init, [float(v) for v in torch.stack(losses).cpu()], rec


def test_c4_bf16_matches_fp32_at_equal_steps(monkeypatch):
    import bench
    val = bench.c4_batch(DEV, 8, seed=1)
    i16, l16, r16 = _run("bf16", "bf16", monkeypatch, val)
    i32, l32, r32 = _run("fp32", "fp32", monkeypatch, val)
    for a, b in zip(i16, i32):
        assert torch.equal(a, b), "the two models must start from the same parameters"
    print("\n[C4 bf16 vs fp32, 200 steps, 32 training slices, 8 validation slices]")
    for s in CHECK:
        print(f"  step {s:3d}: train loss {l16[s]:.6g} vs {l32[s]:.6g}; val loss {r16[s]['val_loss']:.6g} vs "
              f"{r32[s]['val_loss']:.6g}; val PSNR (write_psnr) {r16[s]['psnr']:.3f} vs {r32[s]['psnr']:.3f} dB; "
              f"image PSNR {r16[s]['image_psnr']:.3f} vs {r32[s]['image_psnr']:.3f} dB")
    for s in CHECK:
        slow = s <= 100
        for name, a, b in (("train loss", l16[s], l32[s]), ("val loss", r16[s]["val_loss"], r32[s]["val_loss"])):
            if slow:
                assert a == pytest.approx(b, rel=3e-2), f"{name} at step {s}"
            else:
                assert b / 1.5 <= a <= 1.5 * b, f"{name} at step {s}: outside the fp32 run-to-run spread"
        for key in ("psnr", "image_psnr"):
            d = r16[s][key] - r32[s][key]
            assert abs(d) <= (0.1 if slow else 0.2), f"{key} at step {s}: bf16 - fp32 = {d:.3f} dB"
