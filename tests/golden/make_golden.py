"""Generate golden vectors from the REAL reference (jonbmartin/siren_mri at /root/reference).

Run ONLY in the survey/build container (the reference is not present on the GPU box):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

It imports the reference with in-process stubs for its unused heavy dependencies (SURVEY.md
§A.2: h5py, cv2, skimage, skvideo, cmapy, torchvision, tensorboard) and records, as small
.npz fixtures in tests/golden/, what the reference itself computes (PyTorch 2.10 CPU, fp32):

  mgrid.npz        dataio.get_mgrid / lin2img
  init.npz         SingleBVPNet initial parameters (seeded) — RNG-order pin (modules.py:68-90,641-654)
  forward.npz      SingleBVPNet model_out + diff_operators.gradient + laplace on a 16^2 grid
  losses.npz       image_mse (with/without the 128^2 high-frequency mask), create_circular_mask_torch,
                   gradients_mse, hypernet losses
  train_c1.npz     training.train: 10 steps, 64^2 cameraman, 3x256 (num_hidden_layers=1), Adam 1e-4
  train_c3.npz     training.train: 10 steps, 32^2 cameraman, gradients_mse (sobel GT), 2x64
  psnr_c1.npz      PSNR trajectory at steps 0/50/100/200/500 (64^2 cameraman, nh=3 and nh=1)
  hypernet.npz     ConvolutionalNeuralProcessImplicit2DHypernetFourierFeatures forward (reduced
                   sizes, B=2) on IRData-derived k-space + state_dict + losses
  features.npz     GaussianFourierFeatureTransform + DataConsistencyInKspace
  ../../siren_mri_amd/assets/camera512_u8.npz  the cameraman (uint8, skimage's data dir), config 1 input

The reference's own bugs are worked around exactly as the build documents them:
high_freq=False off 128^2 (bug 0.2), training.train's final UnboundLocalError is caught after it
has written its outputs (bug 0.3), `.cuda()` is a no-op on CPU (bug 0.4), the hypernet is built
without the unsupported `device=` argument (bug 0.5). No reference source is copied.
"""
import os
import shutil
import sys
import tempfile
import types
from functools import partial

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
ASSETS = os.path.join(os.path.dirname(os.path.dirname(OUT)), "siren_mri_amd", "assets")
CAMERA = "/opt/conda/lib/python3.9/site-packages/skimage/data/camera.png"


def import_reference():
    sys.path.insert(0, REF)
    tm = types.ModuleType("torchmeta")
    tm.__path__ = [os.path.join(REF, "torchmeta")]
    sys.modules["torchmeta"] = tm

    class _Stub(types.ModuleType):
        def __getattr__(self, k):
            if k.startswith("__"):
                raise AttributeError(k)
            return _Stub(self.__name__ + "." + k)

        def __call__(self, *a, **k):
            return _Stub("x")

    for n in ["h5py", "cv2", "skimage", "skimage.filters", "skimage.measure", "skvideo", "skvideo.io",
              "cmapy", "torchvision", "torchvision.transforms", "torchvision.utils"]:
        m = _Stub(n)
        m.__path__ = []
        sys.modules[n] = m
    tb = types.ModuleType("torch.utils.tensorboard")

    class SummaryWriter:
        def __init__(self, *a, **k):
            pass

        def __getattr__(self, k):
            return lambda *a, **kw: None

    tb.SummaryWriter = SummaryWriter
    sys.modules["torch.utils.tensorboard"] = tb
    torch.Tensor.cuda = lambda self, *a, **k: self  # bug 0.4 (modules.py:203) on a CPU host
    import builtins
    _print = builtins.print
    builtins.print = lambda *a, **k: None  # SingleBVPNet.__init__ prints the model
    import modules, diff_operators, meta_modules, features, data_consistency, dataio, loss_functions, training, utils  # noqa
    builtins.print = _print
    return types.SimpleNamespace(modules=modules, diff_operators=diff_operators, meta_modules=meta_modules,
                                 features=features, data_consistency=data_consistency, dataio=dataio,
                                 loss_functions=loss_functions, training=training, utils=utils)


def camera_u8():
    from PIL import Image
    return np.array(Image.open(CAMERA).convert("L"), dtype=np.uint8)


def camera_tensor(side):
    """Implicit2DWrapper(Camera) transform restated: PIL bilinear Resize -> ToTensor -> Normalize(.5,.5)."""
    from PIL import Image
    img = Image.fromarray(camera_u8())
    if side != 512:
        img = img.resize((side, side), Image.BILINEAR)
    a = np.asarray(img, dtype=np.float32) / 255.0
    return torch.from_numpy((a - 0.5) / 0.5)[None]  # [1, H, W]


def state_arrays(model, prefix=""):
    return {prefix + k: v.detach().cpu().numpy().copy() for k, v in model.state_dict().items()}


def quiet(fn, *a, **k):
    import builtins
    _p = builtins.print
    builtins.print = lambda *x, **y: None
    try:
        return fn(*a, **k)
    finally:
        builtins.print = _p


def run_train(R, model, coords, gt, loss_fn, steps, lr, clip=False):
    """Drive the reference's own training.train on one full-batch image for `steps` epochs."""
    d = tempfile.mkdtemp()
    mdir = os.path.join(d, "run")
    loader = [({"coords": coords}, gt)]
    try:
        quiet(R.training.train, model=model, train_dataloader=loader, epochs=steps, lr=lr,
              steps_til_summary=10 ** 9, epochs_til_checkpoint=10 ** 9, model_dir=mdir,
              loss_fn=loss_fn, summary_fn=lambda *a, **k: None, clip_grad=clip, device="cpu")
    except UnboundLocalError:
        pass  # bug 0.3: raised after model_final.pth / train_losses_final.txt are written
    losses = np.loadtxt(os.path.join(mdir, "checkpoints", "train_losses_final.txt"))
    final = torch.load(os.path.join(mdir, "checkpoints", "model_final.pth"), weights_only=True)
    shutil.rmtree(d)
    return np.atleast_1d(losses).astype(np.float64), {k: v.numpy() for k, v in final.items()}


def main():
    R = import_reference()
    torch.set_num_threads(8)
    out = {}

    # mgrid / lin2img -----------------------------------------------------------------------
    g5 = R.dataio.get_mgrid(5).numpy()
    g46 = R.dataio.get_mgrid((4, 6)).numpy()
    t = torch.arange(2 * 16 * 3, dtype=torch.float32).view(2, 16, 3)
    np.savez_compressed(os.path.join(OUT, "mgrid.npz"), mgrid5=g5, mgrid4x6=g46,
                        lin2img_in=t.numpy(), lin2img_out=R.dataio.lin2img(t).numpy())

    # init ----------------------------------------------------------------------------------
    init = {}
    for seed, (hid, nh) in [(0, (64, 1)), (1, (64, 1)), (0, (256, 3))]:
        torch.manual_seed(seed)
        m = quiet(R.modules.SingleBVPNet, type="sine", mode="mlp", hidden_features=hid,
                  num_hidden_layers=nh, sidelength=(8, 8))
        for k, v in state_arrays(m).items():
            init[f"s{seed}_h{hid}_n{nh}/{k}"] = v
    np.savez_compressed(os.path.join(OUT, "init.npz"), **init)

    # forward / gradient / laplace ----------------------------------------------------------
    torch.manual_seed(2)
    m = quiet(R.modules.SingleBVPNet, type="sine", mode="mlp", hidden_features=64, num_hidden_layers=2,
              sidelength=(16, 16))
    coords = R.dataio.get_mgrid(16)[None]
    o = m({"coords": coords})
    grad = R.diff_operators.gradient(o["model_out"], o["model_in"])
    lap = R.diff_operators.laplace(o["model_out"], o["model_in"])
    # batched (hypernetwork-style) params through BatchLinear: B=2 perturbed copies
    params = {k: torch.stack([v, v * 1.05]) for k, v in m.state_dict().items()}
    ob = m({"coords": coords.repeat(2, 1, 1)}, params=params)
    np.savez_compressed(os.path.join(OUT, "forward.npz"), coords=coords.numpy(),
                        model_out=o["model_out"].detach().numpy(), gradient=grad.detach().numpy(),
                        laplace=lap.detach().numpy(), batched_out=ob["model_out"].detach().numpy(),
                        **{"param/" + k: v for k, v in state_arrays(m).items()})

    # losses ----------------------------------------------------------------------------------
    gen = torch.Generator().manual_seed(11)
    pred = torch.randn(2, 128 * 128, 2, generator=gen)
    tgt = torch.randn(2, 128 * 128, 2, generator=gen)
    lm = R.loss_functions.image_mse(None, {"model_out": pred}, {"img": tgt})["img_loss"]
    lp = R.loss_functions.image_mse(None, {"model_out": pred}, {"img": tgt}, high_freq=False)["img_loss"]
    mask = R.utils.create_circular_mask_torch(129, 129, center=None, radius=20)
    latent = torch.randn(2, 16, generator=gen)
    hp = {"a": torch.randn(2, 8, 4, generator=gen), "b": torch.randn(2, 8, generator=gen)}
    hl = R.loss_functions.image_hypernetwork_loss(None, 2.78e-8, 6.4e-6,
                                                  {"model_out": pred, "latent_vec": latent, "hypo_params": hp},
                                                  {"img": tgt})
    gsm = R.loss_functions.gradients_mse(o, {"gradients": torch.ones(1, 256, 2) * 0.3})["gradients_loss"]
    lapm = R.loss_functions.laplace_mse(o, {"laplace": torch.ones(1, 256, 1) * 0.1})["laplace_loss"]
    np.savez_compressed(os.path.join(OUT, "losses.npz"), pred=pred.numpy(), tgt=tgt.numpy(),
                        image_mse_hf=lm.item(), image_mse_plain=lp.item(), circ_mask=mask.numpy(),
                        latent=latent.numpy(), hp_a=hp["a"].numpy(), hp_b=hp["b"].numpy(),
                        hyper_img=hl["img_loss"].item(), hyper_latent=hl["latent_loss"].item(),
                        hyper_weight=hl["hypo_weight_loss"].item(), gradients_mse=gsm.item(),
                        laplace_mse=lapm.item())

    # camera image ------------------------------------------------------------------------------
    # (written into the package's data assets: siren_mri_amd/assets/, the product reads it from there)
    np.savez_compressed(os.path.join(ASSETS, "camera512_u8.npz"), img=camera_u8())

    # config 1: training.train 10 steps (64^2, 3x256 = nh 1) ----------------------------------
    img64 = camera_tensor(64)
    gt = {"img": img64.permute(1, 2, 0).reshape(1, -1, 1)}
    coords64 = R.dataio.get_mgrid(64)[None]
    torch.manual_seed(0)
    m = quiet(R.modules.SingleBVPNet, type="sine", mode="mlp", hidden_features=256, num_hidden_layers=1,
              sidelength=(64, 64))
    init_sd = state_arrays(m, "init/")
    loss_fn = partial(R.loss_functions.image_mse, None, high_freq=False)  # bug 0.2 deviation
    losses, final = run_train(R, m, coords64, gt, loss_fn, steps=10, lr=1e-4)
    np.savez_compressed(os.path.join(OUT, "train_c1.npz"), losses=losses, img=gt["img"].numpy(),
                        **init_sd, **{"final/" + k: v for k, v in final.items()})

    # config 3 analogue: gradients_mse, 32^2, 2x64 -----------------------------------------------
    import scipy.ndimage
    img32 = camera_tensor(32) * 10.0
    gx = scipy.ndimage.sobel(img32.numpy(), axis=1).squeeze(0)[..., None]
    gy = scipy.ndimage.sobel(img32.numpy(), axis=2).squeeze(0)[..., None]
    grads = torch.cat((torch.from_numpy(gx).reshape(-1, 1), torch.from_numpy(gy).reshape(-1, 1)), dim=-1)[None]
    torch.manual_seed(3)
    m = quiet(R.modules.SingleBVPNet, type="sine", mode="mlp", hidden_features=64, num_hidden_layers=2,
              sidelength=(32, 32))
    init_sd = state_arrays(m, "init/")
    losses, final = run_train(R, m, R.dataio.get_mgrid(32)[None], {"gradients": grads},
                              R.loss_functions.gradients_mse, steps=10, lr=1e-4)
    np.savez_compressed(os.path.join(OUT, "train_c3.npz"), losses=losses, gradients=grads.numpy(),
                        **init_sd, **{"final/" + k: v for k, v in final.items()})

    # PSNR trajectories -----------------------------------------------------------
    psnr = {}
    for nh in (3, 1):
        torch.manual_seed(0)
        m = quiet(R.modules.SingleBVPNet, type="sine", mode="mlp", hidden_features=256, num_hidden_layers=nh,
                  sidelength=(64, 64))
        opt = torch.optim.Adam(lr=1e-4, params=m.parameters())
        vals, losses = [], []
        for step in range(501):
            o = m({"coords": coords64})
            if step in (0, 50, 100, 200, 500):
                p = R.dataio.lin2img(o["model_out"].detach()).numpy()[0, 0]
                t_ = img64.numpy()[0]
                pp = np.clip(p / 2 + 0.5, 0, 1).astype(np.float64)
                tt = (t_ / 2 + 0.5).astype(np.float64)
                vals.append(10 * np.log10(1.0 / np.mean((pp - tt) ** 2)))
            loss = loss_fn(o, gt)["img_loss"]
            losses.append(loss.item())
            loss.backward()
            opt.step()
            opt.zero_grad()
        psnr[f"nh{nh}_psnr"] = np.array(vals)
        psnr[f"nh{nh}_loss"] = np.array(losses)
    psnr["steps"] = np.array([0, 50, 100, 200, 500])
    np.savez_compressed(os.path.join(OUT, "psnr_c1.npz"), **psnr)

    # hypernetwork forward (config 4 architecture, reduced) ------------------------------------
    import scipy.io as sio
    ir = sio.loadmat(os.path.join(REF, "data", "IRData.mat"))["IRData"]  # [128,128,1,9]
    ks = []
    for s in range(2):
        sl = ir[:, :, 0, s].astype(np.float64)
        sl = sl / np.abs(sl).max()
        k = np.fft.fftshift(np.fft.fft2(sl))
        k = k / np.abs(k).max()
        ks.append(np.stack([k.real, k.imag]).astype(np.float32) * 2.0)
    kspace = torch.from_numpy(np.ascontiguousarray(np.stack(ks))).contiguous()  # [2,2,128,128]
    rs = np.random.RandomState(5)
    mask = torch.zeros_like(kspace)
    for b in range(2):
        rows = rs.permutation(128)[: int(0.3333 * 128)]
        mask[b, :, rows, :] = 1
        mask[b, :, 60:68, :] = 1
    img_sparse = mask * kspace
    torch.manual_seed(0)
    ff = R.features.GaussianFourierFeatureTransform(2, 8, 21, device="cpu")
    Bmat = ff.get_B().clone()
    torch.manual_seed(1)
    model = quiet(R.meta_modules.ConvolutionalNeuralProcessImplicit2DHypernetFourierFeatures,
                  in_features=16, out_features=2, image_resolution=(128, 128), fourier_features_size=16,
                  latent_dim=16, hidden_features=32, num_hidden_layers=1, hyper_hidden_features=16,
                  hyper_hidden_layers=1, conv_kernel_size=3, num_conv_res_blocks=1, w0=30)
    coords = R.dataio.get_mgrid(128)[None].repeat(2, 1, 1)
    mi = {"coords": ff(coords), "img_sparse": img_sparse, "dc_mask": mask}
    o = model(mi)
    gtk = {"img": kspace.permute(0, 2, 3, 1).reshape(2, -1, 2)}
    hl = R.loss_functions.image_hypernetwork_loss(None, 2.78e-8, 6.4e-6, o, gtk)
    total = hl["img_loss"].mean() + hl["latent_loss"].mean() + hl["hypo_weight_loss"].mean()
    total.backward()
    gnorm = {"gradnorm/" + n: np.float64(p.grad.norm().item()) for n, p in model.named_parameters()
             if p.grad is not None}
    np.savez_compressed(os.path.join(OUT, "hypernet.npz"), kspace=kspace.numpy(), mask=mask.numpy().astype(np.uint8),
                        B=Bmat.numpy(), model_out=o["model_out"].detach().numpy(),
                        latent=o["latent_vec"].detach().numpy(), img_loss=hl["img_loss"].item(),
                        latent_loss=hl["latent_loss"].item(), hypo_weight_loss=hl["hypo_weight_loss"].item(),
                        **{"state/" + k: v for k, v in state_arrays(model).items()}, **gnorm)

    # Fourier features + data consistency ------------------------------------------------------------
    x = torch.rand(2, 10, 2, generator=gen) * 2 - 1
    fx = ff(x)
    pred = torch.randn(2, 16, 2, generator=gen)
    k0 = torch.randn(2, 2, 4, 4, generator=gen)
    mk = (torch.rand(2, 2, 4, 4, generator=gen) > 0.5).float()
    dc = R.data_consistency.DataConsistencyInKspace(noise_lvl=None)(pred, k0, mk)
    np.savez_compressed(os.path.join(OUT, "features.npz"), B=Bmat.numpy(), x=x.numpy(), ff=fx.numpy(),
                        pred=pred.numpy(), k0=k0.numpy(), mask=mk.numpy(), dc=dc.numpy())
    for f in sorted(os.listdir(OUT)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(OUT, f)))


if __name__ == "__main__":
    main()
