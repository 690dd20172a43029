"""Counterpart of experiment_scripts/train_poisson_grad_img.py (reference): fit a SIREN to the
Sobel gradients of the 256^2 cameraman (gradients_mse: analytic gradient + its adjoint)."""
from _common import base_parser  # noqa: E402

from torch.utils.data import DataLoader

from siren_mri_amd import dataio, loss_functions, modules, training

opt = base_parser().parse_args()

img_dataset = dataio.Camera()
coord_dataset = dataio.Implicit2DWrapper(img_dataset, sidelength=256, compute_diff="gradients")
dataloader = DataLoader(coord_dataset, shuffle=True, batch_size=opt.batch_size, pin_memory=True, num_workers=0)

if opt.model_type != "sine":
    raise NotImplementedError("the native path covers type='sine'")
model = modules.SingleBVPNet(type="sine", mode="mlp", sidelength=(256, 256), precision=opt.precision)
model.cuda()


def summary_fn(model, model_input, gt, model_output, writer, total_steps):
    print(f"step {total_steps}", flush=True)


training.train(model=model, train_dataloader=dataloader, epochs=opt.num_epochs, lr=opt.lr,
               steps_til_summary=opt.steps_til_summary, epochs_til_checkpoint=opt.epochs_til_ckpt,
               model_dir=f"{opt.logging_root}/{opt.experiment_name}", overwrite=opt.overwrite, loss_fn=loss_functions.gradients_mse,
               summary_fn=summary_fn, double_precision=False)
