"""Counterpart of experiment_scripts/train_img.py (reference): fit a SIREN to the 512^2
cameraman with image_mse + Adam (the BASELINE metric's workload)."""
from _common import base_parser, psnr_summary  # noqa: E402  (also puts the repo on sys.path)

from functools import partial

from torch.utils.data import DataLoader

from siren_mri_amd import dataio, loss_functions, modules, training

opt = base_parser().parse_args()

img_dataset = dataio.Camera()
coord_dataset = dataio.Implicit2DWrapper(img_dataset, sidelength=512, compute_diff="all")
image_resolution = (512, 512)
dataloader = DataLoader(coord_dataset, shuffle=True, batch_size=opt.batch_size, pin_memory=True, num_workers=0)

if opt.model_type in ("sine", "relu", "tanh", "selu", "elu", "softplus"):
    model = modules.SingleBVPNet(type=opt.model_type, mode="mlp", sidelength=image_resolution,
                                 precision=opt.precision)
else:
    raise NotImplementedError(opt.model_type)
model.cuda()

root_path = f"{opt.logging_root}/{opt.experiment_name}"
training.train(model=model, train_dataloader=dataloader, epochs=opt.num_epochs, lr=opt.lr,
               steps_til_summary=opt.steps_til_summary, epochs_til_checkpoint=opt.epochs_til_ckpt,
               model_dir=root_path, overwrite=opt.overwrite, loss_fn=partial(loss_functions.image_mse, None), summary_fn=psnr_summary())
