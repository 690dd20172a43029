"""Counterpart of experiment_scripts/train_mri_neural_process.py (reference, config
'hand_tuned_manual'): conv-encoder hypernetwork + Fourier-feature SIREN on 128^2 k-space with
CS-Cartesian masks. fastMRI is not available: seeded synthetic k-space phantoms (bug 0.7).
The reference wraps the model in nn.DataParallel; here one process drives one GPU (use the
_ddp script for several)."""
from _common import base_parser, psnr_summary  # noqa: E402

from functools import partial

import torch
from torch.utils.data import DataLoader

from siren_mri_amd import dataio, loss_functions, meta_modules, training
from siren_mri_amd.features import GaussianFourierFeatureTransform

p = base_parser(batch_size=100, lr=6e-5, num_epochs=401, epochs_til_ckpt=10, steps_til_summary=100)
p.add_argument("--train_sparsity_range", type=int, nargs="+", default=[2000, 4000])
p.add_argument("--n_slices", type=int, default=1000, help="synthetic training slices")
opt = p.parse_args()

num_fourier_features, kl_weight, fw_weight = 60, 1.07e-9, 1.11e-7
fourier_features_scale, latent_dim = 19, 256
hidden_features_hyper, hidden_layers_hyper, hidden_layers, hidden_features = 512, 1, 3, 256
image_resolution = (128, 128)
device = torch.device("cuda:0")


def make_loader(n, seed, shuffle):
    ds = dataio.SyntheticMRIKspace(n_slices=n, image_resolution=image_resolution, seed=seed)
    coord = dataio.Implicit2DWrapper(ds, sidelength=image_resolution, image=False)
    gen = dataio.ImageGeneralizationWrapper(coord, train_sparsity_range=opt.train_sparsity_range,
                                            test_sparsity="CS_cartesian", generalization_mode="conv_cnp",
                                            device=device, seed=seed)
    return DataLoader(gen, shuffle=shuffle, batch_size=opt.batch_size, pin_memory=False, num_workers=0)


dataloader = make_loader(opt.n_slices, 0, True)
dataloader_val = make_loader(max(opt.batch_size, 16), 1, False)

model = meta_modules.ConvolutionalNeuralProcessImplicit2DHypernetFourierFeatures(
    in_features=2 * num_fourier_features, out_features=2, image_resolution=image_resolution,
    fourier_features_size=2 * num_fourier_features, latent_dim=latent_dim, hidden_features=hidden_features,
    hyper_hidden_features=hidden_features_hyper, hyper_hidden_layers=hidden_layers_hyper,
    num_hidden_layers=hidden_layers, partial_conv=False, precision=opt.precision)
model.to(device)

fourier_transformer = GaussianFourierFeatureTransform(num_input_channels=2, mapping_size_spatial=num_fourier_features,
                                                      scale=fourier_features_scale, device=device)
fourier_transformer.save_B("current_B.pt")

training.train(model=model, train_dataloader=dataloader, val_dataloader=dataloader_val, epochs=opt.num_epochs,
               lr=opt.lr, steps_til_summary=opt.steps_til_summary, epochs_til_checkpoint=opt.epochs_til_ckpt,
               model_dir=f"{opt.logging_root}/{opt.experiment_name}", overwrite=opt.overwrite,
               loss_fn=partial(loss_functions.image_hypernetwork_loss, None, kl_weight, fw_weight),
               summary_fn=psnr_summary(), clip_grad=True, fourier_feat_transformer=fourier_transformer,
               device=device, accumulation_steps=4)
