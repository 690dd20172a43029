"""Counterpart of experiment_scripts/train_mri_neural_process_ddp.py (reference, config
'hyperoptIV_homebrew_small'): one process per GPU, launched by torchrun
(`python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ...`) instead of
mp.spawn; the Fourier matrix B is drawn on rank 0 and broadcast (the reference draws it in the
parent and passes it to the spawned ranks); synthetic k-space replaces fastMRI (bug 0.7)."""
from _common import base_parser, psnr_summary  # noqa: E402

import os
from functools import partial

import torch
import torch.distributed as dist
from torch.utils.data import DataLoader
from torch.utils.data.distributed import DistributedSampler

from siren_mri_amd import checkpoints, dataio, loss_functions, meta_modules, training_ddp
from siren_mri_amd.features import GaussianFourierFeatureTransform

p = base_parser(batch_size=32, lr=5.57e-5, num_epochs=200, epochs_til_ckpt=5, steps_til_summary=100)
p.add_argument("--n_slices", type=int, default=1024)
p.add_argument("--accumulation_steps", type=int, default=1)
opt = p.parse_args()

rank = int(os.environ.get("RANK", 0))
world_size = int(os.environ.get("WORLD_SIZE", 1))
training_ddp.ddp_setup(rank, world_size)
device = torch.device("cuda", torch.cuda.current_device())

num_fourier_features, kl_weight, fw_weight, fourier_features_scale = 60, 2.78e-8, 6.4e-6, 21
latent_dim, hidden_features_hyper, hidden_layers_hyper = 128, 128, 2
hidden_layers, hidden_features, conv_kernel_size, num_conv_res_blocks, w0 = 3, 256, 3, 3, 30
image_resolution = (128, 128)

ds = dataio.SyntheticMRIKspace(n_slices=opt.n_slices, image_resolution=image_resolution, seed=0)
coord = dataio.Implicit2DWrapper(ds, sidelength=image_resolution, image=False)
gen = dataio.ImageGeneralizationWrapper(coord, test_sparsity="CS_cartesian", generalization_mode="conv_cnp",
                                        device=device)
dataloader = DataLoader(gen, shuffle=False, batch_size=opt.batch_size, pin_memory=False, num_workers=0,
                        sampler=DistributedSampler(gen))

model = meta_modules.ConvolutionalNeuralProcessImplicit2DHypernetFourierFeatures(
    in_features=2 * num_fourier_features, out_features=2, image_resolution=image_resolution,
    fourier_features_size=2 * num_fourier_features, latent_dim=latent_dim, hidden_features=hidden_features,
    hyper_hidden_features=hidden_features_hyper, hyper_hidden_layers=hidden_layers_hyper,
    num_hidden_layers=hidden_layers, partial_conv=False, conv_kernel_size=conv_kernel_size,
    num_conv_res_blocks=num_conv_res_blocks, w0=w0, precision=opt.precision)
if opt.checkpoint_path is not None:
    # reference checkpoints from its DDP wrapper carry a "module." prefix (training_ddp.py:89,146)
    checkpoints.load_state_dict_compat(model, opt.checkpoint_path)
model.to(device)

fourier_transformer = GaussianFourierFeatureTransform(num_input_channels=2, mapping_size_spatial=num_fourier_features,
                                                      scale=fourier_features_scale, device=device)
B = fourier_transformer.get_B().contiguous()
dist.broadcast(B, src=0)
fourier_transformer.set_B(B)

model_dir = f"{opt.logging_root}/{opt.experiment_name}"
training_ddp.train_ddp(model=model, train_dataloader=dataloader, epochs=opt.num_epochs, lr=opt.lr,
                       steps_til_summary=opt.steps_til_summary, epochs_til_checkpoint=opt.epochs_til_ckpt,
                       model_dir=model_dir,
                       loss_fn=partial(loss_functions.image_hypernetwork_loss, None, kl_weight, fw_weight),
                       summary_fn=psnr_summary(), clip_grad=True, fourier_feat_transformer=fourier_transformer,
                       device=device, accumulation_steps=opt.accumulation_steps, ddp_run=True)
# every rank's B as <model_dir>/current_B_DDP_mp<rank>.pt, the reference's file names
# (train_mri_neural_process_ddp.py:254-256; its test script loads them,
# test_mri_conv_neural_process_kspace_fourierfeat.py:214-215). Written after training: the
# reference saves them before train_ddp, whose rank 0 then removes model_dir (training_ddp.py:29-31).
# B is identical on every rank (broadcast above), so rank 0 writes all the files.
if rank == 0:
    for r in range(world_size):
        checkpoints.save_b_matrix(fourier_transformer, model_dir, r)
dist.destroy_process_group()
