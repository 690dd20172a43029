"""Counterpart of experiment_scripts/train_mri_neural_process_ddp.py (reference). The reference
selects config 'hyperoptIV_homebrew' (train_mri_neural_process_ddp.py:52,114-128: 8 Fourier
features -> 16 SIREN inputs, k=7 convolutions, 5 residual blocks, 3 x 256 hypo-net, lr 5.57e-5),
which is the default here; --config hyperoptIV_homebrew_small is a lighter variant (60 features,
k=3, 3 blocks) for quick runs.

One process per GPU, launched by torchrun (`python -m torch.distributed.run --nproc-per-node N
--master-addr 127.0.0.1 ...`) instead of mp.spawn. The Fourier matrix B is drawn on rank 0 and
broadcast (the reference draws it in the parent and passes it to the spawned ranks); synthetic
k-space replaces fastMRI (bug 0.7).

B files: every rank's B is written as <model_dir>/current_B_DDP_mp<rank>.pt (the reference's
names, train_mri_neural_process_ddp.py:254-256) as soon as the model directory is prepared, before
the first step, so a crashed or preempted run still has the B its checkpoints were trained with.
On resume (--checkpoint_path) B is read back — from --b_path, or from the checkpoint's run
directory (<run>/checkpoints/model_*.pth -> <run>/current_B_DDP_mp<rank>.pt) — instead of drawing
a new one: the hypernetwork weights only make sense with the B they were trained against."""
from _common import base_parser, psnr_summary  # noqa: E402

import os
from functools import partial

import torch
import torch.distributed as dist
from torch.utils.data import DataLoader
from torch.utils.data.distributed import DistributedSampler

from siren_mri_amd import checkpoints, dataio, loss_functions, meta_modules, training_ddp
from siren_mri_amd.features import GaussianFourierFeatureTransform

CONFIGS = {
    # train_mri_neural_process_ddp.py:114-128
    "hyperoptIV_homebrew": dict(num_fourier_features=8, kl_weight=2.78e-8, fw_weight=6.4e-6, lr=5.57e-5,
                                fourier_features_scale=21, latent_dim=128, hidden_features_hyper=128,
                                hidden_layers_hyper=2, hidden_layers=3, hidden_features=256,
                                conv_kernel_size=7, num_conv_res_blocks=5, w0=30),
    "hyperoptIV_homebrew_small": dict(num_fourier_features=60, kl_weight=2.78e-8, fw_weight=6.4e-6, lr=5.57e-5,
                                      fourier_features_scale=21, latent_dim=128, hidden_features_hyper=128,
                                      hidden_layers_hyper=2, hidden_layers=3, hidden_features=256,
                                      conv_kernel_size=3, num_conv_res_blocks=3, w0=30),
}

p = base_parser(batch_size=32, lr=None, num_epochs=200, epochs_til_ckpt=5, steps_til_summary=100)
p.add_argument("--config", default="hyperoptIV_homebrew", choices=sorted(CONFIGS))
p.add_argument("--n_slices", type=int, default=1024)
p.add_argument("--accumulation_steps", type=int, default=1)
p.add_argument("--b_path", default=None, help="B matrix file to resume with (default: the checkpoint's run dir)")
p.add_argument("--seed", type=int, default=None, help="seed of rank 0's B draw (the reference's is unseeded)")
opt = p.parse_args()
cfg = CONFIGS[opt.config]
lr = opt.lr if opt.lr is not None else cfg["lr"]

rank = int(os.environ.get("RANK", 0))
world_size = int(os.environ.get("WORLD_SIZE", 1))
training_ddp.ddp_setup(rank, world_size)
device = torch.device("cuda", torch.cuda.current_device())

image_resolution = (128, 128)
ds = dataio.SyntheticMRIKspace(n_slices=opt.n_slices, image_resolution=image_resolution, seed=0)
coord = dataio.Implicit2DWrapper(ds, sidelength=image_resolution, image=False)
gen = dataio.ImageGeneralizationWrapper(coord, test_sparsity="CS_cartesian", generalization_mode="conv_cnp",
                                        device=device)
dataloader = DataLoader(gen, shuffle=False, batch_size=opt.batch_size, pin_memory=False, num_workers=0,
                        sampler=DistributedSampler(gen))

nff = cfg["num_fourier_features"]
model = meta_modules.ConvolutionalNeuralProcessImplicit2DHypernetFourierFeatures(
    in_features=2 * nff, out_features=2, image_resolution=image_resolution,
    fourier_features_size=2 * nff, latent_dim=cfg["latent_dim"], hidden_features=cfg["hidden_features"],
    hyper_hidden_features=cfg["hidden_features_hyper"], hyper_hidden_layers=cfg["hidden_layers_hyper"],
    num_hidden_layers=cfg["hidden_layers"], partial_conv=False, conv_kernel_size=cfg["conv_kernel_size"],
    num_conv_res_blocks=cfg["num_conv_res_blocks"], w0=cfg["w0"], precision=opt.precision)

fourier_transformer = GaussianFourierFeatureTransform(num_input_channels=2, mapping_size_spatial=nff,
                                                      scale=cfg["fourier_features_scale"], device=device)
if opt.checkpoint_path is not None:
    # reference checkpoints from its DDP wrapper carry a "module." prefix (training_ddp.py:89,146)
    checkpoints.load_state_dict_compat(model, opt.checkpoint_path)
    b_path = opt.b_path or checkpoints.b_matrix_path(
        os.path.dirname(os.path.dirname(os.path.abspath(opt.checkpoint_path))), rank)
    if not os.path.exists(b_path):
        raise FileNotFoundError(f"resume: no Fourier matrix at {b_path} (pass --b_path)")
    B = torch.load(b_path, map_location="cpu", weights_only=True).contiguous()
else:
    if opt.seed is not None:
        # the transform drew its B at construction; redraw it from the seeded generator
        torch.manual_seed(opt.seed)
        fourier_transformer.set_B(torch.randn((2, nff)) * cfg["fourier_features_scale"])
    B = fourier_transformer.get_B().contiguous()
model.to(device)
B = B.to(device)
dist.broadcast(B, src=0)
fourier_transformer.set_B(B.cpu())


def write_b_files(model_dir):
    # B is identical on every rank (broadcast above), so the writing rank writes every rank's file
    for r in range(world_size):
        checkpoints.save_b_matrix(fourier_transformer, model_dir, r)


model_dir = f"{opt.logging_root}/{opt.experiment_name}"
training_ddp.train_ddp(model=model, train_dataloader=dataloader, epochs=opt.num_epochs, lr=lr,
                       steps_til_summary=opt.steps_til_summary, epochs_til_checkpoint=opt.epochs_til_ckpt,
                       model_dir=model_dir,
                       loss_fn=partial(loss_functions.image_hypernetwork_loss, None, cfg["kl_weight"], cfg["fw_weight"]),
                       summary_fn=psnr_summary(), clip_grad=True, fourier_feat_transformer=fourier_transformer,
                       device=device, accumulation_steps=opt.accumulation_steps, ddp_run=True,
                       model_dir_hook=write_b_files)
dist.destroy_process_group()
