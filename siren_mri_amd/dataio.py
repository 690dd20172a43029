"""Data layouts and producers feeding the SIREN path (dataio.py of jonbmartin/siren_mri).

Restated from the reference:
  get_mgrid                  dataio.py:28-48   row-major grid, x_k = 2 i_k/(S_k - 1) - 1
  lin2img                    dataio.py:51-63   [B, N, C] -> [B, C, H, W]
  Camera                     dataio.py:474-492 (cameraman, siren_mri_amd/assets/camera512_u8.npz)
  MRIImageDomain             dataio.py:507-525 (data/IRData.mat -> siren_mri_amd/assets/irdata.npz)
  Implicit2DWrapper          dataio.py:746-827 (PIL bilinear resize, /255, Normalize; sobel /
                                                laplace ground truth via scipy.ndimage)
  ImageGeneralizationWrapper dataio.py:861-986 (CS-Cartesian masks, conv_cnp inputs)
  FastMRIBrainKspace layout  dataio.py:585-664 (fftshift(fft2(slice)) stacked [H, W, 2])

Deviation (bug 0.7): fastMRI .h5 volumes are not available, so
SyntheticMRIKspace produces k-space of seeded phantoms with the same [H, W, 2] float32 layout:
the reference tree's own IRData slices under the 8 flips/rotations and seeded
random-ellipse phantoms; the CS mask RNG is seeded.
"""
from __future__ import annotations

import os
import random

import numpy as np
import torch
from torch.utils.data import Dataset

# data assets shipped with the package (tools/make_assets.py, tests/golden/make_golden.py)
ASSETS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "assets")


def get_mgrid(sidelen, dim=2):
    if isinstance(sidelen, int):
        sidelen = dim * (sidelen,)
    axes = [np.arange(s, dtype=np.float32) / np.float32(max(s - 1, 1)) for s in sidelen]
    grid = np.stack(np.meshgrid(*axes, indexing="ij"), axis=-1).astype(np.float32)
    grid = (grid - np.float32(0.5)) * np.float32(2.0)
    return torch.from_numpy(np.ascontiguousarray(grid)).view(-1, dim)


def lin2img(tensor, image_resolution=None):
    b, n, c = tensor.shape
    if image_resolution is None:
        h = w = int(np.sqrt(n))
    else:
        h, w = image_resolution
    return tensor.permute(0, 2, 1).reshape(b, c, h, w)


def camera_image() -> np.ndarray:
    """The 512x512 uint8 cameraman (the image skimage.data.camera() returns)."""
    path = os.path.join(ASSETS, "camera512_u8.npz")
    with np.load(path, allow_pickle=False) as d:
        return d["img"]


class Camera(Dataset):
    def __init__(self, downsample_factor=1):
        super().__init__()
        from PIL import Image
        self.img = Image.fromarray(camera_image())
        self.img_channels = 1
        self.downsample_factor = downsample_factor
        if downsample_factor > 1:
            size = (int(512 / downsample_factor),) * 2
            self.img_downsampled = self.img.resize(size, Image.LANCZOS)

    def __len__(self):
        return 1

    def __getitem__(self, idx):
        return self.img_downsampled if self.downsample_factor > 1 else self.img


def irdata() -> np.ndarray:
    """IRData [128, 128, 9] float32 (np.squeeze of data/IRData.mat's 'IRData', dataio.py:519-520)."""
    with np.load(os.path.join(ASSETS, "irdata.npz"), allow_pickle=False) as d:
        return d["IRData"]


class MRIImageDomain(Dataset):
    """dataio.py:507-525: the 9 IRData magnitude slices, item = [128, 128] float32. `split` is
    checked as in the reference and otherwise unused (the reference reads one file for all)."""

    def __init__(self, split="train", downsampled=False):
        assert split in ["train", "test", "val", "val_small"], "Unknown split"
        self.img_channels = 1
        self.downsampled = downsampled
        self.data = irdata()

    def __len__(self):
        return self.data.shape[2]

    def __getitem__(self, idx):
        return np.squeeze(self.data[:, :, idx])


def irdata_image(idx: int = 0, side: int = 256) -> torch.Tensor:
    """Config C2's fitting target (harness-defined since BASELINE.json says
    256x256 and IRData is 128x128): slice idx -> / max -> x2 - 1 -> bilinear resize to side^2
    (F.interpolate, align_corners=False). Returns [side*side, 1] float32 in the flattened
    get_mgrid row order (row-major over (i, j))."""
    import torch.nn.functional as F
    sl = torch.from_numpy(np.ascontiguousarray(MRIImageDomain()[idx]))
    sl = sl / sl.max() * 2 - 1
    img = F.interpolate(sl[None, None], size=(side, side), mode="bilinear", align_corners=False)
    return img.reshape(-1, 1).contiguous()


def smooth_random_image(side: int, n_waves: int = 32, seed: int = 0, max_freq: float = 16.0) -> np.ndarray:
    """Synthetic throughput target: sum of random 2-D sinusoids in [-1, 1]."""
    rs = np.random.RandomState(seed)
    y, x = np.meshgrid(np.linspace(0, 1, side), np.linspace(0, 1, side), indexing="ij")
    img = np.zeros((side, side), np.float64)
    for _ in range(n_waves):
        fx, fy = rs.uniform(0, max_freq, size=2)
        ph = rs.uniform(0, 2 * np.pi)
        img += np.sin(2 * np.pi * (fx * x + fy * y) + ph)
    img = img - img.min()
    img = img / max(img.max(), 1e-12)
    return (img * 2 - 1).astype(np.float32)


def _image_transform(img, sidelength):
    """Resize(sidelength) -> ToTensor -> Normalize(0.5, 0.5) for a PIL image."""
    from PIL import Image
    if isinstance(img, Image.Image):
        if tuple(img.size[::-1]) != tuple(sidelength):
            img = img.resize((sidelength[1], sidelength[0]), Image.BILINEAR)
        a = np.asarray(img, dtype=np.float32)
        if a.ndim == 2:
            a = a[None]
        else:
            a = a.transpose(2, 0, 1)
        a = a / np.float32(255.0)
    else:
        a = np.asarray(img, dtype=np.float32)
        if a.ndim == 2:
            a = a[None]
    return torch.from_numpy((a - np.float32(0.5)) / np.float32(0.5))


class Implicit2DWrapper(Dataset):
    """Image -> {'coords': grid}, {'img': [N, C] (+ 'gradients' / 'laplace')} (dataio.py:746-812)."""

    def __init__(self, dataset, sidelength=None, compute_diff=None, image=True, kspace=False):
        if isinstance(sidelength, int):
            sidelength = (sidelength, sidelength)
        self.sidelength = sidelength
        self.image = image
        self.compute_diff = compute_diff
        self.dataset = dataset
        self.mgrid = get_mgrid(sidelength)

    def __len__(self):
        return len(self.dataset)

    def _transform(self, item):
        if self.image:
            return _image_transform(item, self.sidelength)
        # k-space arrays [H, W, 2]: ToTensor -> [2, H, W]; Normalize(0, 0.5) -> x2
        a = np.asarray(item, dtype=np.float32).transpose(2, 0, 1)
        return torch.from_numpy(np.ascontiguousarray(a)) / 0.5

    def __getitem__(self, idx):
        import scipy.ndimage
        img = self._transform(self.dataset[idx])
        gt = {}
        if self.compute_diff == "gradients":
            img = img * 1e1
        elif self.compute_diff == "laplacian":
            img = img * 1e4
        if self.compute_diff in ("gradients", "all"):
            gx = scipy.ndimage.sobel(img.numpy(), axis=1).squeeze(0)[..., None]
            gy = scipy.ndimage.sobel(img.numpy(), axis=2).squeeze(0)[..., None]
            gt["gradients"] = torch.cat((torch.from_numpy(gx).reshape(-1, 1),
                                         torch.from_numpy(gy).reshape(-1, 1)), dim=-1)
        if self.compute_diff in ("laplacian", "all"):
            lap = scipy.ndimage.laplace(img.numpy()).squeeze(0)[..., None]
            gt["laplace"] = torch.from_numpy(lap).view(-1, 1)
        channels = img.shape[0]
        gt["img"] = img.permute(1, 2, 0).reshape(-1, channels)
        return {"idx": idx, "coords": self.mgrid}, gt

    def get_item_small(self, idx):
        img = self._transform(self.dataset[idx])
        spatial = img.clone()
        channels = img.shape[0]
        return spatial, img.permute(1, 2, 0).reshape(-1, channels), {"img": img.permute(1, 2, 0).reshape(-1, channels)}


def _ellipse_phantom(res: int, rs: np.random.RandomState, n_ellipses: int = 8) -> np.ndarray:
    y, x = np.meshgrid(np.linspace(-1, 1, res), np.linspace(-1, 1, res), indexing="ij")
    img = np.zeros((res, res), np.float64)
    for i in range(n_ellipses):
        a, b = rs.uniform(0.1, 0.8, size=2) if i else (0.85, 0.7)
        cx, cy = rs.uniform(-0.4, 0.4, size=2) if i else (0.0, 0.0)
        th = rs.uniform(0, np.pi)
        val = rs.uniform(-0.4, 1.0) if i else 1.0
        xr = (x - cx) * np.cos(th) + (y - cy) * np.sin(th)
        yr = -(x - cx) * np.sin(th) + (y - cy) * np.cos(th)
        img[(xr / a) ** 2 + (yr / b) ** 2 <= 1] += val
    return img


class SyntheticMRIKspace(Dataset):
    """Seeded synthetic stand-in for FastMRIBrainKspace (bug 0.7): item = float32 [H, W, 2] of
    fftshift(fft2(slice)) stacked real/imag, the reference's layout (dataio.py:654-664).
    Items 0..71 (with irdata=True) are the 9 IRData slices under the 8 flips/rotations of the
    square (normalised to max 1, bilinear-resized when the resolution is not 128); later items
    are seeded random-ellipse phantoms."""

    def __init__(self, n_slices: int = 256, image_resolution=(128, 128), seed: int = 0, irdata: bool = True):
        self.n = n_slices
        self.res = image_resolution
        self.seed = seed
        self.img_channels = 2
        self._ir = globals()["irdata"]() if irdata else None

    def __len__(self):
        return self.n

    def _ir_slice(self, idx):
        sl = self._ir[:, :, idx % 9].astype(np.float64)
        t = idx // 9
        sl = np.rot90(sl, t % 4)
        if t >= 4:
            sl = sl[:, ::-1]
        sl = sl / max(sl.max(), 1e-12)
        if tuple(self.res) != sl.shape:
            import torch.nn.functional as F
            sl = F.interpolate(torch.from_numpy(np.ascontiguousarray(sl))[None, None], size=tuple(self.res),
                               mode="bilinear", align_corners=False)[0, 0].numpy()
        return sl

    def __getitem__(self, idx):
        rs = np.random.RandomState(self.seed * 100003 + idx)
        if self._ir is not None and idx < 72:
            img = self._ir_slice(idx)
        else:
            img = _ellipse_phantom(self.res[0], rs)
        k = np.fft.fftshift(np.fft.fft2(img))
        k = k / max(np.abs(k).max(), 1e-12)
        return np.float32(np.dstack((k.real, k.imag)))


class ImageGeneralizationWrapper(Dataset):
    """conv_cnp inputs with CS-Cartesian sampling (dataio.py:861-986). The row permutation uses
    a per-item seeded RNG (the reference's is unseeded `random.shuffle`)."""

    def __init__(self, dataset, test_sparsity=None, train_sparsity_range=(10, 200),
                 generalization_mode=None, device="cpu", seed: int = 0):
        self.dataset = dataset
        self.sidelength = dataset.sidelength
        self.mgrid = dataset.mgrid
        self.test_sparsity = test_sparsity
        self.train_sparsity_range = train_sparsity_range
        self.generalization_mode = generalization_mode
        self.device = device
        self.seed = seed

    def __len__(self):
        return len(self.dataset)

    def update_test_sparsity(self, test_sparsity):
        self.test_sparsity = test_sparsity

    def get_generalization_in_dict(self, spatial_img, img, idx):
        if self.generalization_mode not in ("conv_cnp", "conv_cnp_test"):
            return {"idx": torch.tensor(idx), "coords": self.mgrid}
        rng = random.Random(self.seed * 1000003 + idx)
        ny = spatial_img.size(1)
        if self.test_sparsity == "full":
            mask = torch.ones_like(spatial_img)
        elif self.test_sparsity == "half":
            mask = torch.ones_like(spatial_img)
            mask[:, ny // 2:, :] = 0
        elif self.test_sparsity in ("CS_cartesian", "CS_cartesian_noACS"):
            rows = list(range(ny))
            rng.shuffle(rows)
            mask = torch.zeros_like(spatial_img)
            mask[:, rows[: int(0.3333 * ny)], :] = 1
            if self.test_sparsity == "CS_cartesian":
                mask[:, int(ny / 2 - 4):int(ny / 2 + 4), :] = 1
        else:
            raise NotImplementedError(f"test_sparsity={self.test_sparsity!r}")
        img_sparse = mask * spatial_img
        z = torch.fft.ifft2(img_sparse[0] + 1j * img_sparse[1])
        ift = torch.stack((torch.abs(z), torch.angle(z)))
        return {"idx": torch.tensor(idx), "coords": self.mgrid, "img_sparse": img_sparse,
                "ift_zfilled": ift, "dc_mask": mask}

    def __getitem__(self, idx):
        spatial_img, img, gt = self.dataset.get_item_small(idx)
        in_dict = self.get_generalization_in_dict(spatial_img, img, idx)
        if "dc_mask" in in_dict:
            gt["dc_mask"] = in_dict["dc_mask"]
        in_dict = {k: v.to(self.device) for k, v in in_dict.items()}
        gt = {k: v.to(self.device) for k, v in gt.items()}
        return in_dict, gt
