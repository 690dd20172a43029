"""siren_mri_amd — MI355X-native (gfx950) SIREN fitting path, a drop-in for the hot path of
jonbmartin/siren_mri (modules.SingleBVPNet/FCBlock, diff_operators, training.train/train_ddp)."""
from .ops import siren_mlp, set_default_precision, get_default_precision  # noqa: F401

__version__ = "0.1.0"
