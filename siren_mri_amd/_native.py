"""ctypes binding of the C ABI in include/siren_mri_amd.h (libsiren_mri_amd.so).

The library is built in-tree by ``__graft_entry__.build()`` (hipcc --offload-arch=gfx950) and
loaded lazily at the first kernel call, after ``torch`` so that the kernels register with the
HIP runtime PyTorch already holds. There is deliberately NO fallback: if the library or a GPU
is missing, every SIREN kernel entry point raises.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch

MAX_LAYERS = 16
PREC_F32 = 0
PREC_BF16 = 1
PREC_F64 = 2  # float64 tensors (siren_mlp64_*): chosen by dtype, not by the precision string
PRECISIONS = {"fp32": PREC_F32, "f32": PREC_F32, "float32": PREC_F32,
              "bf16": PREC_BF16, "bfloat16": PREC_BF16}

LIB_NAME = "libsiren_mri_amd.so"
# SIREN_MRI_AMD_LIB: load another build of the same ABI (A/B timing of kernel variants)
LIB_PATH = os.environ.get("SIREN_MRI_AMD_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), LIB_NAME)

# Every symbol include/siren_mri_amd.h declares (checked by tests/test_native_abi.py).
EXPORTED_SYMBOLS = (
    "siren_mlp_check",
    "siren_mlp_saved_bytes",
    "siren_mlp_workspace_bytes",
    "siren_mlp_forward",
    "siren_mlp_backward",
    "siren_mlp_loss_check",
    "siren_mlp_forward_loss",
    "siren_mlp_backward_ex",
    "siren_mlp64_saved_bytes",
    "siren_mlp64_workspace_bytes",
    "siren_mlp64_forward",
    "siren_mlp64_backward",
    "siren_hyper_saved_bytes",
    "siren_hyper_workspace_bytes",
    "siren_hyper_forward",
    "siren_hyper_backward",
    "siren_jvp_saved_bytes",
    "siren_jvp_workspace_bytes",
    "siren_jvp_forward",
    "siren_jvp_backward",
    "siren_jvp_forward_ex",
    "siren_jvp_backward_ex",
    "siren_timing_enable",
    "siren_timing_collect",
    "siren_timing_disable",
    "siren_config_set",
    "siren_config_get",
    "siren_adam_step",
    "siren_adam_num_blocks",
    "siren_adam_scalars",
    "siren_adam_scalars_table",
    "siren_sse_workspace_bytes",
    "siren_enc_workspace_bytes",
    "siren_conv_wrw_workspace_bytes",
    "siren_conv_wrw_k5",
    "siren_conv_fwd_k5",
    "siren_conv_dgrad_k5_fused",
    "siren_conv_fwd_k5_res",
    "siren_conv_check",
    "siren_conv_fwd",
    "siren_conv_wrw_ws_bytes",
    "siren_conv_wrw",
    "siren_enc_bias_relu",
    "siren_enc_prep",
    "siren_sumsq_workspace_bytes",
    "siren_sumsq_forward",
    "siren_sumsq_backward",
    "siren_enc_relu_bwd",
    "siren_enc_res_fwd",
    "siren_enc_res_bwd",
    "siren_enc_pixfc_fwd",
    "siren_enc_pixfc_bwd",
    "siren_sse_forward",
    "siren_sse_backward",
    "siren_dc_forward",
    "siren_dc_backward",
    "siren_kspace_sse_forward",
    "siren_kspace_sse_backward",
    "siren_fourier_features",
    "siren_sincos_f32",
    "siren_last_error",
    "siren_version",
)

KCLASS_FWD_GEMM = 1
KCLASS_DX_GEMM = 2
KCLASS_DW_GEMM = 3
KCLASS_FWD_FUSED = 4
KCLASS_BWD_FUSED = 5
KCLASS_DX_RING = 6
KCLASS_DW_RING = 7
KCLASS_DX_RING_BOT = 8
KCLASS_DW_RING_REC = 9
KCLASS_DX_RING_TOP = 10
KCLASS_DW_RING_TOP = 11
KCLASS_PAIR_RING = 12
KCLASS_PAIR_RING_TOP = 13
KCLASS_PAIR_RING_BOT = 14


class SirenMLPDesc(ctypes.Structure):
    """Mirror of ``siren_mlp_desc`` (include/siren_mri_amd.h)."""

    _fields_ = [
        ("num_layers", ctypes.c_int32),
        ("dims", ctypes.c_int32 * (MAX_LAYERS + 1)),
        ("outermost_linear", ctypes.c_int32),
        ("prec", ctypes.c_int32),
        ("weights_batched", ctypes.c_int32),
        ("w0", ctypes.c_float),
        ("batch", ctypes.c_int64),
        ("rows_per_batch", ctypes.c_int64),
        ("weight", ctypes.c_void_p * MAX_LAYERS),
        ("bias", ctypes.c_void_p * MAX_LAYERS),
        ("ff_B", ctypes.c_void_p),
        ("ff_in", ctypes.c_int32),
    ]


class SirenLossDesc(ctypes.Structure):
    """Mirror of ``siren_loss_desc`` (include/siren_mri_amd.h)."""

    _fields_ = [
        ("target", ctypes.c_void_p),
        ("k0", ctypes.c_void_p),
        ("mask", ctypes.c_void_p),
        ("hf", ctypes.c_void_p),
        ("hf_len", ctypes.c_int64),
        ("noise", ctypes.c_float),
        ("weight", ctypes.c_float),
        ("y_dc", ctypes.c_void_p),
        ("dy", ctypes.c_void_p),
        ("loss", ctypes.c_void_p),
        ("loss_workspace", ctypes.c_void_p),
        ("loss_workspace_bytes", ctypes.c_int64),
    ]


HYPER_MAXG = 32
HYPER_MAXD = 4


class SirenHyperDesc(ctypes.Structure):
    """Mirror of ``siren_hyper_desc`` (include/siren_mri_amd.h)."""

    _fields_ = [
        ("heads", ctypes.c_int32),
        ("depth", ctypes.c_int32),
        ("rows", ctypes.c_int32),
        ("in_features", ctypes.c_int32),
        ("hidden", ctypes.c_int32),
        ("out_features", ctypes.c_int32 * HYPER_MAXG),
        ("weight", ctypes.c_void_p * (HYPER_MAXG * (HYPER_MAXD + 1))),
        ("bias", ctypes.c_void_p * (HYPER_MAXG * (HYPER_MAXD + 1))),
    ]


ADAM_MAX_TENSORS = 48


class SirenAdamDesc(ctypes.Structure):
    """Mirror of ``siren_adam_desc`` (include/siren_mri_amd.h)."""

    _fields_ = [
        ("num_tensors", ctypes.c_int32),
        ("maximize", ctypes.c_int32),
        ("lr", ctypes.c_float),
        ("beta1", ctypes.c_float),
        ("beta2", ctypes.c_float),
        ("eps", ctypes.c_float),
        ("weight_decay", ctypes.c_float),
        ("one_minus_beta1", ctypes.c_float),
        ("one_minus_beta2", ctypes.c_float),
        ("step_size", ctypes.c_float),
        ("bias_correction2_sqrt", ctypes.c_float),
        ("numel", ctypes.c_int64 * ADAM_MAX_TENSORS),
        ("param", ctypes.c_void_p * ADAM_MAX_TENSORS),
        ("grad", ctypes.c_void_p * ADAM_MAX_TENSORS),
        ("exp_avg", ctypes.c_void_p * ADAM_MAX_TENSORS),
        ("exp_avg_sq", ctypes.c_void_p * ADAM_MAX_TENSORS),
        ("dev_scalars", ctypes.c_void_p),
        ("dev_steps", ctypes.c_void_p),
        ("dev_table", ctypes.c_void_p),
        ("table_n", ctypes.c_int64),

    ]


class NativeError(RuntimeError):
    pass


_lib = None
_lock = threading.Lock()


def _declare(lib):
    P = ctypes.POINTER(SirenMLPDesc)
    vp = ctypes.c_void_p
    i64 = ctypes.c_int64
    lib.siren_mlp_check.argtypes = [P]
    lib.siren_mlp_check.restype = ctypes.c_int
    lib.siren_mlp_saved_bytes.argtypes = [P]
    lib.siren_mlp_saved_bytes.restype = i64
    lib.siren_mlp_workspace_bytes.argtypes = [P]
    lib.siren_mlp_workspace_bytes.restype = i64
    lib.siren_mlp_forward.argtypes = [P, vp, vp, vp, i64, vp, i64, vp]
    lib.siren_mlp_forward.restype = ctypes.c_int
    lib.siren_mlp_backward.argtypes = [P, vp, vp, vp, i64, vp, i64,
                                       ctypes.POINTER(vp), ctypes.POINTER(vp), vp, vp]
    lib.siren_mlp_backward.restype = ctypes.c_int
    ci = ctypes.c_int
    LP = ctypes.POINTER(SirenLossDesc)
    lib.siren_mlp_loss_check.argtypes = [P, LP]
    lib.siren_mlp_loss_check.restype = ci
    lib.siren_mlp_forward_loss.argtypes = [P, LP, vp, vp, vp, i64, vp, i64, vp]
    lib.siren_mlp_forward_loss.restype = ci
    lib.siren_mlp_backward_ex.argtypes = [P, vp, vp, vp, vp, i64, vp, i64, ctypes.POINTER(vp), ctypes.POINTER(vp), vp, vp]
    lib.siren_mlp_backward_ex.restype = ci
    lib.siren_mlp64_saved_bytes.argtypes = [P]
    lib.siren_mlp64_saved_bytes.restype = i64
    lib.siren_mlp64_workspace_bytes.argtypes = [P]
    lib.siren_mlp64_workspace_bytes.restype = i64
    lib.siren_mlp64_forward.argtypes = [P, vp, vp, vp, i64, vp, i64, vp]
    lib.siren_mlp64_forward.restype = ci
    lib.siren_mlp64_backward.argtypes = [P, vp, vp, vp, i64, vp, i64, ctypes.POINTER(vp), ctypes.POINTER(vp), vp, vp]
    lib.siren_mlp64_backward.restype = ci
    HP = ctypes.POINTER(SirenHyperDesc)
    lib.siren_hyper_saved_bytes.argtypes = [HP]
    lib.siren_hyper_saved_bytes.restype = i64
    lib.siren_hyper_workspace_bytes.argtypes = [HP]
    lib.siren_hyper_workspace_bytes.restype = i64
    lib.siren_hyper_forward.argtypes = [HP, vp, ctypes.POINTER(vp), vp, i64, vp]
    lib.siren_hyper_forward.restype = ci
    lib.siren_hyper_backward.argtypes = [HP, vp, ctypes.POINTER(vp), vp, i64, vp, i64, ctypes.POINTER(vp),
                                         ctypes.POINTER(vp), vp, vp]
    lib.siren_hyper_backward.restype = ci
    lib.siren_enc_prep.argtypes = [ci, ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.POINTER(ctypes.c_int64),
                                   ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.POINTER(vp), vp]
    lib.siren_enc_prep.restype = ci
    lib.siren_sumsq_workspace_bytes.argtypes = [i64]
    lib.siren_sumsq_workspace_bytes.restype = i64
    lib.siren_sumsq_forward.argtypes = [ci, ctypes.POINTER(vp), ctypes.POINTER(ctypes.c_int64), vp, vp, i64, vp]
    lib.siren_sumsq_forward.restype = ci
    lib.siren_sumsq_backward.argtypes = [ci, ctypes.POINTER(vp), ctypes.POINTER(ctypes.c_int64), vp,
                                         ctypes.POINTER(vp), vp]
    lib.siren_sumsq_backward.restype = ci
    lib.siren_jvp_saved_bytes.argtypes = [P, ci]
    lib.siren_jvp_saved_bytes.restype = i64
    lib.siren_jvp_workspace_bytes.argtypes = [P, ci]
    lib.siren_jvp_workspace_bytes.restype = i64
    lib.siren_jvp_forward.argtypes = [P, ci, vp, vp, vp, vp, i64, vp, i64, vp]
    lib.siren_jvp_forward.restype = ci
    lib.siren_jvp_forward_ex.argtypes = [P, ci, vp, vp, vp, vp, i64, vp, i64, vp, i64, vp]
    lib.siren_jvp_forward_ex.restype = ci
    lib.siren_jvp_backward.argtypes = [P, ci, vp, vp, vp, i64, vp, i64,
                                       ctypes.POINTER(vp), ctypes.POINTER(vp), vp, vp]
    lib.siren_jvp_backward.restype = ci
    lib.siren_jvp_backward_ex.argtypes = [P, ci, vp, vp, vp, i64, vp, i64,
                                          ctypes.POINTER(vp), ctypes.POINTER(vp), vp, vp, i64, vp]
    lib.siren_jvp_backward_ex.restype = ci
    lib.siren_timing_enable.argtypes = [ctypes.c_int, ctypes.c_int]
    lib.siren_timing_enable.restype = ctypes.c_int
    lib.siren_timing_collect.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(i64)]
    lib.siren_timing_collect.restype = ctypes.c_int
    lib.siren_timing_disable.argtypes = []
    lib.siren_timing_disable.restype = None
    lib.siren_config_set.argtypes = [ctypes.c_char_p, i64]
    lib.siren_config_set.restype = ctypes.c_int
    lib.siren_config_get.argtypes = [ctypes.c_char_p]
    lib.siren_config_get.restype = i64
    lib.siren_adam_step.argtypes = [ctypes.POINTER(SirenAdamDesc), vp]
    lib.siren_adam_step.restype = ctypes.c_int
    lib.siren_adam_num_blocks.argtypes = [ctypes.POINTER(SirenAdamDesc)]
    lib.siren_adam_num_blocks.restype = ctypes.c_int64
    f32 = ctypes.c_float
    f64 = ctypes.c_double
    lib.siren_adam_scalars.argtypes = [vp, f64, f64, f64, vp, vp]
    lib.siren_adam_scalars.restype = ctypes.c_int
    lib.siren_adam_scalars_table.argtypes = [vp, vp, i64, vp, vp]
    lib.siren_adam_scalars_table.restype = ctypes.c_int
    lib.siren_sse_workspace_bytes.argtypes = []
    lib.siren_sse_workspace_bytes.restype = i64
    lib.siren_conv_wrw_workspace_bytes.argtypes = [ci, ci, ci]
    lib.siren_conv_wrw_workspace_bytes.restype = i64
    lib.siren_conv_wrw_k5.argtypes = [vp, vp, ci, ci, ci, ci, vp, vp, i64, vp]
    lib.siren_conv_wrw_k5.restype = ci
    lib.siren_conv_fwd_k5.argtypes = [vp, vp, vp, ci, vp, ci, ci, ci, ci, vp]
    lib.siren_conv_fwd_k5.restype = ci
    lib.siren_conv_dgrad_k5_fused.argtypes = [ci, vp, vp, vp, vp, vp, vp, vp, vp, vp, ci, ci, ci, ci, vp, i64, vp]
    lib.siren_conv_dgrad_k5_fused.restype = ci
    lib.siren_conv_fwd_k5_res.argtypes = [vp, vp, vp, vp, vp, vp, ci, ci, ci, ci, vp]
    lib.siren_conv_fwd_k5_res.restype = ci
    lib.siren_conv_check.argtypes = [ci, ci, ci, ci, ci, ci, ci]
    lib.siren_conv_check.restype = ci
    lib.siren_conv_fwd.argtypes = [vp, vp, vp, ci, vp, ci, ci, ci, ci, ci, ci, vp]
    lib.siren_conv_fwd.restype = ci
    lib.siren_conv_wrw_ws_bytes.argtypes = [ci, ci, ci, ci, ci, ci]
    lib.siren_conv_wrw_ws_bytes.restype = i64
    lib.siren_conv_wrw.argtypes = [vp, vp, ci, ci, ci, ci, ci, ci, vp, vp, i64, vp]
    lib.siren_conv_wrw.restype = ci
    lib.siren_enc_workspace_bytes.argtypes = []
    lib.siren_enc_workspace_bytes.restype = i64
    lib.siren_enc_relu_bwd.argtypes = [vp, vp, vp, vp, vp, i64, ci, vp, i64, vp]
    lib.siren_enc_relu_bwd.restype = ci
    lib.siren_enc_bias_relu.argtypes = [vp, vp, i64, ci, vp]
    lib.siren_enc_bias_relu.restype = ci
    lib.siren_enc_res_fwd.argtypes = [vp, vp, vp, vp, i64, ci, vp]
    lib.siren_enc_res_fwd.restype = ci
    lib.siren_enc_res_bwd.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, i64, ci, vp, i64, vp]
    lib.siren_enc_res_bwd.restype = ci
    lib.siren_enc_pixfc_fwd.argtypes = [vp, vp, vp, vp, vp, ci, i64, ci, vp, i64, vp]
    lib.siren_enc_pixfc_fwd.restype = ci
    lib.siren_enc_pixfc_bwd.argtypes = [vp, vp, vp, vp, vp, vp, vp, ci, i64, ci, vp, i64, vp]
    lib.siren_enc_pixfc_bwd.restype = ci
    lib.siren_sse_forward.argtypes = [vp, vp, vp, i64, i64, f32, vp, vp, vp, i64, vp]
    lib.siren_sse_forward.restype = ctypes.c_int
    lib.siren_sse_backward.argtypes = [vp, vp, i64, i64, vp, f32, vp, vp]
    lib.siren_sse_backward.restype = ctypes.c_int
    lib.siren_dc_forward.argtypes = [vp, vp, vp, i64, i64, ci, f32, vp, vp]
    lib.siren_dc_forward.restype = ci
    lib.siren_dc_backward.argtypes = [vp, vp, i64, i64, ci, f32, vp, vp]
    lib.siren_dc_backward.restype = ci
    lib.siren_kspace_sse_forward.argtypes = [vp, vp, vp, vp, vp, i64, i64, ci, f32, f32, vp, vp, vp, i64, vp]
    lib.siren_kspace_sse_forward.restype = ci
    lib.siren_kspace_sse_backward.argtypes = [vp, vp, vp, i64, i64, ci, f32, vp, f32, vp, vp]
    lib.siren_kspace_sse_backward.restype = ci
    lib.siren_fourier_features.argtypes = [vp, vp, i64, ci, ci, vp, vp]
    lib.siren_fourier_features.restype = ci
    lib.siren_sincos_f32.argtypes = [vp, vp, vp, i64, ci, vp]
    lib.siren_sincos_f32.restype = ci
    lib.siren_last_error.argtypes = []
    lib.siren_last_error.restype = ctypes.c_char_p
    lib.siren_version.argtypes = []
    lib.siren_version.restype = ctypes.c_char_p


def load_library(path: str | None = None):
    """Load (once) and return the native library. Raises if it is missing."""
    global _lib
    with _lock:
        if _lib is not None and path is None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise NativeError(
                f"siren_mri_amd: native library {p} not found. Build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950).")
        lib = ctypes.CDLL(p)
        _declare(lib)
        if path is None:
            _lib = lib
        return lib


def lib():
    return _lib if _lib is not None else load_library()


_OPTIONS_EPOCH = [0]


def options_epoch() -> int:
    """Bumped by every set_option (buffer sizes may depend on the options)."""
    return _OPTIONS_EPOCH[0]


def set_option(key: str, value: int) -> None:
    """siren_config_set: process-wide execution options (e.g. "fused_forward")."""
    _OPTIONS_EPOCH[0] += 1
    if lib().siren_config_set(key.encode(), int(value)) != 0:
        raise NativeError(last_error())


def get_option(key: str) -> int:
    v = lib().siren_config_get(key.encode())
    if v < 0:
        raise NativeError(f"unknown option {key!r}")
    return int(v)


def last_error() -> str:
    return lib().siren_last_error().decode(errors="replace")


def check(rc: int, what: str):
    if rc != 0:
        raise NativeError(f"siren_mri_amd.{what} failed ({rc}): {last_error()}")


def precision_code(precision) -> int:
    if isinstance(precision, int):
        return precision
    try:
        return PRECISIONS[str(precision).lower()]
    except KeyError:
        raise ValueError(f"unknown precision {precision!r}; use 'fp32' or 'bf16'") from None


def stream_handle(device: torch.device) -> int:
    """The current HIP stream of `device` as an integer (torch's raw getter: no Stream object)."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    return torch._C._cuda_getCurrentRawStream(idx)


_SSE_WS: dict = {}


def sse_workspace(device) -> torch.Tensor:
    """The per-(device, stream) partial-sum / hand-off-counter workspace of the deterministic loss
    reductions (siren_sse_workspace_bytes; zeroed once, left zeroed by every launch): two launches
    that may run concurrently never share one."""
    key = (device, torch.cuda.current_stream(device).cuda_stream)
    ws = _SSE_WS.get(key)
    if ws is None:
        ws = torch.zeros(int(lib().siren_sse_workspace_bytes()), dtype=torch.uint8, device=device)
        _SSE_WS[key] = ws
    return ws


_ENC_WS: dict = {}


def enc_workspace(device) -> torch.Tensor:
    """Per-(device, stream) workspace of the encoder passes' channel sums (siren_enc_workspace_bytes;
    zeroed once, left zeroed by every launch)."""
    key = (device, torch.cuda.current_stream(device).cuda_stream)
    ws = _ENC_WS.get(key)
    if ws is None:
        ws = torch.zeros(int(lib().siren_enc_workspace_bytes()), dtype=torch.uint8, device=device)
        _ENC_WS[key] = ws
    return ws


def make_desc(dims, weights, biases, *, w0: float, prec: int, outermost_linear: bool,
              weights_batched: bool, batch: int, rows_per_batch: int, ff_B=None) -> SirenMLPDesc:
    L = len(dims) - 1
    if not 2 <= L <= MAX_LAYERS:
        raise ValueError(f"siren_mri_amd: {L} linear layers outside [2, {MAX_LAYERS}]")
    d = SirenMLPDesc()
    d.num_layers = L
    for i, v in enumerate(dims):
        d.dims[i] = int(v)
    d.outermost_linear = 1 if outermost_linear else 0
    d.prec = int(prec)
    d.weights_batched = 1 if weights_batched else 0
    d.w0 = float(w0)
    d.batch = int(batch)
    d.rows_per_batch = int(rows_per_batch)
    for l in range(L):
        d.weight[l] = weights[l].data_ptr()
        d.bias[l] = biases[l].data_ptr()
    if ff_B is not None:  # Fourier-feature input: x holds the raw coordinates
        d.ff_B = ff_B.data_ptr()
        d.ff_in = int(ff_B.shape[0])
    return d


def describe_only(dims, *, prec: int, outermost_linear: bool = True, weights_batched: bool = False,
                  batch: int = 1, rows_per_batch: int = 1, w0: float = 30.0, ff_in: int = 0):
    """Descriptor with fake (aligned, non-null) pointers — for size queries and validation."""
    L = len(dims) - 1
    d = SirenMLPDesc()
    d.num_layers = L
    for i, v in enumerate(dims):
        d.dims[i] = int(v)
    d.outermost_linear = 1 if outermost_linear else 0
    d.prec = int(prec)
    d.weights_batched = 1 if weights_batched else 0
    d.w0 = float(w0)
    d.batch = int(batch)
    d.rows_per_batch = int(rows_per_batch)
    for l in range(L):
        d.weight[l] = 256 * (l + 1)
        d.bias[l] = 256 * (l + 1) + 64
    if ff_in:
        d.ff_B = 256 * (L + 2)
        d.ff_in = int(ff_in)
    return d


class KernelTimer:
    """Context manager: HIP-event timing of every launch of one kernel class (see
    siren_timing_enable in include/siren_mri_amd.h)."""

    def __init__(self, kernel_class: int, max_launches: int = 4096):
        self.kernel_class = kernel_class
        self.max_launches = max_launches
        self.total_ms = 0.0
        self.launches = 0

    def __enter__(self):
        check(lib().siren_timing_enable(self.kernel_class, self.max_launches), "siren_timing_enable")
        return self

    def __exit__(self, *exc):
        tot = ctypes.c_double(0.0)
        n = ctypes.c_int64(0)
        try:
            check(lib().siren_timing_collect(ctypes.byref(tot), ctypes.byref(n)), "siren_timing_collect")
        finally:
            lib().siren_timing_disable()
        self.total_ms = tot.value
        self.launches = n.value
        return False

    def reset(self):
        """Drop the launches recorded so far and start again (same class and capacity)."""
        lib().siren_timing_disable()
        check(lib().siren_timing_enable(self.kernel_class, self.max_launches), "siren_timing_enable")

    @property
    def avg_ms(self) -> float:
        return self.total_ms / self.launches if self.launches else float("nan")
