"""Adam for the fitting loop (training.py:29: torch.optim.Adam(lr=lr, params=model.parameters())).

`Adam` is torch.optim.Adam — same constructor, param_groups, state keys ('step', 'exp_avg',
'exp_avg_sq') and state_dict, so checkpoints move freely between the two — whose step() runs ONE
native launch (siren_adam_step) over all fp32 CUDA parameters of a group instead of torch's
chain of foreach kernels, with the foreach path's arithmetic (see csrc/siren_adam.hip).
Groups it cannot take (amsgrad, capturable/differentiable/fused flags, non-fp32 or CPU tensors,
sparse gradients, tensor-valued lr/betas) go through torch's own step().
"""
from __future__ import annotations

import ctypes
import math

import torch

from . import _native


def _same_layout(a: torch.Tensor, b: torch.Tensor) -> bool:
    """Same element order in storage: equal strides on every dimension longer than 1 (a 1x1 conv
    weight's channels-last gradient has strides (C, 1, C, C) against the parameter's (C, 1, 1, 1):
    the size-1 dimensions' strides carry no layout)."""
    return a.shape == b.shape and all(sa == sb for n, sa, sb in zip(a.shape, a.stride(), b.stride()) if n > 1)


class Adam(torch.optim.Adam):
    """torch.optim.Adam whose step is one native launch (see the module docstring).

    ``enable_graph_mode()`` makes the step hipGraph-capturable: the bias corrections come from a
    device-side step count instead of host floats baked into the captured launch: each workgroup
    of the update launch advances its own counter and looks the step's scalars up in a table the
    host computed once (siren_adam_desc.dev_steps; no extra launch), or, for betas whose table
    would be too long, a single-thread launch per group advances one counter and computes them
    (siren_adam_scalars). The host-side ``state['step']`` keeps counting eager calls only;
    ``sync_graph_steps()`` copies the device counters back into it."""

    _graph_mode = False
    # graph mode: {step_size, bias_correction2_sqrt} of steps 1, 2, ... up to the step where both
    # bias corrections reach 1 in double (the eager path's expressions; later steps repeat the last
    # entry; siren_adam_scalars_table); betas so close to 1 that this takes more than _TABLE_MAX
    # steps use siren_adam_scalars (the same expressions computed on the device)
    _TABLE_MAX = 1 << 22

    _bias_cache: dict = {}

    @classmethod
    def _bias_corrections(cls, beta1, beta2):
        """(1 - beta1^t, sqrt(1 - beta2^t)) for t = 1 .. the step where both reach 1 in double, as
        float64 arrays (the eager path's expressions, evaluated once per betas), or None when that
        takes more than _TABLE_MAX steps. The table's length depends on the betas only."""
        import numpy as np
        key = (float(beta1), float(beta2), cls._TABLE_MAX)
        if key not in cls._bias_cache:
            bc1s, sq2s = [], []
            t = 1
            while True:
                bc1 = 1 - beta1 ** t
                bc2 = 1 - beta2 ** t
                bc1s.append(bc1)
                sq2s.append(bc2 ** 0.5)
                if (bc1 == 1.0 and bc2 == 1.0) or t >= cls._TABLE_MAX:
                    break
                t += 1
            done = bc1 == 1.0 and bc2 == 1.0
            cls._bias_cache[key] = (np.array(bc1s), np.array(sq2s)) if done else None
        return cls._bias_cache[key]

    @classmethod
    def _scalar_rows(cls, lr, beta1, beta2):
        """Host rows {step_size, bias_correction2_sqrt} of steps 1, 2, ... (float32), or None."""
        import numpy as np
        bc = cls._bias_corrections(beta1, beta2)
        if bc is None:
            return None
        bc1, sq2 = bc
        # (lr / bc1) * -1 elementwise in double: the same IEEE division as the eager expression
        return torch.from_numpy(np.stack([(lr / bc1) * -1, sq2], axis=1).astype(np.float32))

    @classmethod
    def _scalar_table(cls, lr, beta1, beta2, device):
        rows = cls._scalar_rows(lr, beta1, beta2)
        return None if rows is None else rows.to(device)

    def enable_graph_mode(self):
        self._graph_mode = True
        self._dev_step = {}

    def _group_table(self, group, device):
        """The group's device step-scalar table for its current (lr, betas), or None (computed
        form). A table replaced by a betas change stays alive until release_graph_buffers(): a
        hipGraph captured earlier may still point at it. An lr change keeps the table
        (its length depends on the betas only) and rewrites it in place, so an lr schedule
        allocates nothing and a captured graph replays the new lr."""
        lr_now, betas = float(group["lr"]), tuple(float(b) for b in group["betas"])
        tables = self.__dict__.setdefault("_tables", {})
        retired = self.__dict__.setdefault("_retired", [])
        ent = tables.get(id(group))
        if ent is None or ent[0] != betas:
            if ent is not None:
                retired.append(ent[2])
            ent = [betas, lr_now, self._scalar_table(lr_now, *betas, device)]
            tables[id(group)] = ent
        elif ent[1] != lr_now:
            if ent[2] is not None:
                ent[2].copy_(self._scalar_rows(lr_now, *betas))
            ent[1] = lr_now
        return ent[2]

    def update_graph_scalars(self):
        """Graph mode: bring every group's step-scalar table to its current lr without stepping
        (an lr scheduler between replays of a captured step; an eager step() does it itself).
        The table form only: the computed form bakes lr into the captured launch."""
        for group in self.param_groups:
            ent = self.__dict__.get("_tables", {}).get(id(group))
            if ent is not None and ent[2] is not None:
                self._group_table(group, ent[2].device)

    def release_graph_buffers(self):
        """Drop the step-scalar tables and step counters replaced by a betas change or a new
        parameter count. Call it once no hipGraph captured before the change will be replayed
        again (a captured launch keeps pointing at the buffers it was captured with)."""
        self.__dict__.get("_retired", []).clear()

    def sync_graph_steps(self):
        for group in self.param_groups:
            dev = getattr(self, "_dev_step", {}).get(id(group))
            if dev is None:
                continue
            if "t" in dev:
                t = float(dev["t"].item())
            elif dev["steps"]:
                t = float(dev["steps"][0][0].item())
            else:
                continue
            for p in group["params"]:
                if p in self.state and "step" in self.state[p]:
                    self.state[p]["step"].fill_(t)

    def _native_reject(self, group):
        """Why a group cannot take the native step (None when it can)."""
        if group["amsgrad"] or group.get("capturable") or group.get("differentiable") or group.get("fused"):
            return "amsgrad/capturable/differentiable/fused flag"
        if group.get("decoupled_weight_decay", False):
            return "decoupled_weight_decay"
        if any(isinstance(group[k], torch.Tensor) for k in ("lr",)) or any(
                isinstance(b, torch.Tensor) for b in group["betas"]):
            return "tensor-valued lr/betas"
        for p in group["params"]:
            if p.grad is None:
                continue
            if not p.is_cuda or p.dtype != torch.float32 or p.grad.is_sparse or p.grad.dtype != torch.float32:
                return f"param {tuple(p.shape)}: device/dtype ({p.device}, {p.dtype}, grad {p.grad.dtype})"
            # the update is elementwise over the storage: any dense layout (row-major, or the conv
            # encoder's channels-last weights) works when the gradient and the moments share it
            if not (p.is_contiguous() or p.is_contiguous(memory_format=torch.channels_last)):
                return f"param {tuple(p.shape)}: not dense (strides {p.stride()})"
            if not _same_layout(p.grad, p):
                return f"param {tuple(p.shape)}: grad strides {p.grad.stride()} != param strides {p.stride()}"
            st = self.state.get(p)
            if st and "exp_avg" in st and not (_same_layout(st["exp_avg"], p) and _same_layout(st["exp_avg_sq"], p)):
                return f"param {tuple(p.shape)}: moment strides differ from the parameter's"
        return None

    def _native_ok(self, group) -> bool:
        return self._native_reject(group) is None

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        fallback = [g for g in self.param_groups if not self._native_ok(g)]
        fallback_ids = {id(g) for g in fallback}
        if fallback:
            # torch's step over the groups we do not take (the native ones are skipped below)
            saved = self.param_groups
            self.param_groups = fallback
            try:
                super().step()
            finally:
                self.param_groups = saved
        lib = _native.lib()
        for group in self.param_groups:
            if id(group) in fallback_ids:
                continue
            beta1, beta2 = group["betas"]
            params = [p for p in group["params"] if p.grad is not None]
            # lazy state init exactly as torch.optim.Adam._init_group (step on the CPU, fp32)
            for p in params:
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0, dtype=torch.float32)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            # tensors sharing a step count go together (normally: all of them)
            steps = [self.state[p]["step"] for p in params]
            if steps:
                torch._foreach_add_(steps, 1)  # one dispatch for all the CPU step counters
            by_step = {}
            for p, st in zip(params, steps):
                by_step.setdefault(float(st.item()), []).append(p)
            if not params:
                continue
            stream = ctypes.c_void_p(_native.stream_handle(params[0].device))
            dev_scalars = None
            tab = None
            dev = None
            if self._graph_mode:
                if len(by_step) != 1:
                    raise RuntimeError("siren_mri_amd.optim.Adam: graph mode needs one step count per group")
                dev = self._dev_step.get(id(group))
                if dev is None:
                    # {"t0": count before this step, "steps": per-launch workgroup counters (table form),
                    #  "t": the group counter and "scalars" (computed form)}
                    dev = {"t0": next(iter(by_step)) - 1, "steps": {}}
                    self._dev_step[id(group)] = dev
                tab = self._group_table(group, params[0].device)
                if tab is None:
                    if "t" not in dev:
                        dev["t"] = torch.full((1,), dev["t0"], dtype=torch.float64, device=params[0].device)
                        dev["scalars"] = torch.zeros(2, dtype=torch.float32, device=params[0].device)
                    rc = lib.siren_adam_scalars(dev["t"].data_ptr(), float(group["lr"]), float(beta1), float(beta2),
                                                dev["scalars"].data_ptr(), stream)
                    if rc != 0:
                        raise _native.NativeError(_native.last_error())
                    dev_scalars = dev["scalars"].data_ptr()
            for t, plist in by_step.items():
                bc1 = 1 - beta1 ** t
                bc2 = 1 - beta2 ** t
                for i0 in range(0, len(plist), _native.ADAM_MAX_TENSORS):
                    chunk = plist[i0:i0 + _native.ADAM_MAX_TENSORS]
                    d = _native.SirenAdamDesc()
                    d.num_tensors = len(chunk)
                    d.maximize = 1 if group["maximize"] else 0
                    d.lr, d.beta1, d.beta2 = group["lr"], beta1, beta2
                    d.eps, d.weight_decay = group["eps"], group["weight_decay"]
                    d.one_minus_beta1, d.one_minus_beta2 = 1 - beta1, 1 - beta2
                    d.step_size = (group["lr"] / bc1) * -1
                    d.bias_correction2_sqrt = bc2 ** 0.5
                    d.dev_scalars = dev_scalars
                    for k, p in enumerate(chunk):
                        st = self.state[p]
                        d.numel[k] = p.numel()
                        d.param[k] = p.data_ptr()
                        d.grad[k] = p.grad.data_ptr()
                        d.exp_avg[k] = st["exp_avg"].data_ptr()
                        d.exp_avg_sq[k] = st["exp_avg_sq"].data_ptr()
                    if tab is not None:
                        # table form: the launch's workgroups each advance their own counter
                        nblk = lib.siren_adam_num_blocks(ctypes.byref(d))
                        cnt = dev["steps"].get(i0)
                        if cnt is None or cnt.numel() != max(nblk, 1):
                            if cnt is None:
                                cnt = torch.full((max(nblk, 1),), dev["t0"], dtype=torch.float64, device=p.device)
                            else:
                                # carry the device count over (no host sync; every workgroup's
                                # counter holds the same step after a launch)
                                self._retired.append(cnt)
                                cnt = cnt[:1].expand(max(nblk, 1)).clone()
                            dev["steps"][i0] = cnt
                        d.dev_steps = cnt.data_ptr()
                        d.dev_table = tab.data_ptr()
                        d.table_n = tab.shape[0]
                    if lib.siren_adam_step(ctypes.byref(d), stream) != 0:
                        raise _native.NativeError(_native.last_error())
        return loss
