"""Parameter routing for hypernetwork-predicted weights.

Same contract as the torchmeta pieces the reference vendors and uses on the hot path:
  MetaModule.meta_named_parameters   torchmeta/modules/module.py:17-23
  MetaSequential.forward(x, params)  torchmeta/modules/container.py:9-19
  get_subdict(params, key)           torchmeta/modules/utils.py:4-11
Parameter names are therefore identical (``net.net.{i}.0.weight`` for SingleBVPNet), so
HyperNetwork output dicts and state_dicts interoperate with the reference.
get_subdict here is a plain prefix filter (no per-call regex compilation).
"""
from __future__ import annotations

from collections import OrderedDict

from torch import nn


def get_subdict(dictionary, key=None):
    """Entries of `dictionary` under `key.` with the prefix stripped (None passes through)."""
    if dictionary is None:
        return None
    if not key:
        return dictionary
    prefix = key + "."
    n = len(prefix)
    return OrderedDict((k[n:], v) for k, v in dictionary.items() if k.startswith(prefix) and len(k) > n)


class MetaModule(nn.Module):
    """nn.Module whose forward accepts an optional ``params`` dict replacing its parameters."""

    def meta_named_parameters(self, prefix: str = "", recurse: bool = True):
        memo = set()
        modules = self.named_modules(prefix=prefix) if recurse else [(prefix, self)]
        for mod_prefix, module in modules:
            if not isinstance(module, MetaModule):
                continue
            for name, p in module._parameters.items():
                if p is None or p in memo:
                    continue
                memo.add(p)
                yield (mod_prefix + ("." if mod_prefix else "") + name, p)

    def meta_parameters(self, recurse: bool = True):
        for _, p in self.meta_named_parameters(recurse=recurse):
            yield p


class MetaSequential(nn.Sequential, MetaModule):
    """Sequential container that routes ``params`` sub-dicts to MetaModule children."""

    def forward(self, input, params=None):
        for name, module in self._modules.items():
            if isinstance(module, MetaModule):
                input = module(input, params=get_subdict(params, name))
            elif isinstance(module, nn.Module):
                input = module(input)
            else:
                raise TypeError(f"MetaSequential child {name!r} is not an nn.Module")
        return input
