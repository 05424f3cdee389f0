"""Python handle of the persistent int4 decode chain (csrc/decode_chain.hip, C-ABI
``tao_chain_*`` in include/torchao_mi355x.h): dependent M = 1 int4 weight-only linears in one
launch, each workgroup issuing its share of the next linear's weight loads before it waits for
that linear's input.

    chain = DecodeChain([
        ChainPhase(packed, sz, g, x=x_buf, y=qkv, norm_w=attn_norm, eps=1e-5),
        ChainPhase(packed_o, sz_o, g, x=qkv, x_phase=0, y=h, residual=x_buf),
        ...
    ])
    chain.run()            # on torch's current stream; capturable in a HIP graph
    chain.check()          # synchronous: raises if a hand-off timed out

Buffers named by the phases must stay alive (and at fixed addresses) while the chain exists.
"""

import ctypes
from dataclasses import dataclass
from typing import List, Optional

import torch

from torchao import _lib

__all__ = ["ChainPhase", "DecodeChain", "TaoChainPhase"]


class TaoChainPhase(ctypes.Structure):
    _fields_ = [
        ("packed", ctypes.c_void_p),
        ("sz", ctypes.c_void_p),
        ("x", ctypes.c_void_p),
        ("norm_w", ctypes.c_void_p),
        ("residual", ctypes.c_void_p),
        ("y", ctypes.c_void_p),
        ("N", ctypes.c_int64),
        ("K", ctypes.c_int64),
        ("group_size", ctypes.c_int64),
        ("x_phase", ctypes.c_int32),
        ("epilogue", ctypes.c_int32),
        ("eps", ctypes.c_float),
        ("reserved", ctypes.c_int32),
    ]


@dataclass
class ChainPhase:
    """One linear of the chain: y = epi(RMSNorm?(x) @ W^T) (+ residual)."""

    packed: torch.Tensor                 # int32 [N, K/8] (gfx950 row-stream int4)
    scale_and_zero: torch.Tensor         # bf16 [N, K/g, 2]
    group_size: int
    x: torch.Tensor                      # bf16 [K] (or a phase's y holding >= K values)
    y: torch.Tensor                      # bf16 [N] ([N/2] with swiglu)
    x_phase: int = -1                    # index of the phase writing x, -1 = written before run
    norm_w: Optional[torch.Tensor] = None
    eps: float = 1e-5
    residual: Optional[torch.Tensor] = None
    swiglu: bool = False


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


class DecodeChain:
    def __init__(self, phases: List[ChainPhase]):
        arr = (TaoChainPhase * len(phases))()
        self._keep = []  # the tensors the device-side table points at
        for i, p in enumerate(phases):
            N, K8 = p.packed.shape
            for t in (p.packed, p.scale_and_zero, p.x, p.y, p.norm_w, p.residual):
                if t is not None and (not t.is_cuda or not t.is_contiguous()):
                    raise RuntimeError(f"chain phase {i}: operands must be contiguous CUDA tensors")
            out_n = N // 2 if p.swiglu else N
            if p.y.numel() < out_n or p.x.numel() < K8 * 8:
                raise RuntimeError(f"chain phase {i}: x / y too small for [{N}, {K8 * 8}]")
            arr[i] = TaoChainPhase(_ptr(p.packed), _ptr(p.scale_and_zero), _ptr(p.x),
                                   _ptr(p.norm_w), _ptr(p.residual), _ptr(p.y), N, K8 * 8,
                                   int(p.group_size), int(p.x_phase), 1 if p.swiglu else 0,
                                   float(p.eps), 0)
            self._keep.append(p)
        handle = ctypes.c_void_p()
        _lib.call("tao_chain_create", ctypes.cast(arr, ctypes.c_void_p), len(phases),
                  ctypes.byref(handle))
        self._handle = handle
        self.n_phases = len(phases)

    def run(self) -> None:
        _lib.call("tao_chain_run", self._handle, torch.cuda.current_stream().cuda_stream)

    def status(self):
        """(aborted_phase or None, launches completed) — a synchronous device read."""
        ab, n = ctypes.c_int(0), ctypes.c_uint(0)
        _lib.call("tao_chain_status", self._handle, ctypes.byref(ab), ctypes.byref(n))
        return (ab.value - 1 if ab.value else None), n.value

    def check(self) -> None:
        aborted, _ = self.status()
        if aborted is not None:
            raise RuntimeError(f"decode chain: the input of phase {aborted} never arrived "
                               "(hand-off timed out); outputs are invalid, call reset()")

    def profile(self, enable: bool = True) -> Optional[torch.Tensor]:
        """Record per (phase, workgroup) wall-clock stamps on later runs: returns the int64
        [phases, grid, 4] device buffer (start, input ready, tasks done, signalled; 100 MHz)."""
        grid = ctypes.c_int(0)
        if not enable:
            _lib.call("tao_chain_profile", self._handle, None, ctypes.byref(grid))
            self._prof = None
            return None
        _lib.call("tao_chain_profile", self._handle, None, ctypes.byref(grid))
        self._prof = torch.zeros(self.n_phases, grid.value, 4, dtype=torch.int64, device="cuda")
        _lib.call("tao_chain_profile", self._handle, self._prof.data_ptr(), ctypes.byref(grid))
        return self._prof

    def reset(self) -> None:
        _lib.call("tao_chain_reset", self._handle)

    def close(self) -> None:
        if getattr(self, "_handle", None) is not None and self._handle.value:
            _lib.call("tao_chain_destroy", self._handle)
            self._handle = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:  # pragma: no cover - interpreter shutdown
            pass
