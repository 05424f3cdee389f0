"""int4 weight-only layout for MI355X: ``TensorCoreTiledLayout`` on gfx950.

``Int4WeightOnlyConfig()``'s default layout is ``TensorCoreTiledLayout(inner_k_tiles=8)``
(reference quant_api.py:1024). Keeping the class name means a user's config selects this
implementation with no code change; what changes is what the layout packs to and which kernel
its linear calls:

* reference: ``aten._convert_weight_to_int4pack`` tile format ``[N/8][K/(ikt*16)][32][ikt/2]``
  + tinygemm scales ``[K/g][N][2]``, K padded to 1024 and N to 8, linear via
  ``aten._weight_int4pack_mm`` (reference tensor_core_tiled_layout.py:58-114, 117-307);
* here: the gfx950 row-stream layout ``packed_weight`` int32 ``[N][K/8]`` (dword d of row n =
  k 8d..8d+7, bits 4i / 16+4i = q[8d+2i] / q[8d+2i+1]) + ``scale_and_zero`` bf16
  ``[N][K/g][2]``, no padding (K % group_size == 0 is already required by the config), linear
  via ``torch.ops.torchao.int4_weight_only_linear`` (HIP GEMV for M <= 2, or M <= 4 for weights
  of at most 32 Mi elements; bf16 MFMA above — csrc/gemm_mfma.hip ``gemv_max_m``).

``get_plain`` unpacks exactly (HIP kernel / host C++) instead of the reference's K x K identity
matmul through the int4 GEMM (:465-517). ``inner_k_tiles`` is kept as a field (it names the
reference tile format for ``torchao.ops.pack/unpack_tensor_core_tiled_layout``); the gfx950
layout does not depend on it. The packed bytes are device independent, so unlike the reference
(:309-326) ``.to(device)`` moves a quantized weight between CPU and GPU.
"""

from dataclasses import dataclass
from typing import Optional, Tuple

import torch
from torch.utils._python_dispatch import (
    is_traceable_wrapper_subclass,
    return_and_correct_aliasing,
)

from torchao.dtypes.affine_quantized_tensor import AffineQuantizedTensor, register_layout
from torchao.dtypes.utils import AQTTensorImpl, Layout
from torchao.quantization.quant_primitives import ZeroPointDomain
from torchao.quantization.utils import pack_scales_and_zeros_gfx950
from torchao.utils import fill_defaults

aten = torch.ops.aten

__all__ = ["TensorCoreTiledLayout", "TensorCoreTiledAQTTensorImpl",
           "convert_from_tensor_core_tiled"]


def _aqt_is_tensor_core_tile_uint4(aqt) -> bool:
    return aqt.tensor_impl.dtype == torch.int32 and aqt.quant_min == 0 and aqt.quant_max == 15


def _linear_bf16_act_uint4_weight_check(input_tensor, weight_tensor, bias) -> bool:
    return (
        not is_traceable_wrapper_subclass(input_tensor)
        and input_tensor.dtype == torch.bfloat16
        and isinstance(weight_tensor, AffineQuantizedTensor)
        and _aqt_is_tensor_core_tile_uint4(weight_tensor)
        and weight_tensor.dtype == torch.bfloat16
        and len(weight_tensor.shape) == 2
        and weight_tensor.zero_point_domain == ZeroPointDomain.FLOAT
        and isinstance(weight_tensor._layout, TensorCoreTiledLayout)
    )


def _linear_bf16_act_uint4_weight_impl(input_tensor, weight_tensor, bias):
    """y = x @ dequant(W)^T (+ bias) on the gfx950 kernels (reference :74-114)."""
    assert weight_tensor.block_size[0] == 1, (
        f"Requires groupwise quantization, got block_size: {weight_tensor.block_size}"
    )
    assert input_tensor.shape[-1] == weight_tensor.shape[1], (
        f"need input_tensor shape: {input_tensor.shape} final dim to match weight_tensor "
        f"shape: {weight_tensor.shape} second dim"
    )
    impl = weight_tensor.tensor_impl
    orig_dtype = input_tensor.dtype
    if input_tensor.numel() == 0:
        return input_tensor.new_empty((*input_tensor.shape[:-1], weight_tensor.shape[0]))
    x = input_tensor if orig_dtype is torch.bfloat16 else input_tensor.to(torch.bfloat16)
    y = torch.ops.torchao.int4_weight_only_linear(
        x, impl.packed_weight, impl.scale_and_zero, weight_tensor.block_size[-1], bias
    )
    return y if orig_dtype is torch.bfloat16 else y.to(orig_dtype)


def _is_tile_storage(packed_weight: torch.Tensor) -> bool:
    """The reference's storage: int32 [(E,) N/8, K/(ikt*16), 32, ikt/2] (tensor_core_tiled_layout.py
    docstring, :191-211); the gfx950 row-stream storage is [(E,) N, K/8]."""
    return packed_weight.dim() in (4, 5) and packed_weight.shape[-2] == 32


def convert_from_tensor_core_tiled(
    packed_weight: torch.Tensor,
    scale_and_zero: torch.Tensor,
    inner_k_tiles: int,
    shape: Optional[Tuple[int, ...]] = None,
    tile_format=-1,
) -> Tuple[torch.Tensor, torch.Tensor]:
    """Reference ``TensorCoreTiledAQTTensorImpl`` storage -> this layout's storage.

    ``packed_weight`` int32 [(E,) Np/8, Kp/(ikt*16), 32, ikt/2] in the tile format (``tile_format``:
    "cuda" for a checkpoint written by a CUDA build, "rocm" for one written by PyTorch-ROCm; -1 =
    ``torchao.ops.default_tile_format()``), ``scale_and_zero`` bf16 [(E,) Kp/g, Np, 2] (tinygemm
    packing, reference quantization/utils.py:395-409). Returns row-stream ``packed_weight``
    [(E,) N, K/8] and ``scale_and_zero`` [(E,) N, K/g, 2], un-padded to ``shape``'s trailing
    (N, K) (the reference pads K to 1024 and N to 8, tensor_core_tiled_layout.py:127-188).
    Bit-exact: nibbles are moved, scales and zeros copied. Runs on the tensors' device (HIP
    kernels on GPU, host C++ on CPU)."""
    from torchao.ops import unpack_tensor_core_tiled_layout

    lead = packed_weight.shape[:-4]
    Np = packed_weight.shape[-4] * 8
    Kp = packed_weight.shape[-3] * inner_k_tiles * 16
    N, K = (Np, Kp) if shape is None else (int(shape[-2]), int(shape[-1]))
    if N > Np or K > Kp:
        raise ValueError(f"tile storage [{Np}, {Kp}] smaller than the logical shape {(N, K)}")
    if scale_and_zero.shape[-3:-1] != (scale_and_zero.shape[-3], Np) or scale_and_zero.shape[-1] != 2:
        raise ValueError(f"scale_and_zero {tuple(scale_and_zero.shape)} is not [Kp/g, {Np}, 2]")
    groups_p = scale_and_zero.shape[-3]
    g = Kp // groups_p
    if g * groups_p != Kp or K % g:
        raise ValueError(f"group size {Kp}/{groups_p} does not divide K={K}")
    pw = packed_weight.reshape(-1, *packed_weight.shape[-4:])
    rows = []
    for e in range(pw.shape[0]):
        q = unpack_tensor_core_tiled_layout(pw[e].contiguous(), inner_k_tiles, tile_format)
        rows.append(torch.ops.torchao.int4_pack(q[:N, :K].contiguous()))
    packed = torch.stack(rows).reshape(*lead, N, K // 8)
    sz = scale_and_zero.transpose(-3, -2)[..., :N, : K // g, :].contiguous()
    return packed, sz


@dataclass(frozen=True)
class TensorCoreTiledLayout(Layout):
    """int4 layout for the tinygemm-equivalent kernels (gfx950 row-stream packing)."""

    inner_k_tiles: int = 8

    def pre_process(self, input: torch.Tensor) -> torch.Tensor:
        if input.shape[-1] % 32 != 0:
            raise ValueError(
                f"TensorCoreTiledLayout (gfx950) needs in_features % 32 == 0, got {input.shape[-1]}"
            )
        return input

    def extra_repr(self):
        return f"inner_k_tiles={self.inner_k_tiles}"


@register_layout(TensorCoreTiledLayout)
class TensorCoreTiledAQTTensorImpl(AQTTensorImpl):
    """Storage: ``packed_weight`` int32 [(E,) N, K/8], ``scale_and_zero`` bf16 [(E,) N, K/g, 2]."""

    def __new__(
        cls,
        packed_weight: torch.Tensor,
        scale_and_zero: torch.Tensor,
        transposed: bool,
        _layout: Layout,
    ):
        return torch.Tensor._make_wrapper_subclass(
            cls,
            packed_weight.shape,
            device=packed_weight.device,
            layout=packed_weight.layout,
            dtype=packed_weight.dtype,
            requires_grad=False,
        )

    def __init__(
        self,
        packed_weight: torch.Tensor,
        scale_and_zero: torch.Tensor,
        transposed: bool,
        _layout: Layout,
    ):
        self.packed_weight = packed_weight
        self.scale_and_zero = scale_and_zero
        self.transposed = transposed
        self._layout = _layout

    def __tensor_flatten__(self):
        return ["packed_weight", "scale_and_zero"], [self.transposed, self._layout]

    @classmethod
    def _adopt(cls, impl, shape):
        """Called when an AQT is unpickled / unflattened with this impl (AffineQuantizedTensor
        .__setstate__): storage in the reference tile format (a torchao checkpoint) is converted
        to the gfx950 row-stream layout, un-padded to the AQT's logical ``shape``; storage of
        this layout is returned as is. The tile map (CUDA or ROCm build) must have been chosen
        explicitly (``torchao.ops.checkpoint_tile_format`` / ``set_default_tile_format``);
        otherwise this raises rather than guess."""
        if not _is_tile_storage(impl.packed_weight):
            return impl
        from torchao.ops import chosen_checkpoint_tile_format

        packed, sz = convert_from_tensor_core_tiled(
            impl.packed_weight, impl.scale_and_zero, impl._layout.inner_k_tiles, shape,
            chosen_checkpoint_tile_format())
        return cls(packed, sz, impl.transposed, impl._layout)

    @classmethod
    def __tensor_unflatten__(cls, tensor_data_dict, tensor_attributes, outer_size, outer_stride):
        transposed, layout = tensor_attributes
        return cls(
            tensor_data_dict["packed_weight"], tensor_data_dict["scale_and_zero"], transposed, layout
        )

    @classmethod
    def from_plain(
        cls,
        int_data: torch.Tensor,
        scale: torch.Tensor,
        zero_point: Optional[torch.Tensor],
        _layout: Layout,
    ):
        assert isinstance(_layout, TensorCoreTiledLayout)
        assert int_data.dtype == torch.int32, "int4 packing expects int32 values in [0, 15]"
        assert int_data.dim() in (2, 3), f"expected 2D (or 3D MoE) int data, got {int_data.dim()}D"
        lead = int_data.shape[:-1]  # (N,) or (E, N)
        K = int_data.shape[-1]
        # rows are packed independently, so MoE experts pack as one [E*N, K] matrix
        packed = torch.ops.torchao.int4_pack(int_data.reshape(-1, K).contiguous())
        packed = packed.reshape(*lead, K // 8)
        scale = scale.reshape(*lead, -1)
        if zero_point is None:
            zero_point = torch.zeros_like(scale)
        zero_point = zero_point.reshape(*lead, -1)
        sz = pack_scales_and_zeros_gfx950(scale, zero_point.to(scale.dtype), scale.dtype)
        return cls(packed, sz, False, _layout)

    def to(self, *args, **kwargs):
        device = self._get_to_kwargs(*args, **kwargs)["device"]
        return type(self)(
            self.packed_weight.to(device),
            self.scale_and_zero.to(device),
            self.transposed,
            self._layout,
        )

    def _apply_fn_to_data(self, fn):
        return type(self)(
            fn(self.packed_weight), fn(self.scale_and_zero), self.transposed, self._layout
        )

    @property
    def block_size(self) -> Tuple[int, ...]:
        K = self.packed_weight.shape[-1] * 8
        g = K // self.scale_and_zero.shape[-2]
        return tuple([1] * (self.packed_weight.dim() - 1) + [g])

    def get_plain(self) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        K8 = self.packed_weight.shape[-1]
        lead = self.packed_weight.shape[:-1]
        q = torch.ops.torchao.int4_unpack(self.packed_weight.reshape(-1, K8).contiguous())
        q = q.reshape(*lead, K8 * 8)
        scale = self.scale_and_zero[..., 0].contiguous()
        zero = self.scale_and_zero[..., 1].contiguous()
        return q, scale, zero

    def get_layout(self) -> Layout:
        return self._layout

    @classmethod
    def __torch_dispatch__(cls, func, types, args, kwargs):
        kwargs = {} if kwargs is None else kwargs
        if func is aten.detach.default:
            return return_and_correct_aliasing(
                func, args, kwargs, args[0]._apply_fn_to_data(torch.detach)
            )
        if func is aten.clone.default:
            return return_and_correct_aliasing(
                func, args, kwargs, args[0]._apply_fn_to_data(torch.clone)
            )
        if func is aten.copy_.default:
            dst, src = args[0], args[1]
            if (
                isinstance(src, cls)
                and dst.packed_weight.shape == src.packed_weight.shape
                and dst.scale_and_zero.shape == src.scale_and_zero.shape
                and type(dst._layout) is type(src._layout)
            ):
                dst.packed_weight.copy_(src.packed_weight)
                dst.scale_and_zero.copy_(src.scale_and_zero)
                return
            raise ValueError(f"Not supported args for copy_ due to metadata mismatch: {dst, src}")
        if func in (aten.select.int, aten.index.Tensor):
            assert not (func is aten.select.int and args[1] != 0), (
                "aten.select.int currently only has support for dim=0"
            )
            return return_and_correct_aliasing(
                func,
                args,
                kwargs,
                args[0]._apply_fn_to_data(lambda t: func(t, *args[1:], **kwargs)),
            )
        if func is aten.t.default:
            # record the transpose, keep the packing (reference :374-384)
            self = args[0]
            return return_and_correct_aliasing(
                func,
                args,
                kwargs,
                cls(self.packed_weight, self.scale_and_zero, not self.transposed, self._layout),
            )
        if func is aten.slice.Tensor:
            self, dim, start, end, step = fill_defaults(args, 5, [0, None, None, 1])
            return return_and_correct_aliasing(func, args, kwargs, self._slice(dim, start, end, step))
        raise NotImplementedError(
            f"TensorCoreTiledAQTTensorImpl dispatch: attempting to run {func}, this is not supported"
        )

    __torch_function__ = torch._C._disabled_torch_function_impl

    def _slice(self, dim: int, start, end, step):
        """Slice in the logical [N, K] index space: rows map 1:1, k maps to k/8 packed dwords
        and k/g scale groups (start/end must then be multiples of the group size)."""
        assert step == 1, "only step 1 slicing is supported"
        N = self.packed_weight.shape[-2]
        K = self.packed_weight.shape[-1] * 8
        if self.packed_weight.dim() != 2 or dim not in (0, 1):
            raise NotImplementedError(f"slice on dim {dim} of a {self.packed_weight.dim()}D impl")
        size = N if dim == 0 else K
        start = 0 if start is None else start
        end = size if end is None else min(end, size)
        if dim == 0:
            pw = aten.slice.Tensor(self.packed_weight, 0, start, end, 1)
            sz = aten.slice.Tensor(self.scale_and_zero, 0, start, end, 1)
        else:
            g = K // self.scale_and_zero.shape[1]
            if start % g or (end % g and end != K):
                raise ValueError(f"k-slice [{start}, {end}) must align to the group size {g}")
            pw = aten.slice.Tensor(self.packed_weight, 1, start // 8, end // 8, 1)
            sz = aten.slice.Tensor(self.scale_and_zero, 1, start // g, (end + g - 1) // g, 1)
        return type(self)(pw, sz, self.transposed, self._layout)
