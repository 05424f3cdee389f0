"""Write checkpoints of the REFERENCE's own TensorCoreTiledLayout classes as test fixtures.

Run in the build container only (the reference does not exist on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 PYTHONPATH=/root/reference python3 oracle/gen_golden_ckpt.py

Each case runs the reference's own int4 weight path up to the tile pack, exactly as
``Int4WeightOnlyConfig`` -> ``AffineQuantizedTensor.from_hp_to_intx`` does it
(quant_api.py:1126-1138, affine_quantized_tensor.py:287-336):
  * ``TensorCoreTiledLayout(ikt).pre_process`` pads K to 1024 and N to 8
    (tensor_core_tiled_layout.py:127-135);
  * ``_choose_qparams_affine_tinygemm`` / ``_quantize_affine_tinygemm`` on the padded weight;
  * ``post_process`` pads again (:162-185);
  * the scales and zeros are packed by the reference's ``pack_tinygemm_scales_and_zeros``
    (quantization/utils.py:395-409), as ``from_plain`` does (:304-306).
The one step the reference cannot run on CPU is ``aten._convert_weight_to_int4pack`` (PyTorch
core, no CPU kernel): the nibbles go through ``oracle.pack_tile`` instead, the restatement of
that producer pinned nibble by nibble to PyTorch-ROCm's aten op on the MI355X
(tests/golden/aten_tile_map_rocm.npz) for map "rocm", and to the reference .cu unpack kernel's
index math for map "cuda". The reference's own ``TensorCoreTiledAQTTensorImpl`` and
``AffineQuantizedTensor`` are then constructed from that storage, placed in an ``nn.Linear`` the
way ``quantize_`` does (quant_api.py:1155), and its ``state_dict()`` is ``torch.save``d. So the
pickle carries the reference's own attribute set and class paths.

Per case, ``tests/golden/ref_ckpt_<fmt>_<tag>.pt`` (the reference pickle) and
``tests/golden/ref_ckpt_<fmt>_<tag>.npz`` (numbers only: the unpadded q as bytes, s, z, an input
x and the reference dequant -> F.linear output, computed by the reference's own
``_dequantize_affine_tinygemm``).
"""

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(os.path.dirname(HERE), "tests", "golden")

# (fmt, tag, lead (E,) or (), N, K, g, ikt). "rocm" needs N % 16 == 0 (PyTorch-ROCm's packer).
CASES = [
    ("rocm", "N48_K352_g32_ikt8", (), 48, 352, 32, 8),  # K padded 352 -> 1024
    ("rocm", "N64_K2048_g128_ikt2", (), 64, 2048, 128, 2),
    ("rocm", "N256_K4096_g32_ikt8", (), 256, 4096, 32, 8),
    ("cuda", "N40_K352_g32_ikt8", (), 40, 352, 32, 8),  # N % 16 != 0: the CUDA map only
    ("rocm", "E2_N32_K256_g32_ikt4", (2,), 32, 256, 32, 4),  # MoE [E, N, K] (:283-294)
]


def bf16_bits(t: torch.Tensor) -> np.ndarray:
    return t.detach().to(torch.bfloat16).contiguous().view(torch.int16).numpy().view(np.uint16)


def main():
    import torchao  # the reference (PYTHONPATH=/root/reference)

    assert os.path.realpath(torchao.__file__).startswith("/root/reference"), torchao.__file__
    from torchao.dtypes import AffineQuantizedTensor
    from torchao.dtypes.uintx.tensor_core_tiled_layout import (
        TensorCoreTiledAQTTensorImpl,
        TensorCoreTiledLayout,
    )
    from torchao.quantization.quant_primitives import (
        MappingType,
        ZeroPointDomain,
        _choose_qparams_affine_tinygemm,
        _dequantize_affine_tinygemm,
        _quantize_affine_tinygemm,
    )
    from torchao.quantization.utils import pack_tinygemm_scales_and_zeros

    sys.path.insert(0, HERE)
    import oracle  # the deterministic input generators and the tile packer restatement

    for idx, (fmt, tag, lead, N, K, g, ikt) in enumerate(CASES):
        E = lead[0] if lead else 1
        w = torch.stack([oracle.make_linear_weight(N, K, seed=500 + 10 * idx + e)
                         for e in range(E)]).reshape(*lead, N, K)
        layout = TensorCoreTiledLayout(inner_k_tiles=ikt)
        bs = (*([1] * len(lead)), 1, g)
        wp = layout.pre_process(w)
        s, z = _choose_qparams_affine_tinygemm(
            wp, MappingType.ASYMMETRIC, bs, torch.int32, 0, 15, 1e-6,
            zero_point_dtype=torch.bfloat16)
        q = _quantize_affine_tinygemm(wp, bs, s, z, torch.int32, 0, 15)
        q, s, z = layout.post_process(q, s, z, bs)
        Np, Kp = q.shape[-2:]
        # from_plain (:263-307) with the aten packer replaced by its restatement
        qp = q.reshape(E, Np, Kp)
        tiles = [torch.from_numpy(oracle.pack_tile(qp[e].numpy(), ikt, fmt)) for e in range(E)]
        packed = torch.stack(tiles) if lead else tiles[0]
        s2 = s.reshape(*lead, Np, -1)
        z2 = z.reshape(*lead, Np, -1)
        sz = pack_tinygemm_scales_and_zeros(s2, z2, s2.dtype)
        impl = TensorCoreTiledAQTTensorImpl(packed, sz, False, layout)
        aqt = AffineQuantizedTensor(impl, bs, w.shape, 0, 15, ZeroPointDomain.FLOAT,
                                    dtype=torch.bfloat16)
        bias = (torch.randn(*lead, N, generator=torch.Generator().manual_seed(idx)) * 0.1).to(
            torch.bfloat16)
        if lead:
            sd = {"experts.weight": aqt, "experts.bias": bias}
        else:
            lin = torch.nn.Linear(K, N, bias=True, dtype=torch.bfloat16)
            lin.weight = torch.nn.Parameter(aqt, requires_grad=False)  # quant_api.py:1155
            with torch.no_grad():
                lin.bias.copy_(bias)
            sd = lin.state_dict()
        torch.save(sd, os.path.join(OUT, f"ref_ckpt_{fmt}_{tag}.pt"))
        # expected values over the logical extent, from the reference's own dequant
        q_l = qp[:, :N, :K].reshape(*lead, N, K)
        s_l = s2[..., :N, : K // g]
        z_l = z2[..., :N, : K // g]
        wdq = _dequantize_affine_tinygemm(q_l, bs, s_l, z_l, torch.int32, 0, 15,
                                          output_dtype=torch.bfloat16)
        x = oracle.make_activation(3, K, seed=900 + idx)
        y = torch.nn.functional.linear(x, wdq.reshape(-1, N, K)[0], bias.reshape(-1, N)[0])
        qn = q_l.to(torch.uint8)
        np.savez_compressed(
            os.path.join(OUT, f"ref_ckpt_{fmt}_{tag}.npz"),
            fmt=fmt, N=N, K=K, g=g, ikt=ikt, E=E if lead else 0,
            q_u8=(qn[..., 0::2] << 4 | qn[..., 1::2]).numpy(),
            s=bf16_bits(s_l), z=bf16_bits(z_l), bias=bf16_bits(bias),
            x=bf16_bits(x), y_dequant=bf16_bits(y),
            **({"w_dequant": bf16_bits(wdq)} if wdq.numel() <= 256 * 1024 else {}),
        )
        print(fmt, tag, tuple(packed.shape), tuple(sz.shape))


if __name__ == "__main__":
    main()
