"""Generate tests/golden/*.npz by running the REFERENCE torchao (read-only at /root/reference).

Run in the build container only (the reference does not exist on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 PYTHONPATH=/root/reference python3 oracle/gen_golden.py

It imports the reference's own quantize_ / configs / AffineQuantizedTensor on CPU
(Int4CPULayout for int4, since the default TensorCoreTiledLayout has no CPU pack kernel) and
records inputs and outputs as data. bf16 tensors are stored as their uint16 bit patterns.
Nothing of the reference's source is stored; the fixtures are numbers only.
"""

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(os.path.dirname(HERE), "tests", "golden")


def bf16_bits(t: torch.Tensor) -> np.ndarray:
    return t.detach().to(torch.bfloat16).contiguous().view(torch.int16).numpy().view(np.uint16)


def main():
    import torchao  # the reference (PYTHONPATH=/root/reference)

    assert os.path.realpath(torchao.__file__).startswith("/root/reference"), torchao.__file__
    from torchao.dtypes import Int4CPULayout
    from torchao.quantization import (
        Int4WeightOnlyConfig,
        Int8DynamicActivationInt8WeightConfig,
        Int8WeightOnlyConfig,
        quantize_,
    )
    from torchao.quantization.quant_api import _int8_symm_per_token_reduced_range_quant
    from torchao.quantization.quant_primitives import (
        MappingType,
        _choose_qparams_affine_tinygemm,
        _dequantize_affine_tinygemm,
        _quantize_affine_tinygemm,
    )

    sys.path.insert(0, HERE)
    import oracle  # only for the deterministic input generators

    os.makedirs(OUT, exist_ok=True)
    torch.manual_seed(0)

    # ---------------- int4 weight-only ----------------
    int4_cases = [
        # (N, K, g, Ms, weight distribution)
        (64, 256, 32, (1, 3, 16), "linear"),
        (128, 1024, 32, (1, 4, 16), "linear"),
        (96, 1024, 64, (1, 16), "normal"),
        (64, 2048, 128, (1, 5), "linear"),
        (48, 2048, 256, (1, 2), "normal"),
        (64, 4096, 32, (1, 8), "linear"),
        (40, 352, 32, (1, 9), "linear"),  # ragged: N % 8 != 0, K = 11 groups
        (16, 11008, 128, (1,), "linear"),  # Llama-2 FFN width along K
    ]
    for idx, (N, K, g, Ms, dist) in enumerate(int4_cases):
        if dist == "linear":
            w = oracle.make_linear_weight(N, K, seed=idx)
        else:
            gen = torch.Generator().manual_seed(100 + idx)
            w = (torch.randn(N, K, generator=gen) * 0.02).to(torch.bfloat16)
        if idx == 0:
            w[0, :32] = 0.25  # constant group -> scale clamps at eps
            w[1, 32:64] = 0.0
            w[2, :] = torch.linspace(-3, 3, K, dtype=torch.float32).to(torch.bfloat16)
        bias = (torch.randn(N, generator=torch.Generator().manual_seed(7 + idx)) * 0.1).to(
            torch.bfloat16
        )
        lin = torch.nn.Linear(K, N, bias=True).to(torch.bfloat16)
        with torch.no_grad():
            lin.weight.copy_(w)
            lin.bias.copy_(bias)
        # The reference's own primitives, exactly as Int4WeightOnlyConfig calls them
        # (quant_api.py:1126-1138 -> affine_quantized_tensor.py:287-336).
        bs = (1, g)
        s, z = _choose_qparams_affine_tinygemm(
            w, MappingType.ASYMMETRIC, bs, torch.int32, 0, 15, 1e-6,
            zero_point_dtype=torch.bfloat16,
        )
        q = _quantize_affine_tinygemm(w, bs, s, z, torch.int32, 0, 15)
        wdq = _dequantize_affine_tinygemm(
            q, bs, s, z, torch.int32, 0, 15, output_dtype=torch.bfloat16
        )
        has_cpu_layout = N % 16 == 0
        if has_cpu_layout:  # the full quantize_ path must agree with the primitives
            quantize_(lin, Int4WeightOnlyConfig(group_size=g, layout=Int4CPULayout()))
            q2, s2, z2 = lin.weight.tensor_impl.get_plain()
            assert torch.equal(q2, q) and torch.equal(s2, s.reshape(s2.shape))
            assert torch.equal(z2, z.reshape(z2.shape))
            assert torch.equal(lin.weight.dequantize(), wdq)
        qn = q.to(torch.uint8)
        rec = {
            "N": N, "K": K, "g": g, "w": bf16_bits(w), "bias": bf16_bits(bias),
            "q_u8": (qn[:, 0::2] << 4 | qn[:, 1::2]).numpy(),  # q[2i] << 4 | q[2i+1]
            "s": bf16_bits(s), "z": bf16_bits(z),
        }
        if N * K <= 256 * 1024:
            rec["w_dequant"] = bf16_bits(wdq)
        for M in Ms:
            x = oracle.make_activation(M, K, seed=1000 * idx + M)
            y_dq = torch.nn.functional.linear(x, wdq, bias)  # the reference dequant path
            rec[f"x_M{M}"] = bf16_bits(x)
            rec[f"y_dequant_M{M}"] = bf16_bits(y_dq)
            if has_cpu_layout:  # reference AQT linear -> aten._weight_int4pack_mm_for_cpu
                rec[f"y_tinygemm_cpu_M{M}"] = bf16_bits(lin(x))
        np.savez_compressed(os.path.join(OUT, f"int4_N{N}_K{K}_g{g}.npz"), **rec)
        print("int4", N, K, g, Ms)

    # ---------------- int8 weight-only ----------------
    for idx, (N, K, Ms) in enumerate([(64, 256, (1, 4, 16)), (96, 1024, (1, 8, 33))]):
        w = oracle.make_linear_weight(N, K, seed=50 + idx)
        bias = (torch.randn(N, generator=torch.Generator().manual_seed(60 + idx)) * 0.1).to(
            torch.bfloat16
        )
        lin = torch.nn.Linear(K, N, bias=True).to(torch.bfloat16)
        with torch.no_grad():
            lin.weight.copy_(w)
            lin.bias.copy_(bias)
        quantize_(lin, Int8WeightOnlyConfig())
        q, s, zp = lin.weight.tensor_impl.get_plain()
        rec = {"N": N, "K": K, "w": bf16_bits(w), "bias": bf16_bits(bias),
               "q": q.numpy(), "s": bf16_bits(s.reshape(-1)),
               "w_dequant": bf16_bits(lin.weight.dequantize())}
        for M in Ms:
            x = oracle.make_activation(M, K, seed=2000 + 10 * idx + M)
            rec[f"x_M{M}"] = bf16_bits(x)
            rec[f"y_M{M}"] = bf16_bits(lin(x))
        np.savez_compressed(os.path.join(OUT, f"int8wo_N{N}_K{K}.npz"), **rec)
        print("int8wo", N, K, Ms)

    # ---------------- int8 dynamic activation ----------------
    for idx, (N, K, Ms) in enumerate([(64, 256, (32, 48)), (128, 1024, (32, 128))]):
        w = oracle.make_linear_weight(N, K, seed=70 + idx)
        bias = (torch.randn(N, generator=torch.Generator().manual_seed(80 + idx)) * 0.1).to(
            torch.bfloat16
        )
        lin = torch.nn.Linear(K, N, bias=True).to(torch.bfloat16)
        with torch.no_grad():
            lin.weight.copy_(w)
            lin.bias.copy_(bias)
        quantize_(lin, Int8DynamicActivationInt8WeightConfig())
        wq, ws, _ = lin.weight.original_weight_tensor.tensor_impl.get_plain()
        rec = {"N": N, "K": K, "w": bf16_bits(w), "bias": bf16_bits(bias),
               "wq": wq.numpy(), "ws": bf16_bits(ws.reshape(-1))}
        for M in Ms:
            x = oracle.make_activation(M, K, seed=3000 + 10 * idx + M)
            if M == Ms[0]:
                x[0] = 0.0  # all-zero token: scale clamps at eps
                x[1, 5] = 40.0  # outlier token
            xa = _int8_symm_per_token_reduced_range_quant(x)
            xq, xs, _ = xa.tensor_impl.get_plain()
            rec[f"x_M{M}"] = bf16_bits(x)
            rec[f"xq_M{M}"] = xq.numpy()
            rec[f"xs_M{M}"] = bf16_bits(xs.reshape(-1))
            rec[f"y_M{M}"] = bf16_bits(lin(x))
        np.savez_compressed(os.path.join(OUT, f"int8dyn_N{N}_K{K}.npz"), **rec)
        print("int8dyn", N, K, Ms)


if __name__ == "__main__":
    main()
