"""Registration hygiene of the torchao:: operators (reference
test/test_ops.py:297-320, 470-500 run torch.library.opcheck on their tiled-layout ops).

opcheck covers the schema, the fake (meta) impl against the real one, AOT dispatch and
autograd registration for every op this package registers. The compile test runs the
reference harness's mode (generate.py:865-872: torch.compile(fullgraph=True,
mode="reduce-overhead")) over an int4-quantized two-layer MLP and compares with eager.
"""

import pytest
import torch

from oracle import oracle

import torchao.ops  # noqa: F401  (registers torch.ops.torchao.*)

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _int4_args(M=3, N=256, K=512, g=64):
    w = oracle.make_linear_weight(N, K, seed=1)
    s, z = oracle.int4_qparams(w, g)
    q = oracle.int4_quantize(w, s, z, g).to(DEV)
    packed = torch.ops.torchao.int4_pack(q)
    sz = torch.stack([s, z], -1).contiguous().to(DEV)
    x = oracle.make_activation(M, K, seed=2).to(DEV)
    return q, packed, sz, x, s, z, g


def _cases():
    q, packed, sz, x, s, z, g = _int4_args()
    N, K = q.shape
    bias = torch.randn(N, dtype=torch.bfloat16, device=DEV)
    sz_tiny = torch.stack([s, z], -1).transpose(0, 1).contiguous().to(DEV)
    tile = torch.ops.torchao.pack_tensor_core_tiled_layout(q, 8)
    w8 = torch.randint(-128, 128, (N, K), dtype=torch.int8, device=DEV)
    s8 = (torch.rand(N, device=DEV) * 0.01 + 1e-3).to(torch.bfloat16)
    xq, xs = torch.ops.torchao.int8_quantize_per_token(x)
    wbf = oracle.make_linear_weight(N, K, seed=9).to(DEV)
    u8 = ((q[:, ::2] << 4) | q[:, 1::2]).to(torch.uint8).contiguous()
    return {
        "unpack_tensor_core_tiled_layout": (tile, 8),
        "dequantize_tensor_core_tiled_layout": (tile, sz_tiny, g, 8),
        "pack_tensor_core_tiled_layout": (q, 8),
        "int4_pack": (q,),
        "int4_pack_u8": (u8,),
        "int4_unpack": (packed,),
        "int4_dequantize": (packed, sz, g, 0),
        "int4_weight_only_linear": (x, packed, sz, g, bias),
        "int8_weight_only_linear": (x, w8, s8, bias),
        "int8_quantize_per_token": (x,),
        "int4_quantize_pack": (wbf, g, 1e-6),
        "int8_quantize_rows": (wbf, 1e-5),
        "int8_scaled_mm": (xq, xs, w8, s8, bias),
        "int8_dyn_linear": (x[:1], w8, s8, None),
    }


def test_every_registered_op_is_covered():
    defined = {n.split("::")[-1].split(".")[0] for n in torchao.ops.lib._op_defs}
    assert defined and not defined - set(_cases()), sorted(defined - set(_cases()))


@pytest.mark.parametrize("name", [
    "unpack_tensor_core_tiled_layout", "dequantize_tensor_core_tiled_layout",
    "pack_tensor_core_tiled_layout", "int4_pack", "int4_pack_u8", "int4_unpack",
    "int4_dequantize", "int4_weight_only_linear", "int8_weight_only_linear",
    "int8_quantize_per_token", "int4_quantize_pack", "int8_quantize_rows", "int8_scaled_mm",
    "int8_dyn_linear",
])
def test_opcheck(name):
    args = _cases()[name]
    op = getattr(torch.ops.torchao, name).default
    torch.library.opcheck(op, args)


@pytest.mark.timeout(600)
def test_torch_compile_reduce_overhead_int4_mlp_matches_eager():
    """quantize_(Int4WeightOnlyConfig(32)) on a two-layer MLP; torch.compile(fullgraph=True,
    mode="reduce-overhead") traces through AffineQuantizedTensor to the custom op (inside
    inductor's CUDA graph) and gives the eager outputs, at M = 1 (GEMV) and M = 16 (MFMA)."""
    from torchao.quantization import Int4WeightOnlyConfig, quantize_

    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(1024, 2048), torch.nn.ReLU(),
                            torch.nn.Linear(2048, 512, bias=False))
    m = m.eval().to(torch.bfloat16).to(DEV)
    quantize_(m, Int4WeightOnlyConfig(group_size=32))
    cm = torch.compile(m, fullgraph=True, mode="reduce-overhead")
    with torch.no_grad():
        for M in (1, 16):
            x = torch.randn(M, 1024, dtype=torch.bfloat16, device=DEV)
            ref = m(x)
            for _ in range(3):  # warm-up, record, replay
                got = cm(x)
            torch.cuda.synchronize()
            assert torch.equal(got, ref), float((got.float() - ref.float()).abs().max())
