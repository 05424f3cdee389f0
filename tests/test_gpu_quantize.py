"""The fused on-GPU weight quantizers against the torch-op formulation of the
same recipe and against the CPU oracle: bit-exact packed weights, scales and zeros (integer
and byte work, so exact equality is the bar)."""

import pytest
import torch

from oracle import oracle as orc
from torchao.dtypes import AffineQuantizedTensor
from torchao.quantization import (
    Int4WeightOnlyConfig,
    Int8DynamicActivationInt8WeightConfig,
    Int8WeightOnlyConfig,
    quantize_,
)

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _weights(N, K, seed):
    w = orc.make_linear_weight(N, K, seed=seed)
    w[0, :64] = 0.0  # constant group: max == min -> s = eps
    w[1, 5] = 3.0  # an outlier row
    return w


@pytest.mark.parametrize("N,K,g", [(64, 256, 32), (96, 1024, 64), (40, 512, 128),
                                   (8, 2048, 256), (130, 288, 32)])
def test_int4_quantize_pack_matches_oracle(N, K, g):
    w = _weights(N, K, seed=N + K)
    packed, sz = torch.ops.torchao.int4_quantize_pack(w.to(DEV), g, 1e-6)
    s, z = orc.int4_qparams(w, g)
    q = orc.int4_quantize(w, s, z, g)
    assert torch.equal(sz[..., 0].cpu(), s)
    assert torch.equal(sz[..., 1].cpu(), z)
    ref = torch.from_numpy(orc.pack_row_stream(q.numpy()).view("int32"))
    assert torch.equal(packed.cpu(), ref)


def test_int4_quantize_pack_3d_and_tiny_scales():
    w = torch.randn(3, 16, 256, dtype=torch.bfloat16) * 1e-7  # ranges below eps
    packed, sz = torch.ops.torchao.int4_quantize_pack(w.to(DEV), 32, 1e-6)
    assert packed.shape == (3, 16, 32) and sz.shape == (3, 16, 8, 2)
    w2 = w.reshape(48, 256)
    s, z = orc.int4_qparams(w2, 32)
    q = orc.int4_quantize(w2, s, z, 32)
    assert torch.equal(sz.reshape(48, 8, 2)[..., 0].cpu(), s)
    assert torch.equal(sz.reshape(48, 8, 2)[..., 1].cpu(), z)
    ref = torch.from_numpy(orc.pack_row_stream(q.numpy()).view("int32"))
    assert torch.equal(packed.reshape(48, 32).cpu(), ref)


@pytest.mark.parametrize("N,K", [(64, 256), (33, 1000), (512, 4096)])
def test_int8_quantize_rows_matches_oracle(N, K):
    w = _weights(N, K, seed=7 * N + K)
    q, s = torch.ops.torchao.int8_quantize_rows(w.to(DEV), torch.finfo(torch.float32).eps)
    s_ref = orc.int8_weight_qparams(w)
    assert torch.equal(s.cpu(), s_ref)
    assert torch.equal(q.cpu(), orc.int8_weight_quantize(w, s_ref))


def _torch_op_path(lin, config):
    """quantize_ with the fused kernels switched off (the torch-op formulation)."""
    import torchao.dtypes.affine_quantized_tensor as aqt

    saved = aqt._fused_weight_quant
    aqt._fused_weight_quant = lambda *a, **k: None
    try:
        quantize_(lin, config)
    finally:
        aqt._fused_weight_quant = saved
    return lin


@pytest.mark.parametrize("config", [Int4WeightOnlyConfig(group_size=32),
                                    Int4WeightOnlyConfig(group_size=128),
                                    Int8WeightOnlyConfig(),
                                    Int8DynamicActivationInt8WeightConfig()],
                         ids=["int4-g32", "int4-g128", "int8wo", "int8dq"])
def test_quantize_fast_path_is_bit_identical(config):
    torch.manual_seed(0)
    base = torch.nn.Linear(1024, 384, bias=False, dtype=torch.bfloat16, device=DEV)
    fast = torch.nn.Linear(1024, 384, bias=False, dtype=torch.bfloat16, device=DEV)
    slow = torch.nn.Linear(1024, 384, bias=False, dtype=torch.bfloat16, device=DEV)
    with torch.no_grad():
        fast.weight.copy_(base.weight)
        slow.weight.copy_(base.weight)
    quantize_(fast, config)
    _torch_op_path(slow, config)
    wf, ws = fast.weight, slow.weight
    if not isinstance(wf, AffineQuantizedTensor):  # int8 dyn: LinearActivationQuantizedTensor
        wf, ws = wf.original_weight_tensor, ws.original_weight_tensor
    names, _ = wf.tensor_impl.__tensor_flatten__()
    for n in names:
        a, b = getattr(wf.tensor_impl, n), getattr(ws.tensor_impl, n)
        assert a.dtype == b.dtype and a.shape == b.shape, n
        assert torch.equal(a, b), n
    x = torch.randn(3, 1024, dtype=torch.bfloat16, device=DEV)
    assert torch.equal(fast(x), slow(x))


def test_moe_3d_weights_per_expert():
    """3-D [E, N, K] weights (reference per-expert packing, tensor_core_tiled_layout.py:283-294):
    the fused quantizer packs all experts in one launch, each expert slice equals quantizing that
    expert alone, and an expert's linear (AQT index, as the MoE modules do) runs the int4 kernel."""
    import torch.nn.functional as F

    from torchao.dtypes import TensorCoreTiledLayout, to_affine_quantized_intx
    from torchao.quantization.quant_primitives import MappingType, ZeroPointDomain

    def quant(w):
        return to_affine_quantized_intx(
            w, MappingType.ASYMMETRIC, tuple([1] * (w.dim() - 1) + [32]), torch.int32, 0, 15,
            1e-6, zero_point_dtype=torch.bfloat16, preserve_zero=False,
            zero_point_domain=ZeroPointDomain.FLOAT, _layout=TensorCoreTiledLayout(8))

    E, N, K = 4, 256, 512
    w = torch.stack([orc.make_linear_weight(N, K, seed=50 + e) for e in range(E)]).to(DEV)
    qw = quant(w)
    assert qw.shape == (E, N, K) and qw.tensor_impl.packed_weight.shape == (E, N, K // 8)
    x = torch.randn(5, K, dtype=torch.bfloat16, device=DEV)
    for e in range(E):
        alone = quant(w[e].contiguous())
        assert torch.equal(qw[e].tensor_impl.packed_weight, alone.tensor_impl.packed_weight)
        assert torch.equal(qw[e].tensor_impl.scale_and_zero, alone.tensor_impl.scale_and_zero)
        y = F.linear(x, qw[e])
        ref = F.linear(x.float(), qw[e].dequantize().float())
        assert ((y.float() - ref).norm() / ref.norm()) < 1e-2
