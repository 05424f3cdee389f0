"""MoE decode on 3-D int4 weights: the grouped GEMV (tao_int4wo_grouped_gemv_bf16, one launch for
the A activated experts) against the reference's one-token branch of
ConditionalFeedForwardAOQuantizable (_models/mixtral-moe/model.py:360-384: index the 3-D weights
by the top-k experts, then one F.linear per expert on the AQT). Each expert's rows run the plain
M = 1 GEMV body, so the results are bit-identical."""

import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _quant3d(w, g=32):
    from torchao.dtypes import TensorCoreTiledLayout, to_affine_quantized_intx
    from torchao.quantization.quant_primitives import MappingType, ZeroPointDomain

    return to_affine_quantized_intx(
        w, MappingType.ASYMMETRIC, (1, 1, g), torch.int32, 0, 15, 1e-6,
        zero_point_dtype=torch.bfloat16, preserve_zero=False,
        zero_point_domain=ZeroPointDomain.FLOAT, _layout=TensorCoreTiledLayout(8))


def _experts(E, N, K, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    w = (torch.rand(E, N, K, device=DEV, generator=g) * 2 - 1) / math.sqrt(K)
    return _quant3d(w.to(torch.bfloat16))


def _reference_branch(x, w1, w2, w3, expert_indices, expert_weights):
    """The reference module's one-token branch, op for op, on the AQT weights."""
    A = expert_indices.numel()
    idx = expert_indices.view(A)
    w1s, w2s, w3s = w1[idx], w2[idx], w3[idx]
    outs = []
    for i in range(A):
        y1 = F.silu(F.linear(x, w1s[i]))
        y3 = F.linear(x, w3s[i])
        outs.append(F.linear(y1 * y3, w2s[i]))
    return (torch.cat(outs, dim=0) * expert_weights.view(-1, 1)).sum(dim=0).unsqueeze(-1)


@pytest.mark.parametrize("E,A,D,I", [(8, 2, 512, 1024), (4, 4, 1024, 2048), (16, 1, 4096, 1024)])
def test_grouped_moe_ffn_matches_reference_branch(E, A, D, I):
    from torchao._models.llama import kernels

    w1, w3 = _experts(E, I, D, 1), _experts(E, I, D, 2)
    w2 = _experts(E, D, I, 3)
    gen = torch.Generator(device=DEV).manual_seed(4)
    x = torch.randn(1, D, device=DEV, dtype=torch.bfloat16, generator=gen)
    scores = torch.randn(1, E, device=DEV, generator=gen).to(torch.bfloat16)
    ew, ei = torch.topk(F.softmax(scores, dim=-1), A, dim=-1)
    ew = ew / ew.sum(dim=-1, keepdim=True).to(x.dtype)
    ref = _reference_branch(x, w1, w2, w3, ei, ew)
    got = kernels.int4_moe_ffn_decode(x, w1, w2, w3, ei, ew)
    assert got.shape == ref.shape
    assert torch.equal(got, ref)
    # each grouped row is that expert's own linear, bit for bit
    y = kernels.int4_grouped_decode(x, w1.tensor_impl.packed_weight, w1.tensor_impl.scale_and_zero,
                                    32, ei.view(-1))
    for a in range(A):
        assert torch.equal(y[a:a + 1], F.linear(x, w1[int(ei.view(-1)[a])]))
    kernels.check_decode_status()


def test_grouped_graph_replay_and_bad_index():
    """The expert indices are read at replay (graph-capturable routing); an index outside
    [0, E) is clamped and raises from check_decode_status."""
    from torchao._models.llama import kernels

    E, N, K = 8, 1024, 2048
    w = _experts(E, N, K, 7)
    pw, sz = w.tensor_impl.packed_weight, w.tensor_impl.scale_and_zero
    x = torch.randn(3, K, device=DEV, dtype=torch.bfloat16)  # one row per activation
    idx = torch.tensor([0, 5, 2], device=DEV)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        kernels.int4_grouped_decode(x, pw, sz, 32, idx)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            y = kernels.int4_grouped_decode(x, pw, sz, 32, idx)
    torch.cuda.current_stream().wait_stream(s)
    for sel in ([0, 5, 2], [7, 7, 1], [3, 4, 6]):
        idx.copy_(torch.tensor(sel, device=DEV))
        g.replay()
        torch.cuda.synchronize()
        for a, e in enumerate(sel):
            assert torch.equal(y[a:a + 1], F.linear(x[a:a + 1], w[e])), (sel, a)
    kernels.check_decode_status()
    kernels.int4_grouped_decode(x, pw, sz, 32, torch.tensor([0, 8, 1], device=DEV))
    torch.cuda.synchronize()
    with pytest.raises(RuntimeError, match="expert index"):
        kernels.check_decode_status()
    kernels.check_decode_status()
    with pytest.raises(RuntimeError, match="int4_grouped"):
        kernels.int4_grouped_decode(x[:2], pw, sz, 32, idx)
