"""GPU parity of the int4 path (pack / unpack / dequant / linear) against the CPU oracle.

Every op here runs through the C-ABI library (torchao.ops -> torchao._lib -> include/*.h).
Bars: integer/byte work bit-exact; bf16 outputs within the north-star tolerance of 1e-2
relative L2 against the reference CPU dequant -> F.linear path (oracle.int4_linear), and much
tighter against an fp32 accumulation of the same dequantised weights.
"""

import numpy as np
import pytest
import torch

from conftest import bf16, golden_files, golden_ms, load_golden, unpack_u8_nibbles
from oracle import oracle

import torchao
from torchao import _lib

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL_REF = 1e-2  # north_star: within 1e-2 relative on bf16 vs the reference dequant path
TOL_FP32 = 4e-3  # vs fp32 accumulation of the identical dequantised weights


def _qparams(N, K, g, seed=0):
    w = oracle.make_linear_weight(N, K, seed=seed)
    s, z = oracle.int4_qparams(w, g)
    q = oracle.int4_quantize(w, s, z, g)
    return w, q, s, z


def _gpu_weight(q, s, z):
    packed = torch.ops.torchao.int4_pack(q.to(DEV))
    sz = torch.stack([s, z], dim=-1).contiguous().to(DEV)
    return packed, sz


def test_native_library_is_loaded_on_gpu():
    assert _lib.is_available(), _lib.load_error()
    assert _lib.lib().tao_device_count() >= 1
    assert "gfx950" in torch.cuda.get_device_properties(0).gcnArchName


@pytest.mark.parametrize("N,K", [(64, 256), (37, 352), (4096, 4096), (1000, 11008)])
def test_pack_unpack_bit_exact(N, K):
    rng = np.random.default_rng(N + K)
    q = rng.integers(0, 16, size=(N, K), dtype=np.int32)
    packed = torch.ops.torchao.int4_pack(torch.from_numpy(q).to(DEV))
    np.testing.assert_array_equal(packed.cpu().numpy().view(np.uint32), oracle.pack_row_stream(q))
    np.testing.assert_array_equal(torch.ops.torchao.int4_unpack(packed).cpu().numpy(), q)
    # the u8 entry (reference's (q[2i] << 4 | q[2i+1]) operand) packs identically
    qt = torch.from_numpy(q)
    u8 = ((qt[:, 0::2] << 4) | qt[:, 1::2]).to(torch.uint8).to(DEV)
    assert torch.equal(torch.ops.torchao.int4_pack_u8(u8), packed)


@pytest.mark.parametrize("fname", golden_files("int4_"))
def test_dequant_bit_exact_vs_reference(fname):
    rec = load_golden(fname)
    g = int(rec["g"])
    q = unpack_u8_nibbles(rec["q_u8"])
    s, z = bf16(rec["s"]), bf16(rec["z"])
    packed, sz = _gpu_weight(q, s, z)
    w0 = torch.ops.torchao.int4_dequantize(packed, sz, g, 0).cpu()
    assert torch.equal(w0, oracle.int4_dequantize(q, s, z, g))
    if "w_dequant" in rec.files:
        assert torch.equal(w0, bf16(rec["w_dequant"]))  # reference AQT.dequantize(), bit exact
    w1 = torch.ops.torchao.int4_dequantize(packed, sz, g, 1).cpu()
    sz_tiny = torch.stack([s, z], -1).transpose(0, 1)
    assert torch.equal(w1, oracle.dequant_tile_fma(q, sz_tiny, g))


@pytest.mark.parametrize("fname", golden_files("int4_"))
def test_linear_vs_reference_fixtures(fname):
    rec = load_golden(fname)
    g = int(rec["g"])
    q = unpack_u8_nibbles(rec["q_u8"])
    s, z, bias = bf16(rec["s"]), bf16(rec["z"]), bf16(rec["bias"])
    packed, sz = _gpu_weight(q, s, z)
    for M in golden_ms(rec):
        x = bf16(rec[f"x_M{M}"])
        y = torch.ops.torchao.int4_weight_only_linear(x.to(DEV), packed, sz, g, bias.to(DEV)).cpu()
        assert y.shape == (M, int(rec["N"])) and y.dtype == torch.bfloat16
        assert oracle.rel_l2(y, bf16(rec[f"y_dequant_M{M}"])) < TOL_REF
        assert oracle.rel_l2(y, oracle.int4_linear_fp32(x, q, s, z, g, bias)) < TOL_FP32


@pytest.mark.parametrize("M", [1, 2, 3, 4, 5, 7, 8, 9, 16, 17, 33, 64, 128])
@pytest.mark.parametrize("g", [32, 128])
def test_linear_all_m_paths(M, g):
    N, K = 192, 1024
    w, q, s, z = _qparams(N, K, g, seed=M)
    x = oracle.make_activation(M, K, seed=M)
    packed, sz = _gpu_weight(q, s, z)
    y = torch.ops.torchao.int4_weight_only_linear(x.to(DEV), packed, sz, g, None).cpu()
    assert oracle.rel_l2(y, oracle.int4_linear(x, q, s, z, g)) < TOL_REF
    assert oracle.rel_l2(y, oracle.int4_linear_fp32(x, q, s, z, g)) < TOL_FP32


@pytest.mark.parametrize(
    "N,K,g",
    [(4096, 4096, 32), (6144, 4096, 32), (14336, 4096, 32), (4096, 14336, 32),
     (11008, 4096, 32), (4096, 11008, 32), (8192, 28672, 64), (4096, 4096, 256),
     # 70B-style shard launch shapes: few rows with long K (waves split K 8 / 4 ways), a
     # K > 4096 head-like N >= 32768 (8 rows per wave), a 2-rows-per-wave K = 8192 shard
     (1024, 28672, 32), (2048, 14336, 32), (2560, 8192, 32), (33000, 5120, 128)],
)
def test_llama_shapes_m1(N, K, g):
    w, q, s, z = _qparams(N, K, g, seed=N ^ K)
    x = oracle.make_activation(1, K, seed=5)
    packed, sz = _gpu_weight(q, s, z)
    y = torch.ops.torchao.int4_weight_only_linear(x.to(DEV), packed, sz, g, None).cpu()
    assert oracle.rel_l2(y, oracle.int4_linear_fp32(x, q, s, z, g)) < TOL_FP32
    assert oracle.rel_l2(y, oracle.int4_linear(x, q, s, z, g)) < TOL_REF


def test_linearity_and_determinism_full_size():
    """Size-independent properties at 14336 x 4096: run-to-run bit identity and
    additivity y(x1 + x2) ~ y(x1) + y(x2) (up to bf16 output rounding)."""
    N, K, g = 14336, 4096, 32
    w, q, s, z = _qparams(N, K, g, seed=11)
    packed, sz = _gpu_weight(q, s, z)
    x1 = oracle.make_activation(1, K, seed=21).to(DEV)
    x2 = oracle.make_activation(1, K, seed=22).to(DEV)
    f = lambda x: torch.ops.torchao.int4_weight_only_linear(x, packed, sz, g, None).float()
    a = f(x1)
    assert torch.equal(a, f(x1))
    lhs = f((x1.float() + x2.float()).to(torch.bfloat16))
    rel = (lhs - (a + f(x2))).norm() / lhs.norm()
    assert rel < 1e-2


def test_empty_and_bias_and_batched_shapes():
    N, K, g = 64, 256, 32
    w, q, s, z = _qparams(N, K, g)
    packed, sz = _gpu_weight(q, s, z)
    x0 = torch.empty(0, K, dtype=torch.bfloat16, device=DEV)
    assert torch.ops.torchao.int4_weight_only_linear(x0, packed, sz, g, None).shape == (0, N)
    x = oracle.make_activation(6, K, seed=9)
    bias = (torch.randn(N) * 0.5).to(torch.bfloat16)
    y3 = torch.ops.torchao.int4_weight_only_linear(
        x.reshape(2, 3, K).to(DEV), packed, sz, g, bias.to(DEV)
    )
    assert y3.shape == (2, 3, N)
    ref = oracle.int4_linear(x, q, s, z, g, bias).reshape(2, 3, N)
    assert oracle.rel_l2(y3.cpu(), ref) < TOL_REF


def test_bad_arguments_raise():
    packed = torch.zeros(8, 12, dtype=torch.int32, device=DEV)  # K = 96
    sz = torch.zeros(8, 2, 2, dtype=torch.bfloat16, device=DEV)
    x = torch.zeros(1, 96, dtype=torch.bfloat16, device=DEV)
    with pytest.raises(Exception):
        torch.ops.torchao.int4_weight_only_linear(x, packed, sz, 48, None)
    with pytest.raises(Exception):
        torch.ops.torchao.int4_weight_only_linear(x[:, :64], packed, sz, 32, None)


@pytest.mark.parametrize("fmt", ["cuda", "rocm"])
@pytest.mark.parametrize("ikt", [2, 4, 8])
@pytest.mark.parametrize("g", [32, 64, 128, 256])
def test_tile_format_compat_ops(fmt, ikt, g):
    N, K = 256, 1024
    w, q, s, z = _qparams(N, K, g, seed=ikt)
    tile = torch.from_numpy(oracle.pack_tile(q.numpy(), ikt, fmt)).to(DEV)
    assert torch.equal(torchao.ops.pack_tensor_core_tiled_layout(q.to(DEV), ikt, fmt), tile)
    assert torch.equal(torchao.ops.unpack_tensor_core_tiled_layout(tile, ikt, fmt).cpu(), q)
    assert torch.equal(torchao.ops.unpack_tensor_core_tiled_layout(tile.cpu(), ikt, fmt), q)
    sz_tiny = torch.stack([s, z], -1).transpose(0, 1).contiguous()
    d = torchao.ops.dequantize_tensor_core_tiled_layout(tile, sz_tiny.to(DEV), g, ikt, fmt).cpu()
    assert torch.equal(d, oracle.dequant_tile_fma(q, sz_tiny, g))
    # reference test_ops.py:339-402 bar: dequant close to the python dequant
    assert (d.float() - oracle.int4_dequantize(q, s, z, g).float()).abs().max() < 0.1


def test_hip_graph_capture_and_replay():
    N, K, g = 4096, 4096, 32
    w, q, s, z = _qparams(N, K, g, seed=2)
    packed, sz = _gpu_weight(q, s, z)
    x = oracle.make_activation(1, K, seed=3).to(DEV)
    y_eager = torch.ops.torchao.int4_weight_only_linear(x, packed, sz, g, None)
    graph = torch.cuda.CUDAGraph()
    stream = torch.cuda.Stream()
    stream.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(stream):
        torch.ops.torchao.int4_weight_only_linear(x, packed, sz, g, None)  # warm up
        with torch.cuda.graph(graph, stream=stream):
            y_graph = torch.ops.torchao.int4_weight_only_linear(x, packed, sz, g, None)
    torch.cuda.current_stream().wait_stream(stream)
    graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(y_graph, y_eager)


def test_quantize_api_end_to_end_on_gpu():
    from torchao.quantization import Int4WeightOnlyConfig, quantize_

    K, N = 1024, 512
    m = torch.nn.Sequential(torch.nn.Linear(K, N), torch.nn.Linear(N, 256)).to(torch.bfloat16)
    ref_w = [m[0].weight.detach().clone(), m[1].weight.detach().clone()]
    m = m.to(DEV)
    quantize_(m, Int4WeightOnlyConfig(group_size=32))
    x = oracle.make_activation(4, K, seed=4)
    y = m(x.to(DEV)).cpu()
    # oracle: quantize the same weights on CPU, dequant path layer by layer
    h = x
    for i, lin in enumerate(m):
        s, z = oracle.int4_qparams(ref_w[i], 32)
        q = oracle.int4_quantize(ref_w[i], s, z, 32)
        h = oracle.int4_linear(h, q, s, z, 32, lin.bias.detach().cpu())
    assert oracle.rel_l2(y, h) < TOL_REF
    # weights quantized on the GPU carry the same (q, s, z) as the CPU oracle
    q0, s0, z0 = m[0].weight.tensor_impl.get_plain()
    s_ref, z_ref = oracle.int4_qparams(ref_w[0], 32)
    assert torch.equal(s0.cpu(), s_ref) and torch.equal(z0.cpu(), z_ref)
    assert torch.equal(q0.cpu(), oracle.int4_quantize(ref_w[0], s_ref, z_ref, 32))
    # moving a CPU-quantized weight to the GPU keeps working (layout is device independent)
    lin = torch.nn.Linear(K, N, dtype=torch.bfloat16)
    quantize_(lin, Int4WeightOnlyConfig(group_size=64))
    lin = lin.to(DEV)
    assert lin(x.to(DEV)).shape == (4, N)


# ---- experiment knob tao_tune_int4_xlds (x staged once per workgroup in LDS) ------
# Off by default; when switched on the plain M = 1 linear takes the decode prologue's LDS copy of
# x (no norm). Same tolerances as the default path, ragged K and N included; bias falls back.
@pytest.mark.parametrize("N,K,g", [(4096, 4096, 32), (28672, 4096, 32), (4096, 14336, 32),
                                   (40, 352, 32), (1000, 11008, 64)])
def test_xlds_knob_m1(N, K, g):
    w, q, s, z = _qparams(N, K, g, seed=N + K)
    x = oracle.make_activation(1, K, seed=7)
    packed, sz = _gpu_weight(q, s, z)
    ref = oracle.int4_linear_fp32(x, q, s, z, g)
    try:
        _lib.call("tao_tune_int4_xlds", 1)
        y = torch.ops.torchao.int4_weight_only_linear(x.to(DEV), packed, sz, g, None).cpu()
        b = oracle.make_activation(1, N, seed=3).reshape(-1)
        yb = torch.ops.torchao.int4_weight_only_linear(x.to(DEV), packed, sz, g, b.to(DEV)).cpu()
    finally:
        _lib.call("tao_tune_int4_xlds", 0)
    assert oracle.rel_l2(y, ref) < TOL_FP32
    assert oracle.rel_l2(yb, ref + b.float()) < TOL_REF


# ---- pinned to the reference's real producer: PyTorch-ROCm's aten int4 tile ops --------------
# reference test/test_ops.py:260-272: SHAPES x INNERKTILES (x QGROUP_SIZES for the dequant), the
# full grid, plus small shapes (N a multiple of 16: PyTorch-ROCm's packer needs it).
REF_SHAPES = [(4096, 4096), (4096, 11008), (11008, 4096), (4096, 14336), (14336, 4096)]
ATEN_SHAPES = REF_SHAPES + [(16, 128), (32, 512), (64, 1024), (256, 1024)]


@pytest.mark.parametrize("N,K", ATEN_SHAPES)
@pytest.mark.parametrize("ikt", [2, 4, 8])
def test_tile_pack_equals_aten_convert_weight_to_int4pack(N, K, ikt):
    """A11: pack == aten._convert_weight_to_int4pack(u8, ikt) bit for bit (the call at
    tensor_core_tiled_layout.py:279, on this box's PyTorch-ROCm), and unpack inverts it on the
    GPU and on the host (test_ops.py:284-293, the same grid)."""
    if K % (ikt * 16):
        pytest.skip("K not a multiple of ikt * 16")
    g = torch.Generator(device=DEV).manual_seed(N + K + ikt)
    q = torch.randint(0, 16, (N, K), generator=g, dtype=torch.int32, device=DEV)
    u8 = ((q[:, ::2] << 4) | q[:, 1::2]).to(torch.uint8).contiguous()
    ref = torch.ops.aten._convert_weight_to_int4pack(u8, ikt)
    ours = torchao.ops.pack_tensor_core_tiled_layout(q, ikt)  # default map on ROCm: "rocm"
    assert ours.shape == ref.shape and torch.equal(ours, ref.view(torch.int32))
    unpacked = torchao.ops.unpack_tensor_core_tiled_layout(ref.contiguous(), ikt)
    assert torch.equal(unpacked, q)
    # the reference test's own check: re-packed bytes equal the input bytes
    assert torch.equal(((unpacked[:, ::2] << 4) | unpacked[:, 1::2]).to(torch.uint8), u8)
    assert torch.equal(torchao.ops.unpack_tensor_core_tiled_layout(ref.cpu(), ikt), q.cpu())


@pytest.mark.parametrize("N,K", REF_SHAPES + [(256, 1024)])
@pytest.mark.parametrize("ikt", [2, 4, 8])
@pytest.mark.parametrize("g", [32, 64, 128, 256])
def test_tile_dequant_equals_aten_identity_mm(N, K, ikt, g):
    """The reference protocol of test_ops.py:339-402 on the full SHAPES x INNERKTILES x
    QGROUP_SIZES grid: the weight dequantised by aten._weight_int4pack_mm(eye(K)) (this box's
    PyTorch-ROCm, the reference's int4 linear at tensor_core_tiled_layout.py:104) equals the HIP
    dequant op BIT FOR BIT (diff == 0), and both differ from the group-wise python dequant
    (two bf16 roundings) by the same max |diff| < 0.1."""
    from torchao.quantization.utils import (get_groupwise_affine_qparams,
                                            groupwise_affine_dequantize_tensor_from_qparams,
                                            groupwise_affine_quantize_tensor_from_qparams,
                                            pack_tinygemm_scales_and_zeros)
    if K % (ikt * 16):
        pytest.skip("K not a multiple of ikt * 16")
    gen = torch.Generator(device=DEV).manual_seed(N * 7 + K + ikt * 3 + g)
    t = torch.randn(N, K, generator=gen, device=DEV).to(torch.bfloat16)
    s, z = get_groupwise_affine_qparams(t, n_bit=4, groupsize=g, dtype=torch.bfloat16)
    q = groupwise_affine_quantize_tensor_from_qparams(t, s, z, n_bit=4, groupsize=g)
    assert q.dtype == torch.uint8 and q.shape == (N, K // 2)
    packed = torch.ops.aten._convert_weight_to_int4pack(q, ikt)
    sz = pack_tinygemm_scales_and_zeros(s, z)
    assert sz.shape == (K // g, N, 2)
    dq_ao = groupwise_affine_dequantize_tensor_from_qparams(q, s, z, n_bit=4, groupsize=g)
    eye = torch.eye(K, device=DEV, dtype=torch.bfloat16)
    dq_id = torch.ops.aten._weight_int4pack_mm(eye, packed, g, sz).t()
    del eye
    dq_op = torchao.ops.dequantize_tensor_core_tiled_layout(packed, sz, g, ikt)
    diff_ao_id = (dq_id - dq_ao).abs().max()
    diff_op_id = (dq_op - dq_id).abs().max()
    diff_op_ao = (dq_op - dq_ao).abs().max()
    assert diff_op_id == 0
    assert torch.equal(dq_op.view(torch.int16), dq_id.contiguous().view(torch.int16))
    assert diff_op_ao == diff_ao_id
    assert diff_op_ao < 1e-1


# ---- checkpoints written by the reference's own classes (oracle/gen_golden_ckpt.py) -----------
def _ref_ckpt_tags():
    import os

    from conftest import GOLDEN
    return sorted(f[len("ref_ckpt_"):-3] for f in os.listdir(GOLDEN)
                  if f.startswith("ref_ckpt_") and f.endswith(".pt"))


@pytest.mark.parametrize("tag", _ref_ckpt_tags())
def test_reference_written_checkpoint_runs_on_gpu(tag):
    """a state dict pickled by the REFERENCE's TensorCoreTiledAQTTensorImpl /
    AffineQuantizedTensor (tile-format storage, K padded to 1024) loads with
    torch.load(weights_only=True, map_location=cuda) into this package. The tile storage is adopted
    on the GPU (HIP unpack + row-stream pack), get_plain() returns the reference's (q, s, z) bit for
    bit, and the linear matches the reference dequant -> F.linear output stored with it within the
    north-star 1e-2 (and the fp32 accumulation of the same weights within 4e-3)."""
    import os

    import torchao.ops as tops
    from conftest import GOLDEN

    rec = load_golden(f"ref_ckpt_{tag}.npz")
    qu8 = rec["q_u8"]
    q = unpack_u8_nibbles(qu8.reshape(-1, qu8.shape[-1])).reshape(*qu8.shape[:-1], -1)
    s, z, bias = bf16(rec["s"]), bf16(rec["z"]), bf16(rec["bias"])
    N, K, g, E = int(rec["N"]), int(rec["K"]), int(rec["g"]), int(rec["E"])
    path = os.path.join(GOLDEN, f"ref_ckpt_{tag}.pt")
    with tops.checkpoint_tile_format(str(rec["fmt"])):
        # the reference's own flow (test_quant_api.py:746-750, torchtune): load on the CPU (tile
        # storage adopted by the host C++ unpack), then move every tensor to the GPU
        sd = torch.load(path, weights_only=True, map_location="cpu")
        sd = {k: v.to(DEV) for k, v in sd.items()}
        # and straight onto the GPU (adopted by the HIP unpack kernel)
        sd_dev = torch.load(path, weights_only=True, map_location=f"cuda:{torch.cuda.current_device()}")
    aqt = sd["experts.weight" if E else "weight"]
    aqt_dev = sd_dev["experts.weight" if E else "weight"]
    assert aqt.device.type == "cuda" and aqt.tensor_impl.packed_weight.is_cuda
    assert torch.equal(aqt_dev.tensor_impl.packed_weight, aqt.tensor_impl.packed_weight)
    assert torch.equal(aqt_dev.tensor_impl.scale_and_zero, aqt.tensor_impl.scale_and_zero)
    qq, ss, zz = aqt.tensor_impl.get_plain()
    assert torch.equal(qq.cpu(), q) and torch.equal(ss.cpu(), s) and torch.equal(zz.cpu(), z)
    x = bf16(rec["x"])
    if E:  # MoE: expert 0's slice of the adopted [E, N, K/8] storage
        impl = aqt.tensor_impl
        y = torch.ops.torchao.int4_weight_only_linear(
            x.to(DEV), impl.packed_weight[0].contiguous(), impl.scale_and_zero[0].contiguous(), g,
            bias[0].to(DEV)).cpu()
        q0, s0, z0, b0 = q[0], s[0], z[0], bias[0]
    else:
        from torchao.quantization import Int4WeightOnlyConfig, quantize_

        lin = torch.nn.Linear(K, N, dtype=torch.bfloat16, device=DEV)
        quantize_(lin, Int4WeightOnlyConfig(group_size=g))
        lin.load_state_dict(sd, assign=True)  # reference test_quant_api.py:750
        y = lin(x.to(DEV)).cpu()
        q0, s0, z0, b0 = q, s, z, bias
    assert oracle.rel_l2(y, bf16(rec["y_dequant"])) < TOL_REF
    assert oracle.rel_l2(y, oracle.int4_linear_fp32(x, q0, s0, z0, g, b0)) < TOL_FP32


def test_operands_on_another_device_raise():
    """a weight, scale or bias that is not on x's device raises RuntimeError in
    the C++ op kernels and the Python impls, instead of reaching a launch as a foreign pointer."""
    N, K, g = 64, 256, 32
    w, q, s, z = _qparams(N, K, g)
    packed, sz = _gpu_weight(q, s, z)
    x = oracle.make_activation(1, K, seed=1).to(DEV)
    with pytest.raises(RuntimeError, match="same device"):
        torch.ops.torchao.int4_weight_only_linear(x, packed.cpu(), sz, g, None)
    with pytest.raises(RuntimeError, match="same device"):
        torch.ops.torchao.int4_weight_only_linear(x, packed, sz.cpu(), g, None)
    with pytest.raises(RuntimeError, match="same device"):
        torch.ops.torchao.int4_weight_only_linear(x, packed, sz, g, torch.zeros(N, dtype=torch.bfloat16))
    with pytest.raises(RuntimeError, match="same device"):
        torch.ops.torchao.int4_dequantize(packed, sz.cpu(), g, 0)
    s8 = oracle.int8_weight_qparams(w)
    q8 = oracle.int8_weight_quantize(w, s8)
    with pytest.raises(RuntimeError, match="same device"):
        torch.ops.torchao.int8_weight_only_linear(x, q8, s8.to(DEV), None)
    with pytest.raises(RuntimeError, match="same device"):
        torch.ops.torchao.int8_weight_only_linear(x, q8.to(DEV), s8, None)
    xq, xs = torch.ops.torchao.int8_quantize_per_token(x)
    with pytest.raises(RuntimeError, match="same device"):
        torch.ops.torchao.int8_scaled_mm(xq, xs, q8.to(DEV), s8, None)
    with pytest.raises(RuntimeError, match="same device"):
        torch.ops.torchao.int8_scaled_mm(xq, xs.cpu(), q8.to(DEV), s8.to(DEV), None)
    with pytest.raises(RuntimeError, match="same device"):
        torch.ops.torchao.int8_dyn_linear(x, q8, s8.to(DEV), None)


@pytest.mark.gpu
def test_fuse_gate_up_then_quantize_gpu():
    """The reference FeedForward layout merged by fuse_gate_up_ and then quantize_d (int4 g32):
    the merged model's outputs equal the unmerged quantized model's within one GEMV's
    re-association (the merged linear quantizes to the same values; it runs one GEMV launch for
    w1 and w3), and the merged linear dispatches to the HIP int4 op."""
    import copy

    import torch.nn.functional as F

    from torchao.quantization import Int4WeightOnlyConfig, fuse_gate_up_, quantize_

    class FeedForward(torch.nn.Module):
        def __init__(self, d, h):
            super().__init__()
            self.w1 = torch.nn.Linear(d, h, bias=False)
            self.w3 = torch.nn.Linear(d, h, bias=False)
            self.w2 = torch.nn.Linear(h, d, bias=False)

        def forward(self, x):
            return self.w2(F.silu(self.w1(x)) * self.w3(x))

    torch.manual_seed(1)
    ff = FeedForward(1024, 2816).to(device="cuda", dtype=torch.bfloat16)
    merged = copy.deepcopy(ff)
    assert fuse_gate_up_(merged) == 1
    quantize_(ff, Int4WeightOnlyConfig(group_size=32))
    quantize_(merged, Int4WeightOnlyConfig(group_size=32))
    for M in (1, 16):
        x = torch.randn(M, 1024, device="cuda", dtype=torch.bfloat16)
        a, b = ff(x).float(), merged(x).float()
        assert float((a - b).norm() / a.norm()) < 1e-2
