"""The CPU oracle is pinned to the reference's own outputs (tests/golden/, oracle/gen_golden.py).

Quantization math (qparams, quantize, dequantize, activation quant) must match bit for bit.
Matmul outputs are compared with a tight tolerance: the fixtures were produced by F.linear on
the build container's CPU; other hosts may sum in another order.
"""

import numpy as np
import pytest
import torch

from conftest import bf16, golden_files, golden_ms, load_golden, unpack_u8_nibbles
from oracle import oracle


@pytest.mark.parametrize("fname", golden_files("int4_"))
def test_int4_quant_math_bit_exact(fname):
    rec = load_golden(fname)
    g = int(rec["g"])
    w = bf16(rec["w"])
    q_ref = unpack_u8_nibbles(rec["q_u8"])
    s_ref, z_ref = bf16(rec["s"]), bf16(rec["z"])
    s, z = oracle.int4_qparams(w, g)
    assert torch.equal(s, s_ref) and torch.equal(z, z_ref)
    q = oracle.int4_quantize(w, s, z, g)
    assert torch.equal(q, q_ref)
    if "w_dequant" in rec.files:
        assert torch.equal(oracle.int4_dequantize(q, s, z, g), bf16(rec["w_dequant"]))


@pytest.mark.parametrize("fname", golden_files("int4_"))
def test_int4_dequant_path_matches_reference(fname):
    rec = load_golden(fname)
    g = int(rec["g"])
    q = unpack_u8_nibbles(rec["q_u8"])
    s, z, bias = bf16(rec["s"]), bf16(rec["z"]), bf16(rec["bias"])
    for M in golden_ms(rec):
        x = bf16(rec[f"x_M{M}"])
        y = oracle.int4_linear(x, q, s, z, g, bias)
        assert oracle.rel_l2(y, bf16(rec[f"y_dequant_M{M}"])) < 2e-3


@pytest.mark.parametrize("fname", golden_files("int8wo_"))
def test_int8wo_oracle_matches_reference(fname):
    rec = load_golden(fname)
    w = bf16(rec["w"])
    s = oracle.int8_weight_qparams(w)
    assert torch.equal(s, bf16(rec["s"]))
    q = oracle.int8_weight_quantize(w, s)
    assert torch.equal(q, torch.from_numpy(rec["q"]))
    bias = bf16(rec["bias"])
    for M in golden_ms(rec):
        y = oracle.int8wo_linear(bf16(rec[f"x_M{M}"]), q, s, bias)
        assert oracle.rel_l2(y, bf16(rec[f"y_M{M}"])) < 2e-3


@pytest.mark.parametrize("fname", golden_files("int8dyn_"))
def test_int8dyn_oracle_matches_reference(fname):
    rec = load_golden(fname)
    wq, ws = oracle.int8_dyn_weight(bf16(rec["w"]))
    assert torch.equal(wq, torch.from_numpy(rec["wq"]))
    assert torch.equal(ws, bf16(rec["ws"]))
    bias = bf16(rec["bias"])
    for M in golden_ms(rec):
        x = bf16(rec[f"x_M{M}"])
        xq, xs = oracle.int8_act_quant(x)
        assert torch.equal(xq, torch.from_numpy(rec[f"xq_M{M}"]))
        assert torch.equal(xs.reshape(-1), bf16(rec[f"xs_M{M}"]))
        y = oracle.int8_scaled_mm(xq, xs, wq, ws, bias, epilogue="cpu")
        # same integer products and epilogue as the reference CPU branch: bit exact
        assert torch.equal(y, bf16(rec[f"y_M{M}"]))


def test_row_stream_pack_roundtrip_and_bits():
    rng = np.random.default_rng(0)
    q = rng.integers(0, 16, size=(7, 64), dtype=np.int32)
    p = oracle.pack_row_stream(q)
    assert p.dtype == np.uint32 and p.shape == (7, 8)
    np.testing.assert_array_equal(oracle.unpack_row_stream(p), q)
    # hand-checked: k = 0..7 of row 0 -> nibbles (k0,k2,k4,k6) low half, (k1,k3,k5,k7) high half
    q1 = np.arange(8, dtype=np.int32).reshape(1, 8)
    assert int(oracle.pack_row_stream(q1)[0, 0]) == 0x75316420


@pytest.mark.parametrize("ikt", [2, 4, 8])
def test_tile_pack_roundtrip(ikt):
    rng = np.random.default_rng(ikt)
    N, K = 16, ikt * 16 * 3
    q = rng.integers(0, 16, size=(N, K), dtype=np.int32)
    p = oracle.pack_tile(q, ikt)
    assert p.shape == (N // 8, K // (ikt * 16), 32, ikt // 2) and p.dtype == np.int32
    np.testing.assert_array_equal(oracle.unpack_tile(p, ikt), q)


def test_tile_layout_index_math_hand_checked():
    # ikt = 2, one tile: element [0][0][t=5][0] holds row n = 1, ks = {2, 10, 18, 26}
    q = np.zeros((8, 32), dtype=np.int32)
    q[1, 2], q[1, 3], q[1, 10], q[1, 11], q[1, 18], q[1, 19], q[1, 26], q[1, 27] = range(1, 9)
    p = oracle.pack_tile(q, 2).view(np.uint32)
    # bits 4i = q[ks_i], bits 16+4i = q[ks_i + 1]
    assert int(p[0, 0, 5, 0]) == (1 | 3 << 4 | 5 << 8 | 7 << 12 | 2 << 16 | 4 << 20 | 6 << 24 | 8 << 28)
