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


def test_rocm_tile_map_matches_aten_fixture():
    """oracle.pack_tile(fmt="rocm") against the nibble map PyTorch-ROCm's
    aten._convert_weight_to_int4pack produced on the MI355X (experiments/probe_aten_tile_map.py
    -> tests/golden/aten_tile_map_rocm.npz): every nibble of 15 (N, K, inner_k_tiles) cases."""
    m = load_golden("aten_tile_map_rocm.npz")
    assert len(m.files) == 15
    for key in m.files:
        N = int(key.split("_")[0][1:])
        K = int(key.split("_")[1][1:])
        ikt = int(key.split("ikt")[1])
        idx = np.arange(N * K, dtype=np.int64).reshape(N, K)
        # pack the flat index 4 bits at a time, exactly as the probe did, and rebuild the map
        got = np.zeros(m[key].shape, dtype=np.int64)
        for p4 in range((int(N * K - 1).bit_length() + 3) // 4):
            packed = oracle.pack_tile((idx >> (4 * p4)) & 0xF, ikt, "rocm").view(np.uint32)
            nib = np.stack([(packed >> np.uint32(4 * i)) & 0xF for i in range(8)], -1)
            got |= nib.astype(np.int64) << (4 * p4)
        np.testing.assert_array_equal(got, m[key].astype(np.int64), err_msg=key)


@pytest.mark.parametrize("ikt", [2, 4, 8])
def test_rocm_tile_roundtrip(ikt):
    rng = np.random.default_rng(ikt + 100)
    N, K = 48, ikt * 16 * 3
    q = rng.integers(0, 16, size=(N, K), dtype=np.int32)
    p = oracle.pack_tile(q, ikt, "rocm")
    assert p.shape == (N // 8, K // (ikt * 16), 32, ikt // 2)
    np.testing.assert_array_equal(oracle.unpack_tile(p, ikt, "rocm"), q)
    assert not np.array_equal(p, oracle.pack_tile(q, ikt, "cuda"))


def test_llama_oracle_matches_reference_model():
    """oracle/llama_ref.py (the config-4 tolerance anchor) against the reference gpt-fast
    Transformer's own fp32 logits (oracle/gen_golden_llama.py): a 10-token prefill and two KV-
    cache decode steps of a 2-layer GQA model."""
    from oracle import llama_ref

    rec = load_golden("llama_tiny_fp32.npz")
    W = {k[2:]: bf16(rec[k]).float() for k in rec.files if k.startswith("w:")}
    n_layer, n_head, n_kv, base = rec["config"]
    tokens = torch.from_numpy(rec["tokens"]).long()
    logits = llama_ref.llama_forward_fp32(W, int(n_layer), int(n_head), int(n_kv), float(base),
                                          1e-5, tokens)
    ref = torch.from_numpy(rec["logits"])
    assert logits.shape == ref.shape
    torch.testing.assert_close(logits, ref, rtol=2e-5, atol=2e-5)
