"""The end-to-end decode harness (torchao/_models/llama): KV-cache decode == full forward on
CPU (bf16 model, no quantization), and on the GPU with int4 weights: graph-replayed decode ==
eager decode token for token, and int4 logits track the bf16 model's."""

import math

import pytest
import torch

from torchao._models.llama.generate import (
    GraphDecoder,
    GraphPrefill,
    apply_quantization,
    build_model,
    decode_one_token,
    generate,
    prefill,
)
from torchao._models.llama.model import ModelArgs


def test_config_lookup():
    cfg = ModelArgs.from_name("Meta-Llama-3-8B")
    assert (cfg.dim, cfg.n_layer, cfg.n_local_heads, cfg.intermediate_size, cfg.vocab_size) == (
        4096, 32, 8, 14336, 128256)
    assert ModelArgs.from_name("Llama-3.1-70B").rope_scaling is not None
    assert ModelArgs.from_name("stories15M").intermediate_size == 768
    with pytest.raises(ValueError):
        ModelArgs.from_name("no-such-model")


def test_kv_cache_decode_matches_full_forward_cpu():
    torch.manual_seed(0)
    model = build_model("stories15M", torch.device("cpu"), dtype=torch.float32, seed=3)
    P, T = 7, 5
    model.setup_caches(1, P + T)
    ids = torch.randint(0, model.config.vocab_size, (1, P + T))
    full = model(ids, torch.arange(P + T))
    model.setup_caches(1, P + T)
    inc = [model(ids[:, :P], torch.arange(P))]
    for i in range(P, P + T):
        inc.append(model(ids[:, i:i + 1], torch.tensor([i])))
    inc = torch.cat(inc, dim=1)
    torch.testing.assert_close(inc, full, rtol=1e-4, atol=1e-4)


def test_build_model_is_seeded():
    a = build_model("stories15M", torch.device("cpu"), seed=5)
    b = build_model("stories15M", torch.device("cpu"), seed=5)
    assert torch.equal(a.layers[0].attention.wqkv.weight, b.layers[0].attention.wqkv.weight)
    assert torch.equal(a.tok_embeddings.weight, b.tok_embeddings.weight)


@pytest.mark.gpu
@pytest.mark.parametrize("quant", ["int4wo-32", "int8wo", "int8dq"])
def test_graph_decode_matches_eager_gpu(quant):
    dev = torch.device("cuda")
    ref = build_model("stories15M", dev, seed=1)
    model = build_model("stories15M", dev, seed=1)
    apply_quantization(model, quant)
    P, T = 12, 10
    for m in (ref, model):
        m.setup_caches(1, P + T)
    gen = torch.Generator().manual_seed(11)
    prompt = torch.randint(0, model.config.vocab_size, (1, P), generator=gen).to(dev)

    # quantized logits track the bf16 model (quantization error only; int4 g32 on this
    # random-init 6-layer model lands at 14-16 dB depending on the prompt)
    with torch.no_grad():
        lq = model(prompt, torch.arange(P, device=dev))
        lr = ref(prompt, torch.arange(P, device=dev))
    sqnr = 20 * torch.log10(lr.norm() / (lr - lq).norm())
    assert sqnr > (12 if quant.startswith("int4") else 25), float(sqnr)

    eager, _, _ = generate(model, prompt, T, None)
    dec = GraphDecoder(model, 1, P + T, dev)
    dec.reset(prompt, prefill(model, prompt, torch.arange(P, device=dev)))
    dec.capture()
    graphed, _, _ = generate(model, prompt, T, dec)
    assert torch.equal(graphed, eager)
    # a second run replays the same graph from a fresh prefill
    again, _, _ = generate(model, prompt, T, dec)
    assert torch.equal(again, eager)
    # several steps per graph launch (4 here: T - 1 = 9 steps = 2 four-step replays + 1 single)
    dec4 = GraphDecoder(model, 1, P + T, dev, steps_per_graph=4)
    dec4.reset(prompt, prefill(model, prompt, torch.arange(P, device=dev)))
    dec4.capture()
    graphed4, _, _ = generate(model, prompt, T, dec4)
    assert torch.equal(graphed4, eager)
    # the graph-captured prefill gives the same first token and caches; a second prompt
    # through the same prefill graph matches its eager run too
    pre = GraphPrefill(model, (1, P), dev)
    pre.capture(prompt)
    both, _, _ = generate(model, prompt, T, dec, pre)
    assert torch.equal(both, eager)
    prompt2 = torch.randint(0, model.config.vocab_size, (1, P), generator=gen).to(dev)
    eager2, _, _ = generate(model, prompt2, T, None)
    both2, _, _ = generate(model, prompt2, T, dec, pre)
    assert torch.equal(both2, eager2)
    # single step helper agrees with the graph's first produced token
    tok = prefill(model, prompt, torch.arange(P, device=dev))
    nxt = decode_one_token(model, tok, torch.tensor([P], device=dev))
    assert int(nxt) == int(eager[0, P + 1])


# a head_dim-128 GQA model small enough for a unit test (the fused kernels need head_dim 128)
TINY = dict(dim=512, n_layer=2, n_head=4, n_local_heads=2, vocab_size=1000, block_size=256)


def _tiny(dev, seed=2):
    import math

    from torchao._models.llama.model import Transformer

    torch.manual_seed(seed)
    model = Transformer(ModelArgs(**TINY)).to(dev).to(torch.bfloat16)
    with torch.no_grad():
        for mod in model.modules():
            if isinstance(mod, torch.nn.Linear):
                b = 1 / math.sqrt(mod.in_features)
                mod.weight.uniform_(-b, b)
        for blk in model.layers:  # non-trivial norm weights
            blk.attention_norm.weight.uniform_(0.5, 1.5)
            blk.ffn_norm.weight.uniform_(0.5, 1.5)
    return model.eval()


@pytest.mark.gpu
def test_fused_kernels_match_torch_ops_gpu():
    import torch.nn.functional as F

    from torchao._models.llama import kernels
    from torchao._models.llama.model import RMSNorm, _apply_rope, _rope_freqs

    dev = torch.device("cuda")
    x = torch.randn(3, 4096, device=dev, dtype=torch.bfloat16) * 2
    norm = RMSNorm(4096).to(dev).to(torch.bfloat16)
    with torch.no_grad():
        norm.weight.uniform_(0.5, 1.5)
    ref = norm(x)
    got = kernels.rmsnorm(x, norm.weight, norm.eps)
    assert (got.float() - ref.float()).abs().max() <= 2 * ref.float().abs().max() * 2 ** -8

    a = torch.randn(5, 1000, device=dev, dtype=torch.bfloat16) * 3
    b = torch.randn(5, 1000, device=dev, dtype=torch.bfloat16)
    torch.testing.assert_close(kernels.silu_mul(a, b), F.silu(a) * b, rtol=1e-2, atol=1e-2)

    cfg = ModelArgs(**TINY)
    H, Hkv, D, T = cfg.n_head, cfg.n_local_heads, cfg.head_dim, 64
    freqs = _rope_freqs(cfg, cfg.block_size).to(dev)
    qkv = torch.randn(1, 1, (H + 2 * Hkv) * D, device=dev, dtype=torch.bfloat16)
    kc = torch.zeros(1, Hkv, T, D, device=dev, dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    pos = torch.tensor([17], device=dev)
    q = kernels.rope_kv(qkv, freqs, pos, kc, vc, H)
    qr, kr, vr = qkv.split([H * D, Hkv * D, Hkv * D], dim=-1)
    q_ref = _apply_rope(qr.view(1, 1, H, D), freqs[pos]).transpose(1, 2)
    k_ref = _apply_rope(kr.view(1, 1, Hkv, D), freqs[pos]).transpose(1, 2)
    torch.testing.assert_close(q, q_ref, rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(kc[:, :, 17:18], k_ref, rtol=1e-2, atol=1e-2)
    assert torch.equal(vc[:, :, 17:18], vr.view(1, 1, Hkv, D).transpose(1, 2))

    # attention over keys 0..L-1: the single-pass kernel (T <= 1024: L across its 16-key wave
    # steps and 128-key rounds) and the chunk-split pair (T > 1024: L across 64-key chunks)
    for T, L in ((256, 1), (256, 15), (256, 17), (256, 63), (256, 128), (256, 129), (256, 200),
                 (1024, 1024), (1536, 1), (1536, 65), (1536, 1100), (1536, 1536)):
        kc = torch.randn(2, Hkv, T, D, device=dev, dtype=torch.bfloat16)
        vc = torch.randn_like(kc)
        q = torch.randn(2, H, 1, D, device=dev, dtype=torch.bfloat16)
        pos = torch.tensor([L - 1], device=dev)
        got = kernels.attn_decode(q, kc, vc, pos, 1 / math.sqrt(D))
        ref = F.scaled_dot_product_attention(q.float(), kc[:, :, :L].float(), vc[:, :, :L].float(),
                                             enable_gqa=True)
        ref = ref.transpose(1, 2).reshape(2, 1, H * D)
        torch.testing.assert_close(got.float(), ref, rtol=2e-2, atol=2e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("G", [1, 2, 4, 8])
def test_attn_decode_modes_gpu(mode, G):
    """Every decode-attention kernel (tao_tune_attn: 0 f32 single pass (whole-line K loads) up to
    1024 keys, 1 two-launch split) against fp32 SDPA, GQA groups 1..8, lengths across chunk
    edges; run-to-run identical."""
    import torch.nn.functional as F

    from torchao import _lib
    from torchao._models.llama import kernels

    dev = torch.device("cuda")
    Hkv, D = 8 // G if G < 8 else 2, 128
    H = Hkv * G
    _lib.call("tao_tune_attn", mode)
    try:
        for T, L in ((64, 1), (64, 31), (64, 32), (64, 33), (328, 129), (328, 328),
                     (1024, 1000), (1536, 1100)):
            kc = torch.randn(2, Hkv, T, D, device=dev, dtype=torch.bfloat16)
            vc = torch.randn_like(kc)
            q = torch.randn(2, H, 1, D, device=dev, dtype=torch.bfloat16)
            pos = torch.tensor([L - 1], device=dev)
            got = kernels.attn_decode(q, kc, vc, pos, 1 / math.sqrt(D))
            again = kernels.attn_decode(q, kc, vc, pos, 1 / math.sqrt(D))
            ref = F.scaled_dot_product_attention(q.float(), kc[:, :, :L].float(),
                                                 vc[:, :, :L].float(), enable_gqa=True)
            ref = ref.transpose(1, 2).reshape(2, 1, H * D)
            torch.testing.assert_close(got.float(), ref, rtol=2e-2, atol=2e-2)
            assert torch.equal(got, again)
    finally:
        _lib.call("tao_tune_attn", 0)


@pytest.mark.gpu
@pytest.mark.parametrize("quant,split", [(None, 0), ("int4wo-32", 0), ("int4wo-32", 2),
                                         ("int4wo-32", 4), ("int4wo-32", "qkv")])
def test_fused_decode_matches_unfused_gpu(quant, split, monkeypatch):
    """Fused decode (one-pass attention, or with `split` the split attention + merged int4 wo,
    forced for this small cache; "qkv": wqkv + RoPE/KV + attention in one launch,
    kernels.DECODE_QKV_ATTN) against the torch-op forward; graph replay == eager."""
    from torchao._models.llama import kernels

    if split == "qkv":
        monkeypatch.setattr(kernels, "DECODE_QKV_ATTN", True)
        split = 0
    monkeypatch.setattr(kernels, "ATTN_SPLITS", split)
    monkeypatch.setattr(kernels, "ATTN_SPLIT_MIN_T", 0)
    dev = torch.device("cuda")
    model = _tiny(dev)
    apply_quantization(model, quant)
    P, T = 9, 12
    model.setup_caches(1, P + T)
    prompt = torch.randint(0, 1000, (1, P), device=dev)
    pos = torch.arange(P, device=dev)
    assert not model.fused
    model(prompt, pos)
    ref = [model(prompt[:, -1:], torch.tensor([P], device=dev))]
    model.setup_caches(1, P + T)
    assert model.enable_fused_kernels()
    model(prompt, pos)  # fused prefill (rmsnorm / rope_kv / silu_mul kernels)
    got = [model(prompt[:, -1:], torch.tensor([P], device=dev))]
    rel = (got[0] - ref[0]).norm() / ref[0].norm()
    assert rel < 2e-2, float(rel)
    # graph-replayed fused decode == eager fused decode
    eager, _, _ = generate(model, prompt, T, None)
    dec = GraphDecoder(model, 1, P + T, dev)
    dec.reset(prompt, prefill(model, prompt, pos))
    dec.capture()
    graphed, _, _ = generate(model, prompt, T, dec)
    assert torch.equal(graphed, eager)


@pytest.mark.gpu
@pytest.mark.parametrize("P", [37, 200])
@pytest.mark.parametrize("quant,fuse", [(None, True), ("int4wo-32", True), ("int4wo-32", False)])
def test_fused_prefill_matches_torch_ops_gpu(quant, fuse, P):
    """S > 1 tokens on the fused kernels (RMSNorm, RoPE + KV write, SiLU-mul) track the torch-op
    forward: all positions' logits and the KV caches; prefill_next (head at the last position
    only, the last block past wqkv on the one-token kernels) takes the same greedy token wherever
    the top-2 margin decides it. P = 200: more than one 128-row M tile (the single-fetch GEMMs and
    their partials path do not serve it; the MFMA GEMMs do)."""
    dev = torch.device("cuda")
    model = _tiny(dev, seed=7)
    if fuse:
        model.fuse_w13()
    apply_quantization(model, quant)
    model.setup_caches(2, P + 3)
    prompt = torch.randint(0, 1000, (2, P), device=dev)
    pos = torch.arange(P, device=dev)
    with torch.no_grad():
        ref = model(prompt, pos)
        kref = [blk.attention.kv_cache.k_cache.clone() for blk in model.layers]
        assert model.enable_fused_kernels()
        for blk in model.layers:
            blk.attention.kv_cache.k_cache.zero_()
            blk.attention.kv_cache.v_cache.zero_()
        got = model(prompt, pos)
        nxt = model.prefill_next(prompt, pos)
    assert got.shape == ref.shape
    rel = float((got - ref).norm() / ref.norm())
    assert rel < 2e-2, rel
    for blk, k0 in zip(model.layers, kref):
        k1 = blk.attention.kv_cache.k_cache
        assert float((k1 - k0).float().norm() / k0.float().norm()) < 2e-2
    last = ref[:, -1]
    top2 = last.topk(2, dim=-1).values
    for b in range(last.shape[0]):
        if float(top2[b, 0] - top2[b, 1]) > 3e-2 * float(last[b].abs().max()):
            assert int(nxt[b, 0]) == int(last[b].argmax())


def test_fuse_w13_is_exact_cpu():
    model = build_model("stories15M", torch.device("cpu"), dtype=torch.float32, seed=4)
    P = 6
    model.setup_caches(1, P)
    ids = torch.randint(0, model.config.vocab_size, (1, P))
    ref = model(ids, torch.arange(P))
    model.fuse_w13()
    assert model.layers[0].feed_forward.w1 is None
    model.setup_caches(1, P)
    got = model(ids, torch.arange(P))
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("quant", ["int4wo-32", "int8wo"])
def test_fuse_w13_gpu(quant):
    dev = torch.device("cuda")
    ref = _tiny(dev, seed=6)
    model = _tiny(dev, seed=6).fuse_w13()
    for m in (ref, model):
        apply_quantization(m, quant)
        m.setup_caches(1, 16)
        m.enable_fused_kernels()
    prompt = torch.randint(0, 1000, (1, 8), device=dev)
    pos = torch.arange(8, device=dev)
    torch.testing.assert_close(model(prompt, pos), ref(prompt, pos), rtol=2e-2, atol=2e-2)
    one = torch.tensor([8], device=dev)
    a, b = model(prompt[:, -1:], one), ref(prompt[:, -1:], one)
    assert (a - b).norm() / b.norm() < 1e-2


@pytest.mark.gpu
@pytest.mark.parametrize("quant", [None, "int4wo-32"])
def test_decode_past_kv_cache_is_reported_gpu(quant):
    """a decode step at a position past max_seq must not write outside the cache.
    The fused kernels skip the write and report it; check_decode_status() raises."""
    from torchao._models.llama import kernels

    dev = torch.device("cuda")
    model = _tiny(dev, seed=8).fuse_w13()
    apply_quantization(model, quant)
    model.setup_caches(1, 16)
    assert model.enable_fused_kernels()
    T = model.max_seq
    prompt = torch.randint(0, 1000, (1, 8), device=dev)
    model(prompt, torch.arange(8, device=dev))
    kernels.check_decode_status()  # clean so far
    one = torch.tensor([T - 1], device=dev)
    model(prompt[:, -1:], one)  # last valid row
    kernels.check_decode_status()
    caches = [(b.attention.kv_cache.k_cache.clone(), b.attention.kv_cache.v_cache.clone())
              for b in model.layers]
    canary = torch.full((4096,), 7, dtype=torch.int32, device=dev)  # neighbouring allocation
    model(prompt[:, -1:], torch.tensor([T], device=dev))  # one past the end
    torch.cuda.synchronize()
    with pytest.raises(RuntimeError, match="past the KV cache"):
        kernels.check_decode_status()
    kernels.check_decode_status()  # the read cleared it
    for b, (kc, vc) in zip(model.layers, caches):
        assert torch.equal(b.attention.kv_cache.k_cache, kc)
        assert torch.equal(b.attention.kv_cache.v_cache, vc)
    assert bool((canary == 7).all())


@pytest.mark.gpu
@pytest.mark.parametrize("G", [1, 4, 8])
@pytest.mark.parametrize("S,p0,T", [(1, 0, 64), (7, 0, 64), (128, 0, 328), (33, 37, 128),
                                    (200, 50, 1024), (1536, 0, 2048), (17, 1000, 1100)])
def test_attn_prefill_gpu(G, S, p0, T):
    """tao_attn_prefill_bf16: S queries at positions p0 .. p0 + S - 1 against the cache keys
    0..pos (the causal mask of gpt-fast's prefill over the caches), GQA, vs fp32 SDPA with that
    mask; output [B, S, H * D]."""
    import torch.nn.functional as F

    from torchao._models.llama import kernels

    dev = torch.device("cuda")
    B, Hkv, D = 2, 2 if G == 8 else 8 // G, 128
    H = Hkv * G
    g = torch.Generator(device=dev).manual_seed(S + p0 + G)
    kc = torch.randn(B, Hkv, T, D, device=dev, dtype=torch.bfloat16, generator=g)
    vc = torch.randn(B, Hkv, T, D, device=dev, dtype=torch.bfloat16, generator=g)
    q = torch.randn(B, H, S, D, device=dev, dtype=torch.bfloat16, generator=g)
    pos = torch.arange(p0, p0 + S, device=dev)
    got = kernels.attn_prefill(q, kc, vc, pos, 1 / math.sqrt(D))
    mask = torch.arange(T, device=dev)[None, :] <= pos[:, None]  # [S, T]
    ref = F.scaled_dot_product_attention(q.float(), kc.float(), vc.float(), attn_mask=mask,
                                         enable_gqa=True)
    ref = ref.transpose(1, 2).reshape(B, S, H * D)
    torch.testing.assert_close(got.float(), ref, rtol=2e-2, atol=2e-2)
    assert torch.equal(kernels.attn_prefill(q, kc, vc, pos, 1 / math.sqrt(D)), got)
    # each key-split width (waves per query block; wave w takes key blocks w, w + nw, ...; waves
    # past the last block merge an empty state) against the same reference
    from torchao.kernel.tuning import tuning
    for nw in (1, 2, 4):
        with tuning(attn_prefill_nw=nw):
            alt = kernels.attn_prefill(q, kc, vc, pos, 1 / math.sqrt(D))
        torch.testing.assert_close(alt.float(), ref, rtol=2e-2, atol=2e-2)


@pytest.mark.gpu
def test_add_rmsnorm_and_fused_prefill_gpu():
    """tao_add_rmsnorm_bf16 is bit-identical to (x + r, rmsnorm(x + r)); the prefill with the
    residual adds fused into the norms gives logits bit-identical to the unfused prefill."""
    from torchao._models.llama import kernels
    from torchao._models.llama.generate import apply_quantization

    dev = torch.device("cuda")
    # register-resident kernel at 1-4 pieces per thread (ragged 2056), the two-pass one past 8192
    for rows, D in ((1, 4096), (128, 4096), (7, 1024), (3, 8192), (5, 6144), (2, 2056), (2, 16384)):
        g = torch.Generator(device=dev).manual_seed(rows)
        x = torch.randn(rows, D, device=dev, generator=g).to(torch.bfloat16)
        r = torch.randn(rows, D, device=dev, generator=g).to(torch.bfloat16)
        w = (torch.rand(D, device=dev, generator=g) + 0.5).to(torch.bfloat16)
        h, y = kernels.add_rmsnorm(x, r, w, 1e-5)
        assert torch.equal(h, x + r)
        assert torch.equal(y, kernels.rmsnorm(x + r, w, 1e-5))
    model = _tiny(dev)
    apply_quantization(model, "int4wo-32")
    model.setup_caches(1, 48)
    model.enable_fused_kernels()
    prompt = torch.randint(0, model.config.vocab_size, (1, 24), device=dev)
    old = kernels.PREFILL_ADD_NORM
    try:
        outs = []
        for flag in (False, True):
            kernels.PREFILL_ADD_NORM = flag
            with torch.no_grad():
                outs.append(model._layers_prefill(prompt, torch.arange(24, device=dev)))
        assert torch.equal(outs[0], outs[1])
    finally:
        kernels.PREFILL_ADD_NORM = old


@pytest.mark.gpu
@pytest.mark.parametrize("quant,fuse", [(None, True), ("int4wo-32", True), ("int4wo-32", False),
                                        ("int8wo", True)])
def test_prefill_last_row_gpu(quant, fuse):
    """Greedy prefill's last block past wqkv on the one-token kernels (kernels.PREFILL_LAST_ROW):
    the last position's hidden state within bf16 re-association of the all-rows prefill (the
    one-token GEMVs sum K in another order than the M = S GEMMs), the KV caches of every layer
    bit-identical (wqkv still runs over every row), and the same next token where the top-2
    margin of the all-rows logits is decided."""
    from torchao._models.llama import kernels
    from torchao._models.llama.generate import apply_quantization

    dev = torch.device("cuda")
    model = _tiny(dev)
    if fuse:
        model.fuse_w13()
    if quant:
        apply_quantization(model, quant)
    model.setup_caches(1, 64)
    model.enable_fused_kernels()
    pos = torch.arange(40, device=dev)
    prompt = torch.randint(0, model.config.vocab_size, (1, 40), device=dev,
                           generator=torch.Generator(device=dev).manual_seed(5))
    with torch.no_grad():
        full = model._layers_prefill(prompt, pos)[:, -1:].clone()
        caches = [t.clone() for b in model.layers for t in (b.attention.kv_cache.k_cache,
                                                            b.attention.kv_cache.v_cache)]
        last = model._layers_prefill(prompt, pos, last_only=True)
        assert last.shape == full.shape
        assert torch.equal(torch.cat([t.flatten() for b in model.layers for t in (
            b.attention.kv_cache.k_cache, b.attention.kv_cache.v_cache)]),
            torch.cat([t.flatten() for t in caches]))
        rel = ((last.float() - full.float()).norm() / full.float().norm()).item()
        assert rel < 1e-2, rel
        logits = model.output(kernels.rmsnorm(full, model.norm.weight, model.norm.eps)).float()
        top2 = logits[0, -1].topk(2)
        tok = model.prefill_next(prompt, pos)
        if (top2.values[0] - top2.values[1]).item() > 0.05 * top2.values[0].abs().item():
            assert int(tok.item()) == int(top2.indices[0].item())
        old = kernels.PREFILL_LAST_ROW
        try:
            kernels.PREFILL_LAST_ROW = False
            assert torch.equal(model._layers_prefill(prompt, pos, last_only=True)[:, -1:], full)
        finally:
            kernels.PREFILL_LAST_ROW = old


@pytest.mark.gpu
@pytest.mark.parametrize("quant", ["int4wo-32", "int8wo"])
def test_prefill_last_row_first_token_over_prompts_gpu(quant):
    """PREFILL_LAST_ROW (on by default) computes the greedy first token from the
    one-token kernels, which sum K in another order than the all-rows M = S GEMMs of the
    reference's model(idx)[:, -1].argmax. Over 12 seeded prompts the first token with the flag
    on equals the flag-off (all-rows) token wherever the all-rows top-2 margin decides it
    (> 1% of the top logit); near-ties may differ and are counted, not asserted. The switch
    restores the all-rows path (generate.py --prefill_last_row 0)."""
    from torchao._models.llama import kernels
    from torchao._models.llama.generate import apply_quantization

    dev = torch.device("cuda")
    model = _tiny(dev)
    model.fuse_w13()
    apply_quantization(model, quant)
    model.setup_caches(1, 96)
    model.enable_fused_kernels()
    decided = agree = 0
    old = kernels.PREFILL_LAST_ROW
    try:
        for seed in range(12):
            S = 24 + 5 * seed
            pos = torch.arange(S, device=dev)
            prompt = torch.randint(0, model.config.vocab_size, (1, S), device=dev,
                                   generator=torch.Generator(device=dev).manual_seed(100 + seed))
            with torch.no_grad():
                kernels.PREFILL_LAST_ROW = False
                full = model._layers_prefill(prompt, pos)[:, -1:]
                logits = model.output(kernels.rmsnorm(full, model.norm.weight,
                                                      model.norm.eps)).float()[0, -1]
                tok_off = int(model.prefill_next(prompt, pos).item())
                kernels.PREFILL_LAST_ROW = True
                tok_on = int(model.prefill_next(prompt, pos).item())
            top2 = logits.topk(2)
            assert tok_off == int(top2.indices[0].item()) or \
                (top2.values[0] - top2.values[1]).item() <= 1e-2 * top2.values[0].abs().item()
            if (top2.values[0] - top2.values[1]).item() > 1e-2 * top2.values[0].abs().item():
                decided += 1
                agree += tok_on == tok_off
                assert tok_on == tok_off, (seed, tok_on, tok_off)
    finally:
        kernels.PREFILL_LAST_ROW = old
    assert decided >= 6, decided


@pytest.mark.gpu
@pytest.mark.parametrize("fuse", [True, False])
def test_prefill_partials_bit_identical_gpu(fuse):
    """The prefill with wo / w2's K slices summed by the following add + RMSNorm
    (kernels.PREFILL_PARTIALS) gives hidden states and KV caches bit-identical to the in-kernel
    split-K seam (single-fetch GEMM forced on this small model's shapes with 4 K slices)."""
    from torchao import _lib
    from torchao._models.llama import kernels
    from torchao._models.llama.generate import apply_quantization

    dev = torch.device("cuda")
    model = _tiny(dev)
    if fuse:
        model.fuse_w13()
    apply_quantization(model, "int4wo-32")
    model.setup_caches(1, 160)
    model.enable_fused_kernels()
    pos = torch.arange(100, device=dev)
    prompt = torch.randint(0, model.config.vocab_size, (1, 100), device=dev,
                           generator=torch.Generator(device=dev).manual_seed(7))
    old = kernels.PREFILL_PARTIALS
    _lib.call("tao_tune_gemm_sf", 2, 64, 2, 4, 3, 0, 0)
    try:
        outs = []
        for flag in (False, True):
            kernels.PREFILL_PARTIALS = flag
            with torch.no_grad():
                outs.append(model._layers_prefill(prompt, pos).clone())
                outs.append(torch.cat([t.flatten() for b in model.layers for t in (
                    b.attention.kv_cache.k_cache, b.attention.kv_cache.v_cache)]))
        assert torch.equal(outs[0], outs[2]) and torch.equal(outs[1], outs[3])
    finally:
        kernels.PREFILL_PARTIALS = old
        _lib.call("tao_tune_reset")
