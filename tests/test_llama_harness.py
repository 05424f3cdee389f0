"""The end-to-end decode harness (torchao/_models/llama): KV-cache decode == full forward on
CPU (bf16 model, no quantization), and on the GPU with int4 weights: graph-replayed decode ==
eager decode token for token, and int4 logits track the bf16 model's."""

import pytest
import torch

from torchao._models.llama.generate import (
    GraphDecoder,
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
    prompt = torch.randint(0, model.config.vocab_size, (1, P), device=dev)

    # quantized logits track the bf16 model (quantization error only)
    lq = model(prompt, torch.arange(P, device=dev))
    lr = ref(prompt, torch.arange(P, device=dev))
    sqnr = 20 * torch.log10(lr.norm() / (lr - lq).norm())
    assert sqnr > (15 if quant.startswith("int4") else 25), float(sqnr)

    eager, _, _ = generate(model, prompt, T, None)
    dec = GraphDecoder(model, 1, P + T, dev)
    dec.reset(prompt, prefill(model, prompt, torch.arange(P, device=dev)))
    dec.capture()
    graphed, _, _ = generate(model, prompt, T, dec)
    assert torch.equal(graphed, eager)
    # a second run replays the same graph from a fresh prefill
    again, _, _ = generate(model, prompt, T, dec)
    assert torch.equal(again, eager)
    # single step helper agrees with the graph's first produced token
    tok = prefill(model, prompt, torch.arange(P, device=dev))
    nxt = decode_one_token(model, tok, torch.tensor([P], device=dev))
    assert int(nxt) == int(eager[0, P + 1])
