"""Oracle parity for BASELINE configs 4 and 5 on the HIP path.

Config 4 — Llama-3-8B full model, ``quantize_(Int4WeightOnlyConfig(32))``, greedy decode bs=1:
the model is built at the full Llama-3-8B width (dim 4096, 32 heads / 8 kv heads, FFN 14336,
vocabulary 128256) with the layer count cut to 2 so the CPU oracle stays cheap. The prefill runs
the int4 MFMA path; each decode step replays the fused HIP-graph decode (RMSNorm + wqkv +
RoPE/KV, attention, wo, RMSNorm + w1||w3 + SwiGLU, w2, RMSNorm + head) teacher-forced on a fixed
token sequence. Every step's logits are compared with oracle/llama_ref.py: the reference model
restated in fp32 over the reference's own int4 dequantized weights (the CPU "dequant path").

Config 5 — Llama-3-70B linears column-sharded P = 2 / 4 / 8 ways: each shard (a row slice of the
quantized weight, no repacking) through torchao::int4_weight_only_linear, concatenated in rank
order, against the unsharded HIP output and the oracle.
"""

import math

import pytest
import torch

from oracle import llama_ref, oracle

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


def _llama3_8b_truncated(n_layer: int, seed: int):
    from torchao._models.llama.model import ModelArgs, Transformer, llama_configs

    cfg = ModelArgs(**{**llama_configs["Llama-3-8B"], "n_layer": n_layer, "block_size": 256})
    with torch.device("meta"):
        model = Transformer(cfg)
    model = model.to_empty(device=DEV).to(torch.bfloat16)
    gen = torch.Generator(device=DEV).manual_seed(seed)
    with torch.no_grad():
        for name, p in model.named_parameters():
            if name.endswith("norm.weight"):
                p.uniform_(0.5, 1.5, generator=gen)  # non-trivial norm weights
            elif "tok_embeddings" in name:
                p.normal_(0.0, 1.0, generator=gen)
            else:
                b = 1.0 / math.sqrt(p.shape[1])
                p.uniform_(-b, b, generator=gen)
    return model.eval(), cfg


def test_config4_llama3_8b_full_width_int4_graph_decode_vs_oracle():
    from torchao._models.llama.generate import apply_quantization

    torch.manual_seed(0)
    model, cfg = _llama3_8b_truncated(n_layer=2, seed=3)
    g = 32
    # the oracle's weights: the reference's int4 round trip of the same bf16 weights, in fp32
    W = {}
    for name, p in model.named_parameters():
        t = p.detach().cpu()
        if name.endswith(("wqkv.weight", "wo.weight", "w1.weight", "w2.weight", "w3.weight",
                          "output.weight")):
            W[name] = llama_ref.int4_dequant_weight(t, g)
        else:
            W[name] = t.float()
    P, N = 24, 8
    gen = torch.Generator().manual_seed(5)
    seq = torch.randint(0, cfg.vocab_size, (P + N,), generator=gen)
    ref = llama_ref.llama_forward_fp32(W, cfg.n_layer, cfg.n_head, cfg.n_local_heads,
                                       cfg.rope_base, cfg.norm_eps, seq)  # [P + N, V]
    del W

    model.fuse_w13()
    apply_quantization(model, f"int4wo-{g}")
    model.setup_caches(1, P + N)
    assert model.enable_fused_kernels()
    with torch.no_grad():
        pre = model(seq[:P].view(1, P).to(DEV), torch.arange(P, device=DEV))[0].cpu()
    rel_pre = _rel(pre, ref[:P])
    assert rel_pre < 1e-2, rel_pre

    # fused one-token step captured in a HIP graph, teacher-forced
    cur = torch.zeros(1, 1, dtype=torch.int64, device=DEV)
    pos = torch.zeros(1, dtype=torch.int64, device=DEV)
    out = torch.empty(1, 1, cfg.vocab_size, dtype=torch.float32, device=DEV)
    stream = torch.cuda.Stream()
    stream.wait_stream(torch.cuda.current_stream())
    with torch.no_grad(), torch.cuda.stream(stream):
        cur.fill_(int(seq[P]))
        pos.fill_(P)
        out.copy_(model(cur, pos))  # eager warm-up (rewritten below)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=stream):
            out.copy_(model(cur, pos))
    torch.cuda.current_stream().wait_stream(stream)
    worst, agree, decided = 0.0, 0, 0
    for i in range(N):
        cur.fill_(int(seq[P + i]))
        pos.fill_(P + i)
        graph.replay()
        torch.cuda.synchronize()
        got, want = out[0, 0].cpu(), ref[P + i]
        r = _rel(got, want)
        worst = max(worst, r)
        top2 = want.topk(2).values
        if float(top2[0] - top2[1]) > 3e-2 * float(want.abs().max()):  # argmax decided
            decided += 1
            agree += int(got.argmax() == want.argmax())
    assert worst < 1e-2, worst
    assert agree == decided, (agree, decided)
    from torchao._models.llama import kernels

    kernels.check_decode_status()


def test_config4_deeper_greedy_graph_decode_vs_oracle():
    """full Llama-3-8B width, 4 layers, a 128-token prompt, then 32 tokens
    decoded GREEDILY by one captured HIP graph that feeds itself (fused decode step, on-device
    argmax -> next token, position += 1). The oracle (oracle/llama_ref.py, fp32 over the
    reference's int4-dequantized weights) then runs over the prompt plus the decoded tokens:
    every step's logits within 1e-2 relative, and where the oracle's top-2 margin decides the
    argmax, the token the graph picked is the oracle's."""
    from torchao._models.llama.generate import apply_quantization

    torch.manual_seed(0)
    n_layer, P, N, g = 4, 128, 32, 32
    model, cfg = _llama3_8b_truncated(n_layer=n_layer, seed=11)
    W = {}
    for name, p in model.named_parameters():
        t = p.detach().cpu()
        if name.endswith(("wqkv.weight", "wo.weight", "w1.weight", "w2.weight", "w3.weight",
                          "output.weight")):
            W[name] = llama_ref.int4_dequant_weight(t, g)
        else:
            W[name] = t.float()
    prompt = torch.randint(0, cfg.vocab_size, (P,), generator=torch.Generator().manual_seed(9))

    model.fuse_w13()
    apply_quantization(model, f"int4wo-{g}")
    model.setup_caches(1, P + N)
    assert model.enable_fused_kernels()
    with torch.no_grad():
        pre = model(prompt.view(1, P).to(DEV), torch.arange(P, device=DEV))[0].float().cpu()
    cur = torch.zeros(1, 1, dtype=torch.int64, device=DEV)
    pos = torch.zeros(1, dtype=torch.int64, device=DEV)
    out = torch.empty(1, 1, cfg.vocab_size, dtype=torch.float32, device=DEV)
    stream = torch.cuda.Stream()
    stream.wait_stream(torch.cuda.current_stream())
    with torch.no_grad(), torch.cuda.stream(stream):
        cur.fill_(int(pre[-1].argmax()))
        pos.fill_(P)
        out.copy_(model(cur, pos))  # eager warm-up; its cache row is rewritten by the replay
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=stream):
            out.copy_(model(cur, pos))
            cur.copy_(out.argmax(-1))
            pos.add_(1)
    torch.cuda.current_stream().wait_stream(stream)
    tokens, logits = [int(pre[-1].argmax())], []
    cur.fill_(tokens[0])
    pos.fill_(P)
    for _ in range(N):
        graph.replay()
        torch.cuda.synchronize()
        logits.append(out[0, 0].cpu())
        tokens.append(int(cur[0, 0]))
    assert int(pos[0]) == P + N
    seq = torch.cat([prompt, torch.tensor(tokens[:N])])
    ref = llama_ref.llama_forward_fp32(W, cfg.n_layer, cfg.n_head, cfg.n_local_heads,
                                       cfg.rope_base, cfg.norm_eps, seq)  # [P + N, V]
    del W
    assert _rel(pre, ref[:P]) < 1e-2
    worst, agree, decided = 0.0, 0, 0
    for i, got in enumerate([pre[-1]] + logits):
        want = ref[P - 1 + i]
        worst = max(worst, _rel(got, want))
        top2 = want.topk(2).values
        if float(top2[0] - top2[1]) > 3e-2 * float(want.abs().max()):  # argmax decided
            decided += 1
            agree += int(tokens[i] == int(want.argmax()))
        assert tokens[i] == int(got.argmax())  # the graph's on-device pick = host argmax
    assert worst < 1e-2, worst
    assert decided > 0 and agree == decided, (agree, decided)
    from torchao._models.llama import kernels

    kernels.check_decode_status()


# Llama-3-70B linears: wqkv, wo, w1||w3 merged, w2, output head
SHAPES_70B = [(10240, 8192), (8192, 8192), (57344, 8192), (8192, 28672), (128256, 8192)]


@pytest.mark.parametrize("N,K", SHAPES_70B)
def test_config5_llama3_70b_column_shards_match_unsharded_and_oracle(N, K):
    g = 32
    gen = torch.Generator(device=DEV).manual_seed(N + K)
    b = 1.0 / math.sqrt(K)
    w = torch.empty(N, K, device=DEV, dtype=torch.bfloat16).uniform_(-b, b, generator=gen)
    packed, sz = torch.ops.torchao.int4_quantize_pack(w, g, 1e-6)
    x = torch.randn(1, K, generator=torch.Generator().manual_seed(K)).to(torch.bfloat16).to(DEV)
    full = torch.ops.torchao.int4_weight_only_linear(x, packed, sz, g, None)
    scale = float(full.float().abs().max())
    for P in (2, 4, 8):
        n = N // P
        parts = [torch.ops.torchao.int4_weight_only_linear(x, packed[r * n:(r + 1) * n],
                                                             sz[r * n:(r + 1) * n], g, None)
                 for r in range(P)]
        cat = torch.cat(parts, dim=-1)
        # each column's fp32 sum may be re-associated by the shard's launch shape (waves along
        # K, rows per wave): outputs agree to one bf16 rounding, not bit for bit in general
        diff = (cat.float() - full.float()).abs()
        ulp = full.float().abs().clamp_min(scale * 2 ** -8) * 2 ** -7
        assert bool((diff <= ulp).all()), (P, float(diff.max()))
        assert _rel(cat, full) < 2e-3
    # oracle on a sample of rows from every shard of the 8-way split (the CPU dequant path)
    rows = torch.cat([torch.arange(r * (N // 8), r * (N // 8) + 32) for r in range(8)])
    wr = w[rows.to(DEV)].cpu()
    s, z = oracle.int4_qparams(wr, g)
    q = oracle.int4_quantize(wr, s, z, g)
    xc = x.cpu()
    got = full[0, rows.to(DEV)].cpu()
    assert _rel(got, oracle.int4_linear(xc, q, s, z, g)[0]) < 1e-2
    assert _rel(got, oracle.int4_linear_fp32(xc, q, s, z, g)[0]) < 4e-3
