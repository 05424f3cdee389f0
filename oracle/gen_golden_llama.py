"""Generate tests/golden/llama_tiny_fp32.npz by running the REFERENCE gpt-fast model
(read-only at /root/reference, torchao/_models/llama/model.py) — pins oracle/llama_ref.py.

Run in the build container only (the reference does not exist on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 PYTHONPATH=/root/reference python3 oracle/gen_golden_llama.py

A head_dim-64 GQA config small enough for a fixture (dim 128, 2 layers, 2 heads, 1 kv head,
vocab 256, rope base 500000) in fp32 with seeded weights rounded to bf16-representable values
(stored as their bf16 bit patterns, half the bytes): the reference's Transformer with its KV
caches, a 10-token causal prefill at positions 0..9 and two single-token decode steps. The
fixture stores the weights, the token ids and the reference's logits (numbers only).
"""

import os

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(os.path.dirname(HERE), "tests", "golden", "llama_tiny_fp32.npz")


def main():
    from torchao._models.llama.model import ModelArgs, Transformer  # the reference

    import torchao

    assert os.path.realpath(torchao.__file__).startswith("/root/reference"), torchao.__file__
    cfg = ModelArgs(block_size=64, vocab_size=256, n_layer=2, n_head=2, dim=128,
                    intermediate_size=256, n_local_heads=1, rope_base=500000)
    torch.manual_seed(0)
    model = Transformer(cfg).float().eval()
    g = torch.Generator().manual_seed(1)
    with torch.no_grad():
        for name, p in model.named_parameters():
            if name.endswith("norm.weight"):
                p.copy_(torch.rand(p.shape, generator=g) + 0.5)
            elif "tok_embeddings" in name:
                p.copy_(torch.randn(p.shape, generator=g) * 0.5)
            else:
                b = 1.0 / p.shape[1] ** 0.5
                p.copy_((torch.rand(p.shape, generator=g) * 2 - 1) * b)
            p.copy_(p.to(torch.bfloat16).float())  # exactly representable in bf16
    model.setup_caches(max_batch_size=1, max_seq_length=32)
    tokens = torch.randint(0, cfg.vocab_size, (1, 12), generator=g)
    with torch.no_grad():
        pre = model(tokens[:, :10], torch.arange(10))
        d1 = model(tokens[:, 10:11], torch.tensor([10]))
        d2 = model(tokens[:, 11:12], torch.tensor([11]))
    logits = torch.cat([pre, d1, d2], dim=1)[0]
    bits = lambda t: t.to(torch.bfloat16).view(torch.int16).numpy().view(np.uint16)  # noqa: E731
    rec = {f"w:{k}": bits(v.detach()) for k, v in model.state_dict().items()
           if not k.endswith(("k_cache", "v_cache")) and "causal_mask" not in k
           and "freqs_cis" not in k}
    rec["tokens"] = tokens[0].numpy()
    rec["logits"] = logits.numpy()
    rec["config"] = np.array([cfg.n_layer, cfg.n_head, cfg.n_local_heads, cfg.rope_base],
                             dtype=np.float64)
    np.savez_compressed(OUT, **rec)
    print("wrote", OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()
