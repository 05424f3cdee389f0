"""End-to-end greedy decode harness: quantize_ a Llama model, prefill a prompt, decode tokens.

Mirrors the reference's gpt-fast harness (torchao/_models/llama/generate.py: ``-q int4wo-<g>``
/ ``int8wo`` / ``int8dq`` quantization at :395-430, prefill + one-token decode loop at
:111-142, tokens/s and memory-bandwidth accounting at :985-1047) with the MI355X execution
model in place of ``torch.compile(mode="reduce-overhead")`` (:865-875): the one-token decode
step is captured once in a HIP graph and replayed, the next token and position advancing on
the device, so a token costs one graph launch and no host round trip until the end.

No checkpoint or tokenizer travels with the repo (no network): with no ``--checkpoint_path``
the model is random-initialised with nn.Linear-default weights and the prompt is synthetic
token ids (seeded), which exercises exactly the shapes and kernels a real checkpoint would.

    python -m torchao._models.llama.generate --model_name Llama-3-8B -q int4wo-32 \\
        --prompt_length 128 --max_new_tokens 200
"""

import argparse
import json
import math
import time
from pathlib import Path
from typing import Optional

import torch
import torch.nn as nn

from torchao._models.llama.model import ModelArgs, Transformer
from torchao.utils import get_model_size_in_bytes

__all__ = ["build_model", "apply_quantization", "prefill", "decode_one_token", "GraphDecoder",
           "generate", "main"]


def build_model(name: str, device, dtype=torch.bfloat16, checkpoint_path: Optional[Path] = None,
                seed: int = 0, tile_format: Optional[str] = None) -> Transformer:
    """Construct on the meta device, materialise on ``device``; load a state dict if given,
    else random-initialise (nn.Linear default U(-1/sqrt(K), 1/sqrt(K)), embeddings N(0, 0.02)).

    ``tile_format`` ("cuda" | "rocm") names the nibble map of TensorCoreTiledLayout tensors in
    the checkpoint (torchao.ops.checkpoint_tile_format); without it such a checkpoint raises."""
    cfg = ModelArgs.from_name(name)
    with torch.device("meta"):
        model = Transformer(cfg)
    model = model.to_empty(device=device).to(dtype)
    if checkpoint_path is not None:
        import contextlib

        from torchao.ops import checkpoint_tile_format

        ctx = checkpoint_tile_format(tile_format) if tile_format else contextlib.nullcontext()
        with ctx:
            state = torch.load(str(checkpoint_path), map_location=device, weights_only=True,
                               mmap=True)
        model.load_state_dict(state, assign=True)
        return model.eval()
    gen = torch.Generator(device=device).manual_seed(seed)
    with torch.no_grad():
        for mod in model.modules():
            if isinstance(mod, nn.Linear):
                bound = 1.0 / math.sqrt(mod.in_features)
                mod.weight.uniform_(-bound, bound, generator=gen)
            elif isinstance(mod, nn.Embedding):
                mod.weight.normal_(0.0, 0.02, generator=gen)
            elif hasattr(mod, "weight") and mod.__class__.__name__ == "RMSNorm":
                mod.weight.fill_(1.0)
    return model.eval()


def apply_quantization(model: nn.Module, quantization: Optional[str]) -> nn.Module:
    """``-q`` strings of the reference harness: int4wo-<g>, int8wo, int8dq (or none)."""
    if not quantization:
        return model
    from torchao.quantization import (
        Int4WeightOnlyConfig,
        Int8DynamicActivationInt8WeightConfig,
        Int8WeightOnlyConfig,
        quantize_,
    )

    if quantization.startswith("int4wo"):
        parts = quantization.split("-")
        g = int(parts[1]) if len(parts) > 1 else 128
        quantize_(model, Int4WeightOnlyConfig(group_size=g))
    elif quantization == "int8wo":
        quantize_(model, Int8WeightOnlyConfig())
    elif quantization == "int8dq":
        quantize_(model, Int8DynamicActivationInt8WeightConfig())
    else:
        raise ValueError(f"unsupported quantization {quantization!r}")
    return model


@torch.no_grad()
def prefill(model: Transformer, prompt: torch.Tensor, input_pos: torch.Tensor) -> torch.Tensor:
    """prompt [B, P] at positions input_pos [P] -> greedy next token [B, 1]."""
    return model.prefill_next(prompt, input_pos)


@torch.no_grad()
def decode_one_token(model: Transformer, cur: torch.Tensor,
                     input_pos: torch.Tensor) -> torch.Tensor:
    return model.decode_next(cur, input_pos)


class GraphDecoder:
    """One decode step captured in a HIP graph over static buffers: ``cur`` [B, 1] (the token
    fed in, overwritten by the token produced), ``pos`` [1] (its position, incremented in
    place) and ``tokens`` [B, max_len] (each produced token stored at its position), so a
    replay is the whole per-token work with no host involvement."""

    def __init__(self, model: Transformer, batch: int, max_len: int, device,
                 steps_per_graph: int = 1):
        self.model = model
        self.cur = torch.zeros(batch, 1, dtype=torch.int64, device=device)
        self.pos = torch.zeros(1, dtype=torch.int64, device=device)
        self.tokens = torch.zeros(batch, max_len, dtype=torch.int64, device=device)
        self.stream = torch.cuda.Stream(device)
        self.graph = None
        # steps_per_graph > 1: a second graph holds that many steps back to back (the step is
        # device-driven, so k steps replay as one graph launch: one launch overhead per k tokens)
        self.steps_per_graph = max(1, int(steps_per_graph))
        self.graph_k = None

    @torch.no_grad()
    def _step(self):
        if self.model.decode_advance(self.cur, self.pos, self.tokens):
            return  # fused path, batch 1: argmax + bookkeeping in one kernel
        nxt = decode_one_token(self.model, self.cur, self.pos)
        self.pos.add_(1)
        self.tokens.index_copy_(1, self.pos, nxt)
        self.cur.copy_(nxt)

    def capture(self):
        # eager warm-up on the capture stream (allocator pools, library workspaces); the
        # buffers are restored afterwards, and the KV rows it wrote are rewritten by any decode
        saved = (self.cur.clone(), self.pos.clone())
        self.stream.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self.stream):
            self._step()
            self.cur.copy_(saved[0])
            self.pos.copy_(saved[1])
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph, stream=self.stream):
                self._step()
            if self.steps_per_graph > 1:
                self.graph_k = torch.cuda.CUDAGraph()
                with torch.cuda.graph(self.graph_k, stream=self.stream):
                    for _ in range(self.steps_per_graph):
                        self._step()
        torch.cuda.current_stream().wait_stream(self.stream)
        self.cur.copy_(saved[0])
        self.pos.copy_(saved[1])
        torch.cuda.synchronize()

    def reset(self, prompt: torch.Tensor, token: torch.Tensor):
        P = prompt.shape[1]
        self.tokens[:, :P] = prompt
        self.tokens[:, P:P + 1] = token
        self.cur.copy_(token)
        self.pos.fill_(P)

    def step(self):
        self.graph.replay()

    def run(self, n: int):
        """n decode steps: the k-step graph n // k times, then single steps."""
        k = self.steps_per_graph if self.graph_k is not None else 1
        for _ in range(n // k if k > 1 else 0):
            self.graph_k.replay()
        for _ in range(n % k if k > 1 else n):
            self.graph.replay()


class GraphPrefill:
    """The prefill of a fixed prompt shape captured in a HIP graph over static buffers (the
    reference compiles it with ``--compile_prefill``, generate.py:865-875): ``prompt`` [B, P]
    is copied in, the replay writes the KV caches and the first greedy token into ``token``."""

    def __init__(self, model: Transformer, prompt_shape, device):
        self.model = model
        self.prompt = torch.zeros(prompt_shape, dtype=torch.int64, device=device)
        self.pos = torch.arange(prompt_shape[1], device=device)
        self.token = torch.zeros(prompt_shape[0], 1, dtype=torch.int64, device=device)
        self.stream = torch.cuda.Stream(device)
        self.graph = None

    @torch.no_grad()
    def capture(self, prompt: torch.Tensor):
        self.prompt.copy_(prompt)
        self.stream.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self.stream):
            self.token.copy_(prefill(self.model, self.prompt, self.pos))  # eager warm-up
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph, stream=self.stream):
                self.token.copy_(prefill(self.model, self.prompt, self.pos))
        torch.cuda.current_stream().wait_stream(self.stream)
        torch.cuda.synchronize()

    def __call__(self, prompt: torch.Tensor) -> torch.Tensor:
        self.prompt.copy_(prompt)
        self.graph.replay()
        return self.token


@torch.no_grad()
def generate(model: Transformer, prompt: torch.Tensor, max_new_tokens: int,
             decoder: Optional[GraphDecoder] = None, prefiller: Optional[GraphPrefill] = None):
    """Greedy decode. Returns (tokens [B, P + max_new_tokens], prefill_s, decode_s)."""
    B, P = prompt.shape
    device = prompt.device
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if prefiller is not None:
        tok = prefiller(prompt)
    else:
        tok = prefill(model, prompt, torch.arange(P, device=device))
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    _check_status(model)  # a timed-out split-K hand-off in the prefill raises here, not later
    if decoder is not None:
        decoder.reset(prompt, tok)
        decoder.run(max_new_tokens - 1)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        _check_status(model)
        return decoder.tokens[:, :P + max_new_tokens].clone(), t1 - t0, t2 - t1
    out = torch.empty(B, P + max_new_tokens, dtype=prompt.dtype, device=device)
    out[:, :P] = prompt
    out[:, P:P + 1] = tok
    pos = torch.tensor([P], device=device)
    for i in range(1, max_new_tokens):
        tok = decode_one_token(model, tok, pos)
        out[:, P + i:P + i + 1] = tok
        pos += 1
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    _check_status(model)
    return out, t1 - t0, t2 - t1


@torch.no_grad()
def eager_token_check(model: Transformer, prompt: torch.Tensor, graph_tokens: torch.Tensor,
                      n: int):
    """Output check of a graph-decoded run: the first ``n`` greedy tokens decoded again EAGERLY
    (prefill, then one ``model(tok, pos)`` forward per token, fp32 logits, torch argmax) against
    ``graph_tokens`` [B, >= P + n]; also whether every eager step's logits were finite. Returns
    (matching positions, n, first mismatching offset or None, all logits finite)."""
    B, P = prompt.shape
    device = prompt.device
    tok = prefill(model, prompt, torch.arange(P, device=device))
    toks, finite = [tok], True
    pos = torch.tensor([P], device=device)
    for _ in range(1, n):
        logits = model(tok, pos)
        finite = finite and bool(torch.isfinite(logits).all())
        tok = logits[:, -1].argmax(dim=-1, keepdim=True).to(prompt.dtype)
        toks.append(tok)
        pos += 1
    torch.cuda.synchronize()
    _check_status(model)
    eq = (torch.cat(toks, dim=1) == graph_tokens[:, P:P + n]).all(dim=0).cpu()
    bad = (~eq).nonzero()
    return int(eq.sum()), n, (int(bad[0]) if len(bad) else None), finite


def _check_status(model: Transformer) -> None:
    if model.fused:
        from torchao._models.llama import kernels

        kernels.check_decode_status()


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--model_name", default="Llama-3-8B")
    ap.add_argument("--checkpoint_path", type=Path, default=None)
    ap.add_argument("-q", "--quantization", default="int4wo-32")
    ap.add_argument("--prompt_length", type=int, default=128)
    ap.add_argument("--max_new_tokens", type=int, default=200)
    ap.add_argument("--num_samples", type=int, default=3)
    ap.add_argument("--batch_size", type=int, default=1)
    ap.add_argument("--no_graph", action="store_true", help="eager decode (no HIP graph)")
    ap.add_argument("--no_fused", action="store_true",
                    help="torch ops for norms / rope / attention / silu (no fused kernels)")
    ap.add_argument("--no_fuse_w13", action="store_true",
                    help="keep w1 and w3 as two linears (the reference module layout)")
    ap.add_argument("--deferred_norm", action="store_true",
                    help="fused RMSNorm scales the GEMV outputs by rsqrt(mean(x^2)+eps) instead "
                         "of normalising x first (one bf16 rounding fewer; tao_tune_int4_norm 1)")
    ap.add_argument("--sdpa_prefill", action="store_true",
                    help="prefill attention through torch's masked SDPA instead of "
                         "tao_attn_prefill_bf16 (kernels.PREFILL_ATTN = False)")
    ap.add_argument("--prefill_rope", type=int, default=-1,
                    help="1 / 0: fold the prefill RoPE + KV write into the int4 wqkv GEMM's "
                         "epilogue (model.PREFILL_ROPE; -1 = built-in)")
    ap.add_argument("--prefill_swiglu", type=int, default=-1,
                    help="1 / 0: fold the prefill SiLU-mul into the int4 w1||w3 GEMM's epilogue "
                         "(model.PREFILL_SWIGLU; -1 = built-in)")
    ap.add_argument("--prefill_add_norm", type=int, default=-1,
                    help="1 / 0: fuse the prefill residual adds with the next RMSNorm or not "
                         "(kernels.PREFILL_ADD_NORM; -1 = built-in)")
    ap.add_argument("--prefill_last_row", type=int, default=-1,
                    help="1 / 0: the greedy first token from the last block's last row on the "
                         "one-token kernels (a different K summation order than the reference's "
                         "all-rows model(idx)[:, -1].argmax; 0 restores the all-rows path; "
                         "kernels.PREFILL_LAST_ROW; -1 = built-in, on)")
    ap.add_argument("--ffn_engine", type=int, default=-1,
                    help="1 / 0: decode feed-forward on the persistent LDS-DMA engine "
                         "(kernels.DECODE_FFN_ENGINE; -1 = built-in, off)")
    ap.add_argument("--native_prefill_attn", action="store_true",
                    help="prefill attention on tao_attn_prefill_bf16 (kernels.PREFILL_ATTN = True)")
    ap.add_argument("--qkv_attn", type=int, default=-1,
                    help="1 / 0: decode wqkv + RoPE/KV + attention in one launch or two "
                         "(kernels.DECODE_QKV_ATTN; -1 = built-in)")
    ap.add_argument("--head_prologue", action="store_true",
                    help="fuse the final RMSNorm into the output head GEMV (kernels.HEAD_PROLOGUE)")
    ap.add_argument("--steps_per_graph", type=int, default=32,
                    help="decode steps captured back to back in one HIP graph launch (1 = one "
                         "per token; 32: 717.6 vs 710.1 tokens/s, "
                         "profiles/r3_ab_e2e_steps_per_graph.jsonl)")
    ap.add_argument("--attn_mode", type=int, default=-1,
                    help="decode attention kernel (tao_tune_attn; -1 = built-in)")
    ap.add_argument("--check_tokens", type=int, default=32,
                    help="after timing, decode this many tokens again eagerly and report their "
                         "agreement with the graph-decoded tokens (0 = skip)")
    ap.add_argument("--tune", action="append", default=[], metavar="KNOB=V[,V..]",
                    help="launch-shape override for this run (torchao.kernel.tuning knobs; A/B "
                         "measurement only), e.g. --tune cnt_stride=1")
    ap.add_argument("--tile_format", choices=("cuda", "rocm"), default=None,
                    help="nibble map of TensorCoreTiledLayout tensors in --checkpoint_path")
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--write_result", type=Path, default=None)
    args = ap.parse_args(argv)

    if (args.head_prologue or args.sdpa_prefill or args.qkv_attn >= 0
            or args.native_prefill_attn or args.prefill_add_norm >= 0
            or args.prefill_last_row >= 0 or args.ffn_engine >= 0):
        from torchao._models.llama import kernels

        if args.ffn_engine >= 0:
            kernels.DECODE_FFN_ENGINE = bool(args.ffn_engine)
        if args.prefill_last_row >= 0:
            kernels.PREFILL_LAST_ROW = bool(args.prefill_last_row)
        if args.qkv_attn >= 0:
            kernels.DECODE_QKV_ATTN = bool(args.qkv_attn)

        if args.prefill_add_norm >= 0:
            kernels.PREFILL_ADD_NORM = bool(args.prefill_add_norm)
        if args.sdpa_prefill:
            kernels.PREFILL_ATTN = False
        if args.native_prefill_attn:
            kernels.PREFILL_ATTN = True
        if args.head_prologue:
            kernels.HEAD_PROLOGUE = True
    if args.deferred_norm or args.attn_mode >= 0:
        from torchao import _lib

        if args.deferred_norm:
            _lib.call("tao_tune_int4_norm", 1)
        if args.attn_mode >= 0:
            _lib.call("tao_tune_attn", args.attn_mode)
    for kv in args.tune:
        from torchao.kernel.tuning import apply as tune_apply

        knob, _, vals = kv.partition("=")
        tune_apply(knob, *[int(v) for v in vals.split(",")])
    if args.prefill_swiglu >= 0:
        from torchao._models.llama import model as _mdl

        _mdl.PREFILL_SWIGLU = bool(args.prefill_swiglu)
    if args.prefill_rope >= 0:
        from torchao._models.llama import model as _mdl

        _mdl.PREFILL_ROPE = bool(args.prefill_rope)
    device = torch.device(args.device)
    t = time.perf_counter()
    model = build_model(args.model_name, device, checkpoint_path=args.checkpoint_path,
                        seed=args.seed, tile_format=args.tile_format)
    torch.cuda.synchronize()
    t_build = time.perf_counter() - t
    if not args.no_fuse_w13:
        model.fuse_w13()
    t = time.perf_counter()
    apply_quantization(model, args.quantization)
    torch.cuda.synchronize()
    t_quant = time.perf_counter() - t
    model_bytes = get_model_size_in_bytes(model, ignore_embeddings=True)

    B, P, T = args.batch_size, args.prompt_length, args.max_new_tokens
    model.setup_caches(B, P + T)
    if not args.no_fused:
        model.enable_fused_kernels()
    gen = torch.Generator(device="cpu").manual_seed(args.seed + 1)
    prompt = torch.randint(0, model.config.vocab_size, (B, P), generator=gen).to(device)

    decoder = prefiller = None
    if not args.no_graph:
        decoder = GraphDecoder(model, B, P + T, device, steps_per_graph=args.steps_per_graph)
        # capture after an eager prefill so every kernel and workspace has been set up
        decoder.reset(prompt, prefill(model, prompt, torch.arange(P, device=device)))
        decoder.capture()
        prefiller = GraphPrefill(model, (B, P), device)
        prefiller.capture(prompt)

    generate(model, prompt, min(T, 8), decoder, prefiller)  # warm-up
    runs = []
    for _ in range(args.num_samples):
        tokens, t_pre, t_dec = generate(model, prompt, T, decoder, prefiller)
        runs.append((t_pre, t_dec))
    t_pre = sorted(r[0] for r in runs)[len(runs) // 2]
    t_dec = sorted(r[1] for r in runs)[len(runs) // 2]
    dec_tok_s = B * (T - 1) / t_dec
    res = {
        "model": args.model_name,
        "quantization": args.quantization,
        "weights": "checkpoint" if args.checkpoint_path else "random-init (seeded)",
        "batch_size": B,
        "prompt_length": P,
        "max_new_tokens": T,
        "hip_graph": decoder is not None,
        "fused_decode_kernels": model.fused,
        "fused_w13": not args.no_fuse_w13,
        "deferred_norm": args.deferred_norm,
        "decode_tokens_per_s": round(dec_tok_s, 2),
        "decode_ms_per_token": round(t_dec / (T - 1) * 1e3, 3),
        "prefill_ms": round(t_pre * 1e3, 3),
        "tokens_per_s_incl_prefill": round(B * T / (t_pre + t_dec), 2),
        "model_bytes_excl_embeddings": model_bytes,
        "memory_bandwidth_GBps": round(model_bytes * dec_tok_s / B / 1e9, 1),
        "build_s": round(t_build, 2),
        "quantize_s": round(t_quant, 2),
        "sample_tokens": tokens[0, P:P + 16].tolist(),
    }
    if decoder is not None and args.check_tokens > 0:
        n = min(args.check_tokens, T)
        match, n, first_bad, finite = eager_token_check(model, prompt, tokens, n)
        res["graph_eager_token_match"] = f"{match}/{n}"
        res["graph_eager_first_mismatch"] = first_bad
        res["eager_logits_finite"] = finite
    print(json.dumps(res), flush=True)
    if args.write_result:
        with open(args.write_result, "a") as f:
            f.write(json.dumps(res) + "\n")
    return res


if __name__ == "__main__":
    main()
