#!/usr/bin/env python3
"""Benchmark: int4 group-32 weight-only linear GB/s + tokens/s, Llama-3-8B shapes, M = 1 decode.

One "step" = one decoded token through every int4 linear of a Llama-3-8B-shaped stack
(32 layers x {wqkv 6144x4096, wo 4096x4096, w1||w3 28672x4096, w2 4096x14336} + output
128256x4096): 129 launches of the gfx950 int4 GEMV, 4.70 GB of packed weights and scales per
token (> 256 MiB Infinity Cache, so every byte comes from HBM). The gate and up projections
share their input and run as one merged linear, as the e2e harness runs them; --no-fuse-w13
gives the reference's module layout (w1 and w3 apart, 161 launches, the same bytes).
Weights are random-init nn.Linear-distributed bf16, quantized with the
Int4WeightOnlyConfig(group_size=32) math and packed by the HIP pack kernel; activations are
synthetic N(0,1) bf16; everything is resident in HBM before timing. The step is captured once
in a HIP graph and replayed.

N GPUs (torchrun, one rank per GPU): a linear is column-sharded (rank r owns output rows
[r N/P, (r+1) N/P)) with its output all-gathered over RCCL after each GEMV (north star,
SURVEY §8e) when that is faster than running it whole on every rank: at startup every distinct
(N, K) is timed both ways (whole GEMV vs N/P GEMV + all-gather, max over ranks;
--shard-policy auto). An M = 1 gather is latency-bound (~10 µs class), so at 8B sizes only the
large linears can gain. --shard-policy size / all / none override the measurement.
Total work is fixed as P grows ("strong" scaling); value counts the whole model's bytes once
per step.

The line also carries config5_70b: BASELINE config 5's Llama-3-70B linear step (80 layers,
43.4 GB of int4 weights per token). At P = 1 every linear runs whole on the one GPU (the 1-GPU
anchor of the 1/2/4/8 curve); at P > 1 under the Megatron plan (pairs + head gather) and, beside
it as north_star_plan, the north star's plan (every linear column-sharded + RCCL all-gather),
~1/P of the weights per rank, collectives inside the step's HIP graph, with the GEMV-only and
collectives-only times beside the whole step (--no-config5 skips it). --model 70b makes the 70B
the headline instead; the default headline stays the 8B, so the N = 1 point equals BENCH.

Reported (one JSON line, rank 0):
  value        = algorithmic bytes per step x steps / wall time  (GB/s, whole job)
  linear_steps_per_s = steps / wall time (linears only; the model's decode rate is e2e_decode)
  north_star   = BASELINE's per-launch target shape (int4 g32 M=1 4096x4096, wo at 8B): us per
                 launch inside a replayed graph of that shape's launches, and its fraction of
                 8 TB/s (target 0.70, reported unmet while it is), split into the kernel's own
                 span (dispatch-packet events) and the launch-to-launch gap;
                 roofline.per_shape_graph / per_shape_frac hold every shape
  unfused_w13_step = the same 8B step in the reference's module layout (w1, w3 apart: 161
                 launches, the same bytes), one HIP graph
  roofline     = the GEMV kernel: algorithmic bytes per step / GPU time per step of the
                 GEMV-only graph replayed back to back (HIP events on the replay stream, i.e. the
                 sum of the step's kernel durations in the timed regime), against the MI355X
                 HBM3E peak of 8 TB/s; per_shape = one eager step timed per kernel by events the
                 dispatch packets write (tao_profile_*); traffic = HBM bytes per step from the
                 committed rocprofv3 FETCH_SIZE pass (profiles/, gfx950 x2 correction)
  cpu_baseline = the reference's CPU "dequant path" (dequantize -> F.linear, bf16) restated in
                 oracle/, timed on this host's cores over a bounded sample (rank 0, N = 1)
  reference_gpu = the reference's own GPU kernel (PyTorch-ROCm aten._weight_int4pack_mm, which
                 torchao's TensorCoreTiledLayout calls) on the identical weights and step, one
                 HIP graph: its GB/s and the max rel. L2 difference from our outputs
  config2_shapes = BASELINE config 2's shapes (4096x4096, 11008x4096, 4096x11008; int4 g32,
                 M = 1): us per launch in a graph of 32 distinct weights, GB/s, fraction of 8 TB/s
  prefill_mfma = BASELINE config 3 (int8 dyn-act int8-weight linear, M = 128, 4096x4096, the
                 int8 MFMA path) and the int4 g32 linear at M = 128 on its bf16 MFMA path:
                 kernel us, TOPS, fraction of the dense MFMA peak, attainable-roofline fraction
  e2e_decode   = BASELINE config 4: the e2e decode harness (random-init Llama-3-8B, int4wo-32,
                 prompt 128, 200 new tokens, bs = 1, HIP-graph decode) in a child process:
                 decode tokens/s, ms/token, prefill ms (rank 0, N = 1; --no-e2e skips it)
"""

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "torchao-fork_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E, spec (MI355X_MICROARCH.md chip table)
PMC_FILE = os.path.join(ROOT, "profiles", "r6u_pmc_fetch_bench.json")  # --pmc-file overrides

LLAMA3_8B = dict(dim=4096, n_layer=32, n_head=32, n_kv_head=8, head_dim=128,
                 intermediate=14336, vocab=128256)
LLAMA3_70B = dict(dim=8192, n_layer=80, n_head=64, n_kv_head=8, head_dim=128,
                  intermediate=28672, vocab=128256)  # BASELINE config 5 (--model 70b)
MODELS = {"8b": ("Llama-3-8B", LLAMA3_8B), "70b": ("Llama-3-70B", LLAMA3_70B)}


def llama_linears(cfg, fuse_w13=True):
    """(name, N, K) of every nn.Linear quantize_ touches in gpt-fast's Llama (model.py); with
    fuse_w13 the gate and up projections (same input) are one [2I, dim] linear, as the e2e
    harness runs them (torchao/_models/llama/model.py FeedForward.fuse_w13)."""
    d, hd, inter = cfg["dim"], cfg["head_dim"], cfg["intermediate"]
    qkv = (cfg["n_head"] + 2 * cfg["n_kv_head"]) * hd
    out = []
    for layer in range(cfg["n_layer"]):
        out += [
            (f"layers.{layer}.attention.wqkv", qkv, d),
            (f"layers.{layer}.attention.wo", d, d),
        ]
        if fuse_w13:
            out.append((f"layers.{layer}.feed_forward.w13", 2 * inter, d))
        else:
            out += [
                (f"layers.{layer}.feed_forward.w1", inter, d),
                (f"layers.{layer}.feed_forward.w3", inter, d),
            ]
        out.append((f"layers.{layer}.feed_forward.w2", d, inter))
    out.append(("output", cfg["vocab"], d))
    return out


def workload_desc(cfg, fuse_w13=True):
    """'32 layers x {wqkv 6144x4096, ...} + output 128256x4096' for the config."""
    shapes = {}
    for name, N, K in llama_linears(cfg, fuse_w13):
        shapes.setdefault(name.split(".")[-1], (N, K))
    names = {"w13": "w1||w3", "w1": "w1/w3"}
    body = ", ".join(f"{names.get(k, k)} {N}x{K}" for k, (N, K) in shapes.items()
                     if k not in ("output", "w3"))
    N, K = shapes["output"]
    return f"{cfg['n_layer']} layers x {{{body}}} + output {N}x{K}"


def int4_alg_bytes(N, K, g, M=1):
    """N*K/2 + (K/g)*N*4 + M*K*2 + M*N*2 (no bias)."""
    return N * K // 2 + (K // g) * N * 4 + M * K * 2 + M * N * 2


def make_int4_weight(N, K, g, seed, device):
    """Random nn.Linear-init bf16 weight -> tinygemm qparams -> gfx950 packed (HIP pack kernel)."""
    from torchao.quantization.quant_primitives import (
        MappingType,
        _choose_qparams_affine_tinygemm,
        _quantize_affine_tinygemm,
    )

    gen = torch.Generator(device=device).manual_seed(seed)
    bound = 1.0 / (K ** 0.5)
    w = (torch.rand(N, K, generator=gen, device=device) * 2 - 1).mul_(bound).to(torch.bfloat16)
    s, z = _choose_qparams_affine_tinygemm(
        w, MappingType.ASYMMETRIC, (1, g), torch.int32, 0, 15, 1e-6,
        zero_point_dtype=torch.bfloat16)
    q = _quantize_affine_tinygemm(w, (1, g), s, z, torch.int32, 0, 15)
    del w
    packed = torch.ops.torchao.int4_pack(q)
    del q
    sz = torch.stack([s, z], dim=-1).contiguous()
    return packed, sz


def calibrate_sharding(shapes, P, g, device, rehearsal, reps=20, pairs=None):
    """Per (N, K): time the whole-N GEMV and the N/P GEMV + its all-gather, and per Megatron
    pair the replicated pair against colwise + rowwise + all-reduce (GEMVs and RCCL collectives
    each replayed from a HIP graph, as the step runs them; each shape's weights rotated over
    copies past the 256 MiB Infinity Cache; GPU events; max over ranks so every rank takes the
    same decision). An M = 1 collective is latency-bound (~10 µs class), so only linears whose
    GEMV saves more than that are worth sharding. In a gloo rehearsal the collectives are the
    host-staged ones that rehearsal steps take, timed as such: its decision table is real for
    that transport (and says "replicate" for nearly everything)."""
    from torchao import _lib

    lib = _lib.lib()
    sp = torch.cuda.current_stream(device).cuda_stream

    def gemv_us(N, K):
        copies = max(2, min(32, (512 << 20) // max(1, int4_alg_bytes(N, K, g))))
        ws = [make_int4_weight(N, K, g, seed=7 + c, device=device) for c in range(copies)]
        x = torch.randn(1, K, device=device, dtype=torch.bfloat16)
        y = torch.empty(N, device=device, dtype=torch.bfloat16)

        def go(c):
            lib.tao_int4wo_linear_bf16(x.data_ptr(), ws[c][0].data_ptr(), ws[c][1].data_ptr(),
                                       None, y.data_ptr(), 1, N, K, g, sp)

        for c in range(copies):
            go(c)
        # the GEMVs replayed from one HIP graph, as the step runs them (eager launches are
        # host-bound at these sizes: ~5-11 µs per launch against 3-5 µs replayed); no
        # collective is captured here, so every rank issues the same calls either way
        nonlocal sp
        s = torch.cuda.Stream(device)
        s.wait_stream(torch.cuda.current_stream(device))
        sp_eager = sp
        try:
            sp = s.cuda_stream
            with torch.cuda.stream(s):
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph, stream=s):
                    for i in range(reps):
                        go(i % copies)
                graph.replay()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                graph.replay()
                e1.record(s)
            e1.synchronize()
            del graph
            return e0.elapsed_time(e1) * 1e3 / reps
        except Exception:  # graph capture unavailable: eager launches
            torch.cuda.synchronize()
        finally:
            sp = sp_eager
            torch.cuda.current_stream(device).wait_stream(s)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(reps):
            go(i % copies)
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) * 1e3 / reps

    def collective_us(fn):
        """µs per collective: RCCL ones captured `reps` times in one HIP graph and replayed (as
        the step runs them; eager if capture fails); in a gloo rehearsal the host-staged path the
        rehearsal step takes, timed on the host clock."""
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        if rehearsal:
            t0 = time.perf_counter()
            for _ in range(reps):
                fn()
            torch.cuda.synchronize()
            return (time.perf_counter() - t0) * 1e6 / reps
        s = torch.cuda.Stream(device)
        s.wait_stream(torch.cuda.current_stream(device))
        try:
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.stream(s):
                with torch.cuda.graph(graph, stream=s):
                    for _ in range(reps):
                        fn()
                graph.replay()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                graph.replay()
                e1.record(s)
            e1.synchronize()
            del graph
            return e0.elapsed_time(e1) * 1e3 / reps
        except Exception:  # capture of collectives unavailable: eager
            torch.cuda.synchronize()
        finally:
            torch.cuda.current_stream(device).wait_stream(s)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) * 1e3 / reps

    def gather_us(N):
        y_loc = torch.zeros(N // P, device=device, dtype=torch.bfloat16)
        y = torch.empty(N, device=device, dtype=torch.bfloat16)

        def fn():
            if rehearsal:
                parts = [torch.empty_like(y_loc, device="cpu") for _ in range(P)]
                dist.all_gather(parts, y_loc.cpu())
                y.copy_(torch.cat(parts))
            else:
                dist.all_gather_into_tensor(y, y_loc)
        return collective_us(fn)

    def allreduce_us(N):
        y = torch.zeros(N, device=device, dtype=torch.bfloat16)

        def fn():
            if rehearsal:
                t = y.cpu()
                dist.all_reduce(t)
                y.copy_(t)
            else:
                dist.all_reduce(y)
        return collective_us(fn)

    def agree(vals):  # max over ranks so every rank takes the same decision
        t = torch.tensor(vals, dtype=torch.float64, device="cpu" if rehearsal else device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return [float(v) for v in t.tolist()]

    out = {}
    for N, K in shapes:
        if N % P:
            continue
        whole, part, gather = agree([gemv_us(N, K), gemv_us(N // P, K), gather_us(N)])
        out[(N, K)] = {"whole_us": round(whole, 2), "shard_us": round(part, 2),
                       "allgather_us": round(gather, 2), "shard": part + gather < 0.95 * whole}
        torch.cuda.empty_cache()
    # Megatron pairs (colwise A without a gather -> rowwise B + all-reduce), per distinct pair
    for (Na, Ka), (Nb, Kb) in pairs or ():
        if Na % P or Kb % (P * g):
            continue
        wa, wb, pa, pb, ar = agree([gemv_us(Na, Ka), gemv_us(Nb, Kb), gemv_us(Na // P, Ka),
                                    gemv_us(Nb, Kb // P), allreduce_us(Nb)])
        out[("pair", Na, Ka, Nb, Kb)] = {
            "whole_us": round(wa + wb, 2), "colwise_us": round(pa, 2), "rowwise_us": round(pb, 2),
            "allreduce_us": round(ar, 2), "shard": pa + pb + ar < 0.95 * (wa + wb)}
        torch.cuda.empty_cache()
    return out


INT8_PEAK_TOPS = 5000.0   # MI355X dense int8 MFMA, 2x the bf16 rate (MI355X_MICROARCH.md)
BF16_PEAK_TFLOPS = 2500.0  # MI355X dense bf16 MFMA


def reference_gpu_step(plan, xs, g, device, steps):
    """The reference's own GPU kernel on the same step: PyTorch-ROCm's aten._weight_int4pack_mm
    (what torchao's TensorCoreTiledLayout dispatches to, tensor_core_tiled_layout.py:104) on
    the identical weights (repacked by aten._convert_weight_to_int4pack from the same nibbles,
    scales/zeros in its [K/g, N, 2] layout), the 129 calls captured in one HIP graph like ours.
    Returns its GB/s over the same algorithmic bytes and its max relative difference from our
    outputs on the step's linears."""
    packs = []
    for (_, n_loc, K, packed, sz, y_loc, _y, _k) in plan:
        q = torch.ops.torchao.int4_unpack(packed)
        u8 = ((q[:, ::2] << 4) | q[:, 1::2]).to(torch.uint8)
        del q
        packs.append((torch.ops.aten._convert_weight_to_int4pack(u8, 8),
                      sz.transpose(0, 1).contiguous(), K, y_loc))
        del u8
    outs = [None] * len(packs)

    def step():
        for i, (wp, szt, K, _) in enumerate(packs):
            outs[i] = torch.ops.aten._weight_int4pack_mm(xs[K], wp, g, szt)

    stream = torch.cuda.Stream(device)
    stream.wait_stream(torch.cuda.current_stream(device))
    with torch.cuda.stream(stream):
        step()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=stream):
            step()
        for _ in range(3):
            graph.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(steps):
            graph.replay()
        e1.record(stream)
    e1.synchronize()
    ms = e0.elapsed_time(e1) / steps
    diff = max(float((o.float().reshape(-1) - y.float()).norm() / y.float().norm().clamp_min(1e-30))
               for o, (_, _, _, y) in zip(outs, packs))
    del packs, outs, graph
    torch.cuda.empty_cache()
    return ms, diff


def hbm_ceilings(device, nbytes=1 << 30, reps=10):
    """what the chip streams, measured on the box beside the 8 TB/s spec peak, by
    the microarch guide's method (MI355X_MICROARCH.md "HBM": one long launch over a buffer far
    past the 256 MiB Infinity Cache, 16-B accesses). Three numbers, GB/s, HIP events:
      copy_GBps   tao_hbm_copy_probe over 1 GiB (read + write bytes; the guide's float4 copy row),
                  best of a small sweep (grid x cache policy, and a one-pass form);
      read_GBps   tao_hbm_read_probe over 1 GiB in one launch (the GEMV's own load form: 16-B
                  non-temporal loads, 512-thread workgroups);
      torch_copy_GBps  torch's device copy_ of 1 GiB (what rounds 2-4 reported).
    The per-launch floor of the decode step (pure_read_ms_per_step) is the other ceiling: the
    same bytes as one read launch per linear."""
    from torchao import _lib

    lib = _lib.lib()
    a = torch.empty(nbytes // 4, dtype=torch.int32, device=device).fill_(1)
    b = torch.empty_like(a)
    sink = torch.zeros(1024, dtype=torch.int32, device=device)
    sp = torch.cuda.current_stream(device).cuda_stream

    def timed(fn):
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) * 1e-3 / reps

    def copy(grid, mode):
        rc = lib.tao_hbm_copy_probe(a.data_ptr(), b.data_ptr(), nbytes, grid, mode, sp)
        if rc:
            raise RuntimeError(lib.tao_last_error().decode())

    def read():
        rc = lib.tao_hbm_read_probe(a.data_ptr(), nbytes, sink.data_ptr(), sp)
        if rc:
            raise RuntimeError(lib.tao_last_error().decode())

    copies = {(gr, mode): 2 * nbytes / timed(lambda: copy(gr, mode)) / 1e9
              for mode in (0, 1) for gr in (1024, 2048, 4096, 8192)}
    copies[(0, 2)] = 2 * nbytes / timed(lambda: copy(0, 2)) / 1e9
    best = max(copies, key=copies.get)
    out = {"copy_GBps": round(copies[best], 1),
           "copy_best": {"grid": best[0], "mode": ["default policy", "nt", "nt one pass"][best[1]]},
           "copy_sweep_GBps": {f"{['def', 'nt', 'nt1'][m]}_{gr}": round(v, 1)
                               for (gr, m), v in copies.items()},
           "read_GBps": round(nbytes / timed(read) / 1e9, 1),
           "torch_copy_GBps": round(2 * nbytes / timed(lambda: b.copy_(a)) / 1e9, 1),
           "bytes": nbytes}
    del a, b, sink
    torch.cuda.empty_cache()
    return out


def config2_shapes(device, g=32, copies=32, reps=20):
    """BASELINE config 2's named shapes (int4 g32 WO linear, M = 1: 4096x4096, 11008x4096 and
    4096x11008, the 7B-class FFN width): us per launch inside a HIP graph of `copies` launches
    over distinct weights (rotated past the 256 MiB MALL), HIP events on the replay stream."""
    from torchao import _lib

    lib = _lib.lib()
    out = {}
    for (N, K) in ((4096, 4096), (11008, 4096), (4096, 11008)):
        ws = [make_int4_weight(N, K, g, seed=7 * i + N, device=device) for i in range(copies)]
        x = torch.randn(1, K, device=device, dtype=torch.bfloat16)
        y = torch.empty(N, device=device, dtype=torch.bfloat16)
        stream = torch.cuda.Stream(device)

        def run():
            sp = torch.cuda.current_stream(device).cuda_stream
            for packed, sz in ws:
                rc = lib.tao_int4wo_linear_bf16(x.data_ptr(), packed.data_ptr(), sz.data_ptr(),
                                                None, y.data_ptr(), 1, N, K, g, sp)
                if rc:
                    raise RuntimeError(lib.tao_last_error().decode())

        stream.wait_stream(torch.cuda.current_stream(device))
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.stream(stream):
            run()
            with torch.cuda.graph(graph, stream=stream):
                run()
            graph.replay()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(reps):
                graph.replay()
            e1.record(stream)
        e1.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / reps / copies
        b = int4_alg_bytes(N, K, g)
        out[f"{N}x{K}"] = {"us": round(us, 3), "GBps": round(b / (us * 1e-6) / 1e9, 1),
                           "frac": round(b / (us * 1e-6) / 1e9 / HBM_PEAK_GBPS, 4)}
        del graph, ws
    return out


INT8WO_SHAPES = ((4096, 4096), (6144, 4096), (14336, 4096), (4096, 14336))
PMC_INT8WO_FILE = os.path.join(ROOT, "profiles", "r6u_pmc_fetch_int8wo.json")


def int8wo_alg_bytes(N, K, M=1):
    """SURVEY §8(d) for int8 weight-only: N*K + 2N (bf16 scales) + 2MK + 2MN."""
    return N * K + 2 * N + 2 * M * K + 2 * M * N


def int8wo_m1(device, copies_bytes=512 << 20, reps=20, pmc_file=PMC_INT8WO_FILE):
    """The int8 weight-only linear at M = 1 (the int8 GEMV, Int8WeightOnlyConfig's decode path,
    plain_layout.py:250-266) on the Llama-3-8B shapes: us per launch inside a HIP graph over
    distinct weight copies (> 256 MiB MALL), HIP events on the replay stream; GB/s and fraction
    of 8 TB/s over the algorithmic bytes; a pure 16-B read of the same bytes replayed the same way
    beside it (tao_hbm_read_probe); FETCH_SIZE x2 per launch from the committed counter pass of
    this block (--only-int8wo under rocprofv3 --pmc) when present."""
    from torchao import _lib

    lib = _lib.lib()
    pmc = None
    if pmc_file and os.path.exists(pmc_file):
        with open(pmc_file) as f:
            pmc = json.load(f)
    out = {}
    gen = torch.Generator(device=device).manual_seed(11)
    sink = torch.zeros(1024, dtype=torch.int32, device=device)
    for (N, K) in INT8WO_SHAPES:
        b = int8wo_alg_bytes(N, K)
        copies = max(4, min(32, copies_bytes // b))
        ws = [torch.randint(-127, 128, (N, K), dtype=torch.int8, device=device, generator=gen)
              for _ in range(copies)]
        sc = [(torch.rand(N, device=device, generator=gen) * 0.01 + 1e-3).to(torch.bfloat16)
              for _ in range(copies)]
        x = torch.randn(1, K, device=device, dtype=torch.bfloat16, generator=gen)
        y = torch.empty(1, N, device=device, dtype=torch.bfloat16)
        rbufs = [torch.full(((b + 8191) // 8192 * 8192,), 7, dtype=torch.uint8, device=device)
                 for _ in range(copies)]

        def gemv(c):
            sp = torch.cuda.current_stream(device).cuda_stream
            rc = lib.tao_int8wo_linear_bf16(x.data_ptr(), ws[c].data_ptr(), sc[c].data_ptr(), None,
                                            y.data_ptr(), 1, N, K, sp)
            if rc:
                raise RuntimeError(lib.tao_last_error().decode())

        def read(c):
            sp = torch.cuda.current_stream(device).cuda_stream
            rc = lib.tao_hbm_read_probe(rbufs[c].data_ptr(), rbufs[c].numel(), sink.data_ptr(), sp)
            if rc:
                raise RuntimeError(lib.tao_last_error().decode())

        us = graph_us_per_call(gemv, copies, device, reps=reps)
        kern = lib.tao_last_kernel().decode()
        rus = graph_us_per_call(read, copies, device, reps=reps)
        key = f"{N}x{K}"
        rec = {"us": round(us, 3), "GBps": round(b / (us * 1e-6) / 1e9, 1),
               "frac": round(b / (us * 1e-6) / 1e9 / HBM_PEAK_GBPS, 4), "alg_bytes": b,
               "pure_read_us": round(rus, 3), "gemv_over_pure_read": round(us / rus, 3),
               "kernel": kern, "copies": copies}
        if pmc and key in pmc.get("hbm_bytes_per_launch", {}):
            rec["traffic"] = pmc["hbm_bytes_per_launch"][key]
            rec["traffic_over_alg"] = round(rec["traffic"] / b, 3)
        out[key] = rec
        del ws, sc, rbufs
        torch.cuda.empty_cache()
    out["traffic_source"] = os.path.relpath(pmc_file, ROOT) if pmc else None
    return out


def graph_us_per_call(fn, copies, device, reps=3):
    """us per call of fn(c), c over `copies` weight copies, captured once in a HIP graph and
    replayed: events on the replay stream (launch gaps inside the graph included)."""
    s = torch.cuda.Stream(device)
    s.wait_stream(torch.cuda.current_stream(device))
    with torch.cuda.stream(s):
        for c in range(copies):
            fn(c)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=s):
            for c in range(copies):
                fn(c)
        graph.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(reps):
            graph.replay()
        e1.record(s)
    e1.synchronize()
    torch.cuda.current_stream(device).wait_stream(s)
    del graph
    return e0.elapsed_time(e1) * 1e3 / reps / copies


def prefill_mfma(device, M=128, N=4096, K=4096, g=32, reps=40):
    """BASELINE config 3 (int8 dynamic-activation int8-weight linear, M = 128, the MFMA int8
    path) and the int4 g32 linear at the same M on its bf16-MFMA path, timed per kernel by the
    dispatch packets' own events (tao_profile_*, as rocprofv3 reports them), weights rotated
    over copies past the 256 MiB Infinity Cache. Roofline: max(ops / MFMA peak, bytes / HBM
    peak) is the attainable time; `frac` = attainable / measured.

    Beside each, the REFERENCE's own GPU path on the same inputs, both sides captured in one HIP
    graph over the same weight copies (graph_us, launch gaps included for both): config 3 as
    safe_int_mm -> torch._int_mm (hipBLASLt int8) plus the int_scaled_matmul epilogue and the
    weight scale (kernel/intmm.py:82,136-142; plain_layout.py:301-315; the per-token quant is
    ours on both sides), int4 as aten._weight_int4pack_mm on the same nibbles repacked by
    aten._convert_weight_to_int4pack (tensor_core_tiled_layout.py:104)."""
    from torchao import _lib

    def timed(fn, copies, launches):
        for c in range(copies):
            fn(c)
        torch.cuda.synchronize()
        with _lib.KernelTimer(reps * launches) as kt:
            for i in range(reps):
                fn(i % copies)
        torch.cuda.synchronize()
        d = kt.durations_ms
        if len(d) != reps * launches:
            raise RuntimeError(f"prefill_mfma: expected {reps * launches} kernels, got {len(d)}")
        return [sorted(d[j::launches])[len(d[j::launches]) // 2] * 1e3 for j in range(launches)]

    def rel(a, b):
        a, b = a.float(), b.float()
        return round(float((a - b).norm() / b.norm().clamp_min(1e-30)), 5)

    def intake(path, xx, wl, zl, copies):
        """the LDS-DMA intake floor of the single-fetch tile family at this shape
        (tao_sf_intake_probe: the launch shape's per-workgroup bytes through its LDS ring, no
        compute), kernel us over the same rotated weight copies"""
        import ctypes
        shp = (ctypes.c_int * 7)()
        sink = torch.zeros(1024, dtype=torch.int32, device=device)
        h = _lib.lib()

        def probe(c):
            rc = h.tao_sf_intake_probe(path, 0, xx.data_ptr(), wl[c].data_ptr(),
                                       zl[c].data_ptr() if zl else None, M, N, K, g,
                                       ctypes.cast(shp, ctypes.c_void_p), sink.data_ptr(),
                                       torch.cuda.current_stream().cuda_stream)
            if rc != 0:
                raise RuntimeError(h.tao_last_error().decode(errors="replace"))
        try:
            (pus,) = timed(probe, copies, 1)
        except RuntimeError as e:
            return {"unavailable": str(e)[:160]}
        bn, S, ns, a, ld, ks, step_b = list(shp)
        steps = K // ks
        last = steps - a * (S - 1)
        per_wg = step_b * max(a, last)
        return {"us": round(pus, 2), "bn": bn, "k_slices": S, "stages": ns, "loader_waves": ld,
                "k_step": ks, "bytes_per_wg_step": step_b, "bytes_per_wg": per_wg,
                "GBps_per_cu": round(per_wg / (pus * 1e-6) / 1e9, 1)}

    # the floor any launch shows by these events on this box: a one-workgroup 8-KiB read
    # (tao_hbm_read_probe), so each GEMM's roofline can also be read against attainable + floor
    fl_buf = torch.zeros(8192, dtype=torch.uint8, device=device)
    fl_sink = torch.zeros(1024, dtype=torch.int32, device=device)

    def empty_launch(c):
        _lib.call("tao_hbm_read_probe", fl_buf.data_ptr(), 8192, fl_sink.data_ptr(),
                  torch.cuda.current_stream().cuda_stream)

    (floor_us,) = timed(empty_launch, 1, 1)

    out = {}
    # int8 dyn: per-token quant kernel + int8 MFMA GEMM with the fused scale epilogue
    copies = max(2, int(320e6 // (N * K)))
    gen = torch.Generator(device=device).manual_seed(3)
    ws = [torch.randint(-127, 128, (N, K), dtype=torch.int8, device=device, generator=gen)
          for _ in range(copies)]
    wsc = (torch.rand(N, device=device, generator=gen) * 0.01 + 1e-3).to(torch.bfloat16)
    x = torch.randn(M, K, device=device, dtype=torch.bfloat16, generator=gen)

    def int8dyn(c):
        q, s = torch.ops.torchao.int8_quantize_per_token(x)
        torch.ops.torchao.int8_scaled_mm(q, s, ws[c], wsc, None)

    quant_us, gemm_us = timed(int8dyn, copies, 2)
    xq, xs = torch.ops.torchao.int8_quantize_per_token(x)
    torch.ops.torchao.int8_scaled_mm(xq, xs, ws[0], wsc, None)
    kern8 = _lib.lib().tao_last_kernel().decode()
    xs2 = xs.reshape(-1, 1)

    def ours8(c):
        return torch.ops.torchao.int8_scaled_mm(xq, xs, ws[c], wsc, None)

    def ref8(c):  # the reference's GPU ops after the per-token quant
        return ((torch._int_mm(xq, ws[c].t()) * xs2).to(torch.bfloat16)) * wsc

    ref8_us = ours8_graph_us = ref8_diff = None
    try:
        ours8_graph_us = graph_us_per_call(ours8, copies, device)
        ref8_us = graph_us_per_call(ref8, copies, device)
        ref8_diff = rel(ref8(0), ours8(0))
    except Exception as e:  # the hipBLASLt int8 path is build dependent: report, never fail
        ref8_us = f"unavailable: {type(e).__name__}: {str(e)[:120]}"
    ip8 = intake(2, xq, ws, None, copies)
    ops = 2 * M * N * K
    nbytes = N * K + N * 2 + M * K + M * 4 + M * N * 2  # int8 W + scales, int8 x + scales, bf16 y
    att = max(ops / (INT8_PEAK_TOPS * 1e12), nbytes / (HBM_PEAK_GBPS * 1e9)) * 1e6
    out["int8_dyn"] = {
        "config": f"BASELINE config 3: int8 dyn-act int8-weight linear M={M} N={N} K={K}",
        "kernel": f"routed int8 dyn GEMM: {kern8} (v_mfma_i32_16x16x64_i8)",
        "gemm_us": round(gemm_us, 2), "quant_us": round(quant_us, 2),
        "TOPS": round(ops / (gemm_us * 1e-6) / 1e12, 1),
        "mfma_frac": round(ops / (gemm_us * 1e-6) / 1e12 / INT8_PEAK_TOPS, 4),
        "GBps": round(nbytes / (gemm_us * 1e-6) / 1e9, 1),
        "attainable_us": round(att, 2), "roofline_frac": round(att / gemm_us, 4),
        "launch_floor_us": round(floor_us, 2),
        "roofline_frac_with_launch_floor": round((att + floor_us) / gemm_us, 4),
        "graph_us": round(ours8_graph_us, 2) if ours8_graph_us else None,
        "reference_gpu_us": round(ref8_us, 2) if isinstance(ref8_us, float) else ref8_us,
        "reference_gpu_op": "torch._int_mm (hipBLASLt int8, safe_int_mm) * x_scale -> bf16 * w_scale",
        "reference_gpu_rel_l2": ref8_diff,
        # the single-fetch int8 tile family at this shape (config 3 itself stays on the incumbent
        # kernel named above): its LDS-DMA intake alone, no compute
        "intake_probe_sf_int8": ip8,
    }
    del ws
    # int4 g32 weight-only at the same M: bf16 MFMA with in-register nibble dequant
    copies = max(2, int(320e6 // (N * K // 2)))
    w4, wref = [], []
    for c in range(copies):
        q = torch.randint(0, 16, (N, K), dtype=torch.int32, device=device, generator=gen)
        sz = (torch.rand(N, K // g, 2, device=device, generator=gen) * 0.02).to(torch.bfloat16)
        w4.append((torch.ops.torchao.int4_pack(q), sz))
        try:
            u8 = ((q[:, ::2] << 4) | q[:, 1::2]).to(torch.uint8)
            wref.append((torch.ops.aten._convert_weight_to_int4pack(u8, 8),
                         sz.transpose(0, 1).contiguous()))
            del u8
        except Exception:
            wref = None
        del q

    def int4(c):
        return torch.ops.torchao.int4_weight_only_linear(x, w4[c][0], w4[c][1], g, None)

    (us4,) = timed(int4, copies, 1)
    int4(0)
    kern4 = _lib.lib().tao_last_kernel().decode()
    ref4_us = ours4_graph_us = ref4_diff = None
    try:
        ours4_graph_us = graph_us_per_call(int4, copies, device)
        if wref:
            def ref4(c):
                return torch.ops.aten._weight_int4pack_mm(x, wref[c][0], g, wref[c][1])
            ref4_us = graph_us_per_call(ref4, copies, device)
            ref4_diff = rel(ref4(0), int4(0))
    except Exception as e:  # the aten op is build dependent: report, never fail
        ref4_us = f"unavailable: {type(e).__name__}: {str(e)[:120]}"
    ip4 = intake(0, x, [w[0] for w in w4], [w[1] for w in w4], copies)
    if "us" in ip4:
        ip4["gemm_over_intake"] = round(us4 / ip4["us"], 3)
    nbytes4 = int4_alg_bytes(N, K, g, M)
    att4 = max(ops / (BF16_PEAK_TFLOPS * 1e12), nbytes4 / (HBM_PEAK_GBPS * 1e9)) * 1e6
    out["int4_wo"] = {
        "config": f"int4 g{g} weight-only linear M={M} N={N} K={K} (prefill)",
        "kernel": f"routed int4 GEMM: {kern4} (bf16 MFMA)",
        "gemm_us": round(us4, 2),
        "TFLOPS": round(ops / (us4 * 1e-6) / 1e12, 1),
        "mfma_frac": round(ops / (us4 * 1e-6) / 1e12 / BF16_PEAK_TFLOPS, 4),
        "attainable_us": round(att4, 2), "roofline_frac": round(att4 / us4, 4),
        "launch_floor_us": round(floor_us, 2),
        "roofline_frac_with_launch_floor": round((att4 + floor_us) / us4, 4),
        "graph_us": round(ours4_graph_us, 2) if ours4_graph_us else None,
        "reference_gpu_us": round(ref4_us, 2) if isinstance(ref4_us, float) else ref4_us,
        "reference_gpu_op": "aten._weight_int4pack_mm (PyTorch-ROCm)",
        "reference_gpu_rel_l2": ref4_diff,
        # the routed launch shape's LDS-DMA intake alone (same per-workgroup bytes, ring, waits
        # and barriers, no MFMA, no dequantisation, no seam): the floor this tile family reaches
        "intake_probe": ip4,
    }
    del w4, wref
    torch.cuda.empty_cache()
    return out


def e2e_decode(timeout_s=240):
    """BASELINE config 4 beside the linears-only step: the e2e decode harness
    (torchao/_models/llama/generate.py semantics: random-init Llama-3-8B, quantize_ int4wo-32,
    prompt 128, 200 new tokens, bs=1, greedy, HIP-graph decode) in a child process (its own
    model and weights; this process only waits). Its JSON line, trimmed."""
    import subprocess

    # 5 timed samples: generate.py reports the median of each phase (of 2 it took the slower)
    cmd = [sys.executable, "-m", "torchao._models.llama.generate", "-q", "int4wo-32",
           "--num_samples", "5"]
    try:
        out = subprocess.run(cmd, cwd=os.path.join(ROOT, "torchao-fork_amd"), capture_output=True,
                             text=True, timeout=timeout_s, check=True).stdout
        d = json.loads(out.strip().splitlines()[-1])
    except Exception as e:  # reported, never fatal to the bench line
        return {"error": f"{type(e).__name__}: {str(e)[:200]}"}
    keep = ("model", "quantization", "weights", "batch_size", "prompt_length", "max_new_tokens",
            "decode_tokens_per_s", "decode_ms_per_token", "prefill_ms", "tokens_per_s_incl_prefill",
            "graph_eager_token_match", "graph_eager_first_mismatch", "eager_logits_finite")
    rec = {k: d[k] for k in keep if k in d}
    rec["config"] = "BASELINE config 4: Llama-3-8B quantize_(Int4WeightOnlyConfig(32)), greedy bs=1"
    return rec


def host_cpu_info():
    """CPU model, the physical cores this process may run on, and the cgroup CPU quota (the
    GPU box's share of a large host), read from /proc/cpuinfo and /sys/fs/cgroup."""
    allowed = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else []
    model, cores, cur = None, set(), {}
    try:
        with open("/proc/cpuinfo") as f:
            for line in f.read().splitlines() + [""]:
                if not line.strip():
                    if cur.get("processor") is not None and (not allowed or int(cur["processor"]) in allowed):
                        cores.add((cur.get("physical id", "0"), cur.get("core id", cur["processor"])))
                    cur = {}
                    continue
                k, _, v = line.partition(":")
                cur[k.strip()] = v.strip()
                if k.strip() == "model name" and model is None:
                    model = v.strip()
    except OSError:
        pass
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        try:
            with open(path) as f:
                parts = f.read().split()
            if path.endswith("cpu.max") and parts and parts[0] != "max":
                quota = float(parts[0]) / float(parts[1])
            elif path.endswith("quota_us") and parts and int(parts[0]) > 0:
                with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f2:
                    quota = int(parts[0]) / int(f2.read().split()[0])
            break
        except (OSError, ValueError, IndexError):
            continue
    physical = len(cores) or len(allowed) or (os.cpu_count() or 1)
    return {"cpu_model": model, "physical_cores": physical, "logical_cpus": len(allowed) or None,
            "cgroup_cpu_quota": quota}


def cpu_baseline(cfg, g, budget_s=12.0):
    """The reference CPU dequant path (oracle restatement) on one layer's five linears, M = 1,
    plus BASELINE config 1 (one 4096x4096 linear), on every physical core this process may use
    (capped by the cgroup CPU quota: a thread per core the scheduler actually grants)."""
    from oracle import oracle

    info = host_cpu_info()
    cores = info["physical_cores"]
    if info["cgroup_cpu_quota"]:
        cores = max(1, min(cores, int(info["cgroup_cpu_quota"])))
    torch.set_num_threads(cores)
    layer = [lin for lin in llama_linears(cfg) if lin[0].startswith("layers.0.")]
    mats = []
    for i, (_, N, K) in enumerate(layer):
        w = oracle.make_linear_weight(N, K, seed=i)
        s, z = oracle.int4_qparams(w, g)
        q = oracle.int4_quantize(w, s, z, g)
        x = oracle.make_activation(1, K, seed=100 + i)
        mats.append((x, q, s, z, N, K))
    sample_bytes = sum(int4_alg_bytes(N, K, g) for (_, _, _, _, N, K) in mats)
    for (x, q, s, z, _, _) in mats:  # warm up
        oracle.int4_linear(x, q, s, z, g)
    reps, t0 = 0, time.perf_counter()
    while True:
        for (x, q, s, z, _, _) in mats:
            oracle.int4_linear(x, q, s, z, g)
        reps += 1
        if time.perf_counter() - t0 > budget_s or reps >= 200:
            break
    dt = time.perf_counter() - t0
    # PyTorch's own CPU int4 GEMM (what the reference's Int4CPULayout dispatches to), same sample
    # rotated over distinct copies of the packed weights (> 512 MB in all, past the host's L3:
    # a same-weights loop would time a cache-resident working set)
    tg, tg_footprint = None, None
    try:
        packs = [oracle.int4_tinygemm_cpu_pack(q, s, z) + (x,) for (x, q, s, z, _, _) in mats]
        ncopy = max(1, -(-(600 << 20) // sample_bytes))
        rot = [(p.clone(), sz.clone(), x) for _ in range(ncopy) for (p, sz, x) in packs]
        tg_footprint = sum(p.numel() * p.element_size() + sz.numel() * sz.element_size()
                           for (p, sz, _) in rot)
        for p, sz, x in rot:
            oracle.int4_tinygemm_cpu(x, p, sz, g)
        r2, t1 = 0, time.perf_counter()
        while time.perf_counter() - t1 < 3.0:
            for p, sz, x in rot:
                oracle.int4_tinygemm_cpu(x, p, sz, g)
            r2 += 1
        tg = sample_bytes * ncopy * r2 / (time.perf_counter() - t1) / 1e9
        del rot, packs
    except Exception as e:  # pragma: no cover - depends on the host's torch build
        tg = f"unavailable: {type(e).__name__}"
    # BASELINE config 1: a single nn.Linear 4096x4096, int4 g32, the same CPU dequant path
    w1 = oracle.make_linear_weight(4096, 4096, seed=41)
    s1, z1 = oracle.int4_qparams(w1, g)
    q1 = oracle.int4_quantize(w1, s1, z1, g)
    x1 = oracle.make_activation(1, 4096, seed=42)
    oracle.int4_linear(x1, q1, s1, z1, g)
    times = []
    t2 = time.perf_counter()
    while len(times) < 50 and time.perf_counter() - t2 < 3.0:
        t3 = time.perf_counter()
        oracle.int4_linear(x1, q1, s1, z1, g)
        times.append(time.perf_counter() - t3)
    c1 = sorted(times)[len(times) // 2]
    return {
        "value": round(sample_bytes * reps / dt / 1e9, 3),
        "unit": "GB/s",
        "cores": cores,
        "cpu_model": info["cpu_model"],
        "physical_cores": info["physical_cores"],
        "cgroup_cpu_quota": info["cgroup_cpu_quota"],
        "config1_4096x4096": {"ms_median": round(c1 * 1e3, 3),
                              "GBps": round(int4_alg_bytes(4096, 4096, g) / c1 / 1e9, 3),
                              "runs": len(times)},
        "kind": "port",
        "sample": (f"reference CPU dequant path (dequantize -> F.linear bf16, oracle/oracle.py) on "
                   f"layer 0's 5 int4 g{g} linears at M=1, {reps} reps in {dt:.1f}s"),
        "ms_per_token_extrapolated": round(dt / reps * 1e3 * cfg["n_layer"], 1),
        "aten_weight_int4pack_mm_for_cpu_GBps": round(tg, 3) if isinstance(tg, float) else tg,
        "aten_weight_int4pack_mm_for_cpu_footprint_bytes": tg_footprint,
        "aten_weight_int4pack_mm_for_cpu_note": (
            f"PyTorch's CPU int4 GEMM (Int4CPULayout's kernel) on {cores} threads over distinct "
            "copies of layer 0's packed weights rotated per pass (footprint above, beyond L3)"),
    }


def pair_map(lins):
    """Megatron pairs of a Llama block (colwise -> rowwise): wqkv -> wo, w1||w3 (or w1, w3) -> w2.
    {index: ("col", partner) | ("row", first colwise partner)}."""
    pair_of = {}
    for i, (name, N, K) in enumerate(lins):
        if name.endswith("attention.wo"):
            pair_of[i - 1], pair_of[i] = ("col", i), ("row", i - 1)
        elif name.endswith("feed_forward.w2"):
            j = i - 1
            while j >= 0 and lins[j][0].rsplit(".", 1)[0] == name.rsplit(".", 1)[0]:
                pair_of[j] = ("col", i)
                j -= 1
            pair_of[i] = ("row", j + 1)
    return pair_of


def shard_kinds(lins, P, g, policy, calib, shard_min_elems=64 << 20):
    """Per linear: whole (replicated), gather (colwise + all-gather), local (colwise, output
    consumed by its rowwise partner), reduce (rowwise on K/P + all-reduce)."""
    pair_of = pair_map(lins)

    def pair_sharded(i):
        kind, j = pair_of[i]
        a, b = (i, j) if kind == "col" else (j, i)
        (_, Na, Ka), (_, Nb, Kb) = lins[a], lins[b]
        if Na % P or Kb % (P * g):
            return False
        if policy == "tp":
            return True
        return bool(calib.get(("pair", Na, Ka, Nb, Kb), {}).get("shard"))

    kinds = []
    for i, (name, N, K) in enumerate(lins):
        kind = "whole"
        if P > 1 and policy != "none":
            if i in pair_of and policy in ("tp", "auto") and pair_sharded(i):
                kind = "local" if pair_of[i][0] == "col" else "reduce"
            elif policy == "auto" and i not in pair_of and N % P == 0:
                kind = "gather" if calib[(N, K)]["shard"] else "whole"
            elif policy in ("all", "size") and N % P == 0:
                kind = "gather" if policy == "all" or N * K >= shard_min_elems else "whole"
            elif policy == "tp" and i not in pair_of and N % P == 0:
                kind = "gather"
        kinds.append(kind)
    return kinds


class LinearStep:
    """Every int4 linear of one decoded token (M = 1), sharded per `kinds`, with its packed
    weights, inputs and outputs resident in HBM; `step()` issues the GEMVs on the current stream
    and the collectives their kinds need (RCCL; host-staged gloo in a rehearsal)."""

    def __init__(self, lins, kinds, P, rank, g, device, rehearsal):
        from torchao import _lib

        self.lib = _lib.lib()
        self.P, self.g, self.device, self.rehearsal = P, g, device, rehearsal
        self.plan, self.xs, self.bytes_per_step = [], {}, 0
        for i, ((name, N, K), kind) in enumerate(zip(lins, kinds)):
            n_loc = N // P if kind in ("gather", "local") else N
            k_loc = K // P if kind == "reduce" else K
            packed, sz = make_int4_weight(n_loc, k_loc, g,
                                          seed=1000 * i + (rank if kind != "whole" else 0),
                                          device=device)
            if k_loc not in self.xs:
                self.xs[k_loc] = torch.randn(1, k_loc, device=device, dtype=torch.bfloat16)
            y_loc = torch.empty(n_loc, device=device, dtype=torch.bfloat16)  # M = 1 row
            y_full = (torch.empty(N, device=device, dtype=torch.bfloat16) if kind == "gather"
                      else y_loc)
            self.plan.append((name, n_loc, k_loc, packed, sz, y_loc, y_full, kind))
            self.bytes_per_step += int4_alg_bytes(N, K, g)
        self.weight_bytes_per_rank = sum(e[3].numel() * 4 + e[4].numel() * 2 for e in self.plan)
        self.stream = torch.cuda.Stream(device)
        torch.cuda.synchronize()

    def counts(self):
        return {k: sum(e[7] == k for e in self.plan) for k in ("local", "reduce", "gather", "whole")}

    def step(self, do_gemv=True, do_comm=True, only=None):
        sp = torch.cuda.current_stream(self.device).cuda_stream
        g, xs = self.g, self.xs
        for (_, n_loc, K, packed, sz, y_loc, y_full, kind) in self.plan:
            if only is not None and (n_loc, K) != only:
                continue
            if do_gemv:
                rc = self.lib.tao_int4wo_linear_bf16(xs[K].data_ptr(), packed.data_ptr(),
                                                     sz.data_ptr(), None, y_loc.data_ptr(), 1,
                                                     n_loc, K, g, sp)
                if rc:
                    raise RuntimeError(self.lib.tao_last_error().decode())
            if not do_comm or kind in ("whole", "local"):
                continue
            if kind == "gather":
                if self.rehearsal:
                    parts = [torch.empty_like(y_loc, device="cpu") for _ in range(self.P)]
                    dist.all_gather(parts, y_loc.cpu())
                    y_full.copy_(torch.cat(parts))
                else:
                    dist.all_gather_into_tensor(y_full, y_loc)
            elif self.rehearsal:  # reduce
                t = y_loc.cpu()
                dist.all_reduce(t)
                y_loc.copy_(t)
            else:
                dist.all_reduce(y_loc)

    def capture(self, **kw):
        graph = torch.cuda.CUDAGraph()
        self.stream.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(self.stream):
            self.step(**kw)  # warm-up outside capture (RCCL communicators, allocator)
            with torch.cuda.graph(graph, stream=self.stream):
                self.step(**kw)
        torch.cuda.current_stream(self.device).wait_stream(self.stream)
        torch.cuda.synchronize()
        return graph

    def try_capture(self, **kw):
        if self.rehearsal:
            return None
        try:
            return self.capture(**kw)
        except Exception as e:  # graph capture of collectives is runtime dependent
            print(f"[bench] graph capture failed ({e}); timing eager launches", file=sys.stderr)
            torch.cuda.synchronize()
            return None

    def replay_ms(self, graph, reps):
        """GPU time per replay of `graph` back to back (HIP events on the replay stream)."""
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(self.stream):
            graph.replay()
            ev0.record(self.stream)
            for _ in range(reps):
                graph.replay()
            ev1.record(self.stream)
        ev1.synchronize()
        return ev0.elapsed_time(ev1) / reps

    def wall_ms(self, run, steps, warmup):
        """Driver contract: barrier + synchronize on both sides of exactly `steps` runs, max over
        ranks. Returns ms per step."""
        P = self.P

        def barrier():
            if P > 1:
                dist.barrier()
            torch.cuda.synchronize()

        for _ in range(warmup):
            run()
        barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            run()
        barrier()
        elapsed = time.perf_counter() - t0
        if P > 1:
            t = torch.tensor([elapsed], dtype=torch.float64,
                             device="cpu" if self.rehearsal else self.device)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
        return elapsed / steps * 1e3

    def read_probe_graph(self, only=None):
        """The step's launches replayed as PURE 16-B streaming reads of the same algorithmic byte
        counts (tao_hbm_read_probe: one load per thread, 512-thread workgroups, each launch its own
        buffer past the MALL): the floor any one-kernel-per-linear step reaches on this chip,
        measured in the same run as the GEMV step. `only` = (n_loc, K) as step()."""
        if not hasattr(self, "_rbufs"):
            self._rbufs = [torch.empty((int4_alg_bytes(e[1], e[2], self.g) + 8191) // 8192 * 8192,
                                       dtype=torch.uint8, device=self.device) for e in self.plan]
            for b in self._rbufs:
                b.fill_(7)
            self._rsink = torch.zeros(1024, dtype=torch.int32, device=self.device)

        def run():
            sp = torch.cuda.current_stream(self.device).cuda_stream
            for e, b in zip(self.plan, self._rbufs):
                if only is not None and (e[1], e[2]) != only:
                    continue
                rc = self.lib.tao_hbm_read_probe(b.data_ptr(), b.numel(), self._rsink.data_ptr(), sp)
                if rc:
                    raise RuntimeError(self.lib.tao_last_error().decode())
        graph = torch.cuda.CUDAGraph()
        self.stream.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(self.stream):
            run()
            with torch.cuda.graph(graph, stream=self.stream):
                run()
        torch.cuda.current_stream(self.device).wait_stream(self.stream)
        torch.cuda.synchronize()
        return graph

    def release(self):
        self.plan, self.xs = [], {}
        if hasattr(self, "_rbufs"):
            del self._rbufs, self._rsink
        torch.cuda.synchronize()
        torch.cuda.empty_cache()


def parallelism_desc(step, policy):
    c = step.counts()
    return (f"tp{step.P} (shard policy {policy}): "
            + ", ".join(f"{c[k]} {k}" for k in ("local", "reduce", "gather", "whole"))
            + f" of {len(step.plan)} linears (local = colwise feeding its rowwise partner, "
            "reduce = rowwise + RCCL all-reduce, gather = colwise + RCCL all-gather, whole = "
            "replicated)")


def config5_record(P, rank, g, device, rehearsal, steps, warmup, policy="tp"):
    """BASELINE config 5: the 80-layer Llama-3-70B linear step (321 launches, 43.4 GB of int4
    weights per token). At P = 1 every linear runs whole on the one GPU (43 GB fit in 288 GB of
    HBM): the curve's 1-GPU anchor. At P > 1 one of two plans:
      * policy "tp" (Megatron pairs; test_affine_quantized_tensor_parallel.py:49-80):
        wqkv colwise -> wo rowwise + all-reduce, w1||w3 colwise -> w2 rowwise + all-reduce,
        output head colwise + all-gather;
      * policy "all" (the north star's plan): every linear column-sharded, its output
        all-gathered over RCCL.
    ~1/P of the weights per rank either way, the collectives captured in the step's graph. Times
    the whole step (driver contract: barrier, max over ranks), the GEMV-only graph and the
    collectives-only graph separately."""
    _, cfg = MODELS["70b"]
    lins = llama_linears(cfg)
    kinds = shard_kinds(lins, P, g, policy, {}) if P > 1 else ["whole"] * len(lins)
    st = LinearStep(lins, kinds, P, rank, g, device, rehearsal)
    t_build = time.perf_counter()
    graph = st.try_capture()
    ms = st.wall_ms(graph.replay if graph is not None else st.step, steps, warmup)
    gemv_ms = comm_ms = None
    if P > 1:
        ggemv = st.try_capture(do_comm=False)
        gemv_ms = st.replay_ms(ggemv, max(steps, 5)) if ggemv is not None else None
        gcomm = st.try_capture(do_gemv=False)
        comm_ms = st.wall_ms(gcomm.replay if gcomm is not None
                             else (lambda: st.step(do_gemv=False)), steps, 2)
        del ggemv, gcomm
    elif graph is not None:
        gemv_ms = st.replay_ms(graph, max(steps, 5))
    plan = ("single GPU: every linear whole" if P == 1 else
            "Megatron pairs + head all-gather" if policy == "tp" else
            "north star: every linear column-sharded + RCCL all-gather of its output")
    rec = {
        "workload": f"Llama-3-70B int4 g{g} weight-only linears, M=1 decode: "
                    + workload_desc(cfg) + f" ({len(st.plan)} GEMV launches/step)",
        "plan": plan,
        "value": round(st.bytes_per_step / (ms * 1e-3) / 1e9, 2),
        "unit": "GB/s",
        "linear_steps_per_s": round(1e3 / ms, 2),
        "ms_per_step": round(ms, 4),
        "gemv_ms_per_step": round(gemv_ms, 4) if gemv_ms is not None else None,
        "collectives_ms_per_step": round(comm_ms, 4) if comm_ms is not None else 0.0,
        "bytes_per_step": st.bytes_per_step,
        "weight_bytes_per_rank": st.weight_bytes_per_rank,
        "parallelism": parallelism_desc(st, policy) if P > 1 else "single-gpu",
        "n_gpus": P,
        "hip_graph": graph is not None,
        "collectives": ("none" if P == 1 else "RCCL in the step graph" if graph is not None else
                        ("host-staged gloo (rehearsal)" if rehearsal else "RCCL, eager")),
        "scaling": "strong",
    }
    del graph
    st.release()
    rec["setup_s"] = round(time.perf_counter() - t_build, 1)
    return rec


def unfused_record(cfg, g, device, steps):
    """The reference's module layout at P = 1: w1 and w3 as two linears (161 launches, the same
    bytes as the merged step; what a model quantized unchanged runs,
    /root/reference/torchao/_models/llama/model.py:481-486), one HIP graph, replay GPU time and
    wall time per step, its roofline fraction, and per shape the GEMV over a pure read of the
    same bytes (as the headline's per_shape_graph)."""
    lins = llama_linears(cfg, fuse_w13=False)
    st = LinearStep(lins, ["whole"] * len(lins), 1, 0, g, device, False)
    graph = st.capture()
    ms = st.wall_ms(graph.replay, steps, 3)
    reps = max(steps, 10)
    gpu_ms = st.replay_ms(graph, reps)
    gr = st.read_probe_graph()
    pure_ms = st.replay_ms(gr, reps)
    del gr
    per_shape = {}
    for (n_loc, K) in sorted({(e[1], e[2]) for e in st.plan}):
        cnt = sum(1 for e in st.plan if (e[1], e[2]) == (n_loc, K))
        gs_ = st.capture(do_comm=False, only=(n_loc, K))
        us = st.replay_ms(gs_, reps) * 1e3 / cnt
        gr_ = st.read_probe_graph(only=(n_loc, K))
        rus = st.replay_ms(gr_, reps) * 1e3 / cnt
        b = int4_alg_bytes(n_loc, K, g)
        per_shape[f"{n_loc}x{K}"] = {
            "launches": cnt, "us": round(us, 3), "frac": round(b / (us * 1e-6) / 1e9 / HBM_PEAK_GBPS, 4),
            "pure_read_us": round(rus, 3), "gemv_over_pure_read": round(us / rus, 3)}
        del gs_, gr_
    achieved = st.bytes_per_step / (gpu_ms * 1e-3) / 1e9
    rec = {"workload": workload_desc(cfg, False) + f" ({len(st.plan)} GEMV launches/step)",
           "value": round(st.bytes_per_step / (ms * 1e-3) / 1e9, 2), "unit": "GB/s",
           "ms_per_step": round(ms, 4), "kernel_ms_per_step": round(gpu_ms, 4),
           "achieved": round(achieved, 1), "frac": round(achieved / HBM_PEAK_GBPS, 4),
           "pure_read_ms_per_step": round(pure_ms, 4),
           "gemv_over_pure_read": round(gpu_ms / pure_ms, 3),
           "per_shape_graph": per_shape,
           "launches": len(st.plan)}
    del graph
    st.release()
    return rec


def n_launches_expected(args):
    return 161 if args.no_fuse_w13 else 129


def free_port():
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv, script=None, timeout_s=None):
    """`bench.py --gpus N` without torchrun: run `torch.distributed.run --nproc-per-node N
    bench.py ...` as a CHILD process (one rank per GPU, rendezvous on 127.0.0.1) and return its
    exit code. The caller has not initialised the GPU (nothing before this touches HIP) and does
    not exec: the child's stdout (rank 0's JSON line) and stderr stream through unchanged."""
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}",
           script or os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    env.setdefault("OMP_NUM_THREADS", "1")
    proc = subprocess.run(cmd, env=env, timeout=timeout_s)
    return proc.returncode


def rank_census(P, device, rehearsal):
    """Proof of the ranks the line was measured on: the process group's size and, all-gathered
    from every rank, the PCI location of the GPU it drove. Under RCCL the N ranks must sit on N
    distinct devices (asserted); a gloo rehearsal puts every rank on device 0 (recorded as is)."""
    props = torch.cuda.get_device_properties(device)
    mine = f"{props.pci_domain_id:04x}:{props.pci_bus_id:02x}:{props.pci_device_id:02x}"
    seen = dist.get_world_size() if P > 1 else 1
    ids = [mine]
    if P > 1:
        ids = [None] * P
        dist.all_gather_object(ids, mine)
    distinct = sorted(set(ids))
    if P > 1 and not rehearsal and len(distinct) != P:
        raise SystemExit(f"rank census: {P} RCCL ranks on {len(distinct)} distinct GPUs: {ids}")
    return {"ranks_seen": seen, "pci_bus_ids": ids, "distinct_gpus": len(distinct),
            "backend": "single" if P == 1 else ("gloo (rehearsal, shared device)" if rehearsal
                                                 else "nccl (RCCL)")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--group-size", type=int, default=32)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-reference-gpu", action="store_true",
                    help="skip timing PyTorch-ROCm's aten._weight_int4pack_mm on the same step")
    ap.add_argument("--no-prefill", action="store_true",
                    help="skip the config-3 MFMA prefill measurement (prefill_mfma)")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip config2_shapes and the copy-bandwidth probe (profiler passes that "
                         "attribute every launch to the step use this)")
    ap.add_argument("--no-e2e", action="store_true",
                    help="skip the config-4 e2e decode run (e2e_decode, a child process)")
    ap.add_argument("--shard-policy", default="auto",
                    choices=["auto", "tp", "size", "all", "none"],
                    help="P > 1: how to shard. tp = Megatron pairs (wqkv colwise -> wo rowwise + "
                         "all-reduce, w1||w3 colwise -> w2 rowwise + all-reduce) and the output "
                         "head colwise + all-gather; all / size = every (large) linear colwise + "
                         "all-gather; auto = per pair / per head, whichever of {replicated, "
                         "sharded} measured faster at startup (max over ranks)")
    ap.add_argument("--shard-min-elems", type=int, default=64 << 20,
                    help="--shard-policy size: shard when N*K >= this")
    ap.add_argument("--shard-all", action="store_true", help="= --shard-policy all")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo = rehearsal of the P > 1 path on one GPU (all ranks on device 0)")
    ap.add_argument("--model", default="8b", choices=sorted(MODELS),
                    help="8b = the headline workload (BASELINE config 2); 70b = config 5's "
                         "shapes (43 GB of int4 weights per step)")
    ap.add_argument("--no-config5", action="store_true",
                    help="P > 1: skip the Llama-3-70B (BASELINE config 5) sub-record")
    ap.add_argument("--pmc-file", default=PMC_FILE,
                    help="FETCH_SIZE summary (experiments/pmc_summary.py) for roofline.traffic")
    ap.add_argument("--pmc-int8wo-file", default=PMC_INT8WO_FILE,
                    help="FETCH_SIZE summary (experiments/int8wo_pmc.py) for int8wo_m1")
    ap.add_argument("--no-fuse-w13", action="store_true",
                    help="w1 and w3 as two linears (the reference's module layout, 161 launches)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no outer launcher: start one rank per GPU ourselves (a child process; this process has
        # not touched the GPU and never will) and pass rank 0's line through
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # rehearsal of the P > 1 logic on a one-GPU box: every rank on device 0, gloo collectives
    # through host memory (no graph); the real runs use one GPU per rank and RCCL
    rehearsal = args.backend == "gloo"
    if rehearsal:
        local = 0
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if rehearsal:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=device)

    import torchao  # noqa: F401
    from torchao import _lib

    _lib.lib()  # fail loudly if the native library is missing
    census = rank_census(world, device, rehearsal)
    model_name, cfg = MODELS[args.model]
    g, P = args.group_size, world
    lins = llama_linears(cfg, fuse_w13=not args.no_fuse_w13)
    policy = "all" if args.shard_all else args.shard_policy
    pair_of = pair_map(lins)
    calib = {}
    if P > 1 and policy == "auto":
        pairs = sorted({((lins[i][1], lins[i][2]), (lins[j][1], lins[j][2]))
                        for i, (kind, j) in pair_of.items() if kind == "col"})
        calib = calibrate_sharding(sorted({(N, K) for _, N, K in lins}), P, g, device,
                                   rehearsal, pairs=pairs)

    # ---- build the sharded weights, inputs and outputs (all resident in HBM) ----
    st = LinearStep(lins, shard_kinds(lins, P, g, policy, calib, args.shard_min_elems), P, rank,
                    g, device, rehearsal)
    plan, xs, bytes_per_step, stream = st.plan, st.xs, st.bytes_per_step, st.stream
    step, capture = st.step, st.capture

    graph = None if args.no_graph else st.try_capture()
    run = graph.replay if graph is not None else step
    ms = st.wall_ms(run, args.steps, args.warmup)
    elapsed = ms * args.steps * 1e-3

    # ---- roofline: GEMV-only graph replayed back to back, GPU events on the replay stream ----
    groof = graph if (graph is not None and P == 1) else None
    if groof is None and graph is not None:
        groof = capture(do_comm=False)
    kernel_ms = st.replay_ms(groof, max(args.steps, 10)) if groof is not None else None

    # per-shape breakdown: one eager step, events written by each kernel's dispatch packet
    with _lib.KernelTimer(len(plan)) as timer:
        step(do_comm=False)
    torch.cuda.synchronize()
    durs = timer.durations_ms
    assert len(durs) == len(plan)
    gemv_bytes = [int4_alg_bytes(n_loc, K, g) for (_, n_loc, K, *_r) in plan]
    if kernel_ms is None:
        kernel_ms = sum(durs)
    achieved = sum(gemv_bytes) / (kernel_ms * 1e-3) / 1e9
    per_shape = {}
    for (name, n_loc, K, *_r), d, b in zip(plan, durs, gemv_bytes):
        key = f"{n_loc}x{K}"
        e = per_shape.setdefault(key, {"launches": 0, "us": 0.0, "bytes": b})
        e["launches"] += 1
        e["us"] += d * 1e3
    for key, e in per_shape.items():
        e["us"] = round(e["us"] / e["launches"], 3)
        e["GBps"] = round(e["bytes"] / (e["us"] * 1e-6) / 1e9, 1)

    # per-shape cost inside a replayed graph: each shape's launches (its distinct weights, in
    # step order) captured alone and replayed back to back; µs per launch from HIP events on
    # the replay stream. This is the in-step number the north-star target is stated on.
    per_shape_graph = {}
    if graph is not None and P == 1:
        for (n_loc, K) in sorted({(e[1], e[2]) for e in plan}):
            gs_ = capture(do_comm=False, only=(n_loc, K))
            cnt = sum(1 for e in plan if (e[1], e[2]) == (n_loc, K))
            us = st.replay_ms(gs_, max(args.steps, 10)) * 1e3 / cnt
            b = int4_alg_bytes(n_loc, K, g)
            gr_ = st.read_probe_graph(only=(n_loc, K))
            rus = st.replay_ms(gr_, max(args.steps, 10)) * 1e3 / cnt
            per_shape_graph[f"{n_loc}x{K}"] = {
                "launches": cnt, "us": round(us, 3), "GBps": round(b / (us * 1e-6) / 1e9, 1),
                "frac": round(b / (us * 1e-6) / 1e9 / HBM_PEAK_GBPS, 4),
                "pure_read_us": round(rus, 3), "gemv_over_pure_read": round(us / rus, 3)}
            del gs_, gr_
    pure_read_ms = None
    if graph is not None and P == 1:
        # the one-launch-per-linear floor of THIS step, measured now
        gr = st.read_probe_graph()
        pure_read_ms = st.replay_ms(gr, max(args.steps, 10))
        del gr

    # HBM traffic from the committed counter pass (rocprofv3 --pmc FETCH_SIZE of this bench,
    # P = 1 shapes): bytes per step, to set against the algorithmic bytes
    traffic = None
    pmc_file = args.pmc_file
    if P == 1 and args.model == "8b" and pmc_file and os.path.exists(pmc_file):
        with open(pmc_file) as f:
            pmc = json.load(f)
        if pmc.get("launches_per_step", n_launches_expected(args)) == len(plan):
            traffic = pmc.get("hbm_bytes_per_step")

    comm_ms = None
    if P > 1:
        gcomm = st.try_capture(do_gemv=False) if graph is not None else None
        comm_ms = st.wall_ms(gcomm.replay if gcomm is not None else (lambda: step(do_gemv=False)),
                             args.steps, 2)
        del gcomm

    ref_gpu = None
    if P == 1 and not args.no_reference_gpu:
        try:
            # our outputs of the last timed replay are in each plan entry's y_loc
            ref_ms, ref_diff = reference_gpu_step(plan, xs, g, device, args.steps)
            ref_gpu = {
                "op": "aten._weight_int4pack_mm (PyTorch-ROCm; the reference's GPU int4 GEMM, "
                      "tensor_core_tiled_layout.py:104), same weights, same "
                      f"{len(plan)}-call step in one HIP graph",
                "value": round(bytes_per_step / (ref_ms * 1e-3) / 1e9, 2),
                "unit": "GB/s",
                "ms_per_step": round(ref_ms, 4),
                "rel_l2_vs_ours_max": round(ref_diff, 5),
            }
        except Exception as e:  # the aten op is build dependent: report, never fail the bench
            ref_gpu = {"op": "aten._weight_int4pack_mm", "error": f"{type(e).__name__}: {e}"[:300]}

    prefill = None
    if P == 1 and args.model == "8b" and not args.no_prefill:
        prefill = prefill_mfma(device)
    extras = P == 1 and not args.no_extras
    int8wo = (int8wo_m1(device, pmc_file=args.pmc_int8wo_file)
              if extras and args.model == "8b" else None)
    config2 = config2_shapes(device) if extras and args.model == "8b" else None
    ceil = hbm_ceilings(device) if extras else None

    unfused = None
    if P == 1 and args.model == "8b" and not args.no_fuse_w13 and not args.no_extras \
            and graph is not None:
        unfused = unfused_record(cfg, g, device, args.steps)
    config5 = None
    n_launches, has_graph = len(plan), graph is not None
    par_desc = parallelism_desc(st, policy) if P > 1 else "single-gpu"
    if args.model == "8b" and not args.no_config5:
        # release the 8B step's weights first (the 70B step needs 43 GB / P per rank): the
        # plan / inputs / graphs bound here hold them too, so drop those references before
        # st.release() empties the allocator cache
        plan = xs = graph = groof = run = step = capture = None
        st.release()
        c5 = dict(steps=max(2, min(args.steps, 10)), warmup=min(args.warmup, 2))
        config5 = config5_record(P, rank, g, device, rehearsal, policy="tp", **c5)
        if P > 1:
            config5["north_star_plan"] = config5_record(P, rank, g, device, rehearsal,
                                                        policy="all", **c5)

    cpu = None
    if rank == 0 and P == 1 and not args.no_cpu_baseline and args.model == "8b":
        cpu = cpu_baseline(cfg, g)

    if rank == 0:
        rec = {
            "metric": f"int4 WO linear GB/s + tokens/s vs CPU dequant path, {model_name} shapes M=1",
            "value": round(bytes_per_step * args.steps / elapsed / 1e9, 2),
            "unit": "GB/s",
            # linears only (one step = every int4 linear of one decoded token); the model's
            # real decode rate (attention, norms, argmax included) is e2e_decode's
            "linear_steps_per_s": round(args.steps / elapsed, 2),
            "n_gpus": P,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (random-init nn.Linear weights quantized int4 g32; N(0,1) bf16 activations)",
            "config": {
                "workload": f"{model_name} int4 g{g} weight-only linears, M=1 decode: "
                            + workload_desc(cfg, not args.no_fuse_w13)
                            + f" ({n_launches} GEMV launches/step)",
                "model": f"{model_name} (linears only)",
                "global_batch": 1,
                "seq_len": 1,
                "group_size": g,
                "bytes_per_step": bytes_per_step,
                "parallelism": par_desc,
                "hip_graph": has_graph,
            },
            "ranks": census,
            "roofline": {
                "bound": "hbm",
                "kernel": "int4wo_gemv_kernel",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                # what this box streams in one long launch (hbm_ceilings), and the step as a
                # fraction of each ceiling beside the spec-peak fraction
                "measured_copy_GBps": ceil["copy_GBps"] if ceil else None,
                "measured_stream_read_GBps": ceil["read_GBps"] if ceil else None,
                "torch_copy_GBps": ceil["torch_copy_GBps"] if ceil else None,
                "copy_probe": ({"best": ceil["copy_best"], "sweep_GBps": ceil["copy_sweep_GBps"]}
                               if ceil else None),
                "frac": round(achieved / HBM_PEAK_GBPS, 4),
                "frac_of_stream_read": round(achieved / ceil["read_GBps"], 4) if ceil else None,
                "frac_of_copy": round(achieved / ceil["copy_GBps"], 4) if ceil else None,
                "traffic": traffic,
                "traffic_unit": f"HBM bytes per step ({n_launches} launches)",
                "alg_bytes_per_step": bytes_per_step,
                "traffic_source": os.path.relpath(pmc_file, ROOT) if traffic else None,
                "launches": len(durs),
                "kernel_ms_per_step": round(kernel_ms, 4),
                # the same launches as pure 16-B streaming reads of the same bytes, one graph
                # (tao_hbm_read_probe): the floor of a one-kernel-per-linear step, this run
                "pure_read_ms_per_step": round(pure_read_ms, 4) if pure_read_ms else None,
                "gemv_over_pure_read": (round(kernel_ms / pure_read_ms, 3)
                                        if pure_read_ms else None),
                "eager_kernel_ms_per_step": round(sum(durs), 4),
                "per_shape_eager": per_shape,
                "per_shape_graph": per_shape_graph or None,
                # the step rebuilt from the per-shape graph times (launches x us), this run: sits
                # beside kernel_ms_per_step as the in-run check of the step's kernel time
                "per_shape_graph_step_ms": (round(sum(v["launches"] * v["us"]
                                                      for v in per_shape_graph.values()) * 1e-3, 4)
                                            if per_shape_graph else None),
                "per_shape_frac": ({k: v["frac"] for k, v in per_shape_graph.items()}
                                   if per_shape_graph else None),
            },
            "cpu_baseline": cpu,
        }
        ns = per_shape_graph.get("4096x4096") if per_shape_graph else None
        if ns is not None:
            # north_star (BASELINE.json): int4 g32 M=1 4096x4096 at >= 70% of HBM peak per
            # launch; the graph-replayed in-step number (wo's shape at 8B) beside a pure 16-B
            # read of the same 10.5 MB replayed the same way (the floor of one dependent launch
            # on this chip, DESIGN §5.1: launch gap ~1.35 us + one loaded HBM round trip)
            rec["north_star"] = {"shape": f"4096x4096 int4 g{g} M=1",
                                 "us_per_launch": ns["us"], "GBps": ns["GBps"],
                                 "frac": ns["frac"], "target_frac": 0.70, "met": ns["frac"] >= 0.70,
                                 "pure_read_us": ns.get("pure_read_us"),
                                 "pure_read_frac": (round(int4_alg_bytes(4096, 4096, g)
                                                          / (ns["pure_read_us"] * 1e-6) / 1e9
                                                          / HBM_PEAK_GBPS, 4)
                                                    if ns.get("pure_read_us") else None),
                                 "gemv_over_pure_read": ns.get("gemv_over_pure_read"),
                                 "eager_kernel_us": per_shape.get("4096x4096", {}).get("us")}
        if unfused is not None:
            # the reference's module layout (w1, w3 apart): the same bytes in 161 launches
            rec["unfused_w13_step"] = unfused
        if config5 is not None:
            rec["config5_70b"] = config5
        if ref_gpu is not None:
            rec["reference_gpu"] = ref_gpu
            if "value" in ref_gpu:
                rec["speedup_vs_reference_gpu"] = round(rec["value"] / ref_gpu["value"], 2)
        if prefill is not None:
            rec["prefill_mfma"] = prefill
        if config2 is not None:
            rec["config2_shapes"] = config2
        if int8wo is not None:
            rec["int8wo_m1"] = int8wo
        if P == 1 and args.model == "8b" and not args.no_e2e:
            rec["e2e_decode"] = e2e_decode()
        if comm_ms is not None:
            rec["collectives_ms_per_step"] = round(comm_ms, 4)
        if calib:
            rec["shard_calibration_us"] = {
                ("x".join(str(v) for v in key[1:3]) + "->" + "x".join(str(v) for v in key[3:])
                 if key[0] == "pair" else f"{key[0]}x{key[1]}"): v for key, v in calib.items()}
        if cpu is not None:
            rec["speedup_vs_cpu_baseline"] = round(rec["value"] / cpu["value"], 1)
        print(json.dumps(rec), flush=True)

    if P > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
