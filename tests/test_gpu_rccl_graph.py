"""RCCL inside a captured HIP graph, on the box's one GPU (a 1-rank "nccl" process group).

The multi-GPU step (bench.py LinearStep) captures the local int4 GEMVs and the RCCL
collectives of the Megatron pairs (all-reduce of the rowwise partials) and of the head
(all-gather of the column shards) in ONE HIP graph. The driver runs it on 8 GPUs; this test runs
the same call pattern with one rank, so that RCCL's initialisation, its kernels on the capture
stream and graph replay are exercised on MI355X hardware: every replay must equal the eager
step, and a replay after the input changes must recompute (the collectives and GEMVs really
execute inside the graph). With one rank all_reduce is the identity and all_gather a copy, so the
values are also checked against the plain HIP linears. Reference pattern:
test/dtypes/test_affine_quantized_tensor_parallel.py:49-80,120-132.
"""

import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(port, q):
    import sys

    sys.path.insert(0, os.path.join(ROOT, "torchao-fork_amd"))
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    import torch.nn.functional as F

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        from torchao.quantization import Int4WeightOnlyConfig, quantize_

        torch.manual_seed(0)
        D, I, V, g = 1024, 2048, 4096, 32
        lins = {}
        for name, (n, k) in {"w13": (2 * I, D), "w2": (D, I), "head": (V, D)}.items():
            m = torch.nn.Linear(k, n, bias=False).to(torch.bfloat16).to(dev)
            quantize_(m, Int4WeightOnlyConfig(group_size=g))
            lins[name] = m
        x = torch.randn(1, D, dtype=torch.bfloat16, device=dev)
        h = torch.empty(1, D, dtype=torch.bfloat16, device=dev)
        logits = torch.empty(V, dtype=torch.bfloat16, device=dev)

        def step():
            # colwise w1||w3 (no gather) -> SwiGLU -> rowwise w2 partial + all-reduce (+ residual)
            # -> colwise head + all-gather of the column shards: LinearStep's collectives
            ab = F.linear(x, lins["w13"].weight)
            a, b = ab[..., :I], ab[..., I:]
            part = F.linear((F.silu(a.float()) * b.float()).to(torch.bfloat16), lins["w2"].weight)
            dist.all_reduce(part)
            h.copy_(part + x)
            y_loc = F.linear(h, lins["head"].weight).reshape(-1)
            dist.all_gather_into_tensor(logits, y_loc)

        def plain():
            ab = F.linear(x, lins["w13"].weight)
            a, b = ab[..., :I], ab[..., I:]
            part = F.linear((F.silu(a.float()) * b.float()).to(torch.bfloat16), lins["w2"].weight)
            hh = part + x
            return F.linear(hh, lins["head"].weight).reshape(-1)

        stream = torch.cuda.Stream(dev)
        stream.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(stream):
            step()  # warm-up outside capture (communicator, allocator)
            torch.cuda.synchronize()
            eager = logits.clone()
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, stream=stream):
                step()
        torch.cuda.current_stream(dev).wait_stream(stream)
        torch.cuda.synchronize()
        ok_eager = torch.equal(eager, plain())
        logits.zero_()
        replays_equal = True
        for _ in range(3):
            graph.replay()
            torch.cuda.synchronize()
            replays_equal &= torch.equal(logits, eager)
        x.copy_(torch.randn_like(x))
        graph.replay()
        torch.cuda.synchronize()
        ok_new = torch.equal(logits, plain()) and not torch.equal(logits, eager)
        q.put((ok_eager, replays_equal, ok_new, ""))
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback

        q.put((False, False, False, repr(e) + traceback.format_exc()[-1200:]))
    finally:
        dist.destroy_process_group()


def test_rccl_collectives_captured_with_hip_linears():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_free_port(), q))
    p.start()
    ok_eager, replays_equal, ok_new, err = q.get(timeout=300)
    p.join(timeout=60)
    assert not err, err
    assert ok_eager, "eager step with RCCL collectives != the plain HIP linears"
    assert replays_equal, "graph replays of the RCCL + HIP step differ from the eager step"
    assert ok_new, "a replay after the input changed did not recompute"
