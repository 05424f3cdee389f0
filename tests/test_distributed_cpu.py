"""World-size-2 gloo tests (CPU) of the column-sharded path: sharding logic, the all-gather
assembly for M = 1 and M > 1, and that shard-then-quantize equals quantize-then-slice."""

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import sys

    sys.path.insert(0, os.path.join(ROOT, "torchao-fork_amd"))
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle
        from torchao.distributed import ColwiseShardedLinear, parallelize_colwise_
        from torchao.quantization import Int4WeightOnlyConfig, quantize_

        torch.manual_seed(0)  # identical full model on every rank
        full = torch.nn.Sequential(torch.nn.Linear(256, 96), torch.nn.Linear(96, 64)).to(torch.bfloat16)
        x1 = torch.randn(1, 256, dtype=torch.bfloat16)
        x3 = torch.randn(3, 2, 256, dtype=torch.bfloat16)
        ref1, ref3 = full(x1), full(x3)

        import copy

        sharded = parallelize_colwise_(copy.deepcopy(full))
        assert isinstance(sharded[0], ColwiseShardedLinear)
        assert sharded[0].local.weight.shape == (96 // world, 256)
        out1, out3 = sharded(x1), sharded(x3)
        ok_plain = torch.equal(out1, ref1) and torch.equal(out3, ref3)

        # shard-then-quantize == quantize-then-slice (host logic, CPU packer)
        qfull = copy.deepcopy(full)
        quantize_(qfull, Int4WeightOnlyConfig(group_size=32))
        qsh = parallelize_colwise_(copy.deepcopy(full))
        quantize_(qsh, Int4WeightOnlyConfig(group_size=32))
        n = 96 // world
        qa = qsh[0].local.weight.tensor_impl
        qb = qfull[0].weight.tensor_impl
        ok_q = torch.equal(qa.packed_weight, qb.packed_weight[rank * n:(rank + 1) * n]) and torch.equal(
            qa.scale_and_zero, qb.scale_and_zero[rank * n:(rank + 1) * n])

        # sharded int4 forward, local compute by the oracle (no CPU kernel in the product)
        def oracle_linear(x, w, b):
            q, s, z = w.tensor_impl.get_plain()
            return oracle.int4_linear(x, q, s, z, 32, b)

        for m in qsh:
            m.local_fn = oracle_linear
        yq = qsh(x3)
        q0, s0, z0 = qfull[0].weight.tensor_impl.get_plain()
        h = oracle.int4_linear(x3, q0, s0, z0, 32, qfull[0].bias)
        q1, s1, z1 = qfull[1].weight.tensor_impl.get_plain()
        yref = oracle.int4_linear(h, q1, s1, z1, 32, qfull[1].bias)
        ok_int4 = torch.equal(yq, yref)
        q.put((rank, ok_plain, ok_q, ok_int4))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, repr(e), False, False))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_colwise_sharded_linear_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for rank, ok_plain, ok_q, ok_int4 in sorted(results, key=lambda r: r[0]):
        assert ok_plain is True, f"rank {rank}: plain sharded forward mismatch ({ok_plain})"
        assert ok_q, f"rank {rank}: shard-then-quantize differs from quantize-then-slice"
        assert ok_int4, f"rank {rank}: sharded int4 forward differs from the unsharded oracle"
