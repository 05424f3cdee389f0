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


def _colwise_gpu_worker(rank, world, port, q):
    """Column-sharded int4 forward with each rank's local linear on the HIP kernels (cuda:0) and
    the all-gather over gloo on host copies: equals the unsharded HIP forward within one bf16
    rounding per layer (a shard's launch shape follows its own N) and the oracle within 1e-2."""
    import sys

    sys.path.insert(0, os.path.join(ROOT, "torchao-fork_amd"))
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import copy

        import torch.nn.functional as F

        from oracle import oracle
        from torchao.distributed import parallelize_colwise_
        from torchao.quantization import Int4WeightOnlyConfig, quantize_

        dev = torch.device("cuda", 0)
        torch.manual_seed(0)
        full = torch.nn.Sequential(torch.nn.Linear(512, 192), torch.nn.Linear(192, 128)).to(torch.bfloat16)
        xs = [torch.randn(1, 512, dtype=torch.bfloat16), torch.randn(5, 512, dtype=torch.bfloat16)]
        qfull = copy.deepcopy(full)
        quantize_(qfull, Int4WeightOnlyConfig(group_size=32))
        qsh = parallelize_colwise_(copy.deepcopy(full))
        quantize_(qsh, Int4WeightOnlyConfig(group_size=32))

        def hip_linear(x, w, b):
            return F.linear(x.to(dev), w.to(dev), None if b is None else b.to(dev)).cpu()

        for m in qsh:
            m.local_fn = hip_linear
        ok = True
        worst = 0.0
        for x in xs:
            y_sh = qsh(x)
            h = hip_linear(x, qfull[0].weight, qfull[0].bias)
            y_full = hip_linear(h, qfull[1].weight, qfull[1].bias)
            q0, s0, z0 = qfull[0].weight.tensor_impl.get_plain()
            q1, s1, z1 = qfull[1].weight.tensor_impl.get_plain()
            y_ref = oracle.int4_linear(oracle.int4_linear(x, q0, s0, z0, 32, qfull[0].bias),
                                       q1, s1, z1, 32, qfull[1].bias)
            r_full = float((y_sh.float() - y_full.float()).norm() / y_full.float().norm())
            r_ref = float((y_sh.float() - y_ref.float()).norm() / y_ref.float().norm())
            worst = max(worst, r_full, r_ref)
            ok = ok and y_sh.shape == y_full.shape and r_full < 1e-2 and r_ref < 1e-2
        q.put((rank, ok, worst))
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback

        q.put((rank, False, repr(e) + traceback.format_exc()[-800:]))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_colwise_gather_hip_local_compute_gloo():
    """BASELINE config 5's pattern (colwise shards + all-gather of the outputs) with the local
    linears on the HIP kernels; both ranks share the box's one GPU."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_colwise_gpu_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    results = [q.get(timeout=300) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
    for rank, ok, info in sorted(results, key=lambda r: r[0]):
        assert ok is True, f"rank {rank}: sharded HIP forward mismatch ({info})"


def _tp_worker(rank, world, port, q, use_gpu):
    """Megatron pairing on a SwiGLU MLP: w1 / w3 colwise (no gather) -> silu(a) * b on the local
    columns -> w2 rowwise + all-reduce (reference test_affine_quantized_tensor_parallel.py:
    65-80, 120-122). Local compute: the HIP kernels on cuda:0 (use_gpu) or the CPU oracle.
    The gloo collectives run on CPU tensors."""
    import sys

    sys.path.insert(0, os.path.join(ROOT, "torchao-fork_amd"))
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import copy

        import torch.nn.functional as F

        from oracle import oracle
        from torchao.distributed import (
            ColwiseShardedLinear,
            RowwiseShardedLinear,
            shard_linear_colwise,
            shard_linear_rowwise,
            shard_wqkv_by_heads,
        )
        from torchao.quantization import Int4WeightOnlyConfig, quantize_

        dev = torch.device("cuda", 0) if use_gpu else torch.device("cpu")
        g, D, I = 32, 256, 512
        torch.manual_seed(0)  # identical full weights on every rank
        w1 = torch.nn.Linear(D, I, bias=False).to(torch.bfloat16)
        w3 = torch.nn.Linear(D, I, bias=False).to(torch.bfloat16)
        w2 = torch.nn.Linear(I, D, bias=True).to(torch.bfloat16)
        x = torch.randn(1, D, dtype=torch.bfloat16)

        # 1) plain bf16: pairing == unsharded up to the bf16 rounding of the partial sums
        c1 = ColwiseShardedLinear(shard_linear_colwise(w1, rank, world), I, gather=False)
        c3 = ColwiseShardedLinear(shard_linear_colwise(w3, rank, world), I, gather=False)
        r2 = RowwiseShardedLinear(shard_linear_rowwise(w2, rank, world, g), I, w2.bias)
        y_tp = r2(F.silu(c1(x)) * c3(x))
        y_ref = w2(F.silu(w1(x)) * w3(x))
        ok_plain = float((y_tp.float() - y_ref.float()).norm() / y_ref.float().norm()) < 1e-2

        # 2) shard-then-quantize == quantize-then-slice, rowwise (groups along K align)
        qfull = copy.deepcopy(w2)
        quantize_(qfull, Int4WeightOnlyConfig(group_size=g))
        qsh = shard_linear_rowwise(w2, rank, world, g)
        quantize_(qsh, Int4WeightOnlyConfig(group_size=g))
        k = I // world
        fa, fb = qsh.weight.tensor_impl, qfull.weight.tensor_impl
        ok_q = (torch.equal(fa.packed_weight, fb.packed_weight[:, rank * k // 8:(rank + 1) * k // 8])
                and torch.equal(fa.scale_and_zero, fb.scale_and_zero[:, rank * k // g:(rank + 1) * k // g]))

        # 3) int4 forward of the pair: local linears on the HIP kernels (or the oracle), the
        # reduction exact against the sum of the gathered partials
        mods = {}
        for name, lin, mk in (("w1", w1, "col"), ("w3", w3, "col"), ("w2", w2, "row")):
            sh = (shard_linear_colwise(lin, rank, world) if mk == "col"
                  else shard_linear_rowwise(lin, rank, world, g))
            quantize_(sh, Int4WeightOnlyConfig(group_size=g))
            mods[name] = sh.to(dev)

        def lin(m, t):
            if use_gpu:
                return F.linear(t.to(dev), m.weight).cpu()
            qq, ss, zz = m.weight.tensor_impl.get_plain()
            return oracle.int4_linear(t, qq, ss, zz, g)

        a, b = lin(mods["w1"], x), lin(mods["w3"], x)
        h = (F.silu(a.float()) * b.float()).to(torch.bfloat16)
        part = lin(mods["w2"], h)
        parts = [torch.empty_like(part) for _ in range(world)]
        dist.all_gather(parts, part)
        red = part.clone()
        dist.all_reduce(red)
        manual = parts[0].clone()
        for p_ in parts[1:]:
            manual = manual + p_
        ok_reduce = torch.equal(red, manual)
        # against the unsharded int4 MLP through the oracle (the CPU dequant path)
        full = {}
        for name, lin_ in (("w1", w1), ("w3", w3), ("w2", w2)):
            m = copy.deepcopy(lin_)
            quantize_(m, Int4WeightOnlyConfig(group_size=g))
            full[name] = m.weight.tensor_impl.get_plain()
        fa_ = oracle.int4_linear(x, *full["w1"], g)
        fb_ = oracle.int4_linear(x, *full["w3"], g)
        yref = oracle.int4_linear((F.silu(fa_.float()) * fb_.float()).to(torch.bfloat16),
                                  *full["w2"], g)
        ok_int4 = float((red.float() - yref.float()).norm() / yref.float().norm()) < 2e-2

        # 4) head-wise wqkv shard: rank r holds its q, k and v heads
        H, Hkv, hd = 4, 2, 16
        wqkv = torch.nn.Linear(64, (H + 2 * Hkv) * hd, bias=False)
        sq = shard_wqkv_by_heads(wqkv, H, Hkv, hd, rank, world)
        hq, hk = H // world, Hkv // world
        W = wqkv.weight.detach()
        want = torch.cat([W[rank * hq * hd:(rank + 1) * hq * hd],
                          W[H * hd + rank * hk * hd:H * hd + (rank + 1) * hk * hd],
                          W[(H + Hkv) * hd + rank * hk * hd:(H + Hkv) * hd + (rank + 1) * hk * hd]])
        ok_heads = torch.equal(sq.weight, want)
        q.put((rank, ok_plain, ok_q, ok_reduce and ok_int4, ok_heads))
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback

        q.put((rank, repr(e) + traceback.format_exc()[-800:], False, False, False))
    finally:
        dist.destroy_process_group()


def _run_tp(world, use_gpu):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_tp_worker, args=(r, world, port, q, use_gpu)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for rank, ok_plain, ok_q, ok_int4, ok_heads in sorted(results, key=lambda r: r[0]):
        assert ok_plain is True, f"rank {rank}: bf16 colwise->rowwise pairing ({ok_plain})"
        assert ok_q, f"rank {rank}: rowwise shard-then-quantize != quantize-then-slice"
        assert ok_int4, f"rank {rank}: int4 pair forward / reduction mismatch"
        assert ok_heads, f"rank {rank}: head-wise wqkv shard rows"


def test_tp_colwise_rowwise_pairing_gloo():
    _run_tp(2, use_gpu=False)


@pytest.mark.gpu
def test_tp_pairing_hip_local_compute_gloo():
    """The same pairing with each rank's local linears on the HIP kernels (both ranks on the one
    GPU of the box, gloo collectives on host copies)."""
    _run_tp(2, use_gpu=True)
