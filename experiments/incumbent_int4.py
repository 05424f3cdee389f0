"""PyTorch-ROCm's own int4 GEMM (aten._weight_int4pack_mm, the op the reference's
TensorCoreTiledLayout calls on the GPU, tensor_core_tiled_layout.py:104) against this build's
int4 linear on the same box, same shapes, M = 1 and 128: each op's calls captured in one HIP
graph over rotating weight copies (past the 256 MiB Infinity Cache), per-call time = graph
replay time / calls. Checks both against the dequantised fp32 reference. Prints JSON lines."""

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "torchao-fork_amd"))
import torch  # noqa: E402

import torchao  # noqa: E402,F401

G = 32
dev = torch.device("cuda")


def per_call_us(fn, copies, calls=64, reps=10):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for i in range(copies):
            fn(i)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for i in range(calls):
                fn(i % copies)
        g.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(reps):
            g.replay()
        e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (reps * calls)


def main():
    print(json.dumps({"torch": torch.__version__, "hip": torch.version.hip,
                      "device": torch.cuda.get_device_name()}), flush=True)
    for (N, K) in [(4096, 4096), (6144, 4096), (28672, 4096), (4096, 14336), (128256, 4096)]:
        nbytes = N * K // 2 + (K // G) * N * 4
        copies = max(2, min(40, int(400e6 // nbytes)))
        qs = [torch.randint(0, 16, (N, K), dtype=torch.int32, device=dev) for _ in range(copies)]
        s = (torch.rand(N, K // G, device=dev) * 0.01 + 1e-3).to(torch.bfloat16)
        z = (torch.randn(N, K // G, device=dev) * 0.01).to(torch.bfloat16)
        ours = [(torch.ops.torchao.int4_pack(q), torch.stack([s, z], -1).contiguous()) for q in qs]
        rec = {"N": N, "K": K, "bytes": nbytes}
        try:
            u8 = [((q[:, ::2] << 4) | q[:, 1::2]).to(torch.uint8) for q in qs]
            ref_packed = [torch.ops.aten._convert_weight_to_int4pack(u, 8) for u in u8]
            sz_ref = torch.stack([s, z], -1).transpose(0, 1).contiguous()  # [K/g, N, 2]
        except Exception as e:  # pragma: no cover - depends on the torch build
            ref_packed, rec["aten_error"] = None, f"{type(e).__name__}: {str(e)[:200]}"
        for M in (1, 128):
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            w0 = ((qs[0].float() - 8) * s.float().repeat_interleave(G, 1)
                  + z.float().repeat_interleave(G, 1))
            yref = x.float() @ w0.t()
            y = torch.ops.torchao.int4_weight_only_linear(x, ours[0][0], ours[0][1], G, None)
            rec[f"ours_M{M}_relerr"] = float((y.float() - yref).norm() / yref.norm())
            us = per_call_us(lambda i: torch.ops.torchao.int4_weight_only_linear(
                x, ours[i][0], ours[i][1], G, None), copies)
            rec[f"ours_M{M}_us"] = round(us, 2)
            rec[f"ours_M{M}_GBps"] = round(nbytes / us / 1e3, 1)
            if ref_packed is not None:
                try:
                    ya = torch.ops.aten._weight_int4pack_mm(x, ref_packed[0], G, sz_ref)
                    rec[f"aten_M{M}_relerr"] = float((ya.float() - yref).norm() / yref.norm())
                    us = per_call_us(lambda i: torch.ops.aten._weight_int4pack_mm(
                        x, ref_packed[i], G, sz_ref), copies)
                    rec[f"aten_M{M}_us"] = round(us, 2)
                    rec[f"aten_M{M}_GBps"] = round(nbytes / us / 1e3, 1)
                except Exception as e:  # pragma: no cover
                    rec[f"aten_M{M}_error"] = f"{type(e).__name__}: {str(e)[:200]}"
        print(json.dumps(rec), flush=True)
        del qs, ours, ref_packed
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
