"""What does PyTorch-ROCm's aten._convert_weight_to_int4pack produce on gfx950, and does it agree
with the tile format of the reference's unpack kernel (tensor_core_tiled_layout.cu:131-215), as
restated by torchao::pack_tensor_core_tiled_layout? Prints one JSON line per (N, K, ikt).

Also checks the reference's dequant bar (test/test_ops.py:339-402): the tile-format dequant
equals aten._weight_int4pack_mm(eye(K), packed, g, sz).t() exactly."""

import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "torchao-fork_amd"))
import torchao.ops  # noqa: E402,F401


def main():
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(0)
    for (N, K) in ((8, 128), (16, 256), (64, 1024), (256, 512)):
        for ikt in (2, 4, 8):
            if K % (ikt * 16):
                continue
            q = torch.randint(0, 16, (N, K), generator=g, dtype=torch.int32).to(dev)
            u8 = ((q[:, ::2] << 4) | q[:, 1::2]).to(torch.uint8)
            rec = {"N": N, "K": K, "ikt": ikt}
            try:
                a = torch.ops.aten._convert_weight_to_int4pack(u8.contiguous(), ikt)
                rec["aten_shape"] = list(a.shape)
                rec["aten_dtype"] = str(a.dtype)
                ours = torch.ops.torchao.pack_tensor_core_tiled_layout(q, ikt)
                rec["ours_shape"] = list(ours.shape)
                same = a.shape == ours.shape and torch.equal(a.view(torch.int32), ours)
                rec["bit_identical"] = bool(same)
                if a.dtype == torch.int32 and a.dim() == 4 and a.shape[2] == 32:
                    back = torch.ops.torchao.unpack_tensor_core_tiled_layout(a.contiguous(), ikt)
                    rec["unpack_of_aten_equals_q"] = bool(torch.equal(back, q))
                if not same:
                    rec["aten_first"] = [int(v) for v in a.reshape(-1)[:8].view(torch.int32).tolist()]
                    rec["ours_first"] = [int(v) for v in ours.reshape(-1)[:8].tolist()]
                for G in (32, 64, 128):
                    if K % G:
                        continue
                    s = (torch.rand(K // G, N, generator=g) * 0.1 + 0.01).to(torch.bfloat16)
                    z = (torch.rand(K // G, N, generator=g) - 0.5).to(torch.bfloat16)
                    sz = torch.stack([s, z], -1).contiguous().to(dev)
                    eye = torch.eye(K, device=dev, dtype=torch.bfloat16)
                    ref = torch.ops.aten._weight_int4pack_mm(eye, a, G, sz).t().contiguous()
                    if ours.shape == a.shape:
                        mine = torch.ops.torchao.dequantize_tensor_core_tiled_layout(
                            a.view(torch.int32).contiguous(), sz, G, ikt)
                        rec[f"dequant_g{G}_maxdiff_vs_aten_eye_mm"] = float(
                            (mine.float() - ref.float()).abs().max())
            except Exception as e:  # report, keep probing
                rec["error"] = f"{type(e).__name__}: {e}"[:300]
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
