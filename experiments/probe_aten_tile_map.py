"""Recover the nibble map of PyTorch-ROCm's aten._convert_weight_to_int4pack on gfx950.

For each (N, K, inner_k_tiles), packs ceil(log2(N*K)/4) probe matrices whose nibble at (n, k)
is 4 bits of the flat index n*K + k, then reassembles, for every nibble slot of the packed int32
tensor, which (n, k) it holds. Saves the maps to gpurun_out/aten_tile_map.npz (key
"N{N}_K{K}_ikt{ikt}" -> int64 array [*packed.shape, 8] of flat indices, -1 = never written)."""

import json
import os

import numpy as np
import torch


def main():
    dev = torch.device("cuda")
    out = {}
    for (N, K) in ((16, 128), (16, 256), (32, 512), (48, 1024), (64, 2048)):
        for ikt in (2, 4, 8):
            if K % (ikt * 16):
                continue
            idx = torch.arange(N * K, dtype=torch.int64).reshape(N, K)
            nprobe = (int(N * K - 1).bit_length() + 3) // 4
            flat = None
            for p in range(nprobe):
                q = ((idx >> (4 * p)) & 0xF).to(torch.int32).to(dev)
                u8 = ((q[:, ::2] << 4) | q[:, 1::2]).to(torch.uint8).contiguous()
                a = torch.ops.aten._convert_weight_to_int4pack(u8, ikt).view(torch.int32)
                a = a.cpu().numpy().view(np.uint32).astype(np.int64)
                nib = np.stack([(a >> (4 * i)) & 0xF for i in range(8)], axis=-1)
                flat = nib << (4 * p) if flat is None else flat | (nib << (4 * p))
            key = f"N{N}_K{K}_ikt{ikt}"
            out[key] = flat
            uniq = np.unique(flat)
            print(json.dumps({"key": key, "shape": list(flat.shape[:-1]),
                              "bijective": bool(uniq.size == N * K and uniq.min() == 0
                                                and uniq.max() == N * K - 1)}), flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    np.savez_compressed("gpurun_out/aten_tile_map.npz", **out)


if __name__ == "__main__":
    main()
