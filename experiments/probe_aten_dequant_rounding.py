"""Which rounding does PyTorch-ROCm's aten._weight_int4pack_mm apply to the int4 dequant on gfx950?

Runs the reference test_ops.py:339-402 protocol (dequant by an identity-matrix mm) on this box's
aten op and counts, per candidate formula, the elements that differ from aten's output. The
candidates are the ways a kernel can form w = (q - 8) * s + z in bf16 (one or two roundings,
fp32 or bf16 intermediates, the 128 + q "magic number" with a folded zero, RNE or truncating
bf16 conversion). Output: one JSON line per (shape, ikt, g) to gpurun_out/probe_dequant.jsonl,
plus a few mismatching elements of the current restatement for CPU analysis.

    python experiments/probe_aten_dequant_rounding.py
"""

import json
import os
import sys

import torch

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gpurun_out")
BF = torch.bfloat16


def rne(x32):
    return x32.to(BF)


def trunc(x32):
    b = x32.contiguous().view(torch.int32) & ~0xFFFF
    return b.view(torch.float32).to(BF)


def candidates(q, s, z):
    """q int32 [N, K] on device, s/z bf16 [N, K] (expanded per element)."""
    qf = q.float()
    sf, zf = s.float(), z.float()
    d8 = qf - 8.0
    out = {}
    exact = d8.double() * sf.double() + zf.double()
    out["fma_f32_rne"] = rne(exact.float())  # bf16(f32(fma)) == the HIP kernel today
    out["exact_rne"] = exact.to(BF)  # one rounding of the exact value
    out["fma_f32_trunc"] = trunc(exact.float())
    out["two_bf16"] = (d8.to(BF) * s + z)  # python dequant: bf16 mul, bf16 add
    m = (qf + 128.0) * sf  # exact in f32
    z136_f = zf - 136.0 * sf  # f32 rounding
    out["magic_f32"] = rne(m + z136_f)
    out["magic_fma_f32"] = rne((((qf + 128.0).double() * sf.double()) + z136_f.double()).float())
    z136_b = (zf - 136.0 * sf).to(BF).float()
    out["magic_zbf16"] = rne(m + z136_b)
    out["magic_zbf16_fma"] = rne(((qf + 128.0).double() * sf.double() + z136_b.double()).float())
    z8_f = zf - 8.0 * sf
    out["q_fma_z8_f32"] = rne((qf.double() * sf.double() + z8_f.double()).float())
    out["q_mul_add_z8_f32"] = rne(qf * sf + z8_f)
    z8_b = (zf - 8.0 * sf).to(BF).float()
    out["q_fma_z8_bf16"] = rne((qf.double() * sf.double() + z8_b.double()).float())
    out["mul_bf16_add_f32"] = rne((d8 * sf).to(BF).float() + zf)
    return out


def main():
    dev = "cuda"
    os.makedirs(OUT, exist_ok=True)
    shapes = [(4096, 4096), (256, 1024)] if "--randz" in sys.argv else \
        [(4096, 4096), (11008, 4096), (4096, 11008), (256, 1024)]
    rows = []
    mism = {}
    for N, K in shapes:
        for ikt in (2, 8):
            for g in (32, 128):
                gen = torch.Generator(device="cpu").manual_seed(N + K + ikt + g)
                t = torch.randn(N, K, generator=gen).to(BF).to(dev)
                tg = t.reshape(N, K // g, g)
                mn, mx = tg.amin(-1), tg.amax(-1)
                s = torch.clamp((mx - mn) / 15.0, min=1e-6).to(BF)
                z = (mn + s * 8.0).to(BF)
                if "--randz" in sys.argv:  # tests/test_gpu_int4.py's eye-mm distribution
                    s = (torch.rand(N, K // g, generator=gen) * 0.05 + 0.001).to(BF).to(dev)
                    z = ((torch.rand(N, K // g, generator=gen) - 0.5) * 0.2).to(BF).to(dev)
                q = torch.clamp(torch.round((tg - (z - s * 8.0).unsqueeze(-1)) / s.unsqueeze(-1)),
                                0, 15).reshape(N, K).to(torch.int32)
                u8 = ((q[:, ::2] << 4) | q[:, 1::2]).to(torch.uint8).contiguous()
                packed = torch.ops.aten._convert_weight_to_int4pack(u8, ikt)
                sz = torch.stack([s.t(), z.t()], -1).contiguous()  # [K/g, N, 2]
                eye = torch.eye(K, device=dev, dtype=BF)
                ref = torch.ops.aten._weight_int4pack_mm(eye, packed, g, sz).t().contiguous()
                se = s.repeat_interleave(g, 1)
                ze = z.repeat_interleave(g, 1)
                rec = {"N": N, "K": K, "ikt": ikt, "g": g}
                for name, c in candidates(q, se, ze).items():
                    rec[name] = int((c.view(torch.int16) != ref.view(torch.int16)).sum())
                rows.append(rec)
                print(json.dumps(rec), flush=True)
                if (N, K, ikt, g) == (4096, 4096, 8, 32):
                    c = candidates(q, se, ze)["fma_f32_rne"]
                    idx = (c.view(torch.int16) != ref.view(torch.int16)).nonzero()[:64]
                    for n, k in idx.tolist():
                        mism.setdefault("rows", []).append(
                            {"q": int(q[n, k]), "s": float(se[n, k]), "z": float(ze[n, k]),
                             "aten": float(ref[n, k]), "fma": float(c[n, k])})
                del eye, ref
                torch.cuda.empty_cache()
    tag = "_randz" if "--randz" in sys.argv else ""
    with open(os.path.join(OUT, f"probe_dequant{tag}.jsonl"), "w") as f:
        for r in rows:
            f.write(json.dumps(r) + "\n")
        f.write(json.dumps(mism) + "\n")


if __name__ == "__main__":
    sys.exit(main())
