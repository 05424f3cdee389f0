"""Generate tests/golden/groupwise_qparams.npz by running the REFERENCE's
torchao.quantization.utils.get_groupwise_affine_qparams (quantization/utils.py:326-391) on CPU,
for every (zero_point_domain, preserve_zero) branch it has, on weights whose groups include
all-positive, all-negative, constant and mixed-sign values (the cases where the branches differ).
Numbers only (bf16 as uint16 bits, int32 zeros as int32).

    PYTHONDONTWRITEBYTECODE=1 PYTHONPATH=/root/reference python3 oracle/gen_golden_qparams.py
"""
import os

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(os.path.dirname(HERE), "tests", "golden")


def bits(t):
    return t.detach().to(torch.bfloat16).contiguous().view(torch.int16).numpy().view(np.uint16)


def main():
    import torchao

    assert os.path.realpath(torchao.__file__).startswith("/root/reference"), torchao.__file__
    from torchao.quantization.quant_primitives import ZeroPointDomain
    from torchao.quantization.utils import get_groupwise_affine_qparams

    g = torch.Generator().manual_seed(5)
    w = torch.randn(16, 256, generator=g) * 0.05
    w[0, :64] = w[0, :64].abs() + 0.01      # all-positive groups
    w[1, :64] = -w[1, :64].abs() - 0.01     # all-negative groups
    w[2, :32] = 0.25                        # a constant group
    w = w.to(torch.bfloat16)
    rec = {"w": bits(w)}
    for name, zpd, pz in (("float_nopz", ZeroPointDomain.FLOAT, False),
                          ("int_nopz", ZeroPointDomain.INT, False),
                          ("int_pz", ZeroPointDomain.INT, True),
                          ("float_pz", ZeroPointDomain.FLOAT, True)):
        for gs in (32, 64):
            s, z = get_groupwise_affine_qparams(w, 4, gs, torch.bfloat16, zpd, pz)
            rec[f"{name}_g{gs}_s"] = bits(s)
            rec[f"{name}_g{gs}_z"] = z.numpy().view(np.int32) if z.dtype == torch.int32 else bits(z)
            rec[f"{name}_g{gs}_zdtype"] = np.array(str(z.dtype))
    np.savez_compressed(os.path.join(OUT, "groupwise_qparams.npz"), **rec)
    print("groupwise_qparams", sorted(rec))


if __name__ == "__main__":
    main()
