"""Library incumbents for the skinny shapes (run under rocprofv3 --kernel-trace --stats):
torch._int_mm (hipBLASLt int8) and torch.mm bf16 (hipBLASLt) at M in {32, 128}, weights rotated
past the MALL."""
import torch

for (M, N, K) in [(32, 4096, 4096), (128, 4096, 4096), (128, 14336, 4096), (32, 14336, 4096)]:
    copies = max(2, int(300e6 // (N * K)))
    wi = [torch.randint(-127, 128, (N, K), dtype=torch.int8, device="cuda") for _ in range(copies)]
    xi = torch.randint(-127, 128, (M, K), dtype=torch.int8, device="cuda")
    for i in range(30):
        torch._int_mm(xi, wi[i % copies].t())
    del wi
    wb = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) for _ in range(max(2, copies // 2))]
    xb = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    for i in range(30):
        torch.mm(xb, wb[i % len(wb)].t())
    del wb
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    print("done", M, N, K, flush=True)
