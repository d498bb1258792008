"""Probe: the wide-F training step's G^T X (K = 1024 classes, F_aug = 1032, B = 65,536, bf16 in,
f32 accumulate) through the vendor GEMM (torch.mm -> hipBLASLt) vs the shipped gdw kernel's time
in the step (rocprofv3: ~190 us). Prints us per call for each form torch offers here."""
import time

import torch

dev = torch.device("cuda", 0)
B, K, F = 65536, 1024, 1032
G = (torch.randn(B, K, device=dev) * 0.01).to(torch.bfloat16)
X = torch.randn(B, F, device=dev).to(torch.bfloat16)


def bench(fn, name, n=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / n
    print(f"{name:40s} {us:8.1f} us  {2 * B * K * F / us / 1e6:7.1f} TF/s", flush=True)


bench(lambda: torch.mm(G.t(), X), "mm bf16 out (G^T X)")
try:
    bench(lambda: torch.mm(G.t(), X, out_dtype=torch.float32), "mm out_dtype=f32")
except Exception as e:  # noqa: BLE001
    print("out_dtype f32 unsupported:", type(e).__name__, str(e)[:120])
Gt = G.t().contiguous()
bench(lambda: torch.mm(Gt, X), "mm bf16 out (G^T materialised)")
bench(lambda: torch.mm(G.t().float(), X.float()), "mm f32 (upcast, reference)", n=5)
