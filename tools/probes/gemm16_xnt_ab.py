"""A/B of the 16x16 tiles kernel's large-batch X loads (plain default vs nontemporal,
MLAPI_GEMM_XNT16=1) at F = 512 (no 32x32 instantiation), B = 262,144, K = 1000: run once per
setting by tools/probes/r6_xnt16.sh, prints the CUDA-event time per launch."""
import os
import sys

import torch

sys.path.insert(0, ".")
from mlapi_amd.ops import linear as ops  # noqa: E402

dev = torch.device("cuda", 0)
B, F, K = 262144, 512, 1000
X = torch.randn(B, F, device=dev).to(torch.bfloat16)
W = (torch.randn(K, F, device=dev) / 23).to(torch.bfloat16)
b = torch.randn(K, device=dev) * 0.1
out = (torch.empty(B, dtype=torch.int32, device=dev), torch.empty(B, device=dev))
op = ops.GemmSoftmax(B, K, F, dev)
for _ in range(10):
    op(X, W, b, out=out)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(50):
    op(X, W, b, out=out)
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) * 1e3 / 50
print(f"xnt16={os.environ.get('MLAPI_GEMM_XNT16', '0')} F={F} {us:.2f} us {2 * B * K * F / us / 1e6:.1f} TF/s")
