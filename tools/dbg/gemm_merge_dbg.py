"""Debug: gemm_softmax split merge vs the fp64 oracle at one shape; prints the mismatching rows."""
import sys
import torch
import numpy as np
from mlapi_amd.ops import linear as ops
from mlapi_amd.ops import reference as ref
from mlapi_amd.models.linear import Kind

DEV = "cuda"
B, F, K = (int(v) for v in sys.argv[1:4])


def _rand(shape, dtype, seed, scale=1.0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(shape, generator=g, dtype=torch.float64) * scale).to(dtype).to(DEV)


X = _rand((B, F), torch.bfloat16, 9)
W = _rand((K, F), torch.bfloat16, 10, scale=1 / np.sqrt(F))
b = _rand((K,), torch.float32, 11, scale=0.1)
ridx, rp = ref.predict_ref(X, W, b, Kind.MULTINOMIAL)
import time
for it in range(3):
    t0 = time.time()
    idx, p = ops.gemm_softmax(X, W, b, Kind.MULTINOMIAL)
    torch.cuda.synchronize()
    print(f"iter {it}: {time.time() - t0:.3f} s, idx -2: {(idx == -2).sum().item()}, -3: {(idx == -3).sum().item()}")
    bad = (idx != ridx).nonzero().flatten().cpu().numpy()
    pr = (p.double() - rp).abs().max().item()
    print(f"iter {it}: {len(bad)} idx mismatches, max |dp| {pr:.3g}")
    for r in bad[:12]:
        print(f"  row {r} (block {r // 64}, r%64 {r % 64}): idx {idx[r].item()} ref {ridx[r].item()} p {p[r].item():.6f} ref {rp[r].item():.6f}")
    if len(bad):
        blocks = np.unique(bad // 64)
        print("  blocks:", blocks[:40], "rows%64:", np.unique(bad % 64)[:64])
