"""Debug: linear_wide feature-split merge (nfs > 1) with two row tiles."""
import numpy as np
import torch

from mlapi_amd._native import C
from mlapi_amd.models.linear import Kind, LinearModel
from mlapi_amd.ops.linear import LinearWide

torch.cuda.init()
for F, K, kind in ((1500, 33, Kind.OVR), (1500, 33, Kind.MULTINOMIAL), (2048, 16, Kind.MULTINOMIAL), (1100, 40, Kind.MULTINOMIAL)):
    print("plan", F, K, C().linear_wide_plan(0, F, K))
    m = LinearModel.random(F, K, seed=F * 7 + K, kind=kind)
    rng = np.random.default_rng(F + K)
    for fresh in (False, True):
        op = LinearWide(100, F, K, torch.float64, "cuda")
        for B in (1, 7, 16, 17, 32, 100):
            if fresh:
                op = LinearWide(100, F, K, torch.float64, "cuda")
            X = rng.standard_normal((B, F))
            idx, p = op(torch.tensor(X, device="cuda"), torch.tensor(m.W, device="cuda"), torch.tensor(m.b, device="cuda"),
                        int(kind))
            torch.cuda.synchronize()
            ridx, rp = m.predict_max(X)
            bad = np.nonzero(~np.isclose(p.cpu().numpy(), rp, rtol=1e-12, atol=0) | (idx.cpu().numpy() != ridx))[0]
            print(f"  kind {int(kind)} fresh {fresh} B {B}: bad rows {bad.tolist()[:20]}", flush=True)
