"""Debug: linear_wide with many row groups / class blocks (in-kernel class merge)."""
import numpy as np
import torch

from mlapi_amd._native import C
from mlapi_amd.models.linear import Kind, LinearModel
from mlapi_amd.ops.linear import LinearWide

torch.cuda.init()
for F, K, td in ((256, 1000, torch.float32), (4096, 1000, torch.float64), (256, 100, torch.float64)):
    dt = 0 if td == torch.float64 else 1
    print("plan", F, K, td, C().linear_wide_plan(dt, F, K), flush=True)
    m = LinearModel.random(F, K, seed=F + K, kind=Kind.MULTINOMIAL)
    W = m.W.astype(np.float32).astype(np.float64) if dt else m.W
    om = LinearModel(W, m.b, m.classes, m.kind)
    op = LinearWide(256, F, K, td, "cuda")
    rng = np.random.default_rng(3)
    for B in (1, 16, 17, 33, 64, 100, 128, 200, 256, 100, 17):
        X = rng.standard_normal((B, F))
        Xo = X.astype(np.float32).astype(np.float64) if dt else X
        idx, p = op(torch.tensor(X, device="cuda").to(td), torch.tensor(m.W, device="cuda").to(td),
                    torch.tensor(m.b, device="cuda"), int(Kind.MULTINOMIAL))
        torch.cuda.synchronize()
        ridx, rp = om.predict_max(Xo)
        pg = p.cpu().numpy()
        bad = np.nonzero(~np.isclose(pg, rp, rtol=1e-11, atol=0) | (idx.cpu().numpy() != ridx))[0]
        print(f"  B {B}: bad {len(bad)} rows {bad.tolist()[:16]} sample {pg[bad[:3]].tolist()} vs {rp[bad[:3]].tolist()}",
              flush=True)
    ws = op.ws.cpu().numpy().view(np.uint32)
    print("  counters nonzero:", np.nonzero(ws[:1024])[0].tolist()[:20], flush=True)
