"""Debug: compare linear_wide's stored split partials with torch (F=2048, K=16, B=17, f64)."""
import numpy as np
import torch

from mlapi_amd._native import C
from mlapi_amd.models.linear import Kind, LinearModel
from mlapi_amd.ops.linear import LinearWide

torch.cuda.init()
F, K, B = 2048, 16, 17
m = LinearModel.random(F, K, seed=1, kind=Kind.MULTINOMIAL)
X = np.random.default_rng(2).standard_normal((B, F))
op = LinearWide(B, F, K, torch.float64, "cuda")
plan = C().linear_wide_plan(0, F, K)
print(plan)
Xg, Wg, bg = (torch.tensor(a, device="cuda") for a in (X, m.W, m.b))
for it in range(3):
    op.ws.zero_()
    idx, p = op(Xg, Wg, bg, int(Kind.MULTINOMIAL))
    torch.cuda.synchronize()
    ws = op.ws.cpu().numpy()
    part = ws[256:256 + 2 * 512 * 8].view(np.float64).reshape(2, 2, 64, 4)  # [fs][t][lane][r]
    Fh = F // 2
    bad = []
    for fs in range(2):
        Z = X[:, fs * Fh:(fs + 1) * Fh] @ m.W[:, fs * Fh:(fs + 1) * Fh].T  # [B, K]
        for t in range(2):
            for l in range(64):
                for r in range(4):
                    row = min(t * 16 + (l & 15), B - 1)
                    c = (l >> 4) + 4 * r
                    got = part[fs, t, l, r]
                    if not np.isclose(got, Z[row, c], rtol=1e-12, atol=1e-12):
                        bad.append((fs, t, l, r, row, c, float(got), float(Z[row, c])))
    print("iter", it, "bad partials", len(bad))
    for b in bad[:12]:
        print("  ", b)
    ridx, rp = m.predict_max(X)
    print("  bad rows", np.nonzero(~np.isclose(p.cpu().numpy(), rp, rtol=1e-12, atol=0))[0].tolist())
