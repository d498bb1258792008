"""Debug: wide kernel through the engine's direct dispatcher vs hipLaunchKernel - statuses per batch."""
import os, sys
import numpy as np
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from mlapi_amd._native import C
from mlapi_amd._build import hsaco_path
from mlapi_amd.models.linear import Kind, LinearModel

native = C()
F, K = int(sys.argv[1]), int(sys.argv[2])
dt = {"f64": 0, "f32": 1}[sys.argv[3]]
m = LinearModel.random(F, K, seed=F + K, kind=Kind.MULTINOMIAL)
rng = np.random.default_rng(K)
for mode in ("hip", "direct", "direct_nobar"):
    cfg = native.EngineConfig()
    cfg.device = 0
    for k, v in dict(max_batch=256, max_features=F, wide_dtype=dt, hsaco_path=str(hsaco_path()),
                     direct_wide=(mode != "hip"), direct_wide_max_weight_bytes=1 << 30,
                     bar_rows=0 if mode == "direct_nobar" else 32).items():
        setattr(cfg, k, v)
    e = native.Engine(cfg)
    try:
        e.load_model(int(m.kind), m.W, m.b, m.label_json())
        for n in (1, 2, 7, 16, 17, 31, 32, 33, 64, 200):
            X = rng.standard_normal((n, F))
            r = e.predict(X)
            bad = np.nonzero(r[2] != 0)[0]
            print(mode, n, "bad", len(bad), "status", np.unique(r[2]).tolist(), "idx", np.unique(r[0][bad])[:5].tolist(), flush=True)
        print(mode, {k: v for k, v in e.stats().items() if "direct" in k or k == "batches"}, flush=True)
    finally:
        e.stop()
