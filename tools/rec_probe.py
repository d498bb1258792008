import sys, time, numpy as np
sys.path.insert(0, ".")
from mlapi_amd._native import C
from mlapi_amd._build import hsaco_path
from mlapi_amd.models.linear import LinearModel
c = C()
m = LinearModel.random(4, 3, seed=0)
for direct in (False, True):
    for rec in (True, False):
        cfg = c.EngineConfig(); cfg.device = 0; cfg.record_completion = rec; cfg.watchdog_ms = 200
        cfg.hsaco_path = str(hsaco_path()) if direct else ""
        e = c.Engine(cfg)
        e.load_model(int(m.kind), m.W, m.b, m.label_json())
        t = time.time()
        idx, p, st = e.predict(np.ones((3, 4)))
        s = e.stats()
        print("direct", direct, "rec", rec, "status", st.tolist(), "p", p.tolist(), "ref", m.predict_max(np.ones((3,4)))[1].tolist(), "direct_batches", s["direct_batches"], round(time.time()-t, 3), flush=True)
        e.stop()
