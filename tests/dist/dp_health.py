"""torchrun worker: DP serving on ONE shared SO_REUSEPORT port with health-aware dispatch.

Rank MLAPI_FAULT_DROP_RANK fails every batch (fault injection); its health thread takes it out
of the port's SO_REUSEPORT group. When the test creates OUT/recover, the rank stops failing and
its health probe re-admits it. Every rank publishes its server/engine state in OUT/state_<rank>.
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from mlapi_amd.parallel.dp_serve import start_dp_runtime  # noqa: E402
from mlapi_amd.serve.server import NativeServer  # noqa: E402
from mlapi_amd.utils.config import Config  # noqa: E402

out = os.environ["OUT"]
port = int(os.environ["PORT"])
cfg = Config.from_env(device="cpu", port=port, io_threads=2, reload="off")
rt, ctl, key, info = start_dp_runtime(cfg)
srv = NativeServer(Config.from_env(device="cpu", port=port, io_threads=2, reload="off"), runtime=rt)
srv.start()
ctl.start(key)
recovered = False
t0 = time.time()
while not os.path.exists(os.path.join(out, "stop")) and time.time() - t0 < 90:
    if not recovered and os.path.exists(os.path.join(out, "recover")) and cfg.fault_drop_rank == info.rank:
        rt.handle.engine.inject_drop(False)
        recovered = True
    hs, es = srv.http.stats(), rt.handle.stats()
    st = {"rank": info.rank, "accepting": hs["accepting"], "listeners": hs["listeners"],
          "listen_closes": hs["listen_closes"], "healthy": es["healthy"], "requests": es["requests"],
          "metrics": rt.metrics_text()}
    tmp = os.path.join(out, f".state_{info.rank}")
    with open(tmp, "w") as f:
        json.dump(st, f)
    os.replace(tmp, os.path.join(out, f"state_{info.rank}"))
    time.sleep(0.05)
ctl.stop()
srv.stop()
from mlapi_amd.parallel.comm import shutdown  # noqa: E402

shutdown(info)
