"""torchrun worker: DP serving on the CPU backend with per-rank ports and cluster-wide reload."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from mlapi_amd.parallel.dp_serve import start_dp_runtime  # noqa: E402
from mlapi_amd.serve.server import NativeServer  # noqa: E402
from mlapi_amd.utils.config import Config  # noqa: E402

base = int(os.environ["BASE_PORT"])
cfg = Config.from_env(device="cpu", port=0, reload_interval_ms=20)
rt, ctl, key, info = start_dp_runtime(cfg)
srv = NativeServer(Config.from_env(device="cpu", port=base + info.rank, reload_interval_ms=20), runtime=rt)
srv.start()
ctl.start(key)
open(os.path.join(os.environ["OUT"], f"ready_{info.rank}"), "w").close()
stop_file = os.path.join(os.environ["OUT"], "stop")
t0 = time.time()
while not os.path.exists(stop_file) and time.time() - t0 < 60:
    time.sleep(0.05)
ctl.stop()
srv.stop()
from mlapi_amd.parallel.comm import shutdown  # noqa: E402

shutdown(info)
