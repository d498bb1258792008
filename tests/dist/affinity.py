"""launcher worker: records its rank env and CPU affinity."""
import json
import os

out = os.environ["OUT"]
json.dump({"rank": int(os.environ["RANK"]), "world": int(os.environ["WORLD_SIZE"]),
           "cpus": sorted(os.sched_getaffinity(0)), "omp": os.environ.get("OMP_NUM_THREADS")},
          open(os.path.join(out, f"aff_{os.environ['RANK']}.json"), "w"))
if os.environ.get("FAIL_RANK") == os.environ["RANK"]:
    raise SystemExit(7)
if os.environ.get("FAIL_RANK"):
    import time

    time.sleep(60)  # the launcher must stop this rank when the other one fails
