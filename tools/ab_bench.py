"""Run bench.py against the previous build staged in ab_old/ (interleaved A/B sessions)."""
import runpy
import sys

sys.path.insert(0, "ab_old")
sys.argv = ["bench.py"] + sys.argv[1:]
runpy.run_path("bench.py", run_name="__main__")
