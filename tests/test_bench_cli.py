"""Error paths of the benchmark driver and the native server (CPU backend).

A failed pre-check (the workload's oracle check) used to end the process in
``terminate called without an active exception`` (rc 134): the server was started outside the
bench's try/finally, and at interpreter exit the ASGI bridge's daemon pump threads, parked in
HttpServer.next_slow with the GIL released, were torn down by a forced unwind through pybind11's
noexcept GIL guard. Both the bench (try/finally) and NativeServer (atexit stop) now shut down
cleanly; these tests pin that.
"""
import subprocess
import sys
import textwrap

from conftest import ROOT

FAIL_PRECHECK = textwrap.dedent(f"""
    import sys
    sys.path.insert(0, {str(ROOT)!r})
    import mlapi_amd.serve.loadgen as lg

    def boom(*a, **k):
        raise RuntimeError("forced oracle pre-check failure")

    lg.make_workload = boom
    import bench
    sys.exit(bench.main(["--cpu", "--steps", "1", "--warmup", "0", "--reqs-per-conn", "16",
                         "--c1-requests", "10", "--io-threads", "2", "--client-threads", "2"]))
""")

LEAKED_SERVER = textwrap.dedent(f"""
    import sys
    sys.path.insert(0, {str(ROOT)!r})
    from mlapi_amd.serve.server import NativeServer
    from mlapi_amd.utils.config import Config

    srv = NativeServer(Config.from_env(port=0, device="cpu", reload="off", io_threads=2,
                                       model_path="/nonexistent/x.pkl", missing_model="keep"))
    srv.start()
    raise RuntimeError("escaped while the server runs")
""")


def _run(src: str):
    return subprocess.run([sys.executable, "-c", src], capture_output=True, text=True, timeout=240, cwd="/tmp")


def test_bench_failed_precheck_exits_nonzero_without_terminate():
    r = _run(FAIL_PRECHECK)
    assert r.returncode not in (0, 134, -6), (r.returncode, r.stderr[-2000:])
    assert "forced oracle pre-check failure" in r.stderr
    assert "terminate called" not in r.stderr


def test_server_left_running_at_exit_stops_cleanly():
    r = _run(LEAKED_SERVER)
    assert r.returncode == 1, (r.returncode, r.stderr[-2000:])
    assert "escaped while the server runs" in r.stderr
    assert "terminate called" not in r.stderr
