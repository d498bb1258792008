"""The benchmark's out-of-process load generator (mlapi_amd/bin/mlapi-loadgen) against a native CPU
server: every response body is compared with the expected bytes (exactly, or within a relative
tolerance on the trailing probability), and any other body is counted as a mismatch. This is what
makes `bench.py`'s req/s a count of CORRECT responses."""
import numpy as np
import pytest

from mlapi_amd.utils.config import IRIS_FEATURES

ROWS = np.round(np.array([5.84, 3.05, 3.76, 1.2]) + np.random.default_rng(5).standard_normal((40, 4))
                * np.array([0.83, 0.43, 1.76, 0.76]), 1)


@pytest.fixture
def served(iris_cwd):
    from mlapi_amd.ckpt.native import load_model
    from mlapi_amd.serve.loadgen import LoadgenProcess, make_workload
    from mlapi_amd.serve.server import NativeServer
    from mlapi_amd.utils.config import Config

    srv = NativeServer(Config.from_env(port=0, device="cpu", io_threads=2)).start()
    model = load_model(str(iris_cwd / "LRClassifier.pkl"))
    reqs, exp = make_workload(srv.runtime.handle.engine, model, IRIS_FEATURES, ROWS)
    lg = LoadgenProcess()
    try:
        yield srv, lg, reqs, exp
    finally:
        lg.close()
        srv.stop()


def _run(lg, port, conns=8, per_conn=40):
    lg.connect("127.0.0.1", port, conns, 2)
    r = lg.run(per_conn, True)
    lg.cmd("close")
    return r


def test_every_body_validated(served):
    srv, lg, reqs, exp = served
    assert lg.workload(reqs, exp)["entries"] == len(ROWS)
    r = _run(lg, srv.port)
    assert r["completed"] == 8 * 40 and r["ok200"] == 8 * 40
    assert r["body_mismatches"] == 0 and r["errors"] == 0 and r["failed"] == 0
    assert r["n_lat"] == 8 * 40 and r["p50_ns"] > 0


def test_wrong_bodies_are_counted(served):
    srv, lg, reqs, exp = served
    bad = [e.replace(b"Iris", b"Irix") if i % 2 == 0 else e for i, e in enumerate(exp)]
    lg.workload(reqs, bad)
    r = _run(lg, srv.port, conns=4, per_conn=len(ROWS))  # each connection walks the whole workload
    assert r["ok200"] == 4 * len(ROWS)
    assert r["body_mismatches"] == 4 * (len(ROWS) // 2), r


def test_relative_tolerance_on_the_probability(served):
    srv, lg, reqs, exp = served

    def nudge(e, rel):
        head, num = e.rsplit(b":", 1)
        return head + b":" + repr(float(num[:-1]) * (1 + rel)).encode() + b"}"

    close = [nudge(e, 1e-9) for e in exp]
    lg.workload(reqs, close, 1e-6)
    assert _run(lg, srv.port, conns=2, per_conn=len(ROWS))["body_mismatches"] == 0
    lg.workload(reqs, close, 0.0)  # exact comparison: every nudged body differs
    assert _run(lg, srv.port, conns=2, per_conn=len(ROWS))["body_mismatches"] == 2 * len(ROWS)
    far = [nudge(e, 1e-3) for e in exp]
    lg.workload(reqs, far, 1e-6)
    assert _run(lg, srv.port, conns=2, per_conn=len(ROWS))["body_mismatches"] == 2 * len(ROWS)
