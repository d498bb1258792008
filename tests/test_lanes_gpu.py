"""Per-IO-thread dispatch lanes (csrc/runtime/engine.h, Lane): the HTTP IO thread dispatches its
epoll round's rows itself into the engine's multi-producer HSA queue and polls the completion
records in its own loop. Every body is checked byte for byte against the engine's answers (which
make_workload first checks against the float64 oracle); lanes off must give the same bytes."""
import numpy as np
import pytest

from mlapi_amd.models.linear import Kind, LinearModel

pytestmark = pytest.mark.gpu


def _serve(native, model, names, X, *, lanes, conns, threads, reqs_per_conn, dtype="f64", io_threads=4, rtol=None,
           **kw):
    from mlapi_amd.serve.loadgen import make_workload
    from mlapi_amd.serve.server import NativeServer
    from mlapi_amd.utils.config import Config

    cfg = Config.from_env(port=0, device="cuda:0", reload="off", missing_model="keep", io_threads=io_threads,
                          model_path="/nonexistent/lanes.pkl", feature_names=list(names), lanes=lanes, dtype=dtype,
                          **kw)
    with NativeServer(cfg) as srv:
        srv.runtime.handle.load(model)
        if rtol is None:
            rtol = 1e-12 if dtype == "f64" else 1e-5
        reqs, exp = make_workload(srv.runtime.handle.engine, model, names, X, rtol_oracle=rtol, label_margin=1e-5)
        s0 = srv.runtime.handle.stats()
        lg = native.Loadgen("127.0.0.1", srv.port, reqs[0].decode(), conns, threads)
        lg.set_workload([r.decode() for r in reqs], [e.decode() for e in exp], 0.0)
        res = lg.run(reqs_per_conn, True)
        lg.close()
        s1 = srv.runtime.handle.stats()
    d = {k: s1[k] - s0[k] for k in ("requests", "batches", "lane_batches", "idle_batches", "errors")}
    return res, d


@pytest.mark.parametrize("lanes", [1, 0])
def test_lanes_concurrent_bodies_exact(native, lanes):
    names = ["sepal_length", "sepal_width", "petal_length", "petal_width"]
    m = LinearModel.random(4, 3, seed=11, labels=["Iris-setosa", "Iris-versicolor", "Iris-virginica"])
    X = np.round(np.random.default_rng(3).standard_normal((512, 4)) * 2 + 4, 1)
    res, d = _serve(native, m, names, X, lanes=lanes, conns=48, threads=3, reqs_per_conn=200)
    n = 48 * 200
    assert res["failed"] == 0 and res["errors"] == 0 and res["body_mismatches"] == 0, res
    assert res["status_counts"] == {200: n}
    assert d["requests"] == n and d["errors"] == 0, d
    if lanes:
        assert d["lane_batches"] > 0 and d["lane_batches"] <= d["batches"], d
    else:
        assert d["lane_batches"] == 0, d


def test_lanes_batch1_every_request_on_its_lane(native):
    names = ["a", "b", "c", "d", "e", "f", "g", "h"]
    m = LinearModel.random(8, 4, seed=5, kind=Kind.OVR)
    X = np.random.default_rng(9).standard_normal((64, 8))
    res, d = _serve(native, m, names, X, lanes=1, conns=1, threads=1, reqs_per_conn=400, dtype="f32")
    assert res["body_mismatches"] == 0 and res["status_counts"] == {200: 400}, res
    assert d["lane_batches"] == 400 and d["idle_batches"] == 0, d


def test_lanes_skip_wide_models(native):
    """A model off the kernel-argument path (F = 64 binary: the WIDE kernel) never takes a lane: the
    queued path answers it, with the same bytes."""
    F = 64
    names = [f"f{i}" for i in range(F)]
    m = LinearModel.random(F, 2, seed=2)
    X = np.round(np.random.default_rng(4).standard_normal((128, F)), 3)
    res, d = _serve(native, m, names, X, lanes=1, conns=16, threads=2, reqs_per_conn=50, rtol=1e-5)
    assert res["body_mismatches"] == 0 and res["status_counts"] == {200: 800}, res
    assert d["lane_batches"] == 0, d
