"""Serving path on a real GPU: engine (zero-copy batches + fused fp64 kernel) and native HTTP server."""
import json

import numpy as np
import pytest

from mlapi_amd.models.linear import Kind, LinearModel

pytestmark = pytest.mark.gpu


def _engine(native, **kw):
    cfg = native.EngineConfig()
    cfg.device = 0
    for k, v in kw.items():
        setattr(cfg, k, v)
    return native.Engine(cfg)


@pytest.mark.parametrize("dtype", [0, 1])
@pytest.mark.parametrize("kind,K", [(Kind.MULTINOMIAL, 3), (Kind.BINARY, 1), (Kind.OVR, 5), (Kind.BINARY_SOFTMAX, 1)])
def test_engine_gpu_matches_oracle(native, dtype, kind, K):
    m = LinearModel.random(4, 2 if K == 1 else K, seed=K, kind=kind)
    e = _engine(native, dtype=dtype, max_batch=64)
    try:
        e.load_model(int(m.kind), m.W, m.b, m.label_json())
        X = np.random.default_rng(1).standard_normal((5000, 4))
        idx, p, st = e.predict(X)
        ridx, rp = m.predict_max(X)
        assert (st == 0).all()
        np.testing.assert_array_equal(idx, ridx)
        np.testing.assert_allclose(p, rp, rtol=1e-12 if dtype == 0 else 1e-5, atol=0 if dtype == 0 else 1e-6)
        s = e.stats()
        assert s["requests"] == 5000 and s["batches"] >= 5000 // 64
    finally:
        e.stop()


def test_engine_gpu_nonfinite_and_shape(native):
    # logits overflow to +inf for two classes -> inf - inf = NaN probability -> status 1 (A13)
    m = LinearModel(np.array([[1.0, 1, 1, 1], [-1, -1, -1, -1], [0.5, 0.5, 0.5, 0.5]]), np.zeros(3),
                    np.array(["a", "b", "c"], dtype=object), Kind.MULTINOMIAL)
    e = _engine(native)
    try:
        e.load_model(int(m.kind), m.W, m.b, m.label_json())
        idx, p, st = e.predict(np.array([[1e308, 1e308, 1e308, 1e308], [1.0, 2.0, 3.0, 4.0]]))
        assert not np.isfinite(m.predict_max(np.array([[1e308] * 4]))[1][0])
        assert st[0] == 1 and st[1] == 0
        idx, p, st = e.predict(np.ones((3, 5)))
        assert (st == 3).all()
    finally:
        e.stop()


def test_engine_gpu_fault_injection(native):
    m = LinearModel.random(4, 3, seed=0)
    e = _engine(native, fail_every=2, max_batch=1)
    try:
        e.load_model(int(m.kind), m.W, m.b, m.label_json())
        _, _, st = e.predict(np.ones((10, 4)))
        assert (st == 4).sum() == 5
    finally:
        e.stop()


def test_native_server_gpu_end_to_end(iris_cwd, native):
    import httpx

    from mlapi_amd.serve.server import NativeServer
    from mlapi_amd.utils.config import Config

    cfg = Config.from_env(port=0, device="cuda:0")
    with NativeServer(cfg) as srv:
        assert srv.runtime.handle.backend == "hip:0"
        base = f"http://127.0.0.1:{srv.port}"
        r = httpx.post(base + "/predict", json={"sepal_length": 5.1, "sepal_width": 3.5, "petal_length": 1.4,
                                                "petal_width": 0.2})
        assert r.status_code == 200
        assert r.text == '{"prediction":"Iris-setosa","probability":0.979132309910533}'
        body = json.dumps({"sepal_length": 6.7, "sepal_width": 3.0, "petal_length": 5.2, "petal_width": 2.3}).encode()
        req = (b"POST /predict HTTP/1.1\r\nHost: x\r\nContent-Type: application/json\r\nContent-Length: %d\r\n\r\n%s"
               % (len(body), body))
        lg = native.Loadgen("127.0.0.1", srv.port, req.decode(), 32, 2)
        res = lg.run(200, True)
        lg.close()
        assert res["status_counts"] == {200: 6400}
        stats = srv.runtime.handle.stats()
        assert stats["requests"] >= 6400
        assert stats["batches"] < stats["requests"], "concurrent requests must be coalesced into batches"


# ---- persistent (resident-kernel) serving mode -------------------------------------------------
@pytest.mark.parametrize("dtype", [0, 1])
@pytest.mark.parametrize("kind,K", [(Kind.MULTINOMIAL, 3), (Kind.BINARY, 1), (Kind.OVR, 5), (Kind.MULTINOMIAL, 40)])
def test_engine_persistent_matches_oracle(native, dtype, kind, K):
    F = 4 if K < 40 else 48  # K=40/F=48 exercises the generic row path inside the resident kernel
    m = LinearModel.random(F, 2 if K == 1 else K, seed=K, kind=kind)
    e = _engine(native, dtype=dtype, max_batch=64, persistent=True)
    try:
        e.load_model(int(m.kind), m.W, m.b, m.label_json())
        X = np.random.default_rng(2).standard_normal((3000, F))
        idx, p, st = e.predict(X)
        ridx, rp = m.predict_max(X)
        assert (st == 0).all()
        np.testing.assert_array_equal(idx, ridx)
        np.testing.assert_allclose(p, rp, rtol=1e-12 if dtype == 0 else 1e-5, atol=0 if dtype == 0 else 1e-6)
        s = e.stats()
        assert s["requests"] == 3000 and s["kernel_launches"] >= 1
    finally:
        e.stop()


def test_engine_persistent_idle_exit_relaunch_reload_and_sync(native):
    import time

    import torch

    m1, m2 = LinearModel.random(4, 3, seed=1), LinearModel.random(4, 3, seed=2)
    e = _engine(native, persistent=True, persistent_idle_ms=3, max_batch=16)
    try:
        e.load_model(int(m1.kind), m1.W, m1.b, m1.label_json())
        X = np.random.default_rng(3).standard_normal((200, 4))
        np.testing.assert_array_equal(e.predict(X)[0], m1.predict_max(X)[0])
        time.sleep(0.05)  # > idle timeout: the resident kernel leaves ...
        t0 = time.perf_counter()
        torch.cuda.synchronize()  # ... so a device-wide synchronize returns
        assert time.perf_counter() - t0 < 1.0
        e.load_model(int(m2.kind), m2.W, m2.b, m2.label_json())  # hot reload between batches
        idx, p, st = e.predict(X)  # relaunched on demand
        np.testing.assert_array_equal(idx, m2.predict_max(X)[0])
        assert (st == 0).all() and e.stats()["kernel_launches"] >= 2
    finally:
        e.stop()


def test_engine_persistent_fault_injection_keeps_order(native):
    m = LinearModel.random(4, 3, seed=0)
    e = _engine(native, persistent=True, fail_every=3, max_batch=1)
    try:
        e.load_model(int(m.kind), m.W, m.b, m.label_json())
        X = np.random.default_rng(4).standard_normal((12, 4))
        idx, p, st = e.predict(X)
        assert (st == 4).sum() == 4 and (st == 0).sum() == 8  # every 3rd single-row batch fails
        ok = st == 0
        np.testing.assert_array_equal(idx[ok], m.predict_max(X)[0][ok])
    finally:
        e.stop()
