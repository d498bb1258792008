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
        # the Iris model is served by the resident kernel by default: rows, not launched batches
        assert stats["resident_live"] and stats["resident_rows"] >= 6000, stats


# ---- small-model launch modes: kernel-argument batches vs zero-copy pinned rows ------------------
@pytest.mark.parametrize("inline", [True, False])
@pytest.mark.parametrize("max_batch", [16, 256, 1024])
def test_engine_small_inline_and_zero_copy(native, inline, max_batch):
    m = LinearModel.random(4, 3, seed=7)
    e = _engine(native, max_batch=max_batch, inline_args=inline)
    try:
        e.load_model(int(m.kind), m.W, m.b, m.label_json())
        assert e.model_path() == "small"
        X = np.random.default_rng(8).standard_normal((4000, 4))
        idx, p, st = e.predict(X)
        ridx, rp = m.predict_max(X)
        assert (st == 0).all()
        np.testing.assert_array_equal(idx, ridx)
        np.testing.assert_allclose(p, rp, rtol=1e-12, atol=0)
        s = e.stats()
        assert s["path_batches"]["small"] == s["batches"]
        if not inline:
            assert s["inline_batches"] == 0
        elif max_batch == 16:
            assert s["inline_batches"] == s["batches"]  # 16 rows x 4 x f64 always fit
    finally:
        e.stop()


@pytest.mark.parametrize("dtype", [0, 1])
@pytest.mark.parametrize("F,K,kind", [(4, 3, Kind.MULTINOMIAL), (4, 1, Kind.BINARY), (8, 4, Kind.OVR), (10, 5, Kind.MULTINOMIAL)])
def test_engine_direct_dispatch_matches_hip_launch(native, dtype, F, K, kind):
    """Kernel-argument batches written as AQL packets into the engine's own HSA queue (code object
    mlapi_amd/serve_kernels.hsaco) give bit-identical results to the hipLaunchKernel path."""
    from mlapi_amd._build import hsaco_path

    m = LinearModel.random(F, 2 if K == 1 else K, seed=F + K, kind=kind)
    X = np.random.default_rng(F * K).standard_normal((3000, F))
    out = {}
    for mode in ("hip", "direct"):
        e = _engine(native, dtype=dtype, max_batch=32, max_features=F,
                    hsaco_path=str(hsaco_path()) if mode == "direct" else "")
        try:
            e.load_model(int(m.kind), m.W, m.b, m.label_json())
            idx, p, st = e.predict(X)
            assert (st == 0).all()
            s = e.stats()
            assert s["direct_dispatch"] == (mode == "direct")
            assert s["direct_device_kernargs"] == (mode == "direct")  # ring in HBM, not host memory
            assert s["inline_batches"] == s["batches"]
            assert s["direct_batches"] == (s["batches"] if mode == "direct" else 0)
            out[mode] = (idx, p)
        finally:
            e.stop()
    np.testing.assert_array_equal(out["hip"][0], out["direct"][0])
    np.testing.assert_array_equal(out["hip"][1], out["direct"][1])
    ridx, rp = m.predict_max(X)
    np.testing.assert_array_equal(out["direct"][0], ridx)
    np.testing.assert_allclose(out["direct"][1], rp, rtol=1e-12 if dtype == 0 else 1e-5, atol=0 if dtype == 0 else 1e-6)


def test_engine_drop_injection_and_recovery(native):
    m = LinearModel.random(4, 3, seed=0)
    e = _engine(native, max_batch=8)
    try:
        e.load_model(int(m.kind), m.W, m.b, m.label_json())
        e.inject_drop(True)
        _, _, st = e.predict(np.ones((5, 4)))
        assert (st == 4).all() and not e.healthy() and e.stats()["dropped"]
        e.inject_drop(False)
        e.mark_healthy()
        idx, _, st = e.predict(np.ones((5, 4)))
        assert (st == 0).all() and e.healthy()
    finally:
        e.stop()
