"""T4: batching engine semantics on the C++ CPU backend (the "FakeDevice")."""
import asyncio
import threading
import time

import numpy as np
import pytest

from mlapi_amd.models.linear import Kind, LinearModel


def make_engine(native, **kw):
    cfg = native.EngineConfig()
    cfg.device = -1
    for k, v in kw.items():
        setattr(cfg, k, v)
    return native.Engine(cfg)


@pytest.fixture
def model():
    return LinearModel.random(4, 3, seed=1, labels=["a", "b", "c"])


def test_coalesces_concurrent_submits(native, model):
    """Requests submitted while a batch is in progress are coalesced into the next launch."""
    e = make_engine(native, delay_us=2000, max_batch=1024)
    e.load_model(int(model.kind), model.W, model.b, model.label_json())
    sink = native.PySink()
    X = np.random.default_rng(0).normal(size=(500, 4))
    for i in range(500):
        e.submit(X[i], i, sink)
    got = {}
    t0 = time.time()
    while len(got) < 500 and time.time() - t0 < 10:
        for tag, idx, st, p, lat, ver in sink.drain():
            got[tag] = (idx, st, p)
        time.sleep(0.001)
    s = e.stats()
    e.stop()
    assert len(got) == 500 and s["requests"] == 500
    assert s["batches"] <= 10, "500 queued requests must not become 500 launches"
    ridx, rp = model.predict_max(X)
    assert all(got[i][0] == ridx[i] and got[i][1] == 0 for i in range(500))


def test_max_batch_respected(native, model):
    e = make_engine(native, max_batch=7, delay_us=500)
    e.load_model(int(model.kind), model.W, model.b, model.label_json())
    e.predict(np.ones((100, 4)))
    hist = e.stats()["batch_hist"]
    e.stop()
    assert sum(hist[3:]) == 0  # no batch of >= 8 rows


def test_hot_swap_and_unload(native, model):
    e = make_engine(native)
    v1 = e.load_model(int(model.kind), model.W, model.b, model.label_json())
    m2 = LinearModel(model.W, model.b + np.array([100.0, 0, 0]), model.classes, model.kind)
    v2 = e.load_model(int(m2.kind), m2.W, m2.b, m2.label_json())
    assert v2 > v1
    idx, _, st = e.predict(np.zeros((3, 4)))
    assert (idx == 0).all() and (st == 0).all()
    e.unload_model()
    _, _, st = e.predict(np.zeros((2, 4)))
    e.stop()
    assert (st == 2).all()  # ST_NO_MODEL -> HTTP 500 like a missing checkpoint


def test_shape_mismatch_and_fault_injection(native, model):
    e = make_engine(native, fail_every=3, max_batch=1)
    e.load_model(int(model.kind), model.W, model.b, model.label_json())
    _, _, st = e.predict(np.zeros((9, 4)))
    assert (st == 4).sum() == 3
    _, _, st = e.predict(np.zeros((2, 5)))
    e.stop()
    assert (st == 3).all()


def test_many_threads_stress(native, model):
    """Race screen: 8 submitting threads x 2000 requests, every completion accounted for once."""
    e = make_engine(native, max_batch=64)
    e.load_model(int(model.kind), model.W, model.b, model.label_json())
    X = np.random.default_rng(1).normal(size=(2000, 4))
    ridx, rp = model.predict_max(X)
    errors = []

    def worker():
        idx, p, st = e.predict(X)
        if not ((idx == ridx).all() and (st == 0).all() and np.allclose(p, rp, rtol=1e-14)):
            errors.append(1)

    ts = [threading.Thread(target=worker) for _ in range(8)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    s = e.stats()
    e.stop()
    assert not errors and s["requests"] == 16000


def test_stop_is_idempotent_and_rejects(native, model):
    e = make_engine(native)
    e.load_model(int(model.kind), model.W, model.b, model.label_json())
    e.stop()
    e.stop()
    assert e.submit(np.zeros(4), 1, native.PySink()) == 0  # stopping (-1 would mean backpressure)


def test_async_engine(model):
    from mlapi_amd.serve.runtime import AsyncEngine, EngineHandle, PredictionError
    from mlapi_amd.utils.config import Config

    h = EngineHandle(Config.from_env(device="cpu"))
    h.load(model)
    client = AsyncEngine(h)

    async def go():
        rows = np.random.default_rng(2).normal(size=(200, 4))
        res = await asyncio.gather(*(client.predict_one(r) for r in rows))
        with pytest.raises(PredictionError):
            await client.predict_one([float("nan"), 1, 2, 3])
        return rows, res

    rows, res = asyncio.run(go())
    h.close()
    idx, p = model.predict_max(rows)
    assert [r[0] for r in res] == list(model.classes[idx])
    np.testing.assert_allclose([r[1] for r in res], p, rtol=1e-14)


def test_model_store_watch(tmp_path, iris_pickle_bytes):
    from mlapi_amd.serve.runtime import EngineHandle, ModelStore, wait_for
    from mlapi_amd.utils.config import Config

    path = tmp_path / "m.pkl"
    h = EngineHandle(Config.from_env(device="cpu"))
    store = ModelStore(h, str(path))
    assert store.check() is False and "not found" in store.last_error
    store.start_watcher(10)
    path.write_bytes(iris_pickle_bytes)
    assert wait_for(lambda: h.version != 0, 5)
    path.unlink()
    assert wait_for(lambda: h.version == 0, 5)
    path.write_bytes(b"garbage")
    time.sleep(0.1)
    assert h.version == 0 and store.last_error
    store.stop()
    h.close()


def test_max_wait_fills_batches(native, model):
    """max_wait_us > 0: the batcher waits (bounded) for more rows instead of launching at once."""
    e = make_engine(native, max_wait_us=20000, max_batch=64)
    e.load_model(int(model.kind), model.W, model.b, model.label_json())
    sink = native.PySink()
    X = np.random.default_rng(1).normal(size=(64, 4))
    t0 = time.time()
    for i in range(64):  # trickle in: without the wait these would be many small batches
        e.submit(X[i], i, sink)
        time.sleep(0.0001)
    got = 0
    while got < 64 and time.time() - t0 < 10:
        got += len(sink.drain())
        time.sleep(0.001)
    s = e.stats()
    e.stop()
    assert got == 64 and s["batches"] <= 4


def test_backpressure_refuses_beyond_max_queue(native, model):
    e = make_engine(native, max_queue=100, delay_us=50000, max_batch=10)
    e.load_model(int(model.kind), model.W, model.b, model.label_json())
    sink = native.PySink()
    results = [e.submit(np.ones(4), i, sink) for i in range(400)]
    assert results.count(-1) > 0 and results.count(1) >= 100  # queue full -> refused, not dropped
    assert e.stats()["rejected"] == results.count(-1)
    e.stop()


def test_backpressure_http_503(native, model, tmp_path):
    """Native server: a refused submit answers 503 + Retry-After (the request was not queued)."""
    import socket

    e = make_engine(native, max_queue=1, delay_us=200000, max_batch=1)
    e.load_model(int(model.kind), model.W, model.b, model.label_json())
    sc = native.ServerConfig()
    sc.port = 0
    sc.io_threads = 1
    sc.feature_names = ["sepal_length", "sepal_width", "petal_length", "petal_width"]
    srv = native.HttpServer(e, sc)
    srv.start()
    body = b'{"sepal_length":1,"sepal_width":2,"petal_length":3,"petal_width":4}'
    req = (b"POST /predict HTTP/1.1\r\nHost: x\r\nContent-Type: application/json\r\nContent-Length: %d\r\n\r\n%s"
           % (len(body), body))
    socks = []
    try:
        for _ in range(6):
            s = socket.create_connection(("127.0.0.1", srv.port()))
            s.sendall(req)
            socks.append(s)
        codes = []
        for s in socks:
            s.settimeout(10)
            codes.append(s.recv(65536).split(b" ")[1])
        assert b"503" in codes and b"200" in codes
        assert srv.stats()["errors"] >= 1
    finally:
        for s in socks:
            s.close()
        srv.stop()
        e.stop()


def test_direct_wide_knobs_reach_the_engine_config(native, monkeypatch):
    """MLAPI_DIRECT_WIDE / MLAPI_DIRECT_WIDE_MAX_WEIGHT_BYTES (wide batches as AQL packets into the
    engine's HSA queue, csrc/runtime/engine.cpp launch_batch) parse from the environment and the
    native EngineConfig carries them; defaults: on, for W <= 256 KiB."""
    from mlapi_amd.utils.config import Config

    ec = native.EngineConfig()
    assert ec.direct_wide is True and ec.direct_wide_max_weight_bytes == 256 << 10
    cfg = Config.from_env(device="cpu")
    assert cfg.direct_wide is True and cfg.direct_wide_max_weight_bytes == 256 << 10
    monkeypatch.setenv("MLAPI_DIRECT_WIDE", "0")
    monkeypatch.setenv("MLAPI_DIRECT_WIDE_MAX_WEIGHT_BYTES", "1024")
    cfg = Config.from_env(device="cpu")
    assert cfg.direct_wide is False and cfg.direct_wide_max_weight_bytes == 1024
    ec.direct_wide = cfg.direct_wide
    ec.direct_wide_max_weight_bytes = cfg.direct_wide_max_weight_bytes
    e = native.Engine(ec)  # the CPU backend ignores both
    e.stop()
