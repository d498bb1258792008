"""T0: the reference's HTTP contract (Appendix A) against our FastAPI app.

Golden responses in tests/fixtures/reference_contract.json were captured by running an
unmodified copy of the reference main.py (tools/capture_reference_contract.py); every case here
must be byte-identical (status, content type, body).
"""
import json
import os
import pickle
import time

import numpy as np
import pytest
from fastapi.testclient import TestClient

from conftest import FIXTURES

GOLDEN = json.loads((FIXTURES / "reference_contract.json").read_text())
A1 = {"sepal_length": 5.1, "sepal_width": 3.5, "petal_length": 1.4, "petal_width": 0.2}


def _client(**cfg):
    from mlapi_amd.api.app import create_app
    from mlapi_amd.utils.config import Config

    app = create_app(Config.from_env(device="cpu", **cfg))
    return TestClient(app, raise_server_exceptions=False)


def _request(client, req):
    kw = {}
    if "json" in req:
        kw["json"] = req["json"]
    if "content" in req:
        kw["content"] = req["content"].encode()
    if "headers" in req:
        kw["headers"] = req["headers"]
    return client.request(req["method"], req["path"], **kw)


def assert_same_body(got: str, want: str, status: int) -> None:
    """Byte equality, except the last ulps of a 200 probability.

    Logits are bit-identical to numpy/OpenBLAS (same FMA chain), but numpy's SIMD exp and the
    libm/ocml exp differ in the last ulp for ~5% of arguments, so the probability's final digit
    may differ; everything else (label, key order, float formatting) must match exactly.
    """
    if status != 200 or got == want:
        assert got == want
        return
    g, w = json.loads(got), json.loads(want)
    assert list(g) == list(w) and g["prediction"] == w["prediction"]
    assert g["probability"] == pytest.approx(w["probability"], rel=1e-15, abs=0)
    assert got == json.dumps(g, separators=(",", ":"))


@pytest.mark.parametrize("case", [c for c in GOLDEN if c["name"] != "A18"], ids=lambda c: c["name"])
def test_golden_case(iris_cwd, case):
    r = _request(_client(), case["request"])
    assert r.status_code == case["status"]
    assert r.headers.get("content-type") == case["content_type"]
    assert_same_body(r.content.decode(), case["body"], case["status"])


def test_openapi_identical_to_reference(iris_cwd):
    ref = json.loads(next(c for c in GOLDEN if c["name"] == "A18")["body"])
    ours = _client().get("/openapi.json").json()
    assert ours == ref
    assert ours["info"] == {"title": "FastAPI", "version": "0.1.0"}


def test_docs_and_redoc(iris_cwd):
    c = _client()
    for path in ("/docs", "/redoc"):
        r = c.get(path)
        assert r.status_code == 200 and "text/html" in r.headers["content-type"]


def test_missing_checkpoint_is_500_then_recovers(tmp_path, monkeypatch, iris_pickle_bytes):
    """A16: the app starts without LRClassifier.pkl; every request 500s until the file appears."""
    monkeypatch.chdir(tmp_path)
    c = _client()
    r = c.post("/predict", json=A1)
    assert r.status_code == 500 and r.text == "Internal Server Error"
    (tmp_path / "LRClassifier.pkl").write_bytes(iris_pickle_bytes)
    r = c.post("/predict", json=A1)
    assert r.status_code == 200 and r.json()["prediction"] == "Iris-setosa"


def test_hot_swap_by_replacing_the_file(iris_cwd):
    """The reference re-reads the pickle per request (main.py:19): replacing it changes the model."""
    from mlapi_amd.ckpt import export_sklearn_pickle, load_sklearn_pickle

    c = _client()
    assert c.post("/predict", json=A1).json()["prediction"] == "Iris-setosa"
    m = load_sklearn_pickle("LRClassifier.pkl")
    m.b = m.b + np.array([-100.0, 0.0, 100.0])  # force "Iris-virginica"
    time.sleep(0.01)
    export_sklearn_pickle(m, "LRClassifier.pkl")
    r = c.post("/predict", json=A1)
    assert r.json()["prediction"] == "Iris-virginica"
    os.remove("LRClassifier.pkl")
    assert c.post("/predict", json=A1).status_code == 500


def test_backpressure_is_503_with_retry_after(iris_cwd):
    """Not in the reference (no queue): a full engine queue answers 503 instead of queueing forever."""
    c = _client(max_queue=0)
    r = c.post("/predict", json=A1)
    assert r.status_code == 503 and r.headers["retry-after"] == "1"
    assert r.json() == {"detail": "server overloaded, retry later"}


def test_unsafe_checkpoint_is_refused(tmp_path, monkeypatch):
    class Evil:
        def __reduce__(self):
            return (os.system, ("echo pwned > pwned.txt",))

    monkeypatch.chdir(tmp_path)
    (tmp_path / "LRClassifier.pkl").write_bytes(pickle.dumps(Evil()))
    r = _client().post("/predict", json=A1)
    assert r.status_code == 500
    assert not (tmp_path / "pwned.txt").exists()


def test_integer_labels(tmp_path, monkeypatch, iris_data):
    """A17: the reference 500s on integer classes_; we render ints (default) or 500 (parity mode)."""
    from sklearn.linear_model import LogisticRegression

    Xtr, _, ytr, _ = iris_data
    yi = np.searchsorted(np.unique(ytr), ytr)
    (tmp_path / "LRClassifier.pkl").write_bytes(pickle.dumps(LogisticRegression().fit(Xtr, yi)))
    monkeypatch.chdir(tmp_path)
    r = _client().post("/predict", json=A1)
    assert r.status_code == 200 and r.json()["prediction"] == 0
    r = _client(int_labels="error").post("/predict", json=A1)
    assert r.status_code == 500


def test_binary_and_ovr_checkpoints(tmp_path, monkeypatch, iris_data):
    from sklearn.linear_model import LogisticRegression

    Xtr, _, ytr, _ = iris_data
    x = np.array([[A1[k] for k in ("sepal_length", "sepal_width", "petal_length", "petal_width")]])
    monkeypatch.chdir(tmp_path)
    for est, y in ((LogisticRegression(), (ytr == "Iris-setosa").astype(object).astype(str)),
                   (LogisticRegression(solver="liblinear"), ytr)):
        est.fit(Xtr, y)
        (tmp_path / "LRClassifier.pkl").write_bytes(pickle.dumps(est))
        r = _client().post("/predict", json=A1)
        assert r.status_code == 200
        body = r.json()
        assert body["prediction"] == est.predict(x)[0]
        assert body["probability"] == pytest.approx(est.predict_proba(x).max(), rel=1e-13)


def wide_sklearn_checkpoint(tmp_path, F=64, K=10, seed=0, multi_class=None):
    """A wide sklearn LogisticRegression pickle (F features, K classes) in tmp_path, and rows."""
    from sklearn.linear_model import LogisticRegression

    rng = np.random.default_rng(seed)
    X = rng.standard_normal((400, F))
    y = np.array([f"c{i}" for i in range(K)], dtype=object)[np.argmax(X[:, :K] + 0.5 * rng.standard_normal((400, K)), 1)]
    est = LogisticRegression(max_iter=200).fit(X, y) if multi_class is None else \
        LogisticRegression(solver="liblinear").fit(X, y)
    (tmp_path / "LRClassifier.pkl").write_bytes(pickle.dumps(est))
    return est, [f"f{i}" for i in range(F)], np.round(rng.standard_normal((32, F)), 3)


@pytest.mark.parametrize("ovr", [False, True])
def test_wide_sklearn_checkpoint_served_at_float64(tmp_path, monkeypatch, ovr):
    """Models wider than Iris are served at sklearn's precision by default (wide_dtype f64): the
    label is sklearn's predict() and the probability its predict_proba().max() (float64 math; the
    GPU twin is tests/test_serve_wide_gpu.py::test_wide_sklearn_pickle_over_http)."""
    est, names, rows = wide_sklearn_checkpoint(tmp_path, multi_class="ovr" if ovr else None)
    monkeypatch.chdir(tmp_path)
    c = _client(feature_names=names)
    for x in rows:
        r = c.post("/predict", json=dict(zip(names, x.tolist())))
        assert r.status_code == 200, r.text
        body = r.json()
        assert body["prediction"] == est.predict(x[None])[0]
        assert body["probability"] == pytest.approx(est.predict_proba(x[None]).max(), rel=1e-13, abs=0)


# ------------------------------------------------------------------ /files/ (main.py:29-39)
def _files(client, csv: bytes, token="tok", **extra):
    from mlapi_amd.api.multipart import encode_multipart

    fields = {"token": token} if token is not None else {}
    files = {"file": ("data.csv", csv, "text/csv")} if csv is not None else {}
    body, ctype = encode_multipart(fields, files)
    return client.post("/files/", content=body, headers={"content-type": ctype, **extra})


def test_files_echo(iris_cwd, capsys):
    r = _files(_client(), b"a,b\n1.5,x\n2.5,y\n")
    assert r.status_code == 200
    assert r.text == '{"file":{"a":{"0":1.5,"1":2.5},"b":{"0":"x","1":"y"}},"token":"tok"}'
    assert "1.5" in capsys.readouterr().out  # print(df) side effect (main.py:34)


def test_files_missing_fields_422(iris_cwd):
    c = _client()
    r = _files(c, None, token=None)
    assert r.status_code == 422
    assert r.json() == {"detail": [
        {"type": "missing", "loc": ["body", "file"], "msg": "Field required", "input": None},
        {"type": "missing", "loc": ["body", "token"], "msg": "Field required", "input": None}]}
    r = _files(c, b"a\n1.5\n", token="")
    assert r.json()["detail"][0]["loc"] == ["body", "token"]


@pytest.mark.parametrize("csv", [b"a,b\n1,2\n", b"a\nTrue\n", b"a,b\n1.5,\n", b"", b"\xff\xfe,\n"])
def test_files_reference_500_cases(iris_cwd, csv):
    """int / bool / NaN cells, empty and non-UTF-8 uploads are 500 in the reference."""
    assert _files(_client(), csv).status_code == 500


def test_files_lenient_mode(iris_cwd):
    r = _files(_client(files_strict_parity=False), b"a,b\n1,\n")
    assert r.status_code == 200 and r.json()["file"] == {"a": {"0": 1}, "b": {"0": None}}


def test_files_urlencoded(iris_cwd):
    r = _client().post("/files/", content=b"file=a%2Cb%0A1.5%2Cq%0A&token=t",
                       headers={"content-type": "application/x-www-form-urlencoded"})
    assert r.status_code == 200 and r.json() == {"file": {"a": {"0": 1.5}, "b": {"0": "q"}}, "token": "t"}


def test_operational_endpoints(iris_cwd):
    c = _client()
    assert c.get("/healthz").status_code == 200
    r = c.get("/readyz")
    assert r.status_code == 200 and r.json()["ready"] is True
    c.post("/predict", json=A1)
    m = c.get("/metrics").text
    assert "mlapi_requests_total" in m and "mlapi_batch_size_bucket" in m
    assert "mlapi_idle_path_batches_total" in m  # the engine's idle-path counter is exported
    assert c.post("/admin/reload").json()["reloaded"] is True


def test_asgi_fast_path_is_byte_identical_to_the_route(iris_cwd):
    """`uvicorn main:app`'s POST /predict middleware (api/fastpath.py) answers with exactly the
    bytes and headers the FastAPI route sends, and hands every unusual body to the route."""
    import numpy as np

    from mlapi_amd.api.fastpath import PredictFastPath

    fast, route = _client(), _client(asgi_fast_path=False)
    served0 = PredictFastPath.served
    rng = np.random.default_rng(9)
    bodies = [json.dumps(dict(zip(A1, map(float, np.round(r, 2))))) for r in
              rng.normal([5.8, 3.0, 3.8, 1.2], [0.8, 0.4, 1.8, 0.8], (40, 4))]
    bodies += ['{"sepal_length":5,"sepal_width":3,"petal_length":1,"petal_width":0,"extra":[1,{"a":null}]}',
               '{"sepal_length":"5.1","sepal_width":3.5,"petal_length":1.4,"petal_width":0.2}',  # string: route
               '{"sepal_length":5.1,"sepal_width":3.5,"petal_length":1.4}',                       # missing: 422
               '{"sepal_length":NaN,"sepal_width":3.5,"petal_length":1.4,"petal_width":0.2}',     # NaN: route
               '{"sepal_length":1e400,"sepal_width":3.5,"petal_length":1.4,"petal_width":0.2}',   # inf: route
               '[1,2,3]', '', '{"sepal_length":5.1']
    for b in bodies:
        for ctype in ("application/json", "application/vnd.api+json; charset=utf-8", "text/plain"):
            r1 = fast.post("/predict", content=b.encode(), headers={"content-type": ctype})
            r2 = route.post("/predict", content=b.encode(), headers={"content-type": ctype})
            assert (r1.status_code, r1.content, r1.headers.get("content-type"), r1.headers.get("content-length")) == \
                (r2.status_code, r2.content, r2.headers.get("content-type"), r2.headers.get("content-length")), b
    assert PredictFastPath.served - served0 == 2 * 41  # 40 random + the extra-member body, two JSON types
