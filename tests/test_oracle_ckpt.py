"""T1 (oracle vs sklearn) and T2 (checkpoint formats) — CPU only."""
import io
import os
import pickle
import pickletools

import numpy as np
import pytest
from sklearn.linear_model import LogisticRegression, SGDClassifier

from mlapi_amd.ckpt import (TrainState, UnsafeCheckpointError, export_sklearn_pickle, load_model, load_native,
                            load_sklearn_pickle, save_native)
from mlapi_amd.models.linear import Kind, LinearModel


def _sk_from(W, b, classes, **kw):
    m = LogisticRegression(**kw)
    m.coef_, m.intercept_, m.classes_ = np.asarray(W, float), np.asarray(b, float), np.asarray(classes)
    return m


CASES = [
    ("binary", dict(), 1, 2, Kind.BINARY),
    ("multinomial", dict(), 3, 3, Kind.MULTINOMIAL),
    ("ovr_liblinear", dict(solver="liblinear"), 4, 4, Kind.OVR),
    ("many", dict(), 12, 12, Kind.MULTINOMIAL),
]


@pytest.mark.parametrize("name,kw,rows,ncls,kind", CASES, ids=[c[0] for c in CASES])
def test_oracle_matches_sklearn(name, kw, rows, ncls, kind):
    rng = np.random.default_rng(rows)
    W, b = rng.normal(size=(rows, 6)) * 3, rng.normal(size=rows)
    sk = _sk_from(W, b, np.array([f"c{i}" for i in range(ncls)], dtype=object), **kw)
    m = load_sklearn_pickle(pickle.dumps(sk))
    assert m.kind == kind
    X = rng.normal(size=(500, 6)) * 4
    X[:5] = 0  # ties at z = b
    np.testing.assert_array_equal(m.predict(X), sk.predict(X))
    np.testing.assert_allclose(m.predict_proba(X), sk.predict_proba(X), rtol=1e-13, atol=1e-15)
    idx, p = m.predict_max(X)
    np.testing.assert_allclose(p, sk.predict_proba(X).max(1), rtol=1e-13)


def test_oracle_ties_first_max():
    m = LinearModel(np.zeros((3, 2)), np.array([1.0, 1.0, 0.0]), np.array(["a", "b", "c"], dtype=object),
                    Kind.MULTINOMIAL)
    assert m.predict([[0.3, 0.4]])[0] == "a"
    mb = LinearModel(np.zeros((1, 2)), np.zeros(1), np.array(["neg", "pos"], dtype=object), Kind.BINARY)
    assert mb.predict([[1.0, 2.0]])[0] == "neg"  # z == 0 -> class 0 (sklearn: z > 0)


def test_oracle_rejects_nonfinite():
    m = LinearModel.random(4, 3)
    with pytest.raises(ValueError):
        m.predict([[np.nan, 1, 2, 3]])


def test_engine_cpu_backend_matches_oracle(native):
    cfg = native.EngineConfig()
    cfg.device = -1
    for kind, K in ((Kind.BINARY, 1), (Kind.BINARY_SOFTMAX, 1), (Kind.MULTINOMIAL, 5), (Kind.OVR, 4)):
        m = LinearModel.random(7, 2 if K == 1 else K, seed=K, kind=kind)
        e = native.Engine(cfg)
        e.load_model(int(m.kind), m.W, m.b, m.label_json())
        X = np.random.default_rng(0).normal(size=(300, 7)) * 3
        idx, p, st = e.predict(X)
        e.stop()
        ridx, rp = m.predict_max(X)
        np.testing.assert_array_equal(idx, ridx)
        np.testing.assert_allclose(p, rp, rtol=1e-14)
        assert (st == 0).all()


# ------------------------------------------------------------------ T2 checkpoint formats
def test_loads_reference_style_iris_pickle(iris_pickle_bytes, iris_data):
    m = load_sklearn_pickle(iris_pickle_bytes)
    _, Xte, _, yte = iris_data
    assert m.kind == Kind.MULTINOMIAL and m.n_features == 4
    assert m.score(Xte, yte) == 0.9666666666666667  # Logistic Regression.ipynb:13


@pytest.mark.parametrize("protocol", [0, 1, 2, 3, 4, 5])
def test_all_pickle_protocols(iris_sklearn_model, protocol):
    m = load_sklearn_pickle(pickle.dumps(iris_sklearn_model, protocol=protocol))
    np.testing.assert_array_equal(m.W, iris_sklearn_model.coef_)


def test_numpy1x_spelling_and_old_sklearn_module(iris_sklearn_model):
    """Reference-era files: numpy 1.20 writes numpy.core.*, sklearn < 0.22 wrote ...linear_model.logistic."""
    data = pickle.dumps(iris_sklearn_model, protocol=2)
    data = data.replace(b"numpy._core.multiarray", b"numpy.core.multiarray")
    data = data.replace(b"sklearn.linear_model._logistic", b"sklearn.linear_model.logistic")
    m = load_sklearn_pickle(data)
    np.testing.assert_array_equal(m.b, iris_sklearn_model.intercept_)


def test_sgdclassifier_log_loss():
    rng = np.random.default_rng(0)
    X, y = rng.normal(size=(200, 3)), rng.integers(0, 3, 200)
    sk = SGDClassifier(loss="log_loss", random_state=0).fit(X, y)
    m = load_sklearn_pickle(pickle.dumps(sk))
    assert m.kind == Kind.OVR
    np.testing.assert_allclose(m.predict_proba(X), sk.predict_proba(X), rtol=1e-12)


@pytest.mark.parametrize("payload", [
    b"cos\nsystem\n(S'echo hi'\ntR.",
    b"cbuiltins\neval\n(S'1+1'\ntR.",
    pickle.dumps({"a": 1}),
    b"\x80\x04\x95\x1a\x00\x00\x00\x00\x00\x00\x00\x8c\x08builtins\x94\x8c\x04exec\x94\x93\x94.",
])
def test_restricted_unpickler_refuses(payload):
    with pytest.raises((UnsafeCheckpointError, pickle.UnpicklingError)):
        load_sklearn_pickle(payload)


def test_export_round_trip_into_real_sklearn(iris_sklearn_model, iris_data):
    m = load_sklearn_pickle(pickle.dumps(iris_sklearn_model))
    data = export_sklearn_pickle(m)
    ops = {op.name for op, _, _ in pickletools.genops(data)}
    assert "REDUCE" in ops and "BUILD" in ops
    assert b"numpy.core.multiarray" in data  # readable by the reference-era numpy 1.20
    with pytest.warns(Warning):  # sklearn version mismatch warning (0.24.1 -> installed)
        sk2 = pickle.loads(data)  # our own output, trusted
    _, Xte, _, yte = iris_data
    np.testing.assert_array_equal(sk2.predict(Xte), iris_sklearn_model.predict(Xte))
    np.testing.assert_allclose(sk2.predict_proba(Xte), iris_sklearn_model.predict_proba(Xte), rtol=1e-14)
    assert load_sklearn_pickle(data).kind == Kind.MULTINOMIAL


def test_native_format_round_trip_with_train_state(tmp_path):
    m = LinearModel.random(5, 4, seed=3, labels=["w", "x", "y", "z"])
    st = TrainState(step=17, epoch=2, data_cursor=4096, opt={"mom": np.arange(24.0)},
                    rng_state=np.array([1, 2, 3], dtype=np.uint64), config={"lr": 0.1}, extra={"note": "x"})
    p = tmp_path / "m.safetensors"
    save_native(p, m, st)
    m2, st2 = load_native(p)
    np.testing.assert_array_equal(m2.W, m.W)
    assert list(m2.classes) == ["w", "x", "y", "z"] and m2.kind == m.kind
    assert (st2.step, st2.epoch, st2.data_cursor, st2.config) == (17, 2, 4096, {"lr": 0.1})
    np.testing.assert_array_equal(st2.opt["mom"], np.arange(24.0))
    assert load_model(p).n_features == 5


def test_load_model_dispatches_on_format(tmp_path, iris_pickle_bytes):
    p = tmp_path / "LRClassifier.pkl"
    p.write_bytes(iris_pickle_bytes)
    assert load_model(p).kind == Kind.MULTINOMIAL
