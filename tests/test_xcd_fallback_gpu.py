"""The XCD-local split merge (linear_split.h / gemm_softmax.hip xcd_verify) never answers from a
misplaced merge: a row whose merging block read a partial written on another XCD comes back as
XCD_BAD_IDX, the engine fails it (ST_DEVICE_ERROR, counted in stats()["xcd_errors"]) and switches
the protocol off for the device, so the next batches take the agent-scope merge and are right
again. The misplacement is injected (xcd_local_inject: the next launch reports every merged row as
misplaced). Also: class-split batches above one launch's 2048-row cap run in row chunks instead of
throwing. The engine's class-split path serves bf16 models (split_max_rows)."""
import numpy as np
import pytest

from mlapi_amd.models.linear import LinearModel

pytestmark = pytest.mark.gpu

ST_OK, ST_DEVICE_ERROR = 0, 4


def _engine(native, **kw):
    cfg = native.EngineConfig()
    cfg.device = 0
    for k, v in kw.items():
        setattr(cfg, k, v)
    return native.Engine(cfg)


def _check(m, X, idx, p, rtol=1e-4):
    from mlapi_amd.serve.loadgen import bf16_oracle

    om, Xb = bf16_oracle(m, X)  # the model and rows as the bf16 kernel reads them
    ridx, rp = om.predict_max(Xb)
    z = om.decision_function(Xb)
    margin = np.diff(np.sort(z, axis=1)[:, -2:], axis=1)[:, 0]
    assert not ((idx != ridx) & (margin > 1e-3)).any()
    np.testing.assert_allclose(p, rp, rtol=rtol, atol=0)


def test_misplaced_xcd_merge_fails_rows_then_falls_back(native):
    F, K = 256, 200  # 4 class blocks: an in-kernel split merge
    m = LinearModel.random(F, K, seed=21)
    e = _engine(native, max_batch=64, max_features=F, wide_dtype=2, split_max_rows=64, host_merge_rows=0)
    try:
        e.load_model(int(m.kind), m.W, m.b, m.label_json())
        rng = np.random.default_rng(5)
        X = np.round(rng.standard_normal((40, F)), 3)
        idx, p, st = e.predict(X)  # first launch: the placement probe decides the protocol
        assert (st == ST_OK).all()
        _check(m, X, idx, p)
        if native.xcd_placement_state(0) != 1:
            pytest.skip("XCD-local merge is off on this device (placement probe)")
        e0 = native.xcd_local_errors(0)
        native.xcd_local_inject(1)
        idx, p, st = e.predict(X)
        # the injected launch's rows fail (never a silently wrong answer); rows the batcher put in
        # later batches already take the agent-scope merge and are right
        bad = st == ST_DEVICE_ERROR
        assert bad.any() and ((st == ST_OK) | bad).all(), st
        ok = st == ST_OK
        if ok.any():
            _check(m, X[ok], idx[ok], p[ok])
        assert e.stats()["xcd_errors"] == int(bad.sum())
        assert native.xcd_local_errors(0) == e0 + 1 and native.xcd_placement_state(0) == 2
        idx, p, st = e.predict(X)  # agent-scope merge from now on
        assert (st == ST_OK).all()
        _check(m, X, idx, p)
    finally:
        native.xcd_local_inject(0)
        native.xcd_local_reset(0)  # later tests of this process probe the placement afresh
        e.stop()


def test_split_batches_above_one_launch_run_in_chunks(native):
    F, K = 128, 40
    m = LinearModel.random(F, K, seed=8)
    e = _engine(native, max_batch=4096, max_features=F, wide_dtype=2, split_max_rows=4096, max_wait_us=50000)
    try:
        e.load_model(int(m.kind), m.W, m.b, m.label_json())
        X = np.round(np.random.default_rng(2).standard_normal((3000, F)), 3)
        idx, p, st = e.predict(X)
        assert (st == ST_OK).all()
        _check(m, X, idx, p)
        assert e.stats()["batch_hist"][11] >= 1  # at least one batch of >= 2048 rows went through
    finally:
        e.stop()
