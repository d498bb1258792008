"""Wide models on the /predict hot path: the engine routes binary models to the bf16 GEMV kernel
and multiclass models to the MFMA gemm_softmax kernel (reference call sites
/root/reference/main.py:21-22). Every result is compared with the float64 oracle evaluated on the
bf16-rounded inputs the kernel actually sees (tolerance table: labels exact unless the top-2
logit margin is < 1e-3, p_max rel 1e-4)."""
import json
import socket
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from mlapi_amd.models.linear import Kind, LinearModel

pytestmark = pytest.mark.gpu

DT = {"f64": 0, "f32": 1, "bf16": 2}


def bf16_round(a):
    u = np.ascontiguousarray(np.asarray(a, dtype=np.float32)).view(np.uint32).astype(np.uint64)
    u = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return u.astype(np.uint32).view(np.float32).astype(np.float64)


def rounded_oracle(m: LinearModel, X, xdt):
    """The model and rows as the kernel reads them."""
    if xdt == "bf16":
        Wr, Xr, br = bf16_round(m.W), bf16_round(X), m.b.astype(np.float32).astype(np.float64)
    elif xdt == "f32":
        Wr, Xr, br = (a.astype(np.float32).astype(np.float64) for a in (m.W, X, m.b))
    else:
        Wr, Xr, br = m.W, np.asarray(X, dtype=np.float64), m.b
    return LinearModel(Wr, br, m.classes, m.kind), Xr


def check(m: LinearModel, X, idx, p, xdt, rtol=1e-4):
    om, Xr = rounded_oracle(m, X, xdt)
    ridx, rp = om.predict_max(Xr)
    z = om.decision_function(Xr)
    if z.ndim == 1:
        margin = np.abs(z)
    else:
        zs = np.sort(z, axis=1)
        margin = zs[:, -1] - zs[:, -2]
    bad = (idx != ridx) & (margin > 1e-3)
    assert not bad.any(), f"{bad.sum()} label mismatches away from ties"
    np.testing.assert_allclose(p, rp, rtol=rtol, atol=1e-6)


def _engine(native, **kw):
    cfg = native.EngineConfig()
    cfg.device = 0
    for k, v in kw.items():
        setattr(cfg, k, v)
    return native.Engine(cfg)


@pytest.mark.parametrize("stage", [False, True])
@pytest.mark.parametrize("F,K,kind,wide,path", [
    (256, 2, Kind.BINARY, "bf16", "gemv"),
    (256, 2, Kind.BINARY_SOFTMAX, "bf16", "gemv"),
    (100, 2, Kind.BINARY, "bf16", "gemv"),        # F padded to 104
    (256, 2, Kind.BINARY, "f32", "wide"),     # f32 storage, f64 accumulation (f32_gemv: the GEMV)
    (256, 1000, Kind.MULTINOMIAL, "bf16", "gemm"),
    (256, 50, Kind.OVR, "bf16", "gemm"),
    (100, 10, Kind.MULTINOMIAL, "bf16", "gemm"),  # F padded to 128
    (512, 300, Kind.MULTINOMIAL, "bf16", "gemm"),
    (1024, 200, Kind.MULTINOMIAL, "bf16", "gemm"),  # row-group kernel (F looped in slices)
    (700, 30, Kind.OVR, "bf16", "gemm"),            # F padded to 1024
    (48, 40, Kind.MULTINOMIAL, "f32", "wide"),     # f32 storage, f64 MFMA accumulation (linear_wide.h)
    (256, 1000, Kind.MULTINOMIAL, "f32", "wide"),
    (100, 10, Kind.OVR, "f32", "wide"),
    (700, 30, Kind.MULTINOMIAL, "f32", "wide"),
    (3000, 2, Kind.BINARY, "f32", "wide"),          # f32 binary beyond the GEMV's F = 2048
    (48, 40, Kind.OVR, "f64", "wide"),
    (256, 2, Kind.BINARY_SOFTMAX, "f64", "wide"),
    (1024, 300, Kind.MULTINOMIAL, "f64", "wide"),   # feature splits over blocks
    (5000, 20, Kind.MULTINOMIAL, "bf16", "wide"),   # beyond the bf16 kernels' F = 4096: f32 storage
])
def test_engine_wide_paths_match_oracle(native, F, K, kind, wide, path, stage):
    m = LinearModel.random(F, K, seed=F + K, kind=kind)
    e = _engine(native, max_batch=256, max_features=F, wide_dtype=DT[wide], stage_wide=stage)
    try:
        e.load_model(int(m.kind), m.W, m.b, m.label_json())
        assert e.model_path() == path
        X = np.random.default_rng(F * K).standard_normal((3000, F))
        idx, p, st = e.predict(X)
        assert (st == 0).all()
        xdt = ("f32" if wide == "bf16" else wide) if path == "wide" else wide
        # WIDE accumulates in f64: only the rounding of the stored inputs separates it from the oracle
        check(m, X, idx, p, xdt, rtol=1e-11 if path == "wide" else 1e-4)
        s = e.stats()
        assert s["path_batches"][path] == s["batches"] and s["requests"] == 3000
    finally:
        e.stop()


@pytest.mark.parametrize("wide", ["bf16", "f32"])
def test_engine_small_multiclass_batches_take_split_kernel(native, wide):
    """Serving-sized multiclass batches (1..32 rows): bf16 runs the class-split kernel
    (linear_split.h), f32 the f64-accumulating wide kernel (host-merged records up to 16 rows);
    results match the oracle batch by batch."""
    F, K = 256, 1000
    m = LinearModel.random(F, K, seed=5, kind=Kind.MULTINOMIAL)
    e = _engine(native, max_batch=256, max_features=F, wide_dtype=DT[wide])
    try:
        e.load_model(int(m.kind), m.W, m.b, m.label_json())
        assert e.model_path() == ("wide" if wide == "f32" else "gemm")
        rng = np.random.default_rng(9)
        for n in (1, 2, 5, 8, 16, 31, 32, 33):
            X = rng.standard_normal((n, F))
            idx, p, st = e.predict(X)
            assert (st == 0).all()
            check(m, X, idx, p, wide, rtol={"f32": 1e-11, "bf16": 1e-4}[wide])
    finally:
        e.stop()


@pytest.mark.parametrize("wide", ["bf16", "f32"])
@pytest.mark.parametrize("K", [2, 1000])
def test_bar_staged_rows_match_zero_copy(native, wide, K):
    """Small wide batches written into device HBM through the BAR (bar_rows) give the same results
    as zero-copy host reads, across slot reuse (uncached BAR buffers: no stale L2 lines)."""
    F = 256
    m = LinearModel.random(F, K, seed=K + 1, kind=Kind.BINARY if K == 2 else Kind.MULTINOMIAL)
    X = np.random.default_rng(3).standard_normal((400, F))
    outs = {}
    for bar in (32, 0):
        e = _engine(native, max_batch=256, max_features=F, wide_dtype=DT[wide], bar_rows=bar)
        try:
            e.load_model(int(m.kind), m.W, m.b, m.label_json())
            res = [e.predict(X[i:i + 7]) for i in range(0, 400, 7)]
            idx = np.concatenate([r[0] for r in res])
            p = np.concatenate([r[1] for r in res])
            assert all((r[2] == 0).all() for r in res)
            st = e.stats()
            assert (st["bar_batches"] > 0) == (bar > 0 and st["direct_dispatch"] and st["direct_device_kernargs"])
            outs[bar] = (idx, p)
        finally:
            e.stop()
    np.testing.assert_array_equal(outs[32][0], outs[0][0])
    np.testing.assert_array_equal(outs[32][1], outs[0][1])
    check(m, X, outs[32][0], outs[32][1], wide, rtol=1e-11 if wide == "f32" else 1e-4)

@pytest.mark.parametrize("wide", ["bf16", "f32"])
@pytest.mark.parametrize("F,kind", [(256, Kind.BINARY), (64, Kind.BINARY_SOFTMAX), (1024, Kind.BINARY)])
def test_direct_dispatched_gemv_batches_match_hip_launch(native, wide, F, kind):
    """Record-completing binary GEMV batches (>= gemv_record_rows rows) dispatched into the engine's
    HSA queue (mlapi_gemv_* entries, unordered packets) match hipLaunchKernel of the same kernel;
    batch-1 keeps the signal-kernel path on the HIP stream alongside."""
    from mlapi_amd._build import hsaco_path

    m = LinearModel.random(F, 2, seed=F, kind=kind)
    rng = np.random.default_rng(F)
    Xs = [rng.standard_normal((n, F)) for n in (1, 2, 3, 8, 1, 64, 250, 5)]
    outs = {}
    for mode in ("direct", "direct_nobar", "hip"):
        e = _engine(native, max_batch=256, max_features=F, wide_dtype=DT[wide], f32_gemv=True,
                    hsaco_path=str(hsaco_path()), direct_wide=(mode != "hip"),
                    direct_wide_max_weight_bytes=1 << 30, bar_rows=0 if mode == "direct_nobar" else 32)
        try:
            e.load_model(int(m.kind), m.W, m.b, m.label_json())
            assert e.model_path() == "gemv"
            res = [e.predict(X) for X in Xs]
            assert all((r[2] == 0).all() for r in res)
            st = e.stats()
            assert st["direct_dispatch"], "the serving code object did not load"
            assert (st["direct_wide_batches"] > 0) == (mode != "hip")
            outs[mode] = (np.concatenate([r[0] for r in res]), np.concatenate([r[1] for r in res]))
        finally:
            e.stop()
    for mode in ("direct", "direct_nobar"):
        np.testing.assert_array_equal(outs[mode][0], outs["hip"][0])
        np.testing.assert_allclose(outs[mode][1], outs["hip"][1], rtol=1e-6, atol=0)
    check(m, np.concatenate(Xs), outs["direct"][0], outs["direct"][1], wide)


@pytest.mark.parametrize("wide", ["bf16", "f32"])
@pytest.mark.parametrize("F,K,kind", [(256, 1000, Kind.MULTINOMIAL), (64, 40, Kind.OVR), (512, 130, Kind.MULTINOMIAL)])
def test_direct_dispatched_split_batches_match_hip_launch(native, wide, F, K, kind):
    """Class-split batches written as AQL packets into the engine's own HSA queue (the serving code
    object's mlapi_split_* entries, barrier-ordered, kernarg + BAR rows under one HDP flush) give
    the results of hipLaunchKernel of the same kernel (labels exactly), for host-merged (<= 32 rows)
    and in-kernel-merged batches, with and without BAR-staged rows."""
    from mlapi_amd._build import hsaco_path

    m = LinearModel.random(F, K, seed=F + K, kind=kind)
    rng = np.random.default_rng(K)
    sizes = [1, 2, 7, 16, 31, 32, 33, 64, 200, 5, 1]
    Xs = [rng.standard_normal((n, F)) for n in sizes]
    outs = {}
    for mode in ("direct", "direct_nobar", "hip"):
        e = _engine(native, max_batch=256, max_features=F, wide_dtype=DT[wide],
                    hsaco_path=str(hsaco_path()), direct_wide=(mode != "hip"),
                    direct_wide_max_weight_bytes=1 << 30, bar_rows=0 if mode == "direct_nobar" else 32)
        try:
            e.load_model(int(m.kind), m.W, m.b, m.label_json())
            res = [e.predict(X) for X in Xs]
            assert all((r[2] == 0).all() for r in res)
            st = e.stats()
            assert st["direct_dispatch"], "the serving code object did not load"
            if mode == "hip":
                assert st["direct_wide_batches"] == 0
            else:  # f32: every batch is the wide kernel; bf16: beyond split_max_rows the tiles kernel
                assert st["direct_wide_batches"] > 0
                assert wide != "f32" or st["direct_wide_batches"] == st["batches"]
            outs[mode] = (np.concatenate([r[0] for r in res]), np.concatenate([r[1] for r in res]))
        finally:
            e.stop()
    # labels identical; p_max to the last bits only: the engine's batches are whatever rows were
    # queued when the batcher looked, and a row's splits merge on the host (<= 32-row batches) or
    # in the kernel (larger ones), whose float orders differ by an ulp or two
    for mode in ("direct", "direct_nobar"):
        np.testing.assert_array_equal(outs[mode][0], outs["hip"][0])
        np.testing.assert_allclose(outs[mode][1], outs["hip"][1], rtol=1e-6, atol=0)
    check(m, np.concatenate(Xs), outs["direct"][0], outs["direct"][1], wide,
          rtol=1e-11 if wide == "f32" else 1e-4)




def _post(port, bodies):
    out = []
    s = socket.create_connection(("127.0.0.1", port), timeout=30)
    try:
        for body in bodies:
            s.sendall(b"POST /predict HTTP/1.1\r\nHost: t\r\nContent-Type: application/json\r\n"
                      b"Content-Length: %d\r\n\r\n%s" % (len(body), body))
            buf = b""
            while b"\r\n\r\n" not in buf:
                buf += s.recv(65536)
            head, rest = buf.split(b"\r\n\r\n", 1)
            n = int([l.split(b":")[1] for l in head.split(b"\r\n") if l.lower().startswith(b"content-length")][0])
            while len(rest) < n:
                rest += s.recv(65536)
            out.append((int(head.split()[1]), rest[:n]))
    finally:
        s.close()
    return out


@pytest.mark.parametrize("K,kind", [(2, Kind.BINARY), (1000, Kind.MULTINOMIAL)])
def test_native_server_wide_model_every_response(native, K, kind):
    from mlapi_amd.serve.server import NativeServer
    from mlapi_amd.utils.config import Config

    F = 256
    names = [f"f{i}" for i in range(F)]
    m = LinearModel.random(F, K, seed=K, kind=kind, labels=[f"c{i}" for i in range(K)])
    cfg = Config.from_env(port=0, device="cuda:0", feature_names=names, reload="off", missing_model="keep",
                          model_path="/nonexistent/wide.pkl", io_threads=4)
    srv = NativeServer(cfg)
    srv.runtime.handle.load(m)
    srv.start()
    try:
        rng = np.random.default_rng(5)
        X = rng.standard_normal((1024, F))
        bodies = [json.dumps(dict(zip(names, map(float, row))), separators=(",", ":")).encode() for row in X]
        with ThreadPoolExecutor(16) as ex:  # 16 concurrent connections -> coalesced batches
            parts = list(ex.map(lambda j: _post(srv.port, bodies[j::16]), range(16)))
        res = [None] * len(bodies)
        for j, part in enumerate(parts):
            for i, r in enumerate(part):
                res[j + 16 * i] = r
        assert all(st == 200 for st, _ in res)
        got = [json.loads(b) for _, b in res]
        idx = np.array([int(g["prediction"][1:]) for g in got])
        p = np.array([g["probability"] for g in got])
        # the default wide dtype is f32 (bf16 is opt-in): the f64-accumulating wide kernel
        check(m, X, idx, p, "f32", rtol=1e-11)
        st = srv.runtime.handle.stats()
        path = "wide"
        assert st["path_batches"][path] >= 1 and st["path_batches"]["generic"] == 0
        assert st["batches"] < st["requests"]
        assert srv.http.stats()["fast"] >= 1024  # no request fell back to the Python slow path
    finally:
        srv.stop()


@pytest.mark.parametrize("F,K,kind", [(4, 3, Kind.MULTINOMIAL), (256, 2, Kind.BINARY), (256, 1000, Kind.MULTINOMIAL)])
def test_idle_engine_fast_path(native, F, K, kind):
    """One client, one request at a time: the engine is idle at every submit, so the IO thread
    launches the row itself (Engine::run_idle; wide models only because a single connection is
    open). Bodies are identical to the queued path's (idle_inline_rows=0) and match the oracle."""
    from mlapi_amd.serve.server import NativeServer
    from mlapi_amd.utils.config import Config

    names = [f"f{i}" for i in range(F)]
    m = LinearModel.random(F, K, seed=F + K, kind=kind, labels=[f"c{i}" for i in range(K)])
    X = np.round(np.random.default_rng(11).standard_normal((200, F)), 3)
    bodies = [json.dumps(dict(zip(names, map(float, row))), separators=(",", ":")).encode() for row in X]
    out = {}
    for rows in (8, 0):
        # resident off: SMALL models (F = 4) would otherwise take the resident kernel's rings
        # (tests/test_resident.py), never the idle path this test is about
        cfg = Config.from_env(port=0, device="cuda:0", feature_names=names, reload="off", missing_model="keep",
                              model_path="/nonexistent/idle.pkl", io_threads=2, idle_inline_rows=rows,
                              resident="off")
        srv = NativeServer(cfg)
        srv.runtime.handle.load(m)
        srv.start()
        try:
            res = _post(srv.port, bodies)
            assert all(st == 200 for st, _ in res)
            out[rows] = [b for _, b in res]
            st = srv.runtime.handle.stats()
            if rows:
                assert st["idle_batches"] >= 150, st  # nearly every request took the idle path
            else:
                assert st["idle_batches"] == 0
            assert st["requests"] == len(bodies)
        finally:
            srv.stop()
    assert out[8] == out[0]
    got = [json.loads(b) for b in out[8]]
    idx = np.array([int(g["prediction"][1:]) for g in got])
    p = np.array([g["probability"] for g in got])
    if F == 4:  # fp64 small path: exact sklearn parity
        ridx, rp = m.predict_max(X)
        np.testing.assert_array_equal(idx, ridx)
        np.testing.assert_allclose(p, rp, rtol=1e-12, atol=0)
    else:
        check(m, X, idx, p, "f32", rtol=1e-11 if K > 2 else 1e-5)


@pytest.mark.parametrize("F,K,kind", [(256, 2, Kind.BINARY), (256, 40, Kind.MULTINOMIAL),
                                      (1024, 1000, Kind.MULTINOMIAL), (4096, 40, Kind.OVR)])
def test_native_server_f64_wide_models(native, F, K, kind):
    """wide_dtype = f64 (the reference's dtype) over HTTP: every body is the engine's own answer
    rendered byte for byte, labels are the float64 oracle's away from 1e-9 ties and p is within
    rel 1e-12 of it; every batch ran the WIDE kernel (never GENERIC)."""
    from mlapi_amd.serve.loadgen import render_response
    from mlapi_amd.serve.server import NativeServer
    from mlapi_amd.utils.config import Config

    names = [f"f{i}" for i in range(F)]
    m = LinearModel.random(F, K, seed=F + K, kind=kind, labels=[f"c{i}" for i in range(K)])
    cfg = Config.from_env(port=0, device="cuda:0", feature_names=names, reload="off", missing_model="keep",
                          model_path="/nonexistent/wide64.pkl", io_threads=4, wide_dtype="f64")
    srv = NativeServer(cfg)
    srv.runtime.handle.load(m)
    srv.start()
    try:
        X = np.round(np.random.default_rng(F).standard_normal((256, F)), 3)
        bodies = [json.dumps(dict(zip(names, map(float, row))), separators=(",", ":")).encode() for row in X]
        with ThreadPoolExecutor(8) as ex:
            parts = list(ex.map(lambda j: _post(srv.port, bodies[j::8]), range(8)))
        res = [None] * len(bodies)
        for j, part in enumerate(parts):
            for i, r in enumerate(part):
                res[j + 8 * i] = r
        assert all(st == 200 for st, _ in res)
        eidx, ep, est = srv.runtime.handle.engine.predict(X)
        assert (est == 0).all()
        for r, (_, body) in enumerate(res):
            assert body == render_response(m, eidx[r], ep[r]), r
        ridx, rp = m.predict_max(X)
        z = m.decision_function(X)
        margin = np.abs(z) if z.ndim == 1 else np.diff(np.sort(z, axis=1)[:, -2:], axis=1)[:, 0]
        assert not ((eidx != ridx) & (margin > 1e-9)).any()
        np.testing.assert_allclose(ep, rp, rtol=1e-12, atol=0)
        st = srv.runtime.handle.stats()
        assert st["path_batches"]["wide"] >= 1 and st["path_batches"]["generic"] == 0
    finally:
        srv.stop()
