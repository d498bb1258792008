"""The resident SMALL-path kernel (csrc/include/mlapi/resident.h, ServeRing in csrc/runtime/engine.h):
IO threads write parsed /predict rows into per-thread rings that resident waves poll, and render
the answers from the rings' record arrays - no AQL packet, batcher or completer per request.

Every body is checked byte for byte against the engine's answers (which make_workload first
checks against the float64 oracle). The CPU variants run the same ring protocol with the engine's
supervisor thread playing the kernel (resident="on" on the CPU backend); the GPU variants run the
real kernel (serve_resident.h) on the MI355X."""
import threading

import numpy as np
import pytest

from mlapi_amd.models.linear import Kind, LinearModel

IRIS = ["sepal_length", "sepal_width", "petal_length", "petal_width"]
LABELS = ["Iris-setosa", "Iris-versicolor", "Iris-virginica"]
DEVICES = [pytest.param("cpu", id="cpu"), pytest.param("cuda:0", id="gpu", marks=pytest.mark.gpu)]


def _cfg(device, names, **kw):
    from mlapi_amd.utils.config import Config

    base = {"io_threads": 4, "resident": "on", "reload": "off", "missing_model": "keep",
            "model_path": "/nonexistent/resident.pkl"}
    base.update(kw)
    return Config.from_env(port=0, device=device, feature_names=list(names), **base)


def _stats_delta(s0, s1):
    return {k: s1[k] - s0[k] for k in ("requests", "batches", "idle_batches", "errors", "resident_rows",
                                       "resident_stale", "resident_launches")}


def _serve(native, device, model, names, X, *, conns, threads, reqs_per_conn, rtol=1e-12, **kw):
    from mlapi_amd.serve.loadgen import make_workload
    from mlapi_amd.serve.server import NativeServer

    with NativeServer(_cfg(device, names, **kw)) as srv:
        srv.runtime.handle.load(model)
        reqs, exp = make_workload(srv.runtime.handle.engine, model, names, X, rtol_oracle=rtol, label_margin=1e-5)
        lg = native.Loadgen("127.0.0.1", srv.port, reqs[0].decode(), conns, threads)
        lg.set_workload([r.decode() for r in reqs], [e.decode() for e in exp], 0.0)
        lg.run(20, False)  # warm: every IO thread has opened its ring ...
        if kw.get("resident", "on") != "off" and model.n_features <= 32:
            # ... and the supervisor has relaunched the instance over all of them (rows submitted
            # during a relaunch take the engine queue: correct, but not what this test counts)
            import time

            t_end = time.time() + 5
            while time.time() < t_end:
                st = srv.runtime.handle.stats()
                if st["resident_live"] and st["resident_rings"] >= srv.config.io_threads:
                    break
                time.sleep(0.01)
        s0 = srv.runtime.handle.stats()
        res = lg.run(reqs_per_conn, True)
        lg.close()
        s1 = srv.runtime.handle.stats()
    return res, _stats_delta(s0, s1), s1


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("sleep_us", [0, 3], ids=["spin", "sleep"])
def test_resident_concurrent_bodies_exact(native, device, sleep_us):
    """48 connections over 4 IO threads; the IO threads watch their records by spinning
    (io_ring_spin_us) or by sleeping in epoll_pwait2 (io_ring_sleep_us)."""
    m = LinearModel.random(4, 3, seed=11, labels=LABELS)
    X = np.round(np.random.default_rng(3).standard_normal((512, 4)) * 2 + 4, 1)
    res, d, s1 = _serve(native, device, m, IRIS, X, conns=48, threads=3, reqs_per_conn=200, io_ring_sleep_us=sleep_us)
    n = 48 * 200
    assert res["failed"] == 0 and res["errors"] == 0 and res["body_mismatches"] == 0, res
    assert res["status_counts"] == {200: n}
    assert d["requests"] == n and d["errors"] == 0, d
    # every row went through the rings: no batch was launched for them
    assert d["resident_rows"] == n and d["batches"] == 0, d
    assert s1["resident_live"] and s1["resident_rings"] >= 1, s1


@pytest.mark.parametrize("device", DEVICES)
def test_resident_many_rows_per_ring(native, device):
    """64 connections on ONE IO thread: more rows pending than one poll's window (16 rows of 4
    features) - the window slides as the leading rows are answered."""
    m = LinearModel.random(4, 3, seed=12, labels=LABELS)
    X = np.round(np.random.default_rng(4).standard_normal((256, 4)) * 2 + 4, 1)
    res, d, _ = _serve(native, device, m, IRIS, X, conns=64, threads=2, reqs_per_conn=100, io_threads=1)
    assert res["body_mismatches"] == 0 and res["status_counts"] == {200: 6400}, res
    assert d["resident_rows"] == 6400, d


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("F,K,kind,dtype", [(8, 4, Kind.OVR, "f32"), (2, 1, Kind.BINARY, "f64"),
                                            (32, 16, Kind.MULTINOMIAL, "f64"), (5, 1, Kind.BINARY_SOFTMAX, "f32")])
def test_resident_shapes(native, device, F, K, kind, dtype):
    """Every SMALL-path width class (4 / 8 / 32 lanes per row), kind and dtype, batch = 1 and
    concurrent."""
    names = [f"x{i}" for i in range(F)]
    m = LinearModel.random(F, K if K > 1 else 2, seed=5, kind=kind)
    X = np.random.default_rng(9).standard_normal((128, F))
    rtol = 1e-12 if dtype == "f64" else 1e-5
    res, d, _ = _serve(native, device, m, names, X, conns=1, threads=1, reqs_per_conn=300, rtol=rtol, dtype=dtype)
    assert res["body_mismatches"] == 0 and res["status_counts"] == {200: 300}, res
    assert d["resident_rows"] == 300 and d["idle_batches"] == 0 and d["batches"] == 0, d
    res, d, _ = _serve(native, device, m, names, X, conns=24, threads=2, reqs_per_conn=50, rtol=rtol, dtype=dtype)
    assert res["body_mismatches"] == 0 and res["status_counts"] == {200: 1200}, res
    assert d["resident_rows"] == 1200, d


@pytest.mark.parametrize("device", DEVICES)
def test_resident_skips_wide_models(native, device):
    """A model off the SMALL path (F = 64: the WIDE kernel) never takes the rings: the queued path
    answers it, with the same bytes."""
    F = 64
    names = [f"f{i}" for i in range(F)]
    m = LinearModel.random(F, 2, seed=2)
    X = np.round(np.random.default_rng(4).standard_normal((128, F)), 3)
    res, d, s1 = _serve(native, device, m, names, X, conns=16, threads=2, reqs_per_conn=50, rtol=1e-5)
    assert res["body_mismatches"] == 0 and res["status_counts"] == {200: 800}, res
    assert d["resident_rows"] == 0 and d["requests"] == 800, d
    assert not s1["resident_live"], s1


@pytest.mark.parametrize("device", DEVICES)
def test_resident_off_same_bytes(native, device):
    """resident = off: the batcher answers, byte-identical to the resident kernel's answers."""
    m = LinearModel.random(4, 3, seed=11, labels=LABELS)
    X = np.round(np.random.default_rng(3).standard_normal((256, 4)) * 2 + 4, 1)
    res, d, _ = _serve(native, device, m, IRIS, X, conns=16, threads=2, reqs_per_conn=50, resident="off")
    assert res["body_mismatches"] == 0 and res["status_counts"] == {200: 800}, res
    assert d["resident_rows"] == 0 and d["requests"] == 800, d


@pytest.mark.parametrize("device", DEVICES)
def test_resident_hot_reload_under_load(native, device):
    """Models swapped while clients keep posting: every body is the answer of one of the two
    models for its row (rows parsed for the old version are bounced stale and re-answered by the
    engine queue with the current model), nothing fails, and each reload relaunches the instance."""
    import http.client
    import json

    from mlapi_amd.serve.server import NativeServer

    ma = LinearModel.random(4, 3, seed=1, labels=LABELS)
    mb = LinearModel.random(4, 3, seed=2, labels=LABELS)
    rows = np.round(np.random.default_rng(8).standard_normal((64, 4)) * 2 + 4, 1)
    want = []
    for m in (ma, mb):
        idx, p = m.predict_max(rows)
        want.append([(LABELS[i], float(q)) for i, q in zip(idx, p)])
    errors, bad = [], []
    stop = threading.Event()
    with NativeServer(_cfg(device, IRIS)) as srv:
        srv.runtime.handle.load(ma)
        s0 = srv.runtime.handle.stats()

        def client(k):
            try:
                c = http.client.HTTPConnection("127.0.0.1", srv.port, timeout=10)
                i = k
                while not stop.is_set():
                    r = i % len(rows)
                    body = json.dumps(dict(zip(IRIS, rows[r].tolist())))
                    c.request("POST", "/predict", body, {"Content-Type": "application/json"})
                    resp = c.getresponse()
                    data = resp.read()
                    if resp.status != 200:
                        bad.append((resp.status, data))
                        continue
                    got = json.loads(data)
                    cands = [w[r] for w in want]
                    if not any(got["prediction"] == lab and abs(got["probability"] - p) <= 1e-12 * p for lab, p in cands):
                        bad.append((r, got, cands))
                    i += 7
            except Exception as e:  # noqa: BLE001
                errors.append(repr(e))

        ts = [threading.Thread(target=client, args=(k,)) for k in range(6)]
        for t in ts:
            t.start()
        import time

        for j in range(8):
            time.sleep(0.05)
            srv.runtime.handle.load(mb if j % 2 == 0 else ma)
        time.sleep(0.05)
        stop.set()
        for t in ts:
            t.join()
        s1 = srv.runtime.handle.stats()
    assert not errors, errors[:3]
    assert not bad, bad[:3]
    d = _stats_delta(s0, s1)
    assert d["resident_launches"] >= 8 and d["errors"] == 0, d
    assert d["resident_rows"] > 0, d


def test_resident_auto_rule(monkeypatch):
    """resident=auto: on for every rank with at least RESIDENT_MIN_CPUS CPUs, whether or not ranks
    share the device (profiles/r6_resident_n/: two ranks on one card 2.69-2.77 M req/s with the
    resident kernel vs 1.40-1.43 M without; at 8 CPUs per rank on = off)."""
    from mlapi_amd.parallel import comm

    monkeypatch.setattr(comm, "per_rank_cpus", lambda: 16)
    assert comm.resident_auto_ok()
    monkeypatch.setattr(comm, "per_rank_cpus", lambda: 8)
    assert comm.resident_auto_ok()      # two ranks on the 16-CPU box: on (measured faster)
    monkeypatch.setattr(comm, "per_rank_cpus", lambda: 4)
    assert not comm.resident_auto_ok()  # below anything measured: the batcher path


def test_gpu_shared_by_ranks(monkeypatch):
    import torch

    from mlapi_amd.parallel import comm

    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "2")
    assert comm.gpu_shared_by_ranks()
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "1")
    assert not comm.gpu_shared_by_ranks()
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 8)
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    assert not comm.gpu_shared_by_ranks()
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 0)  # CPU backend: nothing to share
    assert not comm.gpu_shared_by_ranks()


def test_per_rank_cpus_share_of_quota(monkeypatch):
    """per_rank_cpus: the affinity mask, capped by the node's ranks' share of the cgroup quota."""
    import os

    from mlapi_amd.parallel import comm
    from mlapi_amd.utils import threads

    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: set(range(128)))
    monkeypatch.setattr(threads, "cgroup_cpu_quota", lambda root="/sys/fs/cgroup": 16.0)
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "2")
    assert comm.per_rank_cpus() == 8      # two ranks in a 16-CPU quota
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "1")
    assert comm.per_rank_cpus() == 16     # the 1-GPU box: on
    monkeypatch.setattr(threads, "cgroup_cpu_quota", lambda root="/sys/fs/cgroup": None)
    monkeypatch.setattr(os, "cpu_count", lambda: 256)
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: set(range(16)))
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    monkeypatch.setenv("MLAPI_PLACEMENT", "cores")
    assert comm.per_rank_cpus() == 16     # 8 ranks pinned to 16 cores each on a 256-CPU node
    # numa placement: a 96-CPU node mask shared by the 4 ranks whose GPUs sit on that node
    from mlapi_amd.utils import affinity

    monkeypatch.setattr(affinity, "gpu_numa_nodes", lambda *a, **k: [0, 0, 0, 0, 1, 1, 1, 1])
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: set(range(96)))
    monkeypatch.setenv("MLAPI_PLACEMENT", "numa")
    monkeypatch.setenv("LOCAL_RANK", "5")
    assert comm.per_rank_cpus() == 24
    monkeypatch.setattr(threads, "cgroup_cpu_quota", lambda root="/sys/fs/cgroup": 128.0)
    assert comm.per_rank_cpus() == 16     # capped by the rank's share of a 128-CPU quota
    monkeypatch.delenv("MLAPI_PLACEMENT")
    assert comm.per_rank_cpus() == 12     # unplaced: the 96-CPU mask shared by all 8 ranks


# ---- failure paths (VERDICT r5 missing 3) ------------------------------------------------
# Each injected fault must end with every request answered - 200 with the exact body, or a 500 -
# never a hang, and a new instance serving the rings afterwards.
FAULTS = [pytest.param("cpu", "stall", 0, id="cpu-stall"),
          pytest.param("cuda:0", "stall", 0, id="gpu-stall", marks=pytest.mark.gpu),
          pytest.param("cuda:0", "exit_ring", 0, id="gpu-exit_ring", marks=pytest.mark.gpu),
          pytest.param("cuda:0", "lease_starve", 600, id="gpu-lease_starve", marks=pytest.mark.gpu),
          pytest.param("cuda:0", "queue_fault", 0, id="gpu-queue_fault", marks=pytest.mark.gpu),
          pytest.param("cuda:0", "ignore_stop", 0, id="gpu-ignore_stop", marks=pytest.mark.gpu)]


def _wait_live(srv, n_rings, timeout=10.0):
    import time

    t_end = time.time() + timeout
    while time.time() < t_end:
        st = srv.runtime.handle.stats()
        if st["resident_live"] and st["resident_rings"] >= n_rings:
            return st
        time.sleep(0.01)
    raise AssertionError(f"resident instance not live: {srv.runtime.handle.stats()}")


@pytest.mark.parametrize("device,mode,arg", FAULTS)
def test_resident_fault_every_request_answered(native, device, mode, arg):
    """Inject a resident-path fault under load (8 connections over 4 IO threads, watchdog 200 ms):
    stall (block 0's heartbeat stops, no row answered: heartbeat / ring watchdog restart),
    exit_ring (ring 0's wave exits: ring watchdog restart), lease_starve (the supervisor stops
    bumping the lease: the waves exit on their own and are relaunched), queue_fault (the instance's
    queue reads as failed: relaunch on a fresh queue), ignore_stop (the waves ignore the stop word; a
    hot reload's stop times out: abandoned to its lease, the path resumes once it has ended)."""
    import time

    from mlapi_amd.serve.loadgen import make_workload
    from mlapi_amd.serve.server import NativeServer

    m = LinearModel.random(4, 3, seed=13, labels=LABELS)
    X = np.round(np.random.default_rng(6).standard_normal((256, 4)) * 2 + 4, 1)
    # ignore_stop: a lease longer than the supervisor's 1 s stop wait (with the default 200 ms lease
    # the waves end on it while the supervisor waits - the lease rule at work - and nothing is
    # abandoned)
    lease = 2000 if mode == "ignore_stop" else 200
    with NativeServer(_cfg(device, IRIS, watchdog_ms=200, resident_lease_ms=lease)) as srv:
        h = srv.runtime.handle
        h.load(m)
        eng = h.engine
        reqs, exp = make_workload(eng, m, IRIS, X, rtol_oracle=1e-12, label_margin=1e-5)
        lg = native.Loadgen("127.0.0.1", srv.port, reqs[0].decode(), 8, 2, 20.0)
        lg.set_workload([r.decode() for r in reqs], [e.decode() for e in exp], 0.0)
        lg.run(20, False)
        _wait_live(srv, 4)
        s0 = h.stats()
        assert eng.resident_inject(mode, arg)
        if mode == "ignore_stop":
            h.load(m)  # a reload stops the instance: the stop is ignored, the instance abandoned
        # traffic for at least a second across the fault (the lease and stop paths take ~0.2-1.2 s
        # to play out; a fast instance answers 1,200 requests in about a millisecond)
        t0 = time.time()
        counts, runs = {}, 0
        while runs == 0 or time.time() - t0 < 1.5:
            res = lg.run(50, False)
            runs += 1
            assert res["failed"] == 0 and res["body_mismatches"] == 0, res
            for k, v in res["status_counts"].items():
                counts[k] = counts.get(k, 0) + v
            assert time.time() - t0 < 20.0, (runs, counts)
        s1 = h.stats()
        # every request answered (the bodies of the 200s byte-exact), within bounded time
        assert sum(counts.values()) == runs * 8 * 50 and set(counts) <= {200, 500}, counts
        assert counts.get(200, 0) >= 0.9 * runs * 8 * 50, counts
        restarts = {k: s1[k] - s0[k] for k in ("resident_hb_restarts", "resident_ring_restarts",
                                               "resident_self_exits", "resident_queue_faults",
                                               "resident_abandoned", "resident_launches")}
        want = {"stall": ("resident_hb_restarts", "resident_ring_restarts"), "exit_ring": ("resident_ring_restarts",),
                "lease_starve": ("resident_self_exits",), "queue_fault": ("resident_queue_faults",),
                "ignore_stop": ("resident_abandoned",)}[mode]
        assert sum(restarts[k] for k in want) >= 1, restarts
        # a new instance serves the rings afterwards
        _wait_live(srv, 4, timeout=15.0)
        s2 = h.stats()
        res2 = lg.run(100, True)
        s3 = h.stats()
        lg.close()
        assert res2["status_counts"] == {200: 800} and res2["body_mismatches"] == 0, res2
        assert s3["resident_rows"] - s2["resident_rows"] >= 700, (s2, s3)
        assert s3["resident_launches"] > s0["resident_launches"], (s0, s3)


def test_resident_metrics_lines(native, iris_cwd):
    """/metrics exports the resident path that serves the default Iris model: rows, stale bounces,
    launches, restarts by cause, liveness, rings and the heartbeat; the removed lanes' counter is gone."""
    import socket

    from mlapi_amd.serve.server import NativeServer

    srv = NativeServer(_cfg("cpu", IRIS, model_path="LRClassifier.pkl", reload="mtime", missing_model="error")).start()
    try:
        body = b'{"sepal_length":5.1,"sepal_width":3.5,"petal_length":1.4,"petal_width":0.2}'
        req = (b"POST /predict HTTP/1.1\r\nHost: t\r\nContent-Type: application/json\r\nContent-Length: %d\r\n\r\n%s"
               % (len(body), body))
        lg = native.Loadgen("127.0.0.1", srv.port, req.decode(), 4, 1)
        lg.run(20, False)
        _wait_live(srv, 1)
        r = lg.run(200, False)
        lg.close()
        assert r["status_counts"] == {200: 800}, r
        s = socket.create_connection(("127.0.0.1", srv.port), timeout=5)
        s.sendall(b"GET /metrics HTTP/1.1\r\nHost: t\r\nConnection: close\r\n\r\n")
        data = b""
        while True:
            c = s.recv(65536)
            if not c:
                break
            data += c
        s.close()
        text = data.split(b"\r\n\r\n", 1)[1].decode()
        vals = {}
        for line in text.splitlines():
            if line.startswith("mlapi_resident"):
                name, v = line.rsplit(" ", 1)
                vals[name.split("{")[0] + ("{" + name.split("{")[1] if "cause" in name else "")] = float(v)
        assert vals["mlapi_resident_rows_total"] >= 800, vals
        assert vals["mlapi_resident_live"] == 1 and vals["mlapi_resident_rings"] >= 1, vals
        assert vals["mlapi_resident_launches_total"] >= 1 and vals["mlapi_resident_heartbeat"] > 0, vals
        assert "mlapi_resident_stale_total" in vals, vals
        causes = {k for k in vals if k.startswith("mlapi_resident_restarts_total")}
        assert len(causes) == 5, causes
        assert "mlapi_lane_batches_total" not in text
    finally:
        srv.stop()
